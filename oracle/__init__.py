"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/mt_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (fluidframework_amd/) never does. See oracle/mt_oracle.cpp for what the oracle
restates and how it is pinned against the reference's own golden vectors.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, cp, i32, u32, u64 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
        L.orc_new.restype = vp
        L.orc_new.argtypes = [cp]
        L.orc_free.argtypes = [vp]
        L.orc_str_free.argtypes = [vp]
        L.orc_apply_json.argtypes = [vp, cp, ctypes.c_size_t]
        L.orc_apply_batch.argtypes = [vp, vp, u32]
        L.orc_load_summary.argtypes = [vp, cp, ctypes.c_size_t]
        L.orc_local_insert_text.argtypes = [vp, i32, cp, cp]
        L.orc_local_insert_marker.argtypes = [vp, i32, i32, cp]
        L.orc_local_remove.argtypes = [vp, i32, i32]
        L.orc_local_annotate.argtypes = [vp, i32, i32, cp]
        L.orc_get_length.argtypes = [vp]
        L.orc_get_length_at.argtypes = [vp, i32, i32]
        for f in ("orc_text", "orc_segments_json"):
            getattr(L, f).restype = vp
            getattr(L, f).argtypes = [vp]
        L.orc_snapshot_json.restype = vp
        L.orc_snapshot_json.argtypes = [vp, u32]
        L.orc_apply_matrix_json.argtypes = [vp, cp, ctypes.c_size_t, cp]
        L.orc_snapshot_vector_json.restype = vp
        L.orc_snapshot_vector_json.argtypes = [vp, u32]
        L.orc_snapshot_legacy_json.restype = vp
        L.orc_snapshot_legacy_json.argtypes = [vp, u32, cp]
        L.orc_checksum.restype = u64
        L.orc_checksum.argtypes = [vp, u32]
        L.orc_ops_applied.restype = u64
        L.orc_ops_applied.argtypes = [vp]
        L.orc_status.argtypes = [vp, cp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_longlong)]
        L.orc_stats.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.orc_generate.argtypes = [vp, u32, u32, u64, u32, u64, vp, vp, ctypes.POINTER(u64)]
        L.orc_generate_batch.restype = u64
        L.orc_generate_batch.argtypes = [u32, vp, vp, u32, u32, u64, i32, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int32)]
        L.orc_replay_list.restype = u64
        L.orc_replay_list.argtypes = [vp, vp, u32, i32, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int32), i32]
        L.orc_matrix_new.restype = vp
        L.orc_matrix_new.argtypes = [cp]
        L.orc_matrix_free.argtypes = [vp]
        L.orc_matrix_apply_json.argtypes = [vp, cp, ctypes.c_size_t]
        L.orc_matrix_vector.restype = vp
        L.orc_matrix_vector.argtypes = [vp, i32]
        L.orc_matrix_load_summary.argtypes = [vp, cp, ctypes.c_size_t]
        L.orc_matrix_snapshot_json.restype = vp
        L.orc_matrix_snapshot_json.argtypes = [vp, u32]
        L.orc_replay_batch.restype = u64
        L.orc_replay_batch.argtypes = [vp, u32, u32, i32, cp, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int32), i32]
        _lib = L
    return _lib


def _take(ptr):
    s = ctypes.string_at(ptr).decode("utf-8")
    lib().orc_str_free(ptr)
    return s


class OracleDoc:
    """One document replayed by the oracle. observer=None => local, non-collaborative tree."""

    def __init__(self, observer="__observer__"):
        self._h = lib().orc_new(observer.encode() if observer is not None else None)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    # -- input
    def apply_json(self, text):
        b = text.encode() if isinstance(text, str) else text
        return lib().orc_apply_json(self._h, b, len(b))

    def load_summary(self, text):
        """SnapshotLoader: resume from a summary ITree (JSON text); the doc must be fresh."""
        b = text.encode() if isinstance(text, str) else text
        return lib().orc_load_summary(self._h, b, len(b))

    def generate(self, kind, gid, n_ops, n_clients=8, seed=0, export=False):
        """Synthetic log (the GPU generator restated), replayed into this (fresh) document. With
        export=True returns (ops numpy records, payload uint16 array)."""
        import numpy as np

        ops = np.zeros(n_ops, dtype=_op_dtype()) if export else None
        pay = np.zeros(8 * n_ops + 1, dtype=np.uint16) if export else None
        pl = ctypes.c_uint64()
        lib().orc_generate(self._h, kind, gid, n_ops, n_clients, seed,
                           ops.ctypes.data if export else None, pay.ctypes.data if export else None, ctypes.byref(pl))
        return (ops, pay[: pl.value]) if export else None

    def apply_batch(self, batch_ptr, doc):
        return lib().orc_apply_batch(self._h, batch_ptr, doc)

    def insert_text_local(self, pos, text, props_json=None):
        return lib().orc_local_insert_text(self._h, pos, text.encode(), props_json.encode() if props_json else None)

    def insert_marker_local(self, pos, ref_type, props_json=None):
        return lib().orc_local_insert_marker(self._h, pos, ref_type, props_json.encode() if props_json else None)

    def remove_local(self, start, end):
        return lib().orc_local_remove(self._h, start, end)

    def annotate_local(self, start, end, props_json):
        return lib().orc_local_annotate(self._h, start, end, props_json.encode())

    # -- outputs
    def length(self):
        return lib().orc_get_length(self._h)

    def length_at(self, ref_seq, short_client):
        return lib().orc_get_length_at(self._h, ref_seq, short_client)

    def text(self):
        return _take(lib().orc_text(self._h))

    def segments_json(self):
        return _take(lib().orc_segments_json(self._h))

    def snapshot_json(self, chunk=10000):
        return _take(lib().orc_snapshot_json(self._h, chunk))

    def apply_matrix_json(self, text, target):
        """SharedMatrix messages (matrix.ts:548-560): this doc is its `target` ("rows" / "cols") vector."""
        b = text.encode() if isinstance(text, str) else text
        return lib().orc_apply_matrix_json(self._h, b, len(b), target.encode())

    def snapshot_vector_json(self, chunk=10000):
        """PermutationVector.snapshot (permutationvector.ts:260-273)."""
        return _take(lib().orc_snapshot_vector_json(self._h, chunk))

    def snapshot_legacy_json(self, chunk=10000, catch_up_name="catchupOps"):
        """SnapshotLegacy ITree (snapshotlegacy.ts): header, body, catch-up messages blob."""
        return _take(lib().orc_snapshot_legacy_json(self._h, chunk, catch_up_name.encode()))

    def checksum(self, chunk=10000):
        return lib().orc_checksum(self._h, chunk)

    def ops_applied(self):
        return lib().orc_ops_applied(self._h)

    def status(self):
        buf = ctypes.create_string_buffer(512)
        fs = ctypes.c_longlong(0)
        code = lib().orc_status(self._h, buf, 512, ctypes.byref(fs))
        return code, buf.value.decode(), fs.value

    def stats(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        lib().orc_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return {"leafCount": a.value, "removedLeafCount": b.value, "maxHeight": c.value}


class _VectorView(OracleDoc):
    """One PermutationVector of an OracleMatrix (owned by it)."""

    def __init__(self, owner, handle):
        self._owner = owner
        self._h = handle

    def __del__(self):
        pass


class OracleMatrix:
    """A SharedMatrix replayed by the oracle (matrix.ts:548-605): both PermutationVectors, their
    HandleTables and the cells SparseArray2D."""

    def __init__(self, observer="__observer__"):
        self._h = lib().orc_matrix_new(observer.encode())
        self.rows = _VectorView(self, lib().orc_matrix_vector(self._h, 0))
        self.cols = _VectorView(self, lib().orc_matrix_vector(self._h, 1))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_matrix_free(self._h)
            self._h = None

    def apply_json(self, text):
        b = text.encode() if isinstance(text, str) else text
        return lib().orc_matrix_apply_json(self._h, b, len(b))

    def load_summary(self, text):
        """SharedMatrix.loadCore (matrix.ts:528-546) from a summary ITree JSON (a fresh matrix)."""
        b = text.encode() if isinstance(text, str) else text
        return lib().orc_matrix_load_summary(self._h, b, len(b))

    def snapshot_json(self, chunk=10000):
        """SharedMatrix.snapshotCore (matrix.ts:405-433) ITree JSON."""
        return _take(lib().orc_matrix_snapshot_json(self._h, chunk))


def _op_dtype():
    import numpy as np

    return np.dtype([("seq", "<i4"), ("ref_seq", "<i4"), ("msn", "<i4"), ("pos1", "<i4"), ("a", "<i4"),
                     ("b", "<u4"), ("props", "<u4"), ("type", "u1"), ("client", "u1"), ("flags", "<u2")])


def generate_batch(kind, gids, n_ops, n_clients=8, seed=0, threads=1):
    """Generate + replay documents with global ids `gids` (op counts n_ops) on the CPU; returns
    (ops, checksums[list], statuses[list])."""
    import numpy as np

    g = np.ascontiguousarray(gids, dtype=np.uint32)
    n = np.ascontiguousarray(n_ops, dtype=np.uint64)
    k = len(g)
    cs = (ctypes.c_uint64 * max(k, 1))()
    st = (ctypes.c_int32 * max(k, 1))()
    ops = lib().orc_generate_batch(kind, g.ctypes.data, n.ctypes.data, k, n_clients, seed, threads, cs, st)
    return ops, list(cs)[:k], list(st)[:k]


def replay_list(batch_ptr, docs, threads=1, with_snapshot=False):
    """Replay the listed documents of an mte_batch (list order, dynamic queue); returns ops applied."""
    import numpy as np

    d = np.ascontiguousarray(docs, dtype=np.uint32)
    return lib().orc_replay_list(batch_ptr, d.ctypes.data, len(d), threads, None, None, 1 if with_snapshot else 0)


def replay_batch(batch_ptr, d0, d1, threads=1, with_snapshot=True):
    """Replay docs [d0, d1) of an mte_batch; returns (ops, checksums[list], statuses[list])."""
    n = d1 - d0
    cs = (ctypes.c_uint64 * max(n, 1))()
    st = (ctypes.c_int32 * max(n, 1))()
    ops = lib().orc_replay_batch(batch_ptr, d0, d1, threads, None, cs, st, 1 if with_snapshot else 0)
    return ops, list(cs)[:n], list(st)[:n]
