"""Python host mirror of the engine's C ABI (include/mte.h), via ctypes.

The reference surface this mirrors is @fluidframework/merge-tree's Client
(packages/dds/merge-tree/src/client.ts): applyMsg (:805-827), getText via MergeTreeTextHelper
(textSegment.ts:154-172), snapshot -> SnapshotV1 (snapshotV1.ts:85-247). Replay always runs on the
GPU through libmte.so; there is no Python or CPU fallback: if the library or the device is missing
these classes raise.
"""
import ctypes
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MTE_LIB=<name> selects an alternative build in _build/<name>/ (csrc/Makefile `prof`: the
# phase-profiling build, engine.hpp MTE_PROFILE; `variant`: experiments with extra flags)
LIB_PATH = os.path.join(_HERE, "_build", os.environ.get("MTE_LIB", ""), "libmte.so")
PROF_NAMES = ["apply", "resolve", "insert_slot", "range", "zamboni", "scour", "heap", "find_seg", "map", "pack",
              "fetch", "lru", "text", "alloc", "ops", "total",
              "n_resolve", "n_dirty", "n_scour", "n_scour_changed", "n_pack", "n_pop", "n_push", "n_split_blk",
              "op_ins", "op_rem", "edit", "split", "zam_edit", "zam_msn", "res_blocks", "res_slot", "blen_dirty",
              "scour_chain", "scour_write", "loop", "n_ins", "n_rem", "apply_pre", "apply_post"]
PROF_SLOTS = 40

MTE_OP_INSERT, MTE_OP_REMOVE, MTE_OP_ANNOTATE, MTE_OP_INSERT_MARKER, MTE_OP_NOOP = 0, 1, 2, 3, 4
MTE_F_END_OF_MSG, MTE_F_REWRITE = 1, 2
DOC_STATUS = {0: "ok", 1: "insert failed", 2: "sequence order", 3: "capacity", 4: "unsupported", 5: "not run"}

OP_DTYPE = np.dtype([("seq", "<i4"), ("ref_seq", "<i4"), ("msn", "<i4"), ("pos1", "<i4"), ("a", "<i4"),
                     ("b", "<u4"), ("props", "<u4"), ("type", "u1"), ("client", "u1"), ("flags", "<u2")])
assert OP_DTYPE.itemsize == 32


class MteError(RuntimeError):
    pass


RCCL_ID_BYTES = 128  # MTE_RCCL_ID_BYTES


def rccl_unique_id():
    buf = (ctypes.c_uint8 * RCCL_ID_BYTES)()
    rc = lib().mte_rccl_unique_id(buf)
    if rc:
        raise MteError(f"mte_rccl_unique_id failed ({rc})")
    return bytes(buf)


def rccl_comm_destroy(comm):
    if comm:
        lib().mte_rccl_comm_destroy(comm)


class mte_batch(ctypes.Structure):
    _fields_ = [
        ("n_docs", ctypes.c_uint32),
        ("doc_op_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("ops", ctypes.c_void_p),
        ("doc_payload_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("payload", ctypes.POINTER(ctypes.c_uint16)),
        ("n_propsets", ctypes.c_uint32),
        ("propsets", ctypes.c_void_p),
        ("prop_keys", ctypes.POINTER(ctypes.c_uint32)),
        ("prop_vals", ctypes.POINTER(ctypes.c_uint32)),
        ("n_keys", ctypes.c_uint32),
        ("key_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("key_text", ctypes.c_void_p),
        ("n_vals", ctypes.c_uint32),
        ("val_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("val_text", ctypes.c_void_p),
        ("doc_client_offsets", ctypes.POINTER(ctypes.c_uint32)),
        ("client_name_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("client_names", ctypes.c_void_p),
        ("doc_msg_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("msg_first_op", ctypes.POINTER(ctypes.c_uint64)),
        ("msg_text_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("msg_text", ctypes.c_void_p),
    ]


class mte_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("chunk_size", ctypes.c_uint32), ("snapshot_format", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 5)]


class mte_stats(ctypes.Structure):
    _fields_ = [("docs", ctypes.c_uint64), ("ops", ctypes.c_uint64), ("messages", ctypes.c_uint64),
                ("failed_docs", ctypes.c_uint64), ("kernel_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double)]


class mte_doc_summary(ctypes.Structure):
    _fields_ = [("checksum", ctypes.c_uint64), ("ops", ctypes.c_uint32), ("length", ctypes.c_uint32),
                ("segments", ctypes.c_uint32), ("snapshot_bytes", ctypes.c_uint32), ("status", ctypes.c_int32),
                ("doc_id", ctypes.c_uint32)]


SUMMARY_DTYPE = np.dtype([("checksum", "<u8"), ("ops", "<u4"), ("length", "<u4"), ("segments", "<u4"),
                          ("snapshot_bytes", "<u4"), ("status", "<i4"), ("doc_id", "<u4")])

# Every symbol declared in include/mte.h (checked by tests/test_abi.py).
EXPORTS = ["mte_abi_version", "mte_build_info", "mte_create", "mte_destroy", "mte_last_error", "mte_load",
           "mte_replay", "mte_generate", "mte_generate_ids", "mte_export_batch", "mte_doc_status", "mte_text", "mte_length", "mte_segments",
           "mte_snapshot_v1", "mte_snapshot_legacy", "mte_snapshot_shared_string", "mte_summaries", "mte_rccl_unique_id",
           "mte_rccl_comm_create", "mte_rccl_comm_destroy", "mte_gather_summaries", "mte_gather_summaries_alloc", "mte_free", "mte_builder_create", "mte_builder_add_doc", "mte_builder_add_doc_from_summary", "mte_builder_add_container_log", "mte_builder_doc_path",
           "mte_builder_add_matrix_log", "mte_builder_add_matrix_from_summary", "mte_snapshot_matrix",
           "mte_builder_batch", "mte_builder_open_doc", "mte_builder_append_messages", "mte_retain",
           "mte_builder_error", "mte_builder_destroy"]

_lib = None


def lib():
    """Load libmte.so; raises (never falls back) when the HIP build is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MteError(f"libmte.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
        L.mte_abi_version.restype = ctypes.c_int
        L.mte_build_info.restype = ctypes.c_char_p
        L.mte_create.argtypes = [ctypes.POINTER(mte_config), ctypes.POINTER(vp)]
        L.mte_destroy.argtypes = [vp]
        L.mte_last_error.argtypes = [vp]
        L.mte_last_error.restype = ctypes.c_char_p
        L.mte_load.argtypes = [vp, ctypes.POINTER(mte_batch)]
        L.mte_replay.argtypes = [vp, ctypes.POINTER(mte_stats)]
        L.mte_generate.argtypes = [vp, u32, u32, u32, ctypes.POINTER(u32), u32, u64]
        L.mte_generate_ids.argtypes = [vp, u32, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32), u32, u64]
        L.mte_export_batch.argtypes = [vp, ctypes.POINTER(mte_batch)]
        L.mte_doc_status.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]
        L.mte_text.argtypes = [vp, u32, ctypes.c_void_p, sz, ctypes.POINTER(sz)]
        L.mte_length.argtypes = [vp, u32, ctypes.POINTER(u64)]
        L.mte_segments_json.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.mte_snapshot_v1.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz), ctypes.POINTER(u32)]
        L.mte_snapshot_shared_string.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.mte_snapshot_legacy.argtypes = [vp, u32, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.mte_summaries.argtypes = [vp, ctypes.c_void_p, sz]
        L.mte_rccl_unique_id.argtypes = [ctypes.c_void_p]
        L.mte_rccl_comm_create.argtypes = [vp, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.mte_rccl_comm_destroy.argtypes = [vp]
        L.mte_rccl_comm_destroy.restype = None
        L.mte_gather_summaries.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_void_p, sz, ctypes.POINTER(sz)]
        L.mte_gather_summaries_alloc.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.mte_free.argtypes = [vp]
        L.mte_free.restype = None
        L.mte_doc_result.argtypes = [vp, u32, ctypes.c_void_p, sz]
        L.mte_run_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64), ctypes.POINTER(u32)]
        L.mte_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
        L.mte_get_info.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
        L.mte_profile.argtypes = [vp, ctypes.c_void_p, sz]
        L.mte_wave_selftest.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, u32]
        L.mte_last_kernel_ms.argtypes = [vp]
        L.mte_last_kernel_ms.restype = ctypes.c_double
        L.mte_builder_create.argtypes = [ctypes.POINTER(vp)]
        L.mte_builder_add_doc.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz]
        L.mte_builder_add_doc_from_summary.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        L.mte_builder_add_container_log.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_uint32)]
        L.mte_builder_add_matrix_log.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz]
        if hasattr(L, "mte_builder_add_matrix_from_summary"):  # (A/B runs load older experiment builds)
            L.mte_builder_add_matrix_from_summary.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        L.mte_snapshot_matrix.argtypes = [vp, u32, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.mte_builder_doc_path.argtypes = [vp, ctypes.c_uint32]
        L.mte_builder_doc_path.restype = ctypes.c_char_p
        L.mte_builder_batch.argtypes = [vp, ctypes.POINTER(mte_batch)]
        if hasattr(L, "mte_builder_open_doc"):  # (A/B runs load older experiment builds)
            L.mte_builder_open_doc.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
            L.mte_builder_append_messages.argtypes = [vp, ctypes.c_uint32, ctypes.c_char_p, sz]
            L.mte_retain.argtypes = [vp, ctypes.c_int]
        L.mte_builder_error.argtypes = [vp]
        L.mte_builder_error.restype = ctypes.c_char_p
        L.mte_builder_destroy.argtypes = [vp]
        _lib = L
    return _lib


class Builder:
    """Op-log ingestion: per-document JSON arrays of ISequencedDocumentMessage -> mte_batch."""

    def __init__(self):
        h = ctypes.c_void_p()
        rc = lib().mte_builder_create(ctypes.byref(h))
        if rc:
            raise MteError(f"mte_builder_create: {rc}")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().mte_builder_destroy(self._h)
            self._h = None

    def add_doc(self, messages, observer="__observer__"):
        """messages: list of message dicts or a JSON string. observer='' => local, non-collab edits."""
        text = messages if isinstance(messages, (str, bytes)) else json.dumps(messages, separators=(",", ":"),
                                                                               ensure_ascii=False)
        b = text.encode() if isinstance(text, str) else text
        rc = lib().mte_builder_add_doc(self._h, observer.encode(), b, len(b))
        if rc:
            raise MteError(f"mte_builder_add_doc: {rc}: {lib().mte_builder_error(self._h).decode()}")

    def add_doc_from_summary(self, summary, messages=None, observer="__observer__"):
        """Catch-up: a SnapshotV1 summary (ITree JSON text or dict) then an op-log suffix
        (SnapshotLoader.initialize + applyMsg, snapshotLoader.ts:38-216)."""
        def enc(x):
            if x is None:
                return None
            t = x if isinstance(x, (str, bytes)) else json.dumps(x, separators=(",", ":"), ensure_ascii=False)
            return t.encode() if isinstance(t, str) else t
        s, m = enc(summary), enc(messages)
        rc = lib().mte_builder_add_doc_from_summary(self._h, observer.encode(), s, len(s), m, len(m) if m else 0)
        if rc:
            raise MteError(f"mte_builder_add_doc_from_summary: {rc}: {lib().mte_builder_error(self._h).decode()}")

    def add_container_log(self, messages, observer="readonly"):
        """Container messages (messages*.json concatenated) -> one document per attached SharedString
        channel (clientReplayTool.ts:113-192). Returns the channel paths of the documents added."""
        t = messages if isinstance(messages, (str, bytes)) else json.dumps(messages, separators=(",", ":"),
                                                                            ensure_ascii=False)
        t = t.encode() if isinstance(t, str) else t
        n = ctypes.c_uint32()
        rc = lib().mte_builder_add_container_log(self._h, observer.encode(), t, len(t), ctypes.byref(n))
        if rc:
            raise MteError(f"mte_builder_add_container_log: {rc}: {lib().mte_builder_error(self._h).decode()}")
        first = self.n_docs() - n.value
        return [lib().mte_builder_doc_path(self._h, first + i).decode() for i in range(n.value)]

    def add_matrix_log(self, messages, observer="readonly"):
        """SharedMatrix messages -> two documents, the rows then the cols PermutationVector
        (matrix.ts:548-560). Returns their indices (rows, cols)."""
        t = messages if isinstance(messages, (str, bytes)) else json.dumps(messages, separators=(",", ":"),
                                                                            ensure_ascii=False)
        t = t.encode() if isinstance(t, str) else t
        rc = lib().mte_builder_add_matrix_log(self._h, observer.encode(), t, len(t))
        if rc:
            raise MteError(f"mte_builder_add_matrix_log: {rc}: {lib().mte_builder_error(self._h).decode()}")
        n = self.n_docs()
        return n - 2, n - 1

    def add_matrix_from_summary(self, summary, messages=None, observer="readonly"):
        """SharedMatrix.loadCore (matrix.ts:528-546) from a summary ITree, then its message suffix:
        two documents, rows then cols. Returns their indices (rows, cols)."""
        def enc(x):
            t = x if isinstance(x, (str, bytes)) else json.dumps(x, separators=(",", ":"), ensure_ascii=False)
            return t.encode() if isinstance(t, str) else t
        s = enc(summary)
        m = enc(messages) if messages is not None else None
        rc = lib().mte_builder_add_matrix_from_summary(self._h, observer.encode(), s, len(s), m, len(m) if m else 0)
        if rc:
            raise MteError(f"mte_builder_add_matrix_from_summary: {rc}: {lib().mte_builder_error(self._h).decode()}")
        n = self.n_docs()
        return n - 2, n - 1

    def open_doc(self, observer="__observer__"):
        """An open document: its log grows with append() (Client.applyMsg, client.ts:805-836); every
        batch() sees it as it is. No other document may be added after it. Returns its index."""
        d = ctypes.c_uint32()
        rc = lib().mte_builder_open_doc(self._h, observer.encode(), ctypes.byref(d))
        if rc:
            raise MteError(f"mte_builder_open_doc: {rc}: {lib().mte_builder_error(self._h).decode()}")
        return d.value

    def append(self, doc, messages):
        """More sequenced messages onto open document `doc` (all or none of them)."""
        text = messages if isinstance(messages, (str, bytes)) else json.dumps(messages, separators=(",", ":"),
                                                                               ensure_ascii=False)
        b = text.encode() if isinstance(text, str) else text
        rc = lib().mte_builder_append_messages(self._h, doc, b, len(b))
        if rc:
            raise MteError(f"mte_builder_append_messages: {rc}: {lib().mte_builder_error(self._h).decode()}")

    def n_docs(self):
        b = mte_batch()
        lib().mte_builder_batch(self._h, ctypes.byref(b))
        return b.n_docs

    def batch(self):
        b = mte_batch()
        lib().mte_builder_batch(self._h, ctypes.byref(b))
        b._owner = self  # keep the builder (which owns the memory) alive
        return b


def batch_ops(b):
    """numpy view of a batch's op records (valid while the owner lives)."""
    n = b.doc_op_offsets[b.n_docs]
    if n == 0:
        return np.zeros(0, OP_DTYPE)
    buf = (ctypes.c_char * (n * 32)).from_address(b.ops)
    return np.frombuffer(buf, dtype=OP_DTYPE, count=n)


class Engine:
    """One engine per GPU: loads/generates batches, replays them with the HIP kernel."""

    def __init__(self, device=0, chunk_size=10000, snapshot_format=0):
        """snapshot_format 0: SnapshotV1 (newMergeTreeSnapshotFormat); 1: SnapshotLegacy (the reference's
        default, client.ts:930-941)."""
        cfg = mte_config(device=device, chunk_size=chunk_size, snapshot_format=snapshot_format)
        h = ctypes.c_void_p()
        rc = lib().mte_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise MteError(f"mte_create failed ({rc}): no HIP device? The replay path has no CPU fallback.")
        self._h = h
        self.n_docs = 0

    def close(self):
        if getattr(self, "_h", None):
            lib().mte_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc, what):
        if rc:
            raise MteError(f"{what} failed ({rc}): {lib().mte_last_error(self._h).decode()}")

    def load(self, batch):
        self._check(lib().mte_load(self._h, ctypes.byref(batch)), "mte_load")
        self.n_docs = batch.n_docs

    def generate(self, kind, n_docs, n_ops, n_clients=8, seed=0, ops_per_doc=None, doc_ids=None):
        """Synthetic logs on the device. doc_ids: GLOBAL ids (default 0..n_docs-1); a
        document's log depends only on its id, op count, kind, n_clients and seed."""
        arr = ids = None
        if ops_per_doc is not None:
            arr = (ctypes.c_uint32 * n_docs)(*[int(x) for x in ops_per_doc])
        if doc_ids is not None:
            ids = (ctypes.c_uint32 * n_docs)(*[int(x) for x in doc_ids])
        self._check(lib().mte_generate_ids(self._h, kind, n_docs, n_ops, arr, ids, n_clients, seed), "mte_generate")
        self.n_docs = n_docs

    def replay(self):
        st = mte_stats()
        self._check(lib().mte_replay(self._h, ctypes.byref(st)), "mte_replay")
        return {"docs": st.docs, "ops": st.ops, "messages": st.messages, "failed_docs": st.failed_docs,
                "kernel_ms": st.kernel_ms, "h2d_ms": st.h2d_ms}

    def export_batch(self):
        b = mte_batch()
        self._check(lib().mte_export_batch(self._h, ctypes.byref(b)), "mte_export_batch")
        b._owner = self
        return b

    def status(self, doc):
        c, s = ctypes.c_int32(), ctypes.c_int64()
        self._check(lib().mte_doc_status(self._h, doc, ctypes.byref(c), ctypes.byref(s)), "mte_doc_status")
        return c.value, s.value

    def text(self, doc):
        n = ctypes.c_size_t()
        self._check(lib().mte_text(self._h, doc, None, 0, ctypes.byref(n)), "mte_text")
        buf = (ctypes.c_uint16 * max(n.value, 1))()
        self._check(lib().mte_text(self._h, doc, buf, n.value, ctypes.byref(n)), "mte_text")
        return np.frombuffer(buf, dtype=np.uint16, count=n.value).tobytes().decode("utf-16-le", "surrogatepass")

    def length(self, doc):
        """Client.getLength(): the observer's visible length, markers counting 1."""
        n = ctypes.c_uint64()
        self._check(lib().mte_length(self._h, doc, ctypes.byref(n)), "mte_length")
        return n.value

    def _str_call(self, fn, doc, *extra):
        n = ctypes.c_size_t()
        self._check(fn(self._h, doc, None, 0, ctypes.byref(n), *extra), fn.__name__)
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(fn(self._h, doc, buf, n.value + 1, ctypes.byref(n), *extra), fn.__name__)
        return buf.raw[: n.value].decode("utf-8")

    def segments_json(self, doc):
        return self._str_call(lib().mte_segments_json, doc)

    def snapshot_json(self, doc):
        nb = ctypes.c_uint32()
        return self._str_call(lib().mte_snapshot_v1, doc, ctypes.byref(nb))

    def snapshot_legacy(self, doc, catch_up_name="catchupOps"):
        """SnapshotLegacy ITree (header, body, catch-up messages) after a snapshot_format 1 replay."""
        n = ctypes.c_size_t()
        name = catch_up_name.encode()
        self._check(lib().mte_snapshot_legacy(self._h, doc, name, None, 0, ctypes.byref(n)), "mte_snapshot_legacy")
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(lib().mte_snapshot_legacy(self._h, doc, name, buf, n.value + 1, ctypes.byref(n)), "mte_snapshot_legacy")
        return buf.raw[: n.value].decode("utf-8")

    def snapshot_matrix(self, rows_doc, cols_doc):
        """SharedMatrix summary tree (matrix.ts:405-430) of a rows / cols document pair."""
        n = ctypes.c_size_t()
        self._check(lib().mte_snapshot_matrix(self._h, rows_doc, cols_doc, None, 0, ctypes.byref(n)), "mte_snapshot_matrix")
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(lib().mte_snapshot_matrix(self._h, rows_doc, cols_doc, buf, n.value + 1, ctypes.byref(n)),
                    "mte_snapshot_matrix")
        return buf.raw[: n.value].decode("utf-8")

    def snapshot_shared_string(self, doc):
        """SharedString summary tree: {"header": intervals "{}", "content": SnapshotV1 tree}."""
        return self._str_call(lib().mte_snapshot_shared_string, doc)

    def summaries(self):
        out = np.zeros(self.n_docs, dtype=SUMMARY_DTYPE)
        self._check(lib().mte_summaries(self._h, out.ctypes.data, self.n_docs), "mte_summaries")
        return out

    def gather_summaries(self, rank=0, world=1, comm=None):
        """Every rank's summary records over RCCL (mte_gather_summaries), rank order. Collective."""
        # one collective call; the library allocates the records (mte_gather_summaries_alloc)
        n, p = ctypes.c_size_t(), ctypes.c_void_p()
        self._check(lib().mte_gather_summaries_alloc(self._h, rank, world, comm, ctypes.byref(p), ctypes.byref(n)),
                    "mte_gather_summaries_alloc")
        try:
            raw = ctypes.string_at(p, n.value * SUMMARY_DTYPE.itemsize) if n.value else b""
        finally:
            lib().mte_free(p)
        return np.frombuffer(raw, dtype=SUMMARY_DTYPE).copy()

    def rccl_comm(self, unique_id, rank, world):
        """RCCL communicator on this engine's device from a MTE_RCCL_ID_BYTES id (rank 0's)."""
        c = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * RCCL_ID_BYTES).from_buffer_copy(bytes(unique_id))
        self._check(lib().mte_rccl_comm_create(self._h, buf, rank, world, ctypes.byref(c)), "mte_rccl_comm_create")
        return c

    DOC_RESULT_FIELDS = ["status", "failing_seq", "ops", "msgs", "min_seq", "cur_seq", "height", "n_lb",
                         "arena_sel", "arena_top", "map_next", "seg_next", "heap_size", "n_gc", "out_off", "n_segs",
                         "max_lb", "mode", "spill_why", "text_off", "cu_n"]

    def doc_result(self, doc):
        buf = (ctypes.c_int32 * 21)()
        self._check(lib().mte_doc_result(self._h, doc, buf, ctypes.sizeof(buf)), "mte_doc_result")
        return dict(zip(self.DOC_RESULT_FIELDS, list(buf)))

    def run_info(self):
        """Last replay/generate: docs that outgrew the LDS plan (re-run HBM-resident) and pass times."""
        sp, a, b, rows, co = ctypes.c_uint32(), ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint32()
        self._check(lib().mte_run_info(self._h, ctypes.byref(sp), ctypes.byref(a), ctypes.byref(b),
                                       ctypes.byref(rows), ctypes.byref(co)), "mte_run_info")
        out = {"spilled": sp.value, "continued": co.value, "lds_ms": a.value, "hbm_ms": b.value,
               "out_rows": rows.value}
        for k in ("lds_groups", "hbm_waves", "hbm_docs", "slot_bytes", "slots", "solo", "solo_us", "solo_lead_us",
                  "solo_tail_us", "lean", "out_text", "rows", "rows_restart_pushed", "rows_restart_popped",
                  "rows_continued"):
            try:
                out[k] = self.get_info(k)
            except MteError:  # (a key an older library build does not know)
                out[k] = -1
        return out

    def get_info(self, key):
        v = ctypes.c_int64()
        self._check(lib().mte_get_info(self._h, key.encode(), ctypes.byref(v)), "mte_get_info")
        return v.value

    def profile(self):
        """Per-doc phase cycle counters (MTE_LIB=prof build), shape (n_docs, len(PROF_NAMES))."""
        out = np.zeros((self.n_docs, PROF_SLOTS), dtype=np.uint64)
        self._check(lib().mte_profile(self._h, out.ctypes.data, out.size), "mte_profile")
        return out[:, : len(PROF_NAMES)]

    def set_option(self, key, value):
        """"force_hbm" (HBM-resident waves only), "pool_limit" (LDS leaf blocks per CU),
        "hbm_waves_per_cu" (HBM-resident waves beside each LDS workgroup), "slot_budget_mb",
        "solo_max" / "solo_min_ops" (solo route), "lean" (0 = never the property-free kernels)."""
        self._check(lib().mte_set_option(self._h, key.encode(), int(value)), "mte_set_option")

    def last_kernel_ms(self):
        return lib().mte_last_kernel_ms(self._h)

    def retain(self, on=True):
        """mte_retain: keep every document's replay state, so a replay of logs that extend the last
        pass's replays only their new ops (get_info("resumed_docs") / "resumed_ops" say how many)."""
        self._check(lib().mte_retain(self._h, int(bool(on))), "mte_retain")

    def wave_selftest(self, values):
        values = np.ascontiguousarray(values, dtype=np.uint32)
        nw = values.size // 64
        out = np.zeros(nw * 64 * 5, dtype=np.uint32)
        self._check(lib().mte_wave_selftest(self._h, values.ctypes.data, out.ctypes.data, nw), "mte_wave_selftest")
        return out.reshape(nw, 5, 64)


class MergeTreeClient:
    """Client-shaped facade for one document (client.ts:42), incremental like Client.applyMsg
    (client.ts:805-836): messages are parsed onto an open builder document as they come, and a read
    (getText, getLength, snapshot) after new messages replays on the GPU only the ops since the last
    read, continuing the document's state from the previous pass (mte_retain). Without new messages
    a read reuses the last results. A document the row engines cannot hold (summary loads, relative
    positions, 64+ clients, ...) replays from its first op instead: same results, not incremental."""

    def __init__(self, observer="__observer__", device=0):
        self.observer = observer
        self._builder = Builder()
        self._doc = self._builder.open_doc(observer)
        self._pending = []
        self._engine = None
        self._device = device
        self._dirty = True
        self.replays = 0  # passes run (a read after new messages runs one)

    def applyMsg(self, msg):  # noqa: N802 (reference name)
        self._pending.append(msg)
        self._dirty = True

    def _run(self):
        if self._dirty:
            if self._pending:
                self._builder.append(self._doc, self._pending)
                self._pending = []
            if self._engine is None:
                self._engine = Engine(self._device)
                self._engine.retain(True)
            self._engine.load(self._builder.batch())
            self._engine.replay()
            self.replays += 1
            code, seq = self._engine.status(0)
            if code:
                raise MteError(f"replay failed at seq {seq}: {DOC_STATUS.get(code, code)}")
            self._dirty = False
        return self._engine

    def resumed_ops(self):
        """Op records the last read did not replay again (continued from the previous pass)."""
        return self._run().get_info("resumed_ops")

    def getText(self):  # noqa: N802
        return self._run().text(0)

    def getLength(self):  # noqa: N802
        return self._run().length(0)

    def snapshot(self):
        return json.loads(self._run().snapshot_json(0))
