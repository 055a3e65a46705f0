"""TEST INFRASTRUCTURE: the register-resident engine (fluidframework_amd/csrc/reg_engine.hpp) built for
the CPU with the emulated wave backend (tests/native/reg_cpu.cpp), plus helpers that replay the same
op records on the oracle and render both results as the segment-table JSON of mte_segments_json."""
import ctypes
import json
import os
import subprocess

import numpy as np

from fluidframework_amd import mte
from oracle import OracleDoc, _op_dtype

_HERE = os.path.dirname(os.path.abspath(__file__))
_NATIVE = os.path.join(_HERE, "native")
_LIB = os.path.join(_NATIVE, "_build", "libregcpu.so")
_lib = None

F_REMOVED, F_MARKER, F_OVL = 1 << 16, 1 << 17, 1 << 18
REG_HANDOFF = 101

DOCRES = np.dtype([("status", "<i4"), ("failing_seq", "<i4"), ("ops", "<u4"), ("msgs", "<u4"), ("min_seq", "<i4"),
                   ("cur_seq", "<i4"), ("height", "<u4"), ("n_lb", "<u4"), ("arena_sel", "<u4"), ("arena_top", "<u4"),
                   ("map_next", "<u4"), ("seg_next", "<u4"), ("heap_size", "<u4"), ("n_gc", "<u4"), ("out_off", "<u4"),
                   ("n_segs", "<u4"), ("max_lb", "<u4"), ("mode", "<u4"), ("spill_why", "<u4"), ("text_off", "<u4"),
                   ("cu_n", "<u4")])


def lib():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", _NATIVE], check=True)
        L = ctypes.CDLL(_LIB)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.regcpu_replay.restype = u64
        L.regcpu_replay.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, vp, u32, vp, u64, vp]
        L.regcpu_replay_paged.restype = u64
        L.regcpu_replay_paged.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, vp, u32, vp, u64, vp, u32]
        L.regcpu_replay_props.restype = u64
        L.regcpu_replay_props.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, vp, u32, vp, u64, vp, u32,
                                          vp, u32, vp, vp, vp, u32, u32, u32, vp, u32]
        L.regcpu_replay_split.restype = u64
        L.regcpu_replay_split.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, vp, u32, vp, u64, vp, u32, u32, u64, vp,
                                          vp, u32, vp, vp, vp, u32, u32, u32, vp]
        L.regcpu_docres_size.restype = u32
        L.regcpu_heap.restype = u32
        L.regcpu_heap.argtypes = [vp, u32, vp]
        assert L.regcpu_docres_size() == DOCRES.itemsize
        _lib = L
    return _lib


def replay(ops, pay, arena_cap=None, pool_rows=None):
    """Replay op records (numpy, oracle._op_dtype) + payload (uint16) on the CPU build of the register
    engine (pool_rows: the PAGED engine of k_rows, rows from a pool of that many). Returns (stop
    index, DocRes record, rows [(vis, aux, ovl)], text uint16 array)."""
    ops = np.ascontiguousarray(ops, dtype=_op_dtype())
    pay = np.ascontiguousarray(pay, dtype=np.uint16)
    n = len(ops)
    seg_cap = 3 * n + 8
    if arena_cap is None:
        arena_cap = 6 * len(pay) + 4096
    cap = seg_cap
    vis = np.zeros((cap, 4), dtype=np.uint32)
    aux = np.zeros((cap, 4), dtype=np.uint32)
    ovl = np.zeros(cap, dtype=np.uint64)
    text = np.zeros(len(pay) + 16, dtype=np.uint16)
    res = np.zeros(1, dtype=DOCRES)
    pay1 = np.concatenate([pay, np.zeros(1, dtype=np.uint16)])
    args = (ops.ctypes.data, n, pay1.ctypes.data, len(pay), seg_cap, arena_cap, vis.ctypes.data, aux.ctypes.data,
            ovl.ctypes.data, cap, text.ctypes.data, len(text), res.ctypes.data)
    if pool_rows is None:
        at = lib().regcpu_replay(*args)
    else:
        at = lib().regcpu_replay_paged(*args, pool_rows)
    r = res[0]
    k = int(r["n_segs"])
    return at, r, (vis[:k], aux[:k], ovl[:k]), text


class GenProps:
    """The generator's property sets (mte_host.cpp build_generator_props, the oracle's genPropset):
    ids 1..28 one key, then 294 two-key sets; value id 0 = null. Interned tables for the engine and
    the oracle's batch."""
    KEYS = ["bold", "italic", "color", "size"]
    VALS = ["null", "true", "false", '"red"', '"blue"', "10", "12"]  # value ids
    GEN_VALS = [1, 2, 3, 4, 5, 6, 0]  # the generator's value order -> value id

    def __init__(self):
        sets = [[]]
        for k in range(4):
            for v in range(7):
                sets.append([(k, self.GEN_VALS[v])])
        for k1 in range(4):
            for k2 in range(k1 + 1, 4):
                for v1 in range(7):
                    for v2 in range(7):
                        sets.append([(k1, self.GEN_VALS[v1]), (k2, self.GEN_VALS[v2])])
        ps, keys, vals = [], [], []
        for st in sets:
            ps += [len(keys), len(st)]
            for k, v in st:
                keys.append(k)
                vals.append(v)
        self.propsets = np.array(ps, dtype=np.uint32)
        self.prop_keys = np.array(keys + [0], dtype=np.uint32)
        self.prop_vals = np.array(vals + [0], dtype=np.uint32)
        self.val_flags = np.array([1 if v in ("null", "false") else 0 for v in self.VALS], dtype=np.uint32)
        self.n_propsets = len(sets)

    def render(self, rec):
        """A map record [n, k0, v0, ...] as JSON.stringify of the property object."""
        n = int(rec[0])
        return "{" + ",".join('"%s":%s' % (self.KEYS[int(rec[1 + 2 * i])], self.VALS[int(rec[2 + 2 * i])])
                              for i in range(n)) + "}"


def replay_props(ops, pay, gp, pool_rows=0, map_words=16, wide=False):
    """The PROPS engine (k_rows' property-carrying form) on the CPU: (stop index, DocRes, rows, text,
    per-row map records)."""
    ops = np.ascontiguousarray(ops, dtype=_op_dtype())
    pay = np.ascontiguousarray(pay, dtype=np.uint16)
    n = len(ops)
    seg_cap = 3 * n + 8
    arena_cap = 6 * len(pay) + 4096
    cap = seg_cap
    vis = np.zeros((cap, 4), dtype=np.uint32)
    aux = np.zeros((cap, 4), dtype=np.uint32)
    ovl = np.zeros(cap, dtype=np.uint64)
    text = np.zeros(len(pay) + 16, dtype=np.uint16)
    res = np.zeros(1, dtype=DOCRES)
    omaps = np.zeros((cap, map_words), dtype=np.uint32)
    pay1 = np.concatenate([pay, np.zeros(1, dtype=np.uint16)])
    map_cap = 2 * n + 64
    at = lib().regcpu_replay_props(ops.ctypes.data, n, pay1.ctypes.data, len(pay), seg_cap, arena_cap,
                                   vis.ctypes.data, aux.ctypes.data, ovl.ctypes.data, cap, text.ctypes.data,
                                   len(text), res.ctypes.data, pool_rows, gp.propsets.ctypes.data, gp.n_propsets,
                                   gp.prop_keys.ctypes.data, gp.prop_vals.ctypes.data, gp.val_flags.ctypes.data,
                                   len(gp.VALS), map_words, map_cap, omaps.ctypes.data, int(wide))
    r = res[0]
    k = int(r["n_segs"])
    return at, r, (vis[:k], aux[:k], ovl[:k]), text, omaps[:k]


def replay_split(ops, pay, cut, kind=0, pool_rows=16, gp=None, map_words=16, arena_cap=None):
    """Incremental replay on the CPU build (reg_engine.hpp ckpt_save / ckpt_resume): ops [0, cut) then a
    fresh engine continuing from the checkpoint. kind 0 lean, 1 paged, 2 PROPS, 3 PROPS paged, 6 / 7
    PROPS + WIDE. Returns (stop index, op the continuation started from, DocRes, rows, text, maps)."""
    ops = np.ascontiguousarray(ops, dtype=_op_dtype())
    pay = np.ascontiguousarray(pay, dtype=np.uint16)
    n = len(ops)
    seg_cap = 3 * n + 8
    if arena_cap is None:
        arena_cap = 6 * len(pay) + 4096
    cap = seg_cap
    vis = np.zeros((cap, 4), dtype=np.uint32)
    aux = np.zeros((cap, 4), dtype=np.uint32)
    ovl = np.zeros(cap, dtype=np.uint64)
    text = np.zeros(len(pay) + 16, dtype=np.uint16)
    res = np.zeros(1, dtype=DOCRES)
    omaps = np.zeros((cap, map_words), dtype=np.uint32)
    pay1 = np.concatenate([pay, np.zeros(1, dtype=np.uint16)])
    resumed = ctypes.c_uint64(0)
    z = np.zeros(2, dtype=np.uint32)
    g = gp if gp is not None else None
    at = lib().regcpu_replay_split(ops.ctypes.data, n, pay1.ctypes.data, len(pay), seg_cap, arena_cap,
                                   vis.ctypes.data, aux.ctypes.data, ovl.ctypes.data, cap, text.ctypes.data, len(text),
                                   res.ctypes.data, pool_rows, kind, cut, ctypes.addressof(resumed),
                                   (g.propsets if g else z).ctypes.data, g.n_propsets if g else 0,
                                   (g.prop_keys if g else z).ctypes.data, (g.prop_vals if g else z).ctypes.data,
                                   (g.val_flags if g else z).ctypes.data, len(g.VALS) if g else 0, map_words,
                                   2 * n + 64, omaps.ctypes.data)
    r = res[0]
    k = int(r["n_segs"])
    return at, int(resumed.value), r, (vis[:k], aux[:k], ovl[:k]), text, omaps[:k]


def rows_json(rows, text, names, props=None):
    """The engine's rows as mte_segments_json renders them (host DocView, mte_host.cpp)."""
    vis, aux, ovl = rows
    out = []
    for i in range(len(vis)):
        ln, seq, rseq, meta = (int(x) for x in vis[i])
        toff = int(aux[i][1])
        kind = "M" if meta & F_MARKER else "T"
        row = {"kind": kind}
        if kind == "M":
            row["refType"] = toff & 0xFFFF
        else:
            row["text"] = text[toff: toff + ln].tobytes().decode("utf-16-le", "surrogatepass")
        row["len"] = ln
        row["seq"] = seq if seq < 2 ** 31 else seq - 2 ** 32
        row["client"] = names[meta & 0xFF]
        if meta & F_REMOVED:
            row["removedSeq"] = rseq if rseq < 2 ** 31 else rseq - 2 ** 32
            row["removedClient"] = names[(meta >> 8) & 0xFF]
        row["overlap"] = [names[b] for b in range(64) if (int(ovl[i]) >> b) & 1]
        row["props"] = props(i) if props and int(aux[i][0]) else None
        out.append(row)
    return json.dumps(out, separators=(",", ":"), ensure_ascii=False)


def engine_text(rows, text):
    vis, _, _ = rows
    total = sum(int(v[0]) for v in vis if not (int(v[3]) & (F_MARKER | F_REMOVED)))
    out = []
    for i in range(len(vis)):
        ln, _, _, meta = (int(x) for x in vis[i])
        if meta & (F_MARKER | F_REMOVED):
            continue
        toff = int(rows[1][i][1])
        out.append(text[toff: toff + ln].tobytes().decode("utf-16-le", "surrogatepass"))
    s = "".join(out)
    assert len(s.encode("utf-16-le")) // 2 == total
    return s


class OneDocBatch:
    """A one-document mte_batch over numpy op records + payload, clients named `names` by short id
    (index 0 = the observer). Keeps its buffers alive."""

    def __init__(self, ops, pay, names, gp=None):
        self.ops = np.ascontiguousarray(ops, dtype=_op_dtype())
        self.pay = np.ascontiguousarray(pay, dtype=np.uint16)
        self.opo = (ctypes.c_uint64 * 2)(0, len(self.ops))
        self.pyo = (ctypes.c_uint64 * 2)(0, len(self.pay))
        self.propsets = (ctypes.c_uint32 * 2)(0, 0)
        self.keyo = (ctypes.c_uint64 * 1)(0)
        self.valo = (ctypes.c_uint64 * 2)(0, 4)
        self.valtext = ctypes.create_string_buffer(b"null")
        enc = [n.encode() for n in names]
        offs = [0]
        for e in enc:
            offs.append(offs[-1] + len(e))
        self.cli = (ctypes.c_uint32 * 2)(0, len(names))
        self.cno = (ctypes.c_uint64 * len(offs))(*offs)
        self.cn = ctypes.create_string_buffer(b"".join(enc))
        b = mte.mte_batch()
        b.n_docs = 1
        b.doc_op_offsets = ctypes.cast(self.opo, ctypes.POINTER(ctypes.c_uint64))
        b.ops = self.ops.ctypes.data
        b.doc_payload_offsets = ctypes.cast(self.pyo, ctypes.POINTER(ctypes.c_uint64))
        b.payload = ctypes.cast(self.pay.ctypes.data, ctypes.POINTER(ctypes.c_uint16))
        b.n_propsets = 1
        b.propsets = ctypes.addressof(self.propsets)
        b.n_keys = 0
        b.key_offsets = ctypes.cast(self.keyo, ctypes.POINTER(ctypes.c_uint64))
        b.n_vals = 1
        b.val_offsets = ctypes.cast(self.valo, ctypes.POINTER(ctypes.c_uint64))
        b.val_text = ctypes.addressof(self.valtext)
        b.doc_client_offsets = ctypes.cast(self.cli, ctypes.POINTER(ctypes.c_uint32))
        b.client_name_offsets = ctypes.cast(self.cno, ctypes.POINTER(ctypes.c_uint64))
        b.client_names = ctypes.addressof(self.cn)
        if gp is not None:  # the generator's property sets
            self.gp = gp
            b.n_propsets = gp.n_propsets
            b.propsets = gp.propsets.ctypes.data
            b.prop_keys = gp.prop_keys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
            b.prop_vals = gp.prop_vals.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
            kt = [('"%s"' % k).encode() for k in gp.KEYS]
            vt = [v.encode() for v in gp.VALS]
            self.keyo = (ctypes.c_uint64 * (len(kt) + 1))(*np.cumsum([0] + [len(x) for x in kt]).tolist())
            self.keytext = ctypes.create_string_buffer(b"".join(kt))
            self.valo = (ctypes.c_uint64 * (len(vt) + 1))(*np.cumsum([0] + [len(x) for x in vt]).tolist())
            self.valtext = ctypes.create_string_buffer(b"".join(vt))
            b.n_keys = len(kt)
            b.key_offsets = ctypes.cast(self.keyo, ctypes.POINTER(ctypes.c_uint64))
            b.key_text = ctypes.addressof(self.keytext)
            b.n_vals = len(vt)
            b.val_offsets = ctypes.cast(self.valo, ctypes.POINTER(ctypes.c_uint64))
            b.val_text = ctypes.addressof(self.valtext)
        self.batch = b

    def oracle(self):
        o = OracleDoc(self.names()[0])
        o.apply_batch(ctypes.addressof(self.batch), 0)
        return o

    def names(self):
        return [self.cn.raw[self.cno[i]: self.cno[i + 1]].decode() for i in range(len(self.cno) - 1)]


def generated(kind, gid, n_ops, n_clients=8, seed=0):
    """A synthetic document log (the GPU generator restated by the oracle): op records + payload."""
    return OracleDoc().generate(kind, gid, n_ops, n_clients=n_clients, seed=seed, export=True)


def compare(ops, pay, names=None, arena_cap=None, pool_rows=None):
    """Replay on the CPU register engine and on the oracle; assert identical status, segment table
    and text. Returns the engine's DocRes record."""
    if names is None:
        nc = int(ops["client"].max()) if len(ops) else 0
        names = ["__observer__"] + [f"w{i}" for i in range(1, max(nc, 1) + 1)]
    at, res, rows, text = replay(ops, pay, arena_cap=arena_cap, pool_rows=pool_rows)
    assert int(res["status"]) != REG_HANDOFF, f"register engine handed off at op {at} (n_lb {res['n_lb']})"
    ob = OneDocBatch(ops, pay, names)
    o = ob.oracle()
    code, err, fseq = o.status()
    assert int(res["status"]) == code, f"status engine={int(res['status'])}@{int(res['failing_seq'])} oracle={code}@{fseq} ({err})"
    if code:
        assert int(res["failing_seq"]) == fseq
        return res
    js, oj = rows_json(rows, text, names), o.segments_json()
    if js != oj:
        a, b = json.loads(js), json.loads(oj)
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                raise AssertionError(f"segment {i} differs:\n engine {x}\n oracle {y}\n ({len(a)} vs {len(b)} rows)")
        raise AssertionError(f"segment count differs: {len(a)} vs {len(b)}")
    assert engine_text(rows, text) == o.text()
    return res


def compare_props(ops, pay, pool_rows=0, wide=False):
    """The PROPS engine against the oracle on a generated kind-3 log: status, segment table with
    each segment's properties (JSON.stringify of the map), text. Returns the DocRes record."""
    gp = GenProps()
    nc = int(ops["client"].max()) if len(ops) else 0
    names = ["__observer__"] + [f"w{i}" for i in range(1, max(nc, 1) + 1)]
    at, res, rows, text, omaps = replay_props(ops, pay, gp, pool_rows=pool_rows, wide=wide)
    assert int(res["status"]) != REG_HANDOFF, f"handed off at op {at} (n_lb {res['n_lb']})"
    o = OneDocBatch(ops, pay, names, gp=gp).oracle()
    code, err, fseq = o.status()
    assert int(res["status"]) == code, f"status engine={int(res['status'])} oracle={code} ({err})"
    if code:
        return res
    js, oj = rows_json(rows, text, names, props=lambda i: gp.render(omaps[i])), o.segments_json()
    if js != oj:
        a, b = json.loads(js), json.loads(oj)
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                raise AssertionError(f"segment {i} differs:\n engine {x}\n oracle {y}\n ({len(a)} vs {len(b)} rows)")
        raise AssertionError(f"segment count differs: {len(a)} vs {len(b)}")
    assert engine_text(rows, text) == o.text()
    return res
