"""Helpers that build ISequencedDocumentMessage logs (protocol.ts:126-166)."""
import json


def msg(client, seq, ref_seq, contents, msn=0, mtype="op"):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref_seq,
            "minimumSequenceNumber": msn, "clientSequenceNumber": 1, "type": mtype, "term": 1,
            "timestamp": 0, "traces": [], "origin": None, "contents": contents}


def ins(pos, seg):
    return {"pos1": pos, "seg": seg, "type": 0}


def rem(a, b):
    return {"pos1": a, "pos2": b, "type": 1}


def ann(a, b, props, combining=None):
    c = {"pos1": a, "pos2": b, "props": props, "type": 2}
    if combining:
        c["combiningOp"] = combining
    return c


def group(*ops):
    return {"ops": list(ops), "type": 3}


def dumps(msgs):
    # JSON.parse(JSON.stringify(msg)) is the wire form (test-runtime-utils mocks.ts:233)
    return json.dumps(msgs, separators=(",", ":"), ensure_ascii=False)


class TestString:
    __test__ = False
    """Mirror of snapshot.spec.ts TestString: one writer, refSeq = previous seq, positions in the
    writer's own view; replayed here by an observer."""

    def __init__(self, writer="fakeId"):
        self.writer = writer
        self.seq = 0
        self.min_seq = 0
        self.msgs = []
        self.text = ""

    def _queue(self, contents, increase_msn):
        ref = self.seq
        self.seq += 1
        if increase_msn:
            self.min_seq = self.seq
        self.msgs.append(msg(self.writer, self.seq, ref, contents, self.min_seq))

    def insert(self, pos, text, increase_msn):
        self._queue(ins(pos, text), increase_msn)
        self.text = self.text[:pos] + text + self.text[pos:]

    def append(self, text, increase_msn):
        self.insert(len(self.text), text, increase_msn)

    def remove_range(self, a, b, increase_msn):
        self._queue(rem(a, b), increase_msn)
        self.text = self.text[:a] + self.text[b:]
