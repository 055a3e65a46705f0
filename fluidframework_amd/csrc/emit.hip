// SnapshotV1 emission on the device: SnapshotV1.extractSync + emit
// (snapshotV1.ts:57-247, snapshotChunks.ts) over each document's final segments, which
// Engine::finish gathered in document order (rows: vis / aux / overlap, the row's property map, the
// text of every row). One wave per document:
//   1. entries (extractSync, :170-228): removed segments at or below minSeq are elided; settled
//      segments (seq <= minSeq, not removed) coalesce into the previous one when both are text,
//      TextSegment.canAppend holds (no trailing '\n', either side <= 256 chars) and matchProperties
//      holds; every other segment is a merge-info entry ({"json":…, seq/client above minSeq,
//      removedSeq/removedClient});
//   2. chunks (:108-168): entries fill a chunk until its length reaches `chunk` characters;
//   3. bytes: the header blob (with headerMetadata) and body_i blobs, JSON exactly as
//      JSON.stringify writes them (UTF-8; '"', '\\', control characters escaped, unpaired
//      surrogates as \uXXXX; property objects in JS key order: array-index keys ascending, then
//      insertion order).
// Legacy format (EmitParams::legacy, SnapshotLegacy.extractSync + emit, snapshotlegacy.ts:103-238): the
// entries are the view at minSeq only (segments inserted at or below minSeq and not removed at or
// below it, coalesced the same way; the others are skipped without breaking a run), a header chunk of
// at least `chunk` characters and ONE body chunk with the rest, in MergeTreeChunkLegacy JSON
// (serializeAsMinSupportedVersion, snapshotChunks.ts:75-111). The catch-up blob is the host's.
// The pass runs twice per list of documents: COUNT sizes every document's blobs (bytes, blob
// count), the host lays the documents out in the output pool, WRITE fills them. Byte-oriented,
// HBM-bound work: lanes encode 64 characters / copy 64 bytes per step, nothing is reshaped for MFMA.
#include "wave_hip.hpp"
#include "emit.h"

namespace mte {
using i64 = long long;

namespace {

struct Out {  // wave-uniform byte cursor; out == nullptr: count only
    char* out;
    u64 pos;
};

MTE_DEV void put_lit(Out& o, const char* s, u32 n) {
    const u32 L = lane_id();
    if (o.out)
        for (u32 i = L; i < n; i += 64) o.out[o.pos + i] = s[i];
    o.pos += n;
}
template <u32 N>
MTE_DEV void put(Out& o, const char (&s)[N]) {
    put_lit(o, s, N - 1);
}
MTE_DEV void put_bytes(Out& o, const char* src, u64 n) {
    const u32 L = lane_id();
    if (o.out)
        for (u64 i = L; i < n; i += 64) o.out[o.pos + i] = src[i];
    o.pos += n;
}
MTE_DEV void put_int(Out& o, i64 v) {  // Number::toString of an integer
    const bool neg = v < 0;
    u64 a = neg ? (u64)(-v) : (u64)v;
    u32 nd = 1;
    for (u64 t = a; t >= 10; t /= 10) nd++;
    const u32 L = lane_id();
    if (o.out) {
        if (neg && L == 0) o.out[o.pos] = '-';
        if (L < nd) {
            u64 t = a;
            for (u32 k = 0; k < nd - 1 - L; k++) t /= 10;
            o.out[o.pos + (neg ? 1 : 0) + L] = (char)('0' + t % 10);
        }
    }
    o.pos += nd + (neg ? 1 : 0);
}

MTE_DEV bool is_hi(u32 c) { return c >= 0xD800 && c < 0xDC00; }
MTE_DEV bool is_lo(u32 c) { return c >= 0xDC00 && c < 0xE000; }

// JSON string of n UTF-16 units (jsonlite.hpp quote, JSON.stringify's escaping), lane = unit
MTE_DEV void put_quoted(Out& o, const u16* s, u64 n) {
    const u32 L = lane_id();
    if (o.out && L == 0) o.out[o.pos] = '"';
    o.pos += 1;
    static constexpr char hx[] = "0123456789abcdef";
    for (u64 base = 0; base < n; base += 64) {
        const u64 i = base + L;
        const bool in = i < n;
        const u32 c = in ? s[i] : 0u;
        const u32 prev = in && i > 0 ? s[i - 1] : 0u;
        const u32 next = in && i + 1 < n ? s[i + 1] : 0u;
        u32 nb = 0;
        if (in) {
            if (c == '"' || c == '\\') nb = 2;
            else if (c < 0x20) nb = (c == '\b' || c == '\f' || c == '\n' || c == '\r' || c == '\t') ? 2 : 6;
            else if (is_hi(c)) nb = is_lo(next) ? 4 : 6;
            else if (is_lo(c)) nb = is_hi(prev) ? 0 : 6;
            else nb = c < 0x80 ? 1 : c < 0x800 ? 2 : 3;
        }
        const u32 incl = wave_scan_incl(nb);
        if (o.out && nb) {
            char* d = o.out + o.pos + (incl - nb);
            if (c == '"' || c == '\\') {
                d[0] = '\\';
                d[1] = (char)c;
            } else if (c < 0x20) {
                if (nb == 2) {
                    d[0] = '\\';
                    d[1] = c == '\b' ? 'b' : c == '\f' ? 'f' : c == '\n' ? 'n' : c == '\r' ? 'r' : 't';
                } else {
                    d[0] = '\\'; d[1] = 'u'; d[2] = '0'; d[3] = '0';
                    d[4] = hx[c >> 4]; d[5] = hx[c & 15];
                }
            } else if (nb == 6) {  // unpaired surrogate
                d[0] = '\\'; d[1] = 'u';
                d[2] = hx[(c >> 12) & 15]; d[3] = hx[(c >> 8) & 15]; d[4] = hx[(c >> 4) & 15]; d[5] = hx[c & 15];
            } else if (nb == 4) {  // surrogate pair -> one 4-byte sequence
                const u32 cp = 0x10000u + ((c - 0xD800u) << 10) + (next - 0xDC00u);
                d[0] = (char)(0xF0 | (cp >> 18));
                d[1] = (char)(0x80 | ((cp >> 12) & 0x3F));
                d[2] = (char)(0x80 | ((cp >> 6) & 0x3F));
                d[3] = (char)(0x80 | (cp & 0x3F));
            } else if (nb == 1) {
                d[0] = (char)c;
            } else if (nb == 2) {
                d[0] = (char)(0xC0 | (c >> 6));
                d[1] = (char)(0x80 | (c & 0x3F));
            } else {
                d[0] = (char)(0xE0 | (c >> 12));
                d[1] = (char)(0x80 | ((c >> 6) & 0x3F));
                d[2] = (char)(0x80 | (c & 0x3F));
            }
        }
        o.pos += wave_read(incl, 63);
    }
    if (o.out && L == 0) o.out[o.pos] = '"';
    o.pos += 1;
}

struct Doc {
    const EmitParams& p;
    u32 d;
    DocRes r;
    u64 row0;  // first row in the output pool
    MTE_DEV Doc(const EmitParams& pp, u32 dd) : p(pp), d(dd) {
        r = p.res[d];
        row0 = r.out_off;
    }
    MTE_DEV const u32* map(u64 row) const { return p.maps + row * p.map_words; }
    // matchProperties (properties.ts:62-93) on two rows' maps (host DocView::match_props)
    MTE_DEV bool val_match(u32 a, u32 b) const {
        if (a == b) return true;
        if (p.val_flags[b] & 2u) {
            const u32 j = p.val_objidx[b];
            return j != NONE && ((p.val_objmatch[a] >> j) & 1ull);
        }
        return false;
    }
    MTE_DEV bool match(u64 ra, bool ha, u64 rb, bool hb) const {
        if (!ha && !hb) return true;
        if (!ha || !hb || !p.maps) return false;
        const u32 *ma = map(ra), *mb = map(rb);
        const u32 n = ma[0];
        if (n != mb[0]) return false;
        for (u32 i = 0; i < n; i++) {
            bool found = false;
            for (u32 q = 0; q < n; q++)
                if (mb[1 + 2 * q] == ma[1 + 2 * i]) {
                    if (!val_match(ma[2 + 2 * i], mb[2 + 2 * q])) return false;
                    found = true;
                }
            if (!found) return false;
        }
        return true;
    }
    // {"k":v,...} in JS key order: array-index keys ascending (repeated minimum; the keys of a map are
    // distinct), then the others in insertion order. Up to (map_words - 1) / 2 pairs.
    MTE_DEV void put_props(Out& o, u64 row) const {
        const u32* m = map(row);
        const u32 cap = (p.map_words - 1) / 2;
        const u32 n = m[0] < cap ? m[0] : cap;
        bool first = true;
        auto pair = [&](u32 i) {
            if (!first) put(o, ",");
            first = false;
            const u32 key = m[1 + 2 * i], val = m[2 + 2 * i];
            put_bytes(o, p.key_text + p.key_off[key], p.key_off[key + 1] - p.key_off[key]);
            put(o, ":");
            put_bytes(o, p.val_text + p.val_off[val], p.val_off[val + 1] - p.val_off[val]);
        };
        put(o, "{");
        bool have = false;
        u32 last = 0;
        for (;;) {
            u32 best = NONE, bidx = 0;
            for (u32 i = 0; i < n; i++) {
                const u32 key = m[1 + 2 * i];
                if (!p.key_is_index[key]) continue;
                const u32 idx = p.key_index[key];
                if ((!have || idx > last) && (best == NONE || idx < bidx)) {
                    best = i;
                    bidx = idx;
                }
            }
            if (best == NONE) break;
            pair(best);
            last = bidx;
            have = true;
        }
        for (u32 i = 0; i < n; i++)
            if (!p.key_is_index[m[1 + 2 * i]]) pair(i);
        put(o, "}");
    }
    MTE_DEV void put_name(Out& o, u32 slot) const {  // getLongClientId, JSON-quoted
        if (slot == NONE) {  // NonCollabClient
            put(o, "\"original\"");
            return;
        }
        const u64 i = (u64)p.name_base[d] + slot;
        if (i >= p.name_base[d + 1]) {
            put(o, "\"\"");
            return;
        }
        put_bytes(o, p.names + p.name_off[i], p.name_off[i + 1] - p.name_off[i]);
    }
    MTE_DEV const u16* row_text(uint4 a) const { return p.text + r.text_off + a.y; }

    // 1. entries: ent[row0 + k] = (first row, last row, length, kind) with kind 0 a settled text
    // run, 1 a settled marker, 2 a merge-info segment, 3 a settled PermutationSegment run (its
    // canAppend, permutationvector.ts:88-94: two unallocated runs, or a handle run continuing the
    // previous one; aux.y = start handle, 0 = unallocated); returns the count
    MTE_DEV u32 build_entries() const {
        const u32 L = lane_id(), n = r.n_segs;
        const i32 minSeq = r.min_seq;
        // a row's last character matters only to TextSegment.canAppend's '\n' test: a document whose
        // payload has no '\n' skips the per-row text read (one 64-B HBM burst per row otherwise)
        const bool nl = p.cfg[d].has_nl != 0;
        u32 ne = 0;
        bool open = false, runText = false, runProps = false, runPerm = false;
        u32 runFirst = 0, runLast = 0, runLen = 0, runLast16 = 0, runStart = 0;
        auto close = [&]() {
            if (open && L == 0) p.ent[row0 + ne] = make_uint4(runFirst, runLast, runLen, runPerm ? 3u : runText ? 0u : 1u);
            ne += open ? 1u : 0u;
            open = false;
        };
        for (u32 base = 0; base < n; base += 64) {
            const u32 k = base + L;
            uint4 v = make_uint4(0, 0, 0, 0), a = make_uint4(0, 0, 0, 0);
            u32 last16 = 0;
            if (k < n) {
                v = p.vis[row0 + k];
                a = p.aux[row0 + k];
                if (nl && !(v.w & (F_MARKER | F_PERM)) && v.x) last16 = row_text(a)[v.x - 1];
            }
            const u32 cnt = n - base < 64 ? n - base : 64u;
            for (u32 j = 0; j < cnt; j++) {
                const u32 len = wave_read(v.x, j), seq = wave_read(v.y, j), rseq = wave_read(v.z, j);
                const u32 meta = wave_read(v.w, j), hasP = wave_read(a.x, j) != 0, start = wave_read(a.y, j);
                const bool removed = (meta & F_REMOVED) != 0, marker = (meta & F_MARKER) != 0, perm = (meta & F_PERM) != 0;
                const u32 row = base + j;
                if (removed && (i32)rseq <= minSeq) continue;  // elided (:184-186)
                if (p.legacy && (i32)seq > minSeq) continue;   // not in the view at minSeq (legacy :195-196)
                if ((i32)seq <= minSeq && (!removed || p.legacy)) {
                    if (open && (runPerm ? perm && start == (runStart ? runStart + runLen : 0u)
                                         : runText && !marker && !perm && !(runLen && runLast16 == u'\n') &&
                                               (runLen <= 256 || len <= 256)) &&
                        match(row0 + runFirst, runProps, row0 + row, hasP)) {
                        runLast = row;  // clone + append (:197-202)
                        runLen += len;
                        if (len) runLast16 = wave_read(last16, j);
                        continue;
                    }
                    close();
                    open = true;
                    runText = !marker && !perm;
                    runPerm = perm;
                    runStart = start;
                    runProps = hasP;
                    runFirst = runLast = row;
                    runLen = len;
                    runLast16 = wave_read(last16, j);
                } else {
                    close();
                    if (L == 0) p.ent[row0 + ne] = make_uint4(row, row, len, 2u);
                    ne++;
                }
            }
        }
        close();
        return ne;
    }

    // a row inside a run's row span that is not part of it: elided (removed at or below minSeq) or,
    // in the legacy view, inserted above minSeq
    MTE_DEV bool skipped(uint4 v) const {
        return ((v.w & F_REMOVED) && (i32)v.z <= r.min_seq) || (p.legacy && (i32)v.y > r.min_seq);
    }
    // the text of a settled run: its rows' text without the elided rows between them, gathered
    // contiguously (in place when no elided text lies inside)
    MTE_DEV const u16* run_text(uint4 e, u64& n) const {
        const u32 L = lane_id();
        const i32 minSeq = r.min_seq;
        const uint4 a0 = p.aux[row0 + e.x];
        const u16* first = row_text(a0);
        bool contiguous = true;
        for (u32 row = e.x + 1; row <= e.y && contiguous; row++) {
            const uint4 v = p.vis[row0 + row];
            contiguous = !(skipped(v) && !(v.w & F_MARKER) && v.x);
        }
        n = e.z;
        if (contiguous) return first;
        u16* dst = p.tscr + r.text_off + a0.y;
        u64 at = 0;
        for (u32 row = e.x; row <= e.y; row++) {
            const uint4 v = p.vis[row0 + row];
            if (skipped(v)) continue;
            const u16* src = row_text(p.aux[row0 + row]);
            for (u32 i = L; i < v.x; i += 64) dst[at + i] = src[i];
            at += v.x;
        }
        wave_sync();
        return dst;
    }
    // quoted text: the bytes from the text (WRITE), or from the rows' emission words (COUNT: tb, the
    // JSON size of the text without its quotes), so COUNT never reads text
    static constexpr u64 NO_TB = ~0ull;  // no precomputed size: COUNT reads the text (legacy format)
    MTE_DEV void put_text(Out& o, const u16* txt, u64 n, u64 tb) const {
        if (o.out || tb == NO_TB) put_quoted(o, txt, n);
        else o.pos += 2 + tb;
    }
    // Segment.toJSONObject of row `row` (vis v, aux a); txt / n / tb: its text (put_text)
    MTE_DEV void put_seg(Out& o, u32 row, uint4 v, uint4 a, const u16* txt, u64 n, u64 tb) const {
        if (v.w & F_PERM) {  // PermutationSegment.toJSONObject (permutationvector.ts:75-77): [length, start]
            put(o, "[");
            put_int(o, (i64)n);
            put(o, ",");
            put_int(o, a.y ? (i64)a.y : (i64)-2147483648LL);  // the start handle, or Handle.unallocated
            put(o, "]");
            return;
        }
        if (v.w & F_MARKER) {
            put(o, "{\"marker\":{\"refType\":");
            put_int(o, a.y & 0xFFFFu);
            put(o, "}");
            if (a.x) {
                put(o, ",\"props\":");
                put_props(o, row0 + row);
            }
            put(o, "}");
        } else if (a.x) {
            put(o, "{\"text\":");
            put_text(o, txt, n, tb);
            put(o, ",\"props\":");
            put_props(o, row0 + row);
            put(o, "}");
        } else {
            put_text(o, txt, n, tb);
        }
    }
    // one entry: e = (first row, last row, length, kind) as build_entries / Walk make them; tb the
    // JSON size of its text (COUNT)
    MTE_DEV void put_entry(Out& o, uint4 e, u64 tb = NO_TB) const {
        const uint4 v = p.vis[row0 + e.x], a = p.aux[row0 + e.x];
        if (e.w == 0 || e.w == 1 || e.w == 3) {  // settled: coalesced text / permutation run or a marker
            u64 n = e.w == 3 ? e.z : 0;
            const u16* t = e.w == 0 && (o.out || tb == NO_TB) ? run_text(e, n) : nullptr;
            if (e.w == 0 && !t) n = e.z;
            put_seg(o, e.x, v, a, t, n, tb);
            return;
        }
        const bool notext = (v.w & (F_MARKER | F_PERM)) != 0;
        put(o, "{\"json\":");
        put_seg(o, e.x, v, a, notext ? nullptr : row_text(a), (v.w & F_MARKER) ? 0 : v.x, tb);
        const bool collab = p.cfg[d].collab != 0;
        if ((i32)v.y > r.min_seq) {
            put(o, ",\"seq\":");
            put_int(o, (i32)v.y);
            put(o, ",\"client\":");
            put_name(o, collab ? (v.w & 0xffu) : NONE);
        }
        if (v.w & F_REMOVED) {
            put(o, ",\"removedSeq\":");
            put_int(o, (i32)v.z);
            put(o, ",\"removedClient\":");
            put_name(o, collab ? ((v.w >> 8) & 0xffu) : NONE);
        }
        put(o, "}");
    }

    // SnapshotLegacy.emit (snapshotlegacy.ts:103-182): getSeqLengthSegs for the header (>= chunk
    // characters) and one body with the rest; MergeTreeChunkLegacy keys in object-literal order,
    // headerMetadata (buildHeaderMetadataForLegecyChunk, snapshotChunks.ts:178-199) on the header only,
    // chunkMinSequenceNumber undefined (omitted)
    MTE_DEV u64 emit_legacy(u32 ne, char* out, u64* blob_off, u32& nblobs) const {
        const u32 L = lane_id();
        u64 total = 0;
        for (u32 q = 0; q < ne; q++) total += p.ent[row0 + q].z;
        u32 c1 = 0;
        u64 l1 = 0;
        while (l1 < p.chunk && c1 < ne) l1 += p.ent[row0 + c1++].z;
        nblobs = c1 < ne ? 2u : 1u;
        Out o{out, 0};
        for (u32 c = 0; c < nblobs; c++) {
            if (blob_off && L == 0) blob_off[c] = o.pos;
            const u32 start = c ? c1 : 0u, cnt = c ? ne - c1 : c1;
            const u64 len = c ? total - l1 : l1;
            put(o, "{\"chunkStartSegmentIndex\":");
            put_int(o, start);
            put(o, ",\"chunkSegmentCount\":");
            put_int(o, cnt);
            put(o, ",\"chunkLengthChars\":");
            put_int(o, (i64)len);
            put(o, ",\"totalLengthChars\":");
            put_int(o, (i64)total);
            put(o, ",\"totalSegmentCount\":");
            put_int(o, ne);
            put(o, ",\"chunkSequenceNumber\":");
            put_int(o, r.min_seq);
            put(o, ",\"segmentTexts\":[");
            for (u32 q = 0; q < cnt; q++) {
                if (q) put(o, ",");
                put_entry(o, p.ent[row0 + start + q]);
            }
            put(o, "]");
            if (c == 0) {
                put(o, ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}");
                if (l1 < total) put(o, ",{\"id\":\"body\"}");
                put(o, "],\"sequenceNumber\":");
                put_int(o, r.min_seq);
                put(o, ",\"totalLength\":");
                put_int(o, (i64)total);
                put(o, ",\"totalSegmentCount\":");
                put_int(o, ne);
                put(o, "}");
            }
            put(o, "}");
        }
        return o.pos;
    }

    // SnapshotV1 COUNT and WRITE without an entries table (extractSync streamed, snapshotV1.ts:170-228):
    // both passes walk the rows in 64-row batches (lane = row: its vis and emission word; aux only for
    // markers and permutation runs). Neither pass reads an entry's rows again: the walk carries the
    // first row's vis, its text offset (the running sum of the text rows' lengths -- Engine::finish
    // lays every text row out in document order), whether it has properties, and the JSON size of the
    // entry's text (the rows' emission words, less 8 bytes per surrogate pair joined across two rows),
    // so COUNT reads no text and WRITE reads only the text it writes. COUNT stores only the chunk table
    // (entry count, length per chunk); WRITE emits each entry as the walk closes it.
    struct Item {
        uint4 e;    // (first row, last row, length, kind) as build_entries makes it
        uint4 v;    // the first row's vis
        u32 ay;     // its text offset in the document's text run, or a marker's refType word / a run's start
        u64 tb;     // the JSON size of the entry's text
        bool props, gap;  // the first row has properties; a run spans an elided text row
    };
    struct Walk {
        const Doc& D;
        const bool counting;  // COUNT: the emission words are made (and stored for WRITE) here
        u32 n, base, j, tcarry;
        uint4 bv;          // this lane's row of the batch: vis
        u32 be, bay, btof;  // ... its emission word, aux.y (markers / permutation runs), text offset
        bool open, pend, filled;
        bool sat;           // a row's JSON text size may not fit ESC_LEN (6 bytes a unit at most): COUNT
                            // gives the walk up and the document takes the entry-table route (emit)
        Item run, pe;       // the open run, and a merge-info entry queued behind it
        bool runText, runPerm, runNL, runHI;
        MTE_DEV Walk(const Doc& d, bool count)
            : D(d), counting(count), n(d.r.n_segs), base(0), j(64), tcarry(0), open(false), pend(false), filled(false),
              sat(false) {}
        MTE_DEV void fill() {
            const u32 L = lane_id(), k = base + L;
            bv = make_uint4(0, 0, 0, 0);
            be = bay = 0;
            u32 ax = 0;
            if (k < n) {
                bv = D.p.vis[D.row0 + k];
                if (counting) {
                    if (bv.w & (F_PERM | F_MARKER)) {
                        const uint4 a = D.p.aux[D.row0 + k];
                        bay = a.y;
                        ax = a.x;
                    } else if (D.p.maps) {
                        ax = D.p.aux[D.row0 + k].x;  // (property-carrying batches only)
                    }
                } else {
                    be = D.p.esc[D.row0 + k];
                    if (bv.w & (F_PERM | F_MARKER)) bay = D.p.aux[D.row0 + k].y;
                }
            }
            const u32 tl = (bv.w & (F_PERM | F_MARKER)) ? 0u : bv.x;
            const u32 incl = wave_scan_incl(tl);
            btof = tcarry + incl - tl;
            tcarry += wave_read(incl, 63);
            if (!counting) return;
            if (wave_ballot(tl > ESC_LEN / 6u)) {
                sat = true;
                return;
            }
            // the emission word of every row of the batch (esc_unit over its text): short rows one
            // per lane, rows longer than 32 units by the whole wave, 64 units per step
            const u16* txt = D.p.text + D.r.text_off;
            u32 tot = 0, first = 0, last = 0;
            if (tl && tl <= 32) {
                const u16* src = txt + btof;
                u32 prev = 0;
                first = src[0];
                for (u32 i = 0; i < tl; i++) {
                    const u32 c = src[i];
                    tot += (u32)esc_unit(c, prev);
                    prev = c;
                }
                last = prev;
            }
            for (u64 lm = wave_ballot(tl > 32); lm; lm &= lm - 1) {
                const u32 l = (u32)__builtin_ctzll(lm);
                const u32 ln = wave_read(tl, l);
                const u16* src = txt + wave_read(btof, l);
                u32 sum = 0, carry = 0;
                for (u32 b0 = 0; b0 < ln; b0 += 64) {
                    const u32 i = b0 + L;
                    const u32 c = i < ln ? src[i] : 0u;
                    u32 pv = __builtin_amdgcn_update_dpp(0u, c, 0x138, 0xf, 0xf, false);  // wave_shr:1
                    if (L == 0) pv = carry;
                    const u32 u = i < ln ? (u32)esc_unit(c, pv) : 0u;
                    sum += wave_read(wave_scan_incl(u), 63);
                    carry = wave_read(c, ln - 1 - b0 < 63 ? ln - 1 - b0 : 63u);
                }
                if (L == l) {
                    tot = sum;
                    first = src[0];
                    last = carry;
                }
            }
            be = (ax ? ESC_PROPS : 0u);
            if (tl)
                be |= (tot & ESC_LEN) | (esc_is_lo(first) ? ESC_LO : 0u) | (esc_is_hi(last) ? ESC_HI : 0u) |
                      (last == (u32)'\n' ? ESC_NL : 0u);
            if (k < n) D.p.esc[D.row0 + k] = be;
        }
        // the next entry into it; false when the document has no more
        MTE_DEV bool next(Item& it) {
            const i32 minSeq = D.r.min_seq;
            for (;;) {
                if (pend && !open) {
                    pend = false;
                    it = pe;
                    return true;
                }
                if (j == 64) {  // the next batch
                    if (filled) base += 64;
                    filled = true;
                    j = 0;
                    if (base < n) fill();
                    if (sat) return false;
                }
                const u32 row = base + j;
                if (row >= n) {  // the end: the open run
                    if (!open) return false;
                    open = false;
                    it = run;
                    return true;
                }
                const uint4 v = make_uint4(wave_read(bv.x, j), wave_read(bv.y, j), wave_read(bv.z, j), wave_read(bv.w, j));
                const u32 ew = wave_read(be, j), ay = wave_read(bay, j), tof = wave_read(btof, j);
                j++;
                const u32 len = v.x, meta = v.w;
                const bool removed = (meta & F_REMOVED) != 0, marker = (meta & F_MARKER) != 0, perm = (meta & F_PERM) != 0;
                const bool hasP = (ew & ESC_PROPS) != 0;
                if (removed && (i32)v.z <= minSeq) {  // elided (:184-186)
                    if (open && runText && !marker && len) run.gap = true;  // run_text gathers around it
                    continue;
                }
                Item cur;
                cur.v = v;
                cur.ay = (marker || perm) ? ay : tof;
                cur.tb = ew & ESC_LEN;
                cur.props = hasP;
                cur.gap = false;
                if ((i32)v.y <= minSeq && !removed) {
                    if (open && (runPerm ? perm && ay == (run.ay ? run.ay + run.e.z : 0u)
                                         : runText && !marker && !perm && !(run.e.z && runNL) && (run.e.z <= 256 || len <= 256)) &&
                        D.match(D.row0 + run.e.x, run.props, D.row0 + row, hasP)) {
                        run.e.y = row;  // clone + append (:197-202)
                        run.e.z += len;
                        // (a high surrogate ending the run meets a low one starting this row: the two
                        // 6-byte escapes become one 4-byte UTF-8 pair; in 64 bits, since a row that is
                        // only that low surrogate adds 6 - 8)
                        run.tb += (u64)(ew & ESC_LEN);
                        if (runHI && (ew & ESC_LO)) run.tb -= 8u;
                        runNL = (ew & ESC_NL) != 0;
                        runHI = (ew & ESC_HI) != 0;
                        continue;
                    }
                    const bool had = open;
                    const Item prev = run;
                    open = true;
                    runText = !marker && !perm;
                    runPerm = perm;
                    runNL = (ew & ESC_NL) != 0;
                    runHI = (ew & ESC_HI) != 0;
                    run = cur;
                    run.e = make_uint4(row, row, len, perm ? 3u : runText ? 0u : 1u);
                    if (had) {
                        it = prev;
                        return true;
                    }
                } else {  // a merge-info entry
                    cur.e = make_uint4(row, row, len, 2u);
                    if (open) {
                        open = false;
                        pend = true;
                        pe = cur;
                        it = run;
                        return true;
                    }
                    it = cur;
                    return true;
                }
            }
        }
    };
    // one streamed entry (put_entry without reading its rows; a run across an elided text row gathers
    // its text through run_text)
    MTE_DEV void put_item(Out& o, const Item& it) const {
        const uint4 a = make_uint4(it.props ? 1u : 0u, it.ay, 0, 0);
        if (it.e.w == 0 || it.e.w == 1 || it.e.w == 3) {  // settled: coalesced text / permutation run or a marker
            u64 n = it.e.z;
            const u16* t = nullptr;
            if (it.e.w == 0 && o.out) t = it.gap ? run_text(it.e, n) : p.text + r.text_off + it.ay;
            put_seg(o, it.e.x, it.v, a, t, n, it.tb);
            return;
        }
        const uint4 v = it.v;
        const bool notext = (v.w & (F_MARKER | F_PERM)) != 0;
        put(o, "{\"json\":");
        put_seg(o, it.e.x, v, a, notext ? nullptr : p.text + r.text_off + it.ay, (v.w & F_MARKER) ? 0 : v.x, it.tb);
        const bool collab = p.cfg[d].collab != 0;
        if ((i32)v.y > r.min_seq) {
            put(o, ",\"seq\":");
            put_int(o, (i32)v.y);
            put(o, ",\"client\":");
            put_name(o, collab ? (v.w & 0xffu) : NONE);
        }
        if (v.w & F_REMOVED) {
            put(o, ",\"removedSeq\":");
            put_int(o, (i32)v.z);
            put(o, ",\"removedClient\":");
            put_name(o, collab ? ((v.w >> 8) & 0xffu) : NONE);
        }
        put(o, "}");
    }

    // n_ent's flag: COUNT found a row too long for the emission words (Walk::sat), so the document's
    // entries are in ent (build_entries) and WRITE takes emit, which reads the text
    static constexpr u32 SAT_ROUTE = 0x80000000u;
    // COUNT (SnapshotV1): byte count and blob count; the chunk table into ent[row0 + c]
    MTE_DEV u64 count_v1(u32& ne, u32& nblobs) const {
        const u32 L = lane_id(), chunk = p.chunk;
        Walk w(*this, true);
        Out o{nullptr, 0};
        u32 nch = 0, cnt = 0, first = 0;
        u64 len = 0, totalLen = 0;
        ne = 0;
        Item it;
        auto close_chunk = [&]() {
            // (a document with no segments owns no rows: its one empty chunk is not stored, since
            // row0 is then the next document's first row; write_v1 rebuilds it as (0, 0, 0))
            if (L == 0 && r.n_segs) p.ent[row0 + nch] = make_uint4(first, cnt, (u32)len, 0u);
            put(o, "{\"version\":\"1\",\"segmentCount\":");
            put_int(o, cnt);
            put(o, ",\"length\":");
            put_int(o, (i64)len);
            put(o, ",\"segments\":[");
            put(o, "],\"startIndex\":");
            put_int(o, first);
            put(o, "}");
            if (cnt > 1) o.pos += cnt - 1;  // the commas between its entries
            totalLen += len;
            nch++;
            first += cnt;
            cnt = 0;
            len = 0;
        };
        while (w.next(it)) {
            put_item(o, it);
            ne++;
            cnt++;
            len += it.e.z;
            if (len >= chunk) close_chunk();
        }
        if (w.sat) {
            ne = SAT_ROUTE;
            return 0;
        }
        if (cnt || nch == 0) close_chunk();
        // the header chunk's metadata
        put(o, ",\"headerMetadata\":{\"minSequenceNumber\":");
        put_int(o, r.min_seq);
        put(o, ",\"sequenceNumber\":");
        put_int(o, r.cur_seq);
        put(o, ",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
        for (u32 b = 1; b < nch; b++) {
            put(o, ",{\"id\":\"body_");
            put_int(o, b - 1);
            put(o, "\"}");
        }
        put(o, "],\"totalLength\":");
        put_int(o, (i64)totalLen);
        put(o, ",\"totalSegmentCount\":");
        put_int(o, ne);
        put(o, "}");
        nblobs = nch;
        return o.pos;
    }
    // WRITE (SnapshotV1) from the chunk table COUNT wrote
    MTE_DEV u64 write_v1(u32 ne, u32 nch, char* out, u64* blob_off) const {
        const u32 L = lane_id();
        Walk w(*this, false);
        Out o{out, 0};
        u64 totalLen = 0;
        const bool empty = r.n_segs == 0;  // (COUNT stored no chunk row: one empty chunk)
        for (u32 c = 0; c < nch && !empty; c++) totalLen += p.ent[row0 + c].z;
        Item it;
        for (u32 c = 0; c < nch; c++) {
            const uint4 ch = empty ? make_uint4(0u, 0u, 0u, 0u) : p.ent[row0 + c];
            if (L == 0) blob_off[c] = o.pos;
            put(o, "{\"version\":\"1\",\"segmentCount\":");
            put_int(o, ch.y);
            put(o, ",\"length\":");
            put_int(o, (i64)ch.z);
            put(o, ",\"segments\":[");
            for (u32 q = 0; q < ch.y; q++) {
                if (!w.next(it)) break;  // (COUNT's walk: never short)
                if (q) put(o, ",");
                put_item(o, it);
            }
            put(o, "],\"startIndex\":");
            put_int(o, ch.x);
            if (c == 0) {
                put(o, ",\"headerMetadata\":{\"minSequenceNumber\":");
                put_int(o, r.min_seq);
                put(o, ",\"sequenceNumber\":");
                put_int(o, r.cur_seq);
                put(o, ",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
                for (u32 b = 1; b < nch; b++) {
                    put(o, ",{\"id\":\"body_");
                    put_int(o, b - 1);
                    put(o, "\"}");
                }
                put(o, "],\"totalLength\":");
                put_int(o, (i64)totalLen);
                put(o, ",\"totalSegmentCount\":");
                put_int(o, ne);
                put(o, "}");
            }
            put(o, "}");
        }
        return o.pos;
    }

    // 2 + 3: chunk plan and bytes; returns the byte count, blob starts into blob_off (WRITE)
    MTE_DEV u64 emit(u32 ne, char* out, u64* blob_off, u32& nblobs) const {
        if (p.legacy) return emit_legacy(ne, out, blob_off, nblobs);
        const u32 L = lane_id();
        const u32 chunk = p.chunk;
        // chunk plan: count, total length, the header chunk's entries
        u32 nch = 0, c0cnt = 0, c0len = 0;
        u64 totalLen = 0;
        {
            u32 i = 0;
            do {
                u32 cnt = 0;
                u64 len = 0;
                while (len < chunk && i < ne) {
                    len += p.ent[row0 + i].z;
                    i++;
                    cnt++;
                }
                if (nch == 0) {
                    c0cnt = cnt;
                    c0len = (u32)len;
                }
                nch++;
                totalLen += len;
            } while (i < ne);
        }
        nblobs = nch;
        Out o{out, 0};
        u32 i = 0;
        for (u32 c = 0; c < nch; c++) {
            if (blob_off && L == 0) blob_off[c] = o.pos;
            // this chunk's entries
            u32 cnt = 0;
            u64 len = 0;
            if (c == 0) {
                cnt = c0cnt;
                len = c0len;
            } else {
                for (u32 q = i; len < chunk && q < ne; q++) {
                    len += p.ent[row0 + q].z;
                    cnt++;
                }
            }
            put(o, "{\"version\":\"1\",\"segmentCount\":");
            put_int(o, cnt);
            put(o, ",\"length\":");
            put_int(o, (i64)len);
            put(o, ",\"segments\":[");
            for (u32 q = 0; q < cnt; q++) {
                if (q) put(o, ",");
                put_entry(o, p.ent[row0 + i + q]);
            }
            put(o, "],\"startIndex\":");
            put_int(o, i);
            if (c == 0) {
                put(o, ",\"headerMetadata\":{\"minSequenceNumber\":");
                put_int(o, r.min_seq);
                put(o, ",\"sequenceNumber\":");
                put_int(o, r.cur_seq);
                put(o, ",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
                for (u32 b = 1; b < nch; b++) {
                    put(o, ",{\"id\":\"body_");
                    put_int(o, b - 1);
                    put(o, "\"}");
                }
                put(o, "],\"totalLength\":");
                put_int(o, (i64)totalLen);
                put(o, ",\"totalSegmentCount\":");
                put_int(o, ne);
                put(o, "}");
            }
            put(o, "}");
            i += cnt;
        }
        return o.pos;
    }
};

}  // namespace

// COUNT: entries, bytes and blob count of every listed document (status 0 only)
__global__ __launch_bounds__(64) void k_emit_count(EmitParams p) {
    const u32 i = blockIdx.x;
    if (i >= p.n_list) return;
    const u32 d = p.list[i];
    Doc doc(p, d);
    u32 ne = 0, nb = 0;
    u64 bytes = 0;
    if (doc.r.status == 0) {
        if (p.legacy || !p.esc) {
            ne = doc.build_entries();
            wave_sync();  // entries written by lane 0, read by every lane
            bytes = doc.emit(ne, nullptr, nullptr, nb);
        } else {
            bytes = doc.count_v1(ne, nb);
            if (ne == Doc::SAT_ROUTE) {
                wave_sync();  // (count_v1's chunk rows are overwritten by the entries)
                ne = doc.build_entries();
                wave_sync();
                bytes = doc.emit(ne, nullptr, nullptr, nb);
                ne |= Doc::SAT_ROUTE;
            }
        }
    }
    if (lane_id() == 0) {
        p.n_ent[d] = ne;
        p.size[d] = bytes;
        p.nblobs[d] = nb;
    }
}

// WRITE: the blobs of every listed document at out + out_off[d], blob starts at blob_off + blob_base[d]
__global__ __launch_bounds__(64) void k_emit_write(EmitParams p) {
    const u32 i = blockIdx.x;
    if (i >= p.n_list) return;
    const u32 d = p.list[i];
    Doc doc(p, d);
    if (doc.r.status != 0 || p.size[d] == 0) return;
    u32 nb = 0;
    const u32 ne = p.n_ent[d];
    if (p.legacy || !p.esc || (ne & Doc::SAT_ROUTE))
        doc.emit(ne & ~Doc::SAT_ROUTE, p.out + p.out_off[d], p.blob_off + p.blob_base[d], nb);
    else doc.write_v1(p.n_ent[d], p.nblobs[d], p.out + p.out_off[d], p.blob_off + p.blob_base[d]);
}

hipError_t launch_emit(const EmitParams& p, bool write, hipStream_t s) {
    if (p.n_list == 0) return hipSuccess;
    void* args[] = {(void*)&p};
    return hipLaunchKernel(write ? (const void*)k_emit_write : (const void*)k_emit_count, dim3(p.n_list), dim3(64),
                           args, 0, s);
}

}  // namespace mte
