// TEST INFRASTRUCTURE ONLY — CPU oracle for the merge-tree replay path.
//
// A restatement of @fluidframework/merge-tree 0.31.0 as a *tree* (the same B-tree object model the
// reference uses: 8-slot blocks, parent pointers, LRU heap, zamboni scour/pack), independent of the
// flat, wave-parallel design of the HIP engine it checks. Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it. Every function cites the reference file:line it follows
// (paths relative to /root/reference/packages/dds/merge-tree/src unless stated).
//
// Parity pinning: the reference is TypeScript and is NOT built here (no tsc in the image; building
// it would need a stand-in compiler). The oracle is pinned by the reference's own golden vectors:
// packages/dds/sequence/src/test/snapshots/v1/*.json (SnapshotV1 bytes, reproduced through the
// local, non-collaborative path of generateSharedStrings.ts:24-98) and by the expected strings of
// the merge-tree spec tests (tests/test_oracle_specs.py). Collaborative merge-info snapshot bytes
// and zamboni boundaries are not covered by any reference fixture: "parity unpinned" for those rows.
//
// The one deliberate replacement: PartialSequenceLengths (partialLengths.ts) is not reproduced; a
// block's length for (refSeq, clientId) is the sum of the leaf visibility predicate
// (mergeTree.ts:1673-1696) over its subtree, which is what the partial-length cache computes when
// each client's refSeq is non-decreasing (deli guarantees it, lambdas/src/deli/lambda.ts:282-295).
#include <algorithm>
#include <atomic>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <sstream>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "../include/mte.h"
#include "jsvalue.hpp"

namespace orc {

// constants.ts:11-15, mergeTree.ts:334,1059-1061
constexpr int MaxNodesInBlock = 8;
constexpr int UniversalSequenceNumber = 0;
constexpr int UnassignedSequenceNumber = -1;
constexpr int TreeMaintenanceSequenceNumber = -2;
constexpr int LocalClientId = -1;
constexpr int NonCollabClient = -2;
constexpr int TextSegmentGranularity = 256;
constexpr int ZamboniSegmentsMaxCount = 2;

struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct Block;

struct Node {
    Block* parent = nullptr;
    int index = 0;
    bool leaf;
    explicit Node(bool l) : leaf(l) {}
};

// BaseSegment / TextSegment / Marker (mergeTree.ts:429-798, textSegment.ts:16-111)
constexpr int HandleUnallocated = INT32_MIN;  // Handle.unallocated (matrix/src/handletable.ts:11)
struct Segment : Node {
    bool marker = false;
    bool perm = false;                            // PermutationSegment (matrix/src/permutationvector.ts:37-127)
    int start = HandleUnallocated;                // its first row/col handle
    int refType = 0;
    u16s text;
    int len = 0;                                  // cachedLength
    bool hasProps = false;                        // properties !== undefined
    JObj props;
    int seq = UniversalSequenceNumber;            // mergeTree.ts:434
    int clientId = LocalClientId;                 // mergeTree.ts:433
    bool removed = false;                         // removedSeq !== undefined
    int removedSeq = 0;
    int removedClientId = 0;
    std::vector<int> overlap;                     // removedClientOverlap
    Segment() : Node(true) {}
};

struct Block : Node {
    Node* children[MaxNodesInBlock] = {};
    int childCount = 0;
    int needsScour = -1;  // -1 undefined, 0 false, 1 true (mergeTree.ts:63)
    Block() : Node(false) {}
};

struct LRUSegment {
    Segment* segment;
    int maxSeq;
};

// collections.ts:213-265 — binary min-heap, 1-based, exactly the reference's sift rules.
struct Heap {
    std::vector<LRUSegment> L{LRUSegment{nullptr, -2}};
    int count() const { return (int)L.size() - 1; }
    const LRUSegment* peek() const { return count() > 0 ? &L[1] : nullptr; }
    static int cmp(const LRUSegment& a, const LRUSegment& b) { return a.maxSeq - b.maxSeq; }  // mergeTree.ts:923-926
    LRUSegment get() {
        LRUSegment x = L[1];
        L[1] = L[count()];
        L.pop_back();
        fixdown(1);
        return x;
    }
    void add(LRUSegment x) {
        L.push_back(x);
        fixup(count());
    }
    void fixup(int k) {
        while (k > 1 && cmp(L[k >> 1], L[k]) > 0) {
            std::swap(L[k >> 1], L[k]);
            k >>= 1;
        }
    }
    void fixdown(int k) {
        while ((k << 1) <= count()) {
            int j = k << 1;
            if (j < count() && cmp(L[j], L[j + 1]) > 0) j++;
            if (cmp(L[k], L[j]) <= 0) break;
            std::swap(L[k], L[j]);
            k = j;
        }
    }
};

// properties.ts:62-93 matchProperties, generalised to JS values for the recursive call.
static std::vector<u16s> for_in_keys(const JV* v) {
    std::vector<u16s> ks;
    if (!v) return ks;
    if (v->t == JV::Obj) return v->o.keys();
    if (v->t == JV::Arr) {
        for (size_t i = 0; i < v->a.size(); i++) {
            std::string d = std::to_string(i);
            ks.push_back(u16s(d.begin(), d.end()));
        }
    } else if (v->t == JV::Str) {
        for (size_t i = 0; i < v->s.size(); i++) {
            std::string d = std::to_string(i);
            ks.push_back(u16s(d.begin(), d.end()));
        }
    }
    return ks;
}
static JVP member(const JV* v, const u16s& k) {
    if (!v) return nullptr;
    if (v->t == JV::Obj) return v->o.get(k);
    uint32_t idx;
    if (!is_array_index(k, &idx)) return nullptr;
    if (v->t == JV::Arr) return idx < v->a.size() ? v->a[idx] : nullptr;
    if (v->t == JV::Str) return idx < v->s.size() ? JV::str(u16s(1, v->s[idx])) : nullptr;
    return nullptr;
}
static bool strict_equal(const JV* a, const JV* b) {  // b is a primitive here
    if (!a || !b) return a == b;
    if (a->t != b->t) return false;
    switch (a->t) {
        case JV::Null: return true;
        case JV::Bool: return a->b == b->b;
        case JV::Num: return a->n == b->n;
        case JV::Str: return a->s == b->s;
        default: return a == b;
    }
}
static bool match_values(const JV* a, const JV* b) {
    if (truthy(a)) {
        if (!truthy(b)) return false;
        for (auto& k : for_in_keys(a)) {
            JVP bk = member(b, k);
            JVP ak = member(a, k);
            if (!bk) return false;
            if (bk->t == JV::Obj || bk->t == JV::Arr || bk->t == JV::Null) {
                if (!match_values(ak.get(), bk.get())) return false;
            } else if (!strict_equal(bk.get(), ak.get())) {
                return false;
            }
        }
        for (auto& k : for_in_keys(b))
            if (!member(a, k)) return false;
    } else {
        if (truthy(b)) return false;
    }
    return true;
}
static bool matchProperties(const Segment* a, const Segment* b) {
    JV av, bv;
    av.t = JV::Obj; av.o = a->props;
    bv.t = JV::Obj; bv.o = b->props;
    return match_values(a->hasProps ? &av : nullptr, b->hasProps ? &bv : nullptr);
}

// TextSegment.append / PermutationSegment.append (textSegment.ts:74-85, permutationvector.ts:96-102)
static void appendSeg(Segment* prev, const Segment* s) {
    if (prev->perm) {
        prev->len += s->len;
        return;
    }
    prev->text += s->text;
    prev->len = (int)prev->text.size();
}
// textSegment.ts:63-68
static bool canAppend(const Segment* prev, const Segment* seg) {
    if (prev->marker) return false;  // Marker.canAppend (mergeTree.ts:793-795)
    if (prev->perm)                  // PermutationSegment.canAppend (permutationvector.ts:88-94): handle runs
        return seg->perm && (prev->start == HandleUnallocated ? seg->start == HandleUnallocated
                                                               : seg->start == prev->start + prev->len);
    return !(prev->text.size() && prev->text.back() == u'\n') && !seg->marker && !seg->perm &&
           (prev->len <= TextSegmentGranularity || seg->len <= TextSegmentGranularity);
}

struct CollabWindow {  // mergeTree.ts:822-839
    int clientId = LocalClientId;
    bool collaborating = false;
    int minSeq = 0;
    int currentSeq = 0;
};

struct SegmentChanges {
    Segment* replaceCurrent = nullptr;
    Node* next = nullptr;
};

struct InsertCtx {
    bool splitMode;          // ensureIntervalBoundary (leaf = splitLeafSegment) vs blockInsert (onLeaf)
    Segment* candidate = nullptr;
    bool continuePredicate = false;
};

class MergeTree {
   public:
    Block* root;
    CollabWindow cw;
    Heap heap;
    std::deque<Segment> segPool;
    std::deque<Block> blockPool;
    std::vector<std::string>* longIds = nullptr;  // getLongClientId
    // mergeTreeDeltaCallback (mergeTree.ts:1981-1987, 2592-2598, 2705-2711): operation (0 insert,
    // 1 remove, 2 annotate) and the delta segments in walk order, each with its propertyDeltas keys
    typedef std::vector<std::pair<Segment*, std::vector<u16s>>> Deltas;
    std::function<void(int, Deltas&)> onDelta;
    // mergeTreeMaintenanceCallback's UNLINK (mergeTree.ts:1309-1315): a removed segment zamboni drops
    std::function<void(Segment*)> onUnlink;

    MergeTree() { root = makeBlock(0); }

    // getContainingSegment (mergeTree.ts:1623-1634) -> searchBlock (:1797-1829): the first child whose
    // length in the (refSeq, clientId) view exceeds the remaining position
    Segment* containingSegment(int pos, int refSeq, int clientId, int& offset) const {
        const Block* b = root;
        for (;;) {
            const Node* hit = nullptr;
            for (int i = 0; i < b->childCount; i++) {
                const Node* c = b->children[i];
                const int len = nodeLength(c, refSeq, clientId);
                if (pos < len) {
                    hit = c;
                    break;
                }
                pos -= len;
            }
            if (!hit) return nullptr;
            if (hit->leaf) {
                offset = pos;
                return (Segment*)hit;
            }
            b = (const Block*)hit;
        }
    }

    Block* makeBlock(int childCount) {  // mergeTree.ts:1114-1123
        blockPool.emplace_back();
        Block* b = &blockPool.back();
        b->childCount = childCount;
        return b;
    }
    Segment* newSegment() {
        segPool.emplace_back();
        return &segPool.back();
    }

    void startCollaboration(int localClientId, int minSeq, int currentSeq) {  // mergeTree.ts:1254-1271
        cw.clientId = localClientId;
        cw.minSeq = minSeq;
        cw.collaborating = true;
        cw.currentSeq = currentSeq;
        heap = Heap();
    }

    // reloadFromSegments (mergeTree.ts:1195-1251): the B-tree is built bottom-up, level by level,
    // MaxNodesInBlock - 1 = 7 children per block, until one block remains (the root).
    void reloadFromSegments(std::vector<Node*> nodes) {
        const int maxChildren = MaxNodesInBlock - 1;
        if (nodes.empty()) {
            root = makeBlock(0);
            return;
        }
        for (;;) {
            std::vector<Node*> blocks;
            for (size_t ni = 0; ni < nodes.size();) {
                Block* b = makeBlock(0);
                for (int c = 0; c < maxChildren && ni < nodes.size(); c++, ni++) assignChild(b, nodes[ni], b->childCount++);
                blocks.push_back(b);
            }
            if (blocks.size() == 1) {
                root = (Block*)blocks[0];
                break;
            }
            nodes.swap(blocks);
        }
        root->parent = nullptr;
        root->index = 0;
    }

    // mergeTree.ts:1161-1172
    int localNetLength(const Segment* s) const { return s->removed ? 0 : s->len; }

    int localLength(const Node* n) const {
        if (n->leaf) return localNetLength((const Segment*)n);
        const Block* b = (const Block*)n;
        int t = 0;
        for (int i = 0; i < b->childCount; i++) t += localLength(b->children[i]);
        return t;
    }

    // mergeTree.ts:1659-1699 (branch ids are all 0 for an observer; origin is never set)
    int nodeLength(const Node* node, int refSeq, int clientId) const {
        if (!cw.collaborating || cw.clientId == clientId) return localLength(node);
        if (!node->leaf) {
            const Block* b = (const Block*)node;
            int t = 0;
            for (int i = 0; i < b->childCount; i++) t += nodeLength(b->children[i], refSeq, clientId);
            return t;  // == partialLengths.getPartialLength(refSeq, clientId)
        }
        const Segment* s = (const Segment*)node;
        if (s->clientId == clientId || (s->seq != UnassignedSequenceNumber && s->seq <= refSeq)) {
            if (s->removed) {
                if (s->removedClientId == clientId ||
                    std::find(s->overlap.begin(), s->overlap.end(), clientId) != s->overlap.end() ||
                    (s->removedSeq != UnassignedSequenceNumber && s->removedSeq <= refSeq))
                    return 0;
                return s->len;
            }
            return s->len;
        }
        return 0;
    }

    int getLength(int refSeq, int clientId) const { return nodeLength(root, refSeq, clientId); }

    void assignChild(Block* b, Node* child, int index) {  // mergeTree.ts:375-382
        child->parent = b;
        child->index = index;
        b->children[index] = child;
    }

    // mergeTree.ts:2248-2277
    bool breakTie(int pos, const Node* node, int refSeq, int clientId) const {
        if (node->leaf) {
            if (pos == 0) {
                const Segment* s = (const Segment*)node;
                if (s->removed && s->removedSeq != 0 && s->removedSeq <= refSeq &&
                    s->removedSeq != UnassignedSequenceNumber)
                    return false;
                if (clientId == cw.clientId) return true;
                if (s->seq != UnassignedSequenceNumber) return true;
            }
            return false;
        }
        return true;
    }

    // TextSegment.createSplitSegmentAt + BaseSegment.splitAt (textSegment.ts:103-111, mergeTree.ts:524-568)
    Segment* splitAt(Segment* s, int pos) {
        if (!(pos > 0) || s->marker) return nullptr;
        Segment* r = newSegment();
        if (s->perm) {  // PermutationSegment.createSplitSegmentAt (permutationvector.ts:104-115)
            r->perm = true;
            r->len = s->len - pos;
            r->start = s->start == HandleUnallocated ? HandleUnallocated : s->start + pos;
            s->len = pos;
        } else {
            r->text = s->text.substr(pos);
            s->text = s->text.substr(0, pos);
            s->len = (int)s->text.size();
            r->len = (int)r->text.size();
        }
        if (s->hasProps) { r->hasProps = true; r->props = s->props; }  // segmentPropertiesManager.ts:113-128
        r->parent = s->parent;
        r->removedClientId = s->removedClientId;
        r->removedSeq = s->removedSeq;
        r->removed = s->removed;
        r->seq = s->seq;
        r->clientId = s->clientId;
        r->overlap = s->overlap;
        return r;
    }

    SegmentChanges leafAction(InsertCtx& ctx, Segment* segment, int pos) {
        SegmentChanges ch;
        if (ctx.splitMode) {  // splitLeafSegment, mergeTree.ts:2225-2239
            if (!(pos > 0)) return ch;
            ch.next = splitAt(segment, pos);
            return ch;
        }
        if (segment) {  // onLeaf, mergeTree.ts:2180-2190
            ch.replaceCurrent = ctx.candidate;
            ch.next = segment;
        } else {
            ch.next = ctx.candidate;
        }
        return ch;
    }

    // rightExcursion + checkSegmentIsLocal (mergeTree.ts:2143-2161, 2313-2343)
    bool continueFrom(Block* node) {
        Node* start = node;
        Block* parent = start->parent;
        while (parent) {
            bool matched = false;
            for (int i = 0; i < parent->childCount; i++) {
                Node* c = parent->children[i];
                if (matched) {
                    Segment* first = firstLeaf(c);
                    if (first) return first->seq == UnassignedSequenceNumber;
                    if (c->leaf) return ((Segment*)c)->seq == UnassignedSequenceNumber;
                } else {
                    matched = (c == start);
                }
            }
            start = parent;
            parent = parent->parent;
        }
        return false;
    }
    Segment* firstLeaf(Node* n) {
        if (n->leaf) return (Segment*)n;
        Block* b = (Block*)n;
        for (int i = 0; i < b->childCount; i++) {
            Segment* s = firstLeaf(b->children[i]);
            if (s) return s;
        }
        return nullptr;
    }

    Block* const UNFINISHED = (Block*)(intptr_t)1;

    // mergeTree.ts:2476-2489
    Block* split(Block* node) {
        int half = MaxNodesInBlock / 2;
        Block* nn = makeBlock(half);
        node->childCount = half;
        for (int i = 0; i < half; i++) {
            assignChild(nn, node->children[half + i], i);
            node->children[half + i] = nullptr;
        }
        return nn;
    }

    // mergeTree.ts:2345-2474
    Block* insertingWalk(Block* block, int pos, int refSeq, int clientId, int seq, InsertCtx& ctx) {
        int childIndex;
        Node* newNode = nullptr;
        for (childIndex = 0; childIndex < block->childCount; childIndex++) {
            Node* child = block->children[childIndex];
            int len = nodeLength(child, refSeq, clientId);
            if (pos < len || (pos == len && breakTie(pos, child, refSeq, clientId))) {
                if (!child->leaf) {
                    Block* splitNode = insertingWalk((Block*)child, pos, refSeq, clientId, seq, ctx);
                    if (splitNode == nullptr) return nullptr;
                    if (splitNode == UNFINISHED) {
                        pos -= len;
                        continue;
                    }
                    newNode = splitNode;
                    childIndex++;
                } else {
                    Segment* segment = (Segment*)child;
                    SegmentChanges ch = leafAction(ctx, segment, pos);
                    if (ch.replaceCurrent) assignChild(block, ch.replaceCurrent, childIndex);
                    if (ch.next) {
                        newNode = ch.next;
                        childIndex++;
                    } else {
                        return nullptr;
                    }
                }
                break;
            } else {
                pos -= len;
            }
        }
        if (!newNode) {
            if (pos == 0) {
                if (seq != UnassignedSequenceNumber && ctx.continuePredicate && continueFrom(block)) {
                    return UNFINISHED;
                }
                SegmentChanges ch = leafAction(ctx, nullptr, pos);
                newNode = ch.next;
            }
        }
        if (newNode) {
            for (int i = block->childCount; i > childIndex; i--) {
                block->children[i] = block->children[i - 1];
                block->children[i]->index = i;
            }
            assignChild(block, newNode, childIndex);
            block->childCount++;
            if (block->childCount < MaxNodesInBlock) return nullptr;
            return split(block);
        }
        return nullptr;
    }

    void updateRoot(Block* splitNode) {  // mergeTree.ts:1876-1887
        if (splitNode != nullptr && splitNode != UNFINISHED) {
            Block* nr = makeBlock(2);
            assignChild(nr, root, 0);
            assignChild(nr, splitNode, 1);
            root = nr;
        }
    }

    void ensureIntervalBoundary(int pos, int refSeq, int clientId) {  // mergeTree.ts:2241-2245
        InsertCtx ctx{true};
        Block* s = insertingWalk(root, pos, refSeq, clientId, TreeMaintenanceSequenceNumber, ctx);
        updateRoot(s);
    }

    // mergeTree.ts:1273-1283
    void addToLRUSet(Segment* seg, int seq) {
        if (seg->parent->needsScour != 1 && seq > cw.currentSeq) {
            seg->parent->needsScour = 1;
            heap.add(LRUSegment{seg, seq});
        }
    }

    // mergeTree.ts:2141-2224
    void blockInsert(int pos, int refSeq, int clientId, int seq, std::vector<Segment*>& segs) {
        int insertPos = pos;
        for (Segment* ns : segs) {
            if (ns->len > 0) {
                ns->seq = seq;
                ns->clientId = clientId;
                InsertCtx ctx{false, ns, true};
                Block* splitNode = insertingWalk(root, insertPos, refSeq, clientId, seq, ctx);
                if (ns->parent == nullptr) {
                    throw EngineError(MTE_DOC_INSERT_FAILED, "MergeTree insert failed");
                }
                updateRoot(splitNode);
                // saveIfLocal (:2164-2179)
                if (cw.collaborating) {
                    if (!(ns->seq == UnassignedSequenceNumber && clientId == cw.clientId) && ns->seq > cw.minSeq)
                        addToLRUSet(ns, ns->seq);
                }
                insertPos += ns->len;
            }
        }
    }

    // mergeTree.ts:1968-1998
    void insertSegments(int pos, std::vector<Segment*>& segs, int refSeq, int clientId, int seq) {
        ensureIntervalBoundary(pos, refSeq, clientId);
        blockInsert(pos, refSeq, clientId, seq, segs);
        if (onDelta) {
            Deltas d;
            for (Segment* x : segs) d.emplace_back(x, std::vector<u16s>());
            onDelta(0, d);
        }
        if (cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments();
    }

    // nodeMap (mergeTree.ts:2903-2965) restricted to leaf actions (post actions only update caches)
    template <class F>
    bool nodeMap(Block* node, int pos, int refSeq, int clientId, int start, int end, F& leaf) {
        bool go = true;
        for (int ci = 0; ci < node->childCount; ci++) {
            Node* child = node->children[ci];
            int len = nodeLength(child, refSeq, clientId);
            if (go && end > 0 && len > 0 && start < len) {
                if (!child->leaf) {
                    if (go) go = nodeMap((Block*)child, pos, refSeq, clientId, start, end, leaf);
                } else {
                    go = leaf((Segment*)child, pos, start, end);
                }
            }
            if (!go) break;
            pos += len;
            start -= len;
            end -= len;
        }
        return go;
    }

    // mergeTree.ts:2607-2719 (observer / non-collab paths; branch 0)
    void markRangeRemoved(int start, int end, int refSeq, int clientId, int seq) {
        ensureIntervalBoundary(start, refSeq, clientId);
        ensureIntervalBoundary(end, refSeq, clientId);
        Deltas removed;
        auto markRemoved = [&](Segment* s, int, int, int) {
            if (s->removed) {
                if (s->removedSeq == UnassignedSequenceNumber) {
                    s->removedClientId = clientId;
                    s->removedSeq = seq;
                } else {
                    s->overlap.push_back(clientId);  // addOverlappingClient :2544-2552
                }
            } else {
                s->removed = true;
                s->removedClientId = clientId;
                s->removedSeq = seq;
                removed.emplace_back(s, std::vector<u16s>());  // removedSegments (:2639)
            }
            if (cw.collaborating) {
                if (!(s->removedSeq == UnassignedSequenceNumber && clientId == cw.clientId)) addToLRUSet(s, seq);
            }
            return true;
        };
        nodeMap(root, 0, refSeq, clientId, start, end, markRemoved);
        if (onDelta) onDelta(1, removed);
        if (cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments();
    }

    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111), remote / non-collab
    // Returns the keys of the propertyDeltas it builds, in their insertion order.
    static std::vector<u16s> addProperties(Segment* s, const JObj& newProps, bool rewrite) {
        std::vector<u16s> deltas;
        if (!s->hasProps) {
            s->hasProps = true;
            s->props = JObj();
        }
        if (rewrite) {
            for (auto& k : s->props.keys()) {
                JVP nv = newProps.get(k);
                if (!truthy(nv.get())) {
                    s->props.del(k);
                    deltas.push_back(k);
                }
            }
        }
        for (auto& k : newProps.keys()) {
            JVP nv = newProps.get(k);
            if (std::find(deltas.begin(), deltas.end(), k) == deltas.end()) deltas.push_back(k);
            if (nv->t == JV::Null) s->props.del(k);
            else s->props.set(k, nv);
        }
        return deltas;
    }

    // mergeTree.ts:2565-2605
    void annotateRange(int start, int end, const JObj& props, bool rewrite, int refSeq, int clientId, int seq) {
        ensureIntervalBoundary(start, refSeq, clientId);
        ensureIntervalBoundary(end, refSeq, clientId);
        Deltas annotated;
        auto annotate = [&](Segment* s, int, int, int) {
            annotated.emplace_back(s, addProperties(s, props, rewrite));
            if (cw.collaborating && seq != UnassignedSequenceNumber) addToLRUSet(s, seq);
            return true;
        };
        nodeMap(root, 0, refSeq, clientId, start, end, annotate);
        if (onDelta) onDelta(2, annotated);
        if (cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments();
    }

    bool underflow(const Block* b) const { return b->childCount < MaxNodesInBlock / 2; }  // :1285-1287

    // mergeTree.ts:1289-1365 (observer: segmentGroups/trackingCollection empty, all branch 0)
    void scourNode(Block* node, std::vector<Node*>& hold) {
        Segment* prev = nullptr;
        for (int k = 0; k < node->childCount; k++) {
            Node* cn = node->children[k];
            if (!cn->leaf) {
                hold.push_back(cn);
                prev = nullptr;
                continue;
            }
            Segment* s = (Segment*)cn;
            if (s->removed) {
                if (s->removedSeq > cw.minSeq) {
                    hold.push_back(s);
                } else {
                    if (onUnlink) onUnlink(s);
                    s->parent = nullptr;
                }
                prev = nullptr;
            } else if (s->seq <= cw.minSeq) {
                bool ok = prev && canAppend(prev, s) && matchProperties(prev, s) && localNetLength(s) > 0;
                if (ok) {
                    appendSeg(prev, s);  // TextSegment.append (textSegment.ts:74-85)
                    s->parent = nullptr;
                } else {
                    hold.push_back(s);
                    prev = localNetLength(s) > 0 ? s : nullptr;
                }
            } else {
                hold.push_back(s);
                prev = nullptr;
            }
        }
    }

    // mergeTree.ts:1368-1420
    void pack(Block* block) {
        Block* parent = block->parent;
        std::vector<Node*> hold;
        for (int ci = 0; ci < parent->childCount; ci++) {
            Block* cb = (Block*)parent->children[ci];
            scourNode(cb, hold);
            cb->parent = nullptr;
        }
        int total = (int)hold.size();
        int half = MaxNodesInBlock / 2;
        int childCount = std::min(MaxNodesInBlock - 1, total / half);
        if (childCount < 1) childCount = 1;
        int baseCount = total / childCount;
        int extra = total % childCount;
        Block* packed[MaxNodesInBlock] = {};
        int rd = 0;
        for (int ni = 0; ni < childCount; ni++) {
            int nc = baseCount;
            if (extra > 0) { nc++; extra--; }
            Block* pb = makeBlock(nc);
            for (int pi = 0; pi < nc; pi++) assignChild(pb, hold[rd++], pi);
            pb->parent = parent;
            packed[ni] = pb;
        }
        for (int j = 0; j < MaxNodesInBlock; j++) parent->children[j] = nullptr;
        for (int j = 0; j < childCount; j++) assignChild(parent, packed[j], j);
        parent->childCount = childCount;
        if (underflow(parent) && parent->parent) pack(parent);
    }

    // mergeTree.ts:1422-1478
    void zamboniSegments() {
        if (!cw.collaborating) return;
        for (int i = 0; i < ZamboniSegmentsMaxCount; i++) {
            const LRUSegment* top = heap.peek();
            if (!top || top->maxSeq > cw.minSeq) break;
            LRUSegment e = heap.get();
            if (e.segment->parent && e.segment->parent->needsScour != 0) {
                Block* block = e.segment->parent;
                std::vector<Node*> copy;
                scourNode(block, copy);
                block->needsScour = 0;
                int nc = (int)copy.size();
                if (nc < block->childCount) {
                    for (int j = 0; j < MaxNodesInBlock; j++) block->children[j] = nullptr;
                    block->childCount = nc;
                    for (int j = 0; j < nc; j++) assignChild(block, copy[j], j);
                    if (underflow(block) && block->parent) pack(block);
                }
            }
        }
    }

    // mergeTree.ts:1718-1736
    void setMinSeq(int minSeq) {
        if (minSeq > cw.currentSeq) throw EngineError(MTE_DOC_SEQ_ORDER, "minSeq > currentSeq");
        if (minSeq < cw.minSeq) throw EngineError(MTE_DOC_SEQ_ORDER, "minSeq moved backwards");
        if (minSeq > cw.minSeq) {
            cw.minSeq = minSeq;
            zamboniSegments();
        }
    }

    template <class F>
    bool walkAllSegments(Block* b, F& f) {  // mergeTree.ts:2969-2983
        bool go = true;
        for (int i = 0; go && i < b->childCount; i++) {
            Node* c = b->children[i];
            go = c->leaf ? f((Segment*)c) : walkAllSegments((Block*)c, f);
        }
        return go;
    }

    // getStats (mergeTree.ts:1484-1527): leafCount, removedLeafCount, maxHeight
    void stats(Block* b, int& leaves, int& removed, int& height) {
        int h = 0;
        for (int i = 0; i < b->childCount; i++) {
            Node* c = b->children[i];
            int ch = 1;
            if (!c->leaf) {
                int l2 = 0, r2 = 0, h2 = 0;
                stats((Block*)c, l2, r2, h2);
                leaves += l2;
                removed += r2;
                ch = 1 + h2;
            } else {
                leaves++;
                if (((Segment*)c)->removed) removed++;
            }
            h = std::max(h, ch);
        }
        height = h;
    }
};

// ---- JSON of a segment (TextSegment.toJSONObject textSegment.ts:48-54, Marker mergeTree.ts:652-656)
static void props_json(std::string& o, const JObj& p) {
    JV v;
    v.t = JV::Obj;
    v.o = p;
    js_stringify(o, v);
}
static void segment_json(std::string& o, const Segment* s) {
    if (s->perm) {  // PermutationSegment.toJSONObject (permutationvector.ts:75-77): [length, start]
        o += "[" + js_number(s->len) + "," + js_number(s->start) + "]";
        return;
    }
    if (s->marker) {
        o += "{\"marker\":{\"refType\":" + js_number(s->refType) + "}";
        if (s->hasProps) { o += ",\"props\":"; props_json(o, s->props); }
        o += "}";
    } else if (s->hasProps) {
        o += "{\"text\":";
        js_quote(o, s->text);
        o += ",\"props\":";
        props_json(o, s->props);
        o += "}";
    } else {
        js_quote(o, s->text);
    }
}

// FNV-1a-64
// Buffer.toString("utf8") of the decoded base64 bytes (fromBase64ToUtf8,
// common/lib/common-utils/src/base64Encoding.ts): the WHATWG UTF-8 decoder, each maximal invalid subpart becomes U+FFFD.
// Re-encoded as UTF-8 for the JSON parser.
static std::string utf8ReplaceInvalid(const std::string& in) {
    std::string out;
    out.reserve(in.size());
    auto put = [&](uint32_t cp) {
        if (cp < 0x80) {
            out.push_back((char)cp);
        } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    };
    uint32_t need = 0, seen = 0, cp = 0, lo = 0x80, hi = 0xBF;
    for (size_t i = 0; i < in.size();) {
        const uint32_t b = (unsigned char)in[i];
        if (need == 0) {
            i++;
            if (b < 0x80) put(b);
            else if (b >= 0xC2 && b <= 0xDF) { need = 1; cp = b & 0x1F; }
            else if (b >= 0xE0 && b <= 0xEF) { if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; need = 2; cp = b & 0xF; }
            else if (b >= 0xF0 && b <= 0xF4) { if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; need = 3; cp = b & 0x7; }
            else put(0xFFFD);
            continue;
        }
        if (b < lo || b > hi) {  // the byte starts over (not consumed)
            need = seen = cp = 0;
            lo = 0x80;
            hi = 0xBF;
            put(0xFFFD);
            continue;
        }
        i++;
        lo = 0x80;
        hi = 0xBF;
        cp = (cp << 6) | (b & 0x3F);
        if (++seen == need) {
            put(cp);
            need = seen = cp = 0;
        }
    }
    if (need) put(0xFFFD);
    return out;
}

static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}

class Doc {
   public:
    MergeTree mt;
    std::vector<std::string> shortIds;                 // shortClientIdMap (client.ts:644-668)
    std::unordered_map<std::string, int> nameToShort;  // clientNameToIds
    std::string observer;
    bool collab = false;
    int status = 0;
    long long failingSeq = -1;
    std::string error;
    uint64_t opsApplied = 0;
    // idToSegment (mergeTree.ts:1098, 1185-1187) by the builder's marker tag (include/mte.h
    // MTE_OP_RELPOS): the builder leaves unmapped every id the reference could tie to two markers
    std::unordered_map<uint32_t, Segment*> tagged;

    // ---- legacy snapshot catch-up messages (SharedSegmentSequence.processMergeTreeMsg,
    // sequence.ts:597-634, with newMergeTreeSnapshotFormat unset): every op message is stashed in
    // messagesSinceMSNChange; one whose refSeq is not seq - 1 is stashed with refSeq = seq - 1 and its
    // contents rebuilt from its sequenceDelta events (createOpsFromDelta, sequence.ts:58-100).
    std::vector<JVP> catchup;
    bool transforming = false;
    std::vector<JVP> xops;  // ops built from the current message's delta events
    static JVP jnum(double x) {
        JVP v = std::make_shared<JV>();
        v->t = JV::Num;
        v->n = x;
        return v;
    }
    static JVP jobj() {
        JVP v = std::make_shared<JV>();
        v->t = JV::Obj;
        return v;
    }
    // SequenceDeltaEvent.ranges (sequenceDeltaEvent.ts:26-46): delta segments in document order, each
    // at client.getPosition(segment) = getPosition(segment, currentSeq, local client) -- the op is
    // not yet in currentSeq, so its own inserts count 0 and its own removals still count
    void deltaOps(int op, MergeTree::Deltas& d) {
        if (!transforming) return;
        for (auto& e : d) {
            Segment* seg = e.first;
            const int pos = seg->parent ? getPosition(seg, mt.cw.currentSeq, mt.cw.clientId) : -1;
            const double len = seg->len;
            JVP last = xops.empty() ? nullptr : xops.back();
            if (op == 0) {  // createInsertOp(pos, segment.clone().toJSONObject())
                std::string sj;
                segment_json(sj, seg);
                JVP o = jobj();
                o->o.set(u"pos1", jnum(pos));
                o->o.set(u"seg", parse(sj.data(), sj.size()));
                o->o.set(u"type", jnum(0));
                xops.push_back(o);
            } else if (op == 1) {  // lastRem?.pos1 === r.position ? lastRem.pos2 += len : createRemoveRangeOp
                JVP p1 = last ? last->o.get(u"pos1") : nullptr;
                if (p1 && p1->t == JV::Num && p1->n == pos) {
                    JVP p2 = last->o.get(u"pos2");
                    last->o.set(u"pos2", jnum(p2 && p2->t == JV::Num ? p2->n + len : NAN));
                } else {
                    JVP o = jobj();
                    o->o.set(u"pos1", jnum(pos));
                    o->o.set(u"pos2", jnum(pos + len));
                    o->o.set(u"type", jnum(1));
                    xops.push_back(o);
                }
            } else {  // props[key] = segment.properties[key] ?? null over the propertyDeltas keys
                JVP props = jobj();
                for (auto& k : e.second) {
                    JVP v = seg->hasProps ? seg->props.get(k) : nullptr;
                    props->o.set(k, v ? v : std::make_shared<JV>());
                }
                JVP p2 = last ? last->o.get(u"pos2") : nullptr;
                JVP lp = last ? last->o.get(u"props") : nullptr;
                if (p2 && p2->t == JV::Num && p2->n == pos && match_values(lp.get(), props.get())) {
                    last->o.set(u"pos2", jnum(p2->n + len));
                } else {
                    JVP o = jobj();
                    o->o.set(u"pos1", jnum(pos));
                    o->o.set(u"pos2", jnum(pos + len));
                    o->o.set(u"props", props);
                    o->o.set(u"type", jnum(2));
                    xops.push_back(o);
                }
            }
        }
    }
    // processMinSequenceNumberChanged (sequence.ts:640-650)
    void trimCatchup(int minSeq) {
        size_t i = 0;
        while (i < catchup.size() && num(catchup[i]->o, u"sequenceNumber") <= minSeq) i++;
        if (i) catchup.erase(catchup.begin(), catchup.begin() + i);
    }

    // posFromRelativePos (mergeTree.ts:1943-1966) -> getPosition (:1586-1603). An unmapped id is
    // unsupported. A marker zamboni dropped is unlinked (scourNode sets its parent undefined,
    // mergeTree.ts:1317): getPosition's walk up the parents is empty and gives 0, so the position is
    // 0 + cachedLength + offset, or 0 - offset before it (client.getPostion.spec.ts:41-57 pins the
    // unlinking).
    int markerPos(uint32_t tag, int refSeq, int clientId) {
        auto it = tag && tag <= 0xFFFFu ? tagged.find(tag) : tagged.end();
        if (it == tagged.end()) throw EngineError(MTE_DOC_UNSUPPORTED, "relative position: marker id not mapped");
        return getPosition(it->second, refSeq, clientId);
    }
    int getPosition(Node* node, int refSeq, int clientId) {
        if (!node->parent) return 0;  // unlinked by zamboni
        for (Node* n = node; n != mt.root; n = n->parent) {
            bool linked = false;
            for (int ci = 0; n->parent && ci < n->parent->childCount; ci++) linked |= n->parent->children[ci] == n;
            if (!linked) throw EngineError(MTE_DOC_UNSUPPORTED, "relative position: marker dropped from the tree");
        }
        int total = 0;
        Block* parent = node->parent;
        Node* prevParent = nullptr;
        while (parent) {
            for (int ci = 0; ci < parent->childCount; ci++) {
                Node* child = parent->children[ci];
                if ((prevParent && child == prevParent) || child == node) break;
                total += mt.nodeLength(child, refSeq, clientId);
            }
            prevParent = parent;
            parent = parent->parent;
        }
        return total;
    }
    // Client.getValidOpRange (client.ts:493-510): positions from the RELPOS record before the op
    void relPositions(const mte_batch* b, uint64_t i, uint32_t d, mte_op& op) {
        if (i == b->doc_op_offsets[d] || b->ops[i - 1].type != MTE_OP_RELPOS)
            throw EngineError(MTE_DOC_UNSUPPORTED, "MTE_F_REL without a RELPOS record");
        const mte_op& r = b->ops[i - 1];
        if (r.pos1) {
            const int q = markerPos((uint32_t)r.pos1, op.ref_seq, op.client);
            op.pos1 = (r.flags & MTE_F_REL_BEFORE1) ? q - r.msn : q + 1 + r.msn;  // Marker cachedLength 1
        }
        if (r.a) {
            const int q = markerPos((uint32_t)r.a, op.ref_seq, op.client);
            op.a = (r.flags & MTE_F_REL_BEFORE2) ? q - (int32_t)r.props : q + 1 + (int32_t)r.props;
        }
        // a position before 0 (an unlinked marker, "before" with an offset) sends the reference's walks
        // below the tree's start: not modelled
        if ((r.pos1 && op.pos1 < 0) || (r.a && op.a < 0))
            throw EngineError(MTE_DOC_UNSUPPORTED, "relative position before the document start");
    }
    void tag(Segment* s, uint32_t word) {
        s->refType = (int)(word & 0xFFFFu);
        if (word >> 16) tagged[word >> 16] = s;
    }

    explicit Doc(const char* observerName) {
        mt.longIds = &shortIds;
        if (observerName) {  // startOrUpdateCollaboration(observer) (client.ts:1059-1079)
            observer = observerName;
            collab = true;
            getOrAddShortClientId(observer);
            mt.startCollaboration(0, 0, 0);
            mt.onDelta = [this](int op, MergeTree::Deltas& d) { deltaOps(op, d); };
        }
    }

    int getOrAddShortClientId(const std::string& name) {
        auto it = nameToShort.find(name);
        if (it != nameToShort.end()) return it->second;
        int id = (int)shortIds.size();
        shortIds.push_back(name);
        nameToShort[name] = id;
        return id;
    }
    std::string longId(int shortId) const { return shortId >= 0 ? shortIds[shortId] : "original"; }

    // The JSON path's idToSegment, keyed by the id string itself (the record path above uses the
    // builder's tags): mapped at insert and for live loaded markers; an id mapped to two markers, and
    // any id after an annotate that sets "markerId", is ambiguous -- blockUpdate re-maps live markers
    // (mergeTree.ts:2748-2768, 275-284) in an order this restatement does not model -- and a relative
    // position naming it is unsupported, as in the builder (include/mte.h MTE_OP_RELPOS).
    std::unordered_map<u16s, Segment*> idToSegment;
    std::unordered_set<u16s> idAmbiguous;
    bool idAnnotated = false;
    void mapIdToSegment(Segment* s) {
        if (!s->marker || !s->hasProps) return;
        JVP v = s->props.get(u"markerId");
        if (!v || v->t != JV::Str || v->s.empty()) return;
        auto it = idToSegment.find(v->s);
        if (it != idToSegment.end() && it->second != s) idAmbiguous.insert(v->s);
        idToSegment[v->s] = s;
    }
    int posFromRelativePos(const JV& rp, int refSeq, int clientId) {  // mergeTree.ts:1943-1966
        JVP id = rp.t == JV::Obj ? rp.o.get(u"id") : nullptr;
        if (!id || id->t != JV::Str || id->s.empty() || idAnnotated || idAmbiguous.count(id->s) ||
            !idToSegment.count(id->s))
            throw EngineError(MTE_DOC_UNSUPPORTED, "relative position: marker id not mapped");
        int pos = getPosition(idToSegment[id->s], refSeq, clientId);
        JVP before = rp.o.get(u"before"), off = rp.o.get(u"offset");
        const int o = off && off->t == JV::Num ? (int)off->n : 0;
        return truthy(before.get()) ? pos - o : pos + 1 + o;
    }

    // a SharedMatrix row / col vector (PermutationVector, permutationvector.ts:129-146) instead of a
    // SharedString: specs are PermutationSegment JSON
    bool permutation = false;
    // its HandleTable (handletable.ts:19-86): handles[0] is the free-list head
    std::vector<int> handles{1};
    int allocateHandle() {  // :35-40
        const int fr = handles[0];
        handles[0] = fr < (int)handles.size() ? handles[fr] : fr + 1;  // handles[free] ?? free + 1
        if (fr == (int)handles.size()) handles.push_back(0);
        else handles[fr] = 0;
        return fr;
    }
    void freeHandle(int h) {  // :56-59
        handles[h] = handles[0];
        handles[0] = h;
    }
    // PermutationVector.adjustPosition (permutationvector.ts:198-209); -1 = undefined
    int adjustPosition(int pos, int refSeq, int clientId) {
        int off = 0;
        Segment* s = mt.containingSegment(pos, refSeq, clientId, off);
        if (!s || s->removed) return -1;
        return getPosition(s, mt.cw.currentSeq, mt.cw.clientId) + off;
    }
    // PermutationVector.getAllocatedHandle (permutationvector.ts:176-196)
    int getAllocatedHandle(int pos) {
        int off = 0;
        Segment* s = mt.containingSegment(pos, mt.cw.currentSeq, mt.cw.clientId, off);
        if (!s) throw EngineError(MTE_DOC_UNSUPPORTED, "getAllocatedHandle beyond the vector");
        if (s->start != HandleUnallocated) return s->start + off;
        // walkSegments(pos, pos + 1, splitRange) -> mapRange (mergeTree.ts:2797-2807)
        if (pos) mt.ensureIntervalBoundary(pos, mt.cw.currentSeq, mt.cw.clientId);
        mt.ensureIntervalBoundary(pos + 1, mt.cw.currentSeq, mt.cw.clientId);
        int h = HandleUnallocated;
        auto leaf = [&](Segment* seg, int, int, int) {
            seg->start = h = allocateHandle();
            return true;
        };
        mt.nodeMap(mt.root, 0, mt.cw.currentSeq, mt.cw.clientId, pos, pos + 1, leaf);
        return h;
    }
    Segment* makeSegment(const JV& spec) {  // SharedStringFactory.segmentFromSpec (sequenceFactory.ts:31-37)
        Segment* s = mt.newSegment();
        if (permutation) {  // PermutationSegment.fromJSONObject (permutationvector.ts:41-44): [length, start]
            if (spec.t != JV::Arr || spec.a.empty() || !spec.a[0] || spec.a[0]->t != JV::Num)
                throw EngineError(MTE_DOC_UNSUPPORTED, "not a PermutationSegment spec");
            s->perm = true;
            s->len = (int)spec.a[0]->n;
            s->start = HandleUnallocated;  // onDelta resets every inserted segment's handles (:302-309)
            return s;
        }
        if (spec.t == JV::Str) {
            s->text = spec.s;
            s->len = (int)s->text.size();
            return s;
        }
        if (spec.t == JV::Obj) {
            JVP m = spec.o.get(u"marker");
            JVP t = spec.o.get(u"text");
            JVP p = spec.o.get(u"props");
            if (m) {
                s->marker = true;
                JVP rt = m->t == JV::Obj ? m->o.get(u"refType") : nullptr;
                s->refType = rt && rt->t == JV::Num ? (int)rt->n : 0;
                s->len = 1;
            } else if (t && t->t == JV::Str) {
                s->text = t->s;
                s->len = (int)s->text.size();
            } else {
                throw EngineError(MTE_DOC_UNSUPPORTED, "unknown segment spec");
            }
            if (truthy(p.get())) MergeTree::addProperties(s, p->o, false);
            return s;
        }
        throw EngineError(MTE_DOC_UNSUPPORTED, "unknown segment spec");
    }

    static int num(const JObj& o, const char16_t* k, bool* has = nullptr) {
        JVP v = o.get(k);
        if (has) *has = v && v->t == JV::Num;
        return v && v->t == JV::Num ? (int)v->n : 0;
    }

    // Client.applyRemoteOp (client.ts:776-803) -> applyInsertOp/RemoveRange/AnnotateRange (:328-449)
    void applyRemoteOp(const JObj& op, int clientId, int refSeq, int seq) {
        if (op.get(u"register")) throw EngineError(MTE_DOC_UNSUPPORTED, "registers are out of scope");
        int type = num(op, u"type");
        bool hasPos1 = false;
        int pos1 = num(op, u"pos1", &hasPos1);
        int pos2 = num(op, u"pos2");
        // Client.getValidOpRange (client.ts:493-510)
        auto relPositions = [&]() {
            JVP rp1 = op.get(u"relativePos1"), rp2 = op.get(u"relativePos2");
            if (!op.get(u"pos1") && rp1 && truthy(rp1.get())) {
                pos1 = posFromRelativePos(*rp1, refSeq, clientId);
                if (pos1 < 0) throw EngineError(MTE_DOC_UNSUPPORTED, "relative position before the document start");
            }
            if (type != 0 && !op.get(u"pos2") && rp2 && truthy(rp2.get())) {
                pos2 = posFromRelativePos(*rp2, refSeq, clientId);
                if (pos2 < 0) throw EngineError(MTE_DOC_UNSUPPORTED, "relative position before the document start");
            }
        };
        switch (type) {
            case 0: {
                JVP seg = op.get(u"seg");
                if (!seg) return;
                relPositions();
                std::vector<Segment*> segs{makeSegment(*seg)};
                mapIdToSegment(segs[0]);
                mt.insertSegments(pos1, segs, refSeq, clientId, seq);
                opsApplied++;
                break;
            }
            case 1:
                relPositions();
                mt.markRangeRemoved(pos1, pos2, refSeq, clientId, seq);
                opsApplied++;
                break;
            case 2: {
                relPositions();
                JVP props = op.get(u"props");
                if (props && props->t == JV::Obj && props->o.get(u"markerId")) idAnnotated = true;
                JVP comb = op.get(u"combiningOp");
                bool rewrite = false;
                if (comb) {
                    JVP name = comb->t == JV::Obj ? comb->o.get(u"name") : nullptr;
                    if (name && name->t == JV::Str && name->s == u"rewrite") rewrite = true;
                    else throw EngineError(MTE_DOC_UNSUPPORTED, "combiningOp other than rewrite");
                }
                JObj empty;
                mt.annotateRange(pos1, pos2, props && props->t == JV::Obj ? props->o : empty, rewrite, refSeq,
                                 clientId, seq);
                opsApplied++;
                break;
            }
            case 3: {
                JVP ops = op.get(u"ops");
                if (ops && ops->t == JV::Arr)
                    for (auto& m : ops->a) applyRemoteOp(m->o, clientId, refSeq, seq);
                break;
            }
            default: break;
        }
    }

    // Client.applyMsg + updateSeqNumbers (client.ts:805-836)
    void applyMsg(const JV& msg) {
        if (status) return;
        const JObj& m = msg.o;
        JVP cid = m.get(u"clientId");
        std::string clientName = cid && cid->t == JV::Str ? u16_to_utf8(cid->s) : "";
        int seq = num(m, u"sequenceNumber");
        int refSeq = num(m, u"referenceSequenceNumber");
        int msn = num(m, u"minimumSequenceNumber");
        try {
            int shortId = getOrAddShortClientId(clientName);
            JVP type = m.get(u"type");
            if (type && type->t == JV::Str && type->s == u"op") {
                if (clientName == observer) throw EngineError(MTE_DOC_UNSUPPORTED, "observer never submits ops");
                if (!(mt.cw.currentSeq < seq)) throw EngineError(MTE_DOC_SEQ_ORDER, "seq <= currentSeq");
                JVP contents = m.get(u"contents");
                transforming = refSeq != seq - 1;
                xops.clear();
                if (contents && contents->t == JV::Obj) applyRemoteOp(contents->o, shortId, refSeq, seq);
                transforming = false;
                updateSeqNumbers(msn, seq);
                JVP stash = std::make_shared<JV>(msg);
                if (refSeq != seq - 1) {
                    stash->o.set(u"referenceSequenceNumber", jnum(seq - 1));
                    if (xops.size() == 1) {
                        stash->o.set(u"contents", xops[0]);
                    } else {  // createGroupOp(...ops)
                        JVP g = jobj(), arr = std::make_shared<JV>();
                        arr->t = JV::Arr;
                        arr->a = xops;
                        g->o.set(u"ops", arr);
                        g->o.set(u"type", jnum(3));
                        stash->o.set(u"contents", g);
                    }
                }
                xops.clear();
                catchup.push_back(stash);
                // "Do GC every once in a while" (sequence.ts:628-632)
                if (catchup.size() > 20 && num(catchup[20]->o, u"sequenceNumber") < msn) trimCatchup(msn);
                return;
            }
            updateSeqNumbers(msn, seq);
        } catch (EngineError& e) {
            status = e.code;
            failingSeq = seq;
            error = e.what();
        }
    }

    // ---- resume from a summary (SnapshotLoader, snapshotLoader.ts) ----------------------------
    // specToSegment (snapshotLoader.ts:79-111): merge info (hasMergeInfo, snapshotChunks.ts:71-73)
    // carries client / seq / removedSeq / removedClient; a bare spec is universal and NonCollab.
    // A PermutationSegment keeps its start handle when loaded (PermutationSegment.fromJSONObject,
    // permutationvector.ts:41-44; loading inserts with no op args, so onDelta's reset, :302-309, does
    // not run); Handle.unallocated stays unallocated.
    Segment* loadSegment(const JV& spec) {
        Segment* s = makeSegment(spec);
        if (permutation && spec.a.size() > 1 && spec.a[1] && spec.a[1]->t == JV::Num) s->start = (int)spec.a[1]->n;
        return s;
    }
    Segment* loadSpec(const JV& spec) {
        JVP json = spec.t == JV::Obj ? spec.o.get(u"json") : nullptr;
        if (!json) {
            Segment* s = loadSegment(spec);
            s->seq = UniversalSequenceNumber;
            s->clientId = NonCollabClient;
            return s;
        }
        Segment* s = loadSegment(*json);
        JVP c = spec.o.get(u"client"), sq = spec.o.get(u"seq"), rs = spec.o.get(u"removedSeq"),
            rc = spec.o.get(u"removedClient");
        s->clientId = c && c->t == JV::Str ? getOrAddShortClientId(u16_to_utf8(c->s)) : NonCollabClient;
        s->seq = sq && sq->t == JV::Num ? (int)sq->n : UniversalSequenceNumber;
        if (rs && rs->t == JV::Num) {
            s->removed = true;
            s->removedSeq = (int)rs->n;
        }
        if (rc && rc->t == JV::Str) s->removedClientId = getOrAddShortClientId(u16_to_utf8(rc->s));
        return s;
    }
    static JVP treeEntry(const JV& tree, const u16s& path) {
        JVP es = tree.t == JV::Obj ? tree.o.get(u"entries") : nullptr;
        if (!es || es->t != JV::Arr) return nullptr;
        for (auto& e : es->a) {
            JVP p = e->t == JV::Obj ? e->o.get(u"path") : nullptr;
            if (p && p->t == JV::Str && p->s == path) return e;
        }
        return nullptr;
    }
    // An ITree blob's text: storage.read(path) + fromBase64ToUtf8 (snapshotV1.ts:255,267,
    // snapshotLoader.ts:225) for { contents, encoding: "utf-8" | "base64" }; base64 read as Node's
    // Buffer.from(s, "base64") does (both alphabets, whitespace skipped, '=' ends the data).
    static std::string blobText(JVP v, const char* missing) {
        JVP c = v && v->t == JV::Obj ? v->o.get(u"contents") : nullptr;
        JVP enc = v && v->t == JV::Obj ? v->o.get(u"encoding") : nullptr;
        if (!c || c->t != JV::Str) throw EngineError(MTE_DOC_UNSUPPORTED, missing);
        if (!enc || (enc->t == JV::Str && enc->s == u"utf-8")) return u16_to_utf8(c->s);
        if (!(enc->t == JV::Str && enc->s == u"base64")) throw EngineError(MTE_DOC_UNSUPPORTED, "blob encoding");
        static const std::string A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
        std::string out;
        unsigned acc = 0, nb = 0;
        for (char16_t ch : c->s) {
            if (ch == u'=') break;
            if (ch == u' ' || ch == u'\n' || ch == u'\r' || ch == u'\t') continue;
            const char16_t cc = ch == u'-' ? u'+' : (ch == u'_' ? u'/' : ch);
            const size_t d = cc < 128 ? A.find((char)cc) : std::string::npos;
            if (d == std::string::npos) throw EngineError(MTE_DOC_UNSUPPORTED, "bad base64 blob");
            acc = (acc << 6) | (unsigned)d;
            nb += 6;
            if (nb >= 8) {
                nb -= 8;
                out.push_back((char)((acc >> nb) & 0xff));
            }
        }
        return utf8ReplaceInvalid(out);
    }
    // storage.read(path) + SnapshotV1.processChunk (snapshotV1.ts:249-270)
    static JVP chunkAt(const JV& tree, const u16s& path) {  // (legacy chunks converted to v1)
        JVP e = treeEntry(tree, path);
        JVP v = e ? e->o.get(u"value") : nullptr;
        std::string s = blobText(v, "summary blob missing");
        JVP ch = parse(s.data(), s.size());
        JVP ver = ch->t == JV::Obj ? ch->o.get(u"version") : nullptr;
        if (!ver && ch->t == JV::Obj && ch->o.get(u"segmentTexts")) {  // toLatestVersion (snapshotChunks.ts:135-176)
            auto v1 = std::make_shared<JV>();
            v1->t = JV::Obj;
            v1->o.set(u"version", JV::str(u"1"));
            v1->o.set(u"segments", ch->o.get(u"segmentTexts"));
            JVP md = ch->o.get(u"headerMetadata");
            if (!md && path == u"header") {  // buildHeaderMetadataForLegecyChunk (:158-176)
                md = std::make_shared<JV>();
                md->t = JV::Obj;
                auto ids = std::make_shared<JV>();
                ids->t = JV::Arr;
                auto id = [&](const char16_t* n) {
                    auto o = std::make_shared<JV>();
                    o->t = JV::Obj;
                    o->o.set(u"id", JV::str(n));
                    ids->a.push_back(o);
                };
                id(u"header");
                JVP cl = ch->o.get(u"chunkLengthChars"), tl = ch->o.get(u"totalLengthChars");
                if (cl && tl && cl->n < tl->n) id(u"body");
                md->o.set(u"orderedChunkMetadata", ids);
                if (JVP m = ch->o.get(u"chunkMinSequenceNumber")) md->o.set(u"minSequenceNumber", m);
                if (JVP q = ch->o.get(u"chunkSequenceNumber")) md->o.set(u"sequenceNumber", q);
            }
            if (md) v1->o.set(u"headerMetadata", md);
            return v1;
        }
        if (!ver || ver->t != JV::Str || ver->s != u"1") throw EngineError(MTE_DOC_UNSUPPORTED, "chunk version");
        return ch;
    }
    // SnapshotLoader.initialize: loadHeader (:113-148) then loadBody (:150-216).
    void loadSnapshot(const JV& summary) {
        const JV* t = &summary;
        JVP content = treeEntry(summary, u"content"), inner;
        if (content) {  // SharedString summary: the merge-tree lives under "content" (sequence.ts:413-438)
            inner = content->o.get(u"value");
            if (inner) t = inner.get();
        }
        JVP header = chunkAt(*t, u"header");
        JVP md = header->o.get(u"headerMetadata");
        if (!md || md->t != JV::Obj) throw EngineError(MTE_DOC_UNSUPPORTED, "header metadata not available");
        std::vector<Node*> segs;
        JVP hs = header->o.get(u"segments");
        if (hs && hs->t == JV::Arr)
            for (auto& sp : hs->a) segs.push_back(loadSpec(*sp));
        mt.reloadFromSegments(segs);
        for (Node* n : segs)  // addNodeReferences maps the live markers (mergeTree.ts:275-284)
            if (!((Segment*)n)->removed) mapIdToSegment((Segment*)n);
        bool hasMin = false;
        const int cur = num(md->o, u"sequenceNumber");
        const int minSeq = num(md->o, u"minSequenceNumber", &hasMin);
        mt.startCollaboration(0, hasMin ? minSeq : cur, cur);
        // loadBody (snapshotLoader.ts:150-216): nothing when the header holds every segment
        // (:159-161; the shipAsserts on the lengths only log); otherwise every later chunk's segments
        JVP ocm = md->o.get(u"orderedChunkMetadata");
        std::vector<Segment*> bodySegs;
        bool hasCount = false, hasTotal = false;
        const int segCount = num(header->o, u"segmentCount", &hasCount);
        const int totalSegs = num(md->o, u"totalSegmentCount", &hasTotal);
        if (!(hasCount && hasTotal && segCount == totalSegs)) {
            for (size_t i = 1; ocm && ocm->t == JV::Arr && i < ocm->a.size(); i++) {
                JVP id = ocm->a[i]->t == JV::Obj ? ocm->a[i]->o.get(u"id") : nullptr;
                if (!id || id->t != JV::Str) throw EngineError(MTE_DOC_UNSUPPORTED, "chunk id");
                JVP ch = chunkAt(*t, id->s);
                JVP cs = ch->o.get(u"segments");
                if (!cs || cs->t != JV::Arr) continue;
                for (auto& sp : cs->a) bodySegs.push_back(loadSpec(*sp));
            }
        }
        // append(segments, cli, seq) = insertSegments(root.cachedLength, segments, refSeq 0, cli, seq):
        // blockInsert walks each segment to insertPos and advances insertPos by its length. A segment
        // object already in the tree (flushBatch never clears `batch`, :196-199) keeps its parent:
        // when the walk fails it is skipped without error; when the walk finds pos the reference links
        // the same object a second time -- a tree the engine does not model, so both report it as
        // unsupported.
        std::unordered_set<Segment*> linked;
        auto append = [&](const std::vector<Segment*>& v, int cli, int seq) {
            int insertPos = mt.localLength(mt.root);
            for (Segment* sg : v) {
                if (sg->len <= 0) continue;
                if (linked.count(sg)) {
                    if (mt.getLength(UniversalSequenceNumber, cli) >= insertPos)
                        throw EngineError(MTE_DOC_UNSUPPORTED, "loadBody re-links a segment object");
                    insertPos += sg->len;
                    continue;
                }
                std::vector<Segment*> one{sg};
                mapIdToSegment(sg);  // blockInsert (mergeTree.ts:2199-2205)
                mt.insertSegments(insertPos, one, UniversalSequenceNumber, cli, seq);
                linked.insert(sg);
                insertPos += sg->len;
            }
        };
        std::vector<Segment*> batch;
        auto flushBatch = [&]() {
            if (!batch.empty()) append(batch, NonCollabClient, UniversalSequenceNumber);
        };
        for (Segment* sg : bodySegs) {
            if (sg->clientId == NonCollabClient && sg->seq == UniversalSequenceNumber) {
                batch.push_back(sg);
            } else {
                flushBatch();
                append({sg}, sg->clientId, sg->seq);
            }
        }
        flushBatch();
        // loadBodyAndCatchupOps (snapshotLoader.ts:55-77): a blob beyond the chunks holds catch-up
        // messages, applied after the load (sequence.ts:499-527, processMergeTreeMsg -> applyMsg)
        JVP es = t->t == JV::Obj ? t->o.get(u"entries") : nullptr;
        size_t nBlobs = 0, nChunks = ocm && ocm->t == JV::Arr ? ocm->a.size() : 1;
        JVP extra;
        for (auto& e : es && es->t == JV::Arr ? es->a : std::vector<JVP>{}) {
            JVP ty = e->o.get(u"type"), p = e->o.get(u"path");
            if (!ty || ty->t != JV::Str || ty->s != u"Blob" || !p) continue;
            nBlobs++;
            bool isChunk = false;
            for (size_t i = 0; ocm && ocm->t == JV::Arr && i < ocm->a.size(); i++) {
                JVP id = ocm->a[i]->o.get(u"id");
                isChunk |= id && id->t == JV::Str && id->s == p->s;
            }
            if (!isChunk) extra = e;
        }
        if (nBlobs != nChunks + 1 && nBlobs != nChunks) throw EngineError(MTE_DOC_UNSUPPORTED, "Unexpected blobs in snapshot");
        if (nBlobs == nChunks + 1 && extra) {
            std::string txt = blobText(extra->o.get(u"value"), "catch-up ops blob");
            JVP msgs = parse(txt.data(), txt.size());
            if (msgs->t == JV::Arr)
                for (auto& m : msgs->a) applyMsg(*m);
        }
    }
    int loadSnapshotJson(const char* json, size_t len) {
        try {
            JVP v = parse(json, len);
            loadSnapshot(*v);
        } catch (EngineError& e) {
            status = e.code;
            error = e.what();
        } catch (std::exception& e) {
            status = MTE_DOC_UNSUPPORTED;
            error = e.what();
        }
        return status;
    }

    void updateSeqNumbers(int msn, int seq) {
        if (seq < mt.cw.currentSeq) throw EngineError(MTE_DOC_SEQ_ORDER, "seq < currentSeq");
        mt.cw.currentSeq = seq;
        if (msn > seq) throw EngineError(MTE_DOC_SEQ_ORDER, "msn > seq");
        mt.setMinSeq(msn);
    }

    // ---- binary batch input (include/mte.h records) ----------------------------------------
    JObj propset(const mte_batch* b, uint32_t id) {
        JObj o;
        if (id == 0 || id >= b->n_propsets) return o;
        const mte_propset& ps = b->propsets[id];
        for (uint32_t i = 0; i < ps.count; i++) {
            uint32_t k = b->prop_keys[ps.first + i], v = b->prop_vals[ps.first + i];
            std::string ktxt(b->key_text + b->key_offsets[k], b->key_text + b->key_offsets[k + 1]);
            std::string vtxt(b->val_text + b->val_offsets[v], b->val_text + b->val_offsets[v + 1]);
            JVP kv = parse(ktxt);
            o.set(kv->s, parse(vtxt));
        }
        return o;
    }

    void applyBatch(const mte_batch* b, uint32_t d) {
        // client names in short-id order; the observer is short id 0
        uint32_t c0 = b->doc_client_offsets[d], c1 = b->doc_client_offsets[d + 1];
        std::vector<std::string> names;
        for (uint32_t c = c0; c < c1; c++)
            names.emplace_back(b->client_names + b->client_name_offsets[c],
                               b->client_names + b->client_name_offsets[c + 1]);
        const uint16_t* payload = b->payload + b->doc_payload_offsets[d];
        std::vector<Node*> loadSegs;
        std::vector<Segment*> bodySegs;
        int bodyClient = NonCollabClient;
        int appendPos = 0;
        for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1] && !status; i++) {
            mte_op op = b->ops[i];
            try {
                if (op.client >= names.size()) throw EngineError(MTE_DOC_UNSUPPORTED, "client id out of range");
                int shortId = getOrAddShortClientId(names[op.client]);
                if (shortId != op.client) throw EngineError(MTE_DOC_UNSUPPORTED, "client ids not in first-appearance order");
                if (op.type >= MTE_OP_LOAD_SEG && op.type != MTE_OP_RELPOS) {  // summary records (include/mte.h; loadSnapshot above)
                    if (op.type == MTE_OP_LOAD_NODE) continue;  // the engine's shape hint; rebuilt here
                    if (op.type == MTE_OP_LOAD_END) {
                        mt.reloadFromSegments(loadSegs);
                        loadSegs.clear();
                        mt.startCollaboration(0, op.msn, op.seq);
                        if (!bodySegs.empty())  // loadBody's single flush (snapshotLoader.ts:203-213)
                            mt.insertSegments(mt.localLength(mt.root), bodySegs, 0, bodyClient, 0);
                        bodySegs.clear();
                        continue;
                    }
                    if (op.type == MTE_OP_LOAD_APPEND) {  // loadBody's appends (loadSnapshot above)
                        const int len = (op.flags & MTE_F_LOAD_MARKER) ? 1 : (int)op.b;
                        if (op.flags & MTE_F_APPEND_FIRST) appendPos = mt.localLength(mt.root);
                        const int pos = appendPos;
                        appendPos += len;
                        if (len == 0) continue;
                        if (op.flags & MTE_F_APPEND_REPEAT) {
                            if (mt.getLength(UniversalSequenceNumber, op.client) >= pos)
                                throw EngineError(MTE_DOC_UNSUPPORTED, "loadBody re-links a segment object");
                            continue;
                        }
                    } else if (op.type != MTE_OP_LOAD_SEG) {
                        throw EngineError(MTE_DOC_UNSUPPORTED, "unknown record");
                    }
                    Segment* s = mt.newSegment();
                    if (op.flags & MTE_F_LOAD_MARKER) {
                        s->marker = true;
                        tag(s, (uint32_t)op.a);
                        s->len = 1;
                    } else {
                        s->text.assign((const char16_t*)payload + op.a, op.b);
                        s->len = (int)op.b;
                    }
                    if (op.props) MergeTree::addProperties(s, propset(b, op.props), false);
                    if (op.flags & MTE_F_LOAD_BODY) {
                        bodySegs.push_back(s);
                        bodyClient = op.client;
                        continue;
                    }
                    if (op.type == MTE_OP_LOAD_APPEND) {
                        if (op.flags & MTE_F_LOAD_REMOVED) {
                            if (op.pos1 < 0 || (size_t)op.pos1 >= names.size() ||
                                getOrAddShortClientId(names[op.pos1]) != op.pos1)
                                throw EngineError(MTE_DOC_UNSUPPORTED, "removed client id");
                            s->removed = true;
                            s->removedSeq = op.ref_seq;
                            s->removedClientId = op.pos1;
                        }
                        std::vector<Segment*> one{s};
                        mt.insertSegments(appendPos - s->len, one, UniversalSequenceNumber, op.client, op.seq);
                        continue;
                    }
                    s->seq = op.seq;
                    s->clientId = op.client;
                    if (op.flags & MTE_F_LOAD_REMOVED) {
                        if (op.pos1 < 0 || (size_t)op.pos1 >= names.size() ||
                            getOrAddShortClientId(names[op.pos1]) != op.pos1)
                            throw EngineError(MTE_DOC_UNSUPPORTED, "removed client id");
                        s->removed = true;
                        s->removedSeq = op.ref_seq;
                        s->removedClientId = op.pos1;
                    }
                    loadSegs.push_back(s);
                    continue;
                }
                // a cell op needs both vectors (orc_matrix_* replays a matrix from its messages)
                if (op.type == MTE_OP_CELL) throw EngineError(MTE_DOC_UNSUPPORTED, "cell record in a one-document replay");
                if (op.type != MTE_OP_NOOP && !(mt.cw.currentSeq < op.seq))
                    throw EngineError(MTE_DOC_SEQ_ORDER, "seq <= currentSeq");
                if (op.flags & MTE_F_REL) relPositions(b, i, d, op);
                switch (op.type) {
                    case MTE_OP_INSERT:
                    case MTE_OP_INSERT_MARKER: {
                        Segment* s = mt.newSegment();
                        if (op.type == MTE_OP_INSERT && (op.flags & MTE_F_PERM)) {  // permutation run, handles unallocated
                            s->perm = true;
                            s->len = (int)op.b;
                        } else if (op.type == MTE_OP_INSERT) {
                            s->text.assign((const char16_t*)payload + op.a, op.b);
                            s->len = (int)op.b;
                        } else {
                            s->marker = true;
                            tag(s, op.b);
                            s->len = 1;
                        }
                        if (op.props) MergeTree::addProperties(s, propset(b, op.props), false);
                        std::vector<Segment*> segs{s};
                        mt.insertSegments(op.pos1, segs, op.ref_seq, op.client, op.seq);
                        opsApplied++;
                        break;
                    }
                    case MTE_OP_REMOVE:
                        mt.markRangeRemoved(op.pos1, op.a, op.ref_seq, op.client, op.seq);
                        opsApplied++;
                        break;
                    case MTE_OP_ANNOTATE:
                        mt.annotateRange(op.pos1, op.a, propset(b, op.props), (op.flags & MTE_F_REWRITE) != 0,
                                         op.ref_seq, op.client, op.seq);
                        opsApplied++;
                        break;
                    default: break;
                }
                if (op.flags & MTE_F_END_OF_MSG) updateSeqNumbers(op.msn, op.seq);
            } catch (EngineError& e) {
                status = e.code;
                failingSeq = op.seq;
                error = e.what();
            }
        }
    }

    // ---- synthetic workload ------------------------------------------------------
    // A CPU restatement of the GPU generator (fluidframework_amd/csrc/engine.hpp generate_run; the
    // generator is this build's own code, not the reference's): 8 writers draw each op from their own
    // view getLength(refSeq, client) of the tree as it stands, and the op is applied at once. Used to
    // check that a document's log depends only on its global id (multi-GPU sharding) and that the
    // device generator emits exactly these records.
    struct GenRng {  // xoshiro256** seeded through splitmix64
        uint64_t s[4];
        static uint64_t splitmix(uint64_t& x) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            return z ^ (z >> 31);
        }
        explicit GenRng(uint64_t x) {
            for (int i = 0; i < 4; i++) s[i] = splitmix(x);
        }
        static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
        uint64_t next() {
            uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
            s[2] ^= s[0];
            s[3] ^= s[1];
            s[1] ^= s[2];
            s[0] ^= s[3];
            s[2] ^= t;
            s[3] = rotl(s[3], 45);
            return r;
        }
        uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
    };
    // The generator's property sets in the host's interning order (mte_host.cpp
    // build_generator_props): ids 1..28 one key, then every two-key set.
    static constexpr uint32_t kGenPropsets = 28 + 6 * 49;
    static JObj genPropset(uint32_t id) {
        static const char* keys[4] = {"bold", "italic", "color", "size"};
        static const char* vals[7] = {"true", "false", "\"red\"", "\"blue\"", "10", "12", "null"};
        std::string j;
        if (id >= 1 && id <= 28) {
            j = std::string("{\"") + keys[(id - 1) / 7] + "\":" + vals[(id - 1) % 7] + "}";
        } else {
            uint32_t q = id - 29, pair = q / 49, k1 = 0, k2 = 1;
            for (uint32_t a = 0, n = 0; a < 4; a++)
                for (uint32_t b2 = a + 1; b2 < 4; b2++, n++)
                    if (n == pair) k1 = a, k2 = b2;
            j = std::string("{\"") + keys[k1] + "\":" + vals[(q % 49) / 7] + ",\"" + keys[k2] + "\":" + vals[q % 7] + "}";
        }
        return parse(j)->o;
    }
    // kind 2: C2 insert/remove around a 2048-char target; 3: C3 annotate + forced ties/overlaps;
    // 5: the C2 mix with every writer's refSeq within 64 of the current seq.
    void generate(uint32_t kind, uint32_t gid, uint64_t nops, uint32_t nc, uint64_t seed, mte_op* opsOut,
                  std::vector<uint16_t>* payOut) {
        GenRng rng(0xF1D0C0DEull ^ (uint64_t)gid ^ (seed * 0x9E3779B97F4A7C15ull));
        std::vector<int> ref(nc, 0), sidOf(nc, 0);
        int nextShort = 1, lastC = -1, lastR = 0, lastPos = 0;
        uint32_t pay = 0;
        for (uint64_t step = 0; step < nops && !status; step++) {
            const int seq = (int)step + 1, cur = seq - 1;
            const uint32_t c = rng.below(nc);
            if (rng.below(4) == 0) {
                ref[c] = cur;
            } else {
                int nr = ref[c] + (int)rng.below(5);
                ref[c] = nr < cur ? nr : cur;
            }
            if (kind == 5 && ref[c] < cur - 64) ref[c] = cur - 64;
            bool forced = false;  // (short-circuit order: the draw happens only past the first tests)
            if (kind == 3 && lastC >= 0 && (uint32_t)lastC != c && rng.below(100) < 15 && lastR >= ref[c]) {
                ref[c] = lastR;
                forced = true;
            }
            if (sidOf[c] == 0) {
                sidOf[c] = nextShort++;
                getOrAddShortClientId("client-" + std::to_string(c));
            }
            const int C = sidOf[c], R = ref[c];
            const int len = mt.getLength(R, C);
            const uint32_t roll = rng.below(100);
            uint32_t type;
            if (len == 0) type = MTE_OP_INSERT;
            else if (kind == 3) type = roll < 45 ? MTE_OP_INSERT : (roll < 80 ? MTE_OP_REMOVE : MTE_OP_ANNOTATE);
            else type = roll < (len < 2048 ? 60u : 40u) ? MTE_OP_INSERT : MTE_OP_REMOVE;
            mte_op op{};
            op.seq = seq;
            op.ref_seq = R;
            op.client = (uint8_t)C;
            op.flags = MTE_F_END_OF_MSG;
            op.type = (uint8_t)type;
            try {
                if (type == MTE_OP_INSERT) {
                    const int pos = forced ? (lastPos < len ? lastPos : len) : (int)rng.below((uint32_t)len + 1);
                    const uint32_t n = 1 + rng.below(8);
                    op.pos1 = pos;
                    op.a = (int32_t)pay;
                    op.b = n;
                    Segment* s = mt.newSegment();
                    for (uint32_t i = 0; i < n; i++) {
                        const char16_t ch = (char16_t)(u'a' + rng.below(26));
                        s->text.push_back(ch);
                        if (payOut) payOut->push_back((uint16_t)ch);
                    }
                    s->len = (int)n;
                    pay += n;
                    if (kind == 3 && rng.below(4) == 0) op.props = 1 + rng.below(kGenPropsets);
                    if (op.props) MergeTree::addProperties(s, genPropset(op.props), false);
                    std::vector<Segment*> segs{s};
                    mt.insertSegments(pos, segs, R, C, seq);
                } else {
                    const int a = forced ? (lastPos < len ? lastPos : len - 1) : (int)rng.below((uint32_t)len);
                    const int n = 1 + (int)rng.below(16);
                    op.pos1 = a;
                    op.a = a + n < len ? a + n : len;
                    if (type == MTE_OP_ANNOTATE) {
                        op.props = 1 + rng.below(kGenPropsets);
                        mt.annotateRange(op.pos1, op.a, genPropset(op.props), false, R, C, seq);
                    } else {
                        mt.markRangeRemoved(op.pos1, op.a, R, C, seq);
                    }
                }
                opsApplied++;
                int msn = ref[0];
                for (uint32_t q = 1; q < nc; q++) msn = ref[q] < msn ? ref[q] : msn;
                op.msn = msn;
                lastC = (int)c;
                lastR = R;
                lastPos = op.pos1;
                if (opsOut) opsOut[step] = op;
                updateSeqNumbers(msn, seq);
            } catch (EngineError& e) {
                status = e.code;
                failingSeq = seq;
                error = e.what();
            }
        }
    }

    // ---- local, non-collaborative ops (SharedString before attach; generateSharedStrings.ts) --
    void localInsert(int pos, Segment* s) {
        std::vector<Segment*> segs{s};
        mt.insertSegments(pos, segs, mt.cw.currentSeq, mt.cw.clientId, UniversalSequenceNumber);
    }

    // ---- outputs ------------------------------------------------------------------------------
    u16s text() {  // MergeTreeTextHelper.getText(currentSeq, clientId) (textSegment.ts:154-172)
        u16s out;
        auto f = [&](Segment* s) {
            if (!s->marker && !s->removed) out += s->text;
            return true;
        };
        mt.walkAllSegments(mt.root, f);
        return out;
    }

    std::string segmentsJson() {
        std::string o = "[";
        bool first = true;
        auto f = [&](Segment* s) {
            if (!first) o += ",";
            first = false;
            o += "{\"kind\":";
            o += s->marker ? "\"M\"" : s->perm ? "\"P\"" : "\"T\"";
            if (s->marker) o += ",\"refType\":" + std::to_string(s->refType);
            else if (s->perm) o += ",\"start\":" + std::to_string(s->start);
            else { o += ",\"text\":"; js_quote(o, s->text); }
            o += ",\"len\":" + std::to_string(s->len) + ",\"seq\":" + std::to_string(s->seq) + ",\"client\":";
            js_quote(o, utf8_to_u16(longId(s->clientId).data(), longId(s->clientId).size()));
            if (s->removed) {
                o += ",\"removedSeq\":" + std::to_string(s->removedSeq) + ",\"removedClient\":";
                std::string rc = longId(s->removedClientId);
                js_quote(o, utf8_to_u16(rc.data(), rc.size()));
            }
            std::vector<int> ov = s->overlap;
            std::sort(ov.begin(), ov.end());
            o += ",\"overlap\":[";
            for (size_t i = 0; i < ov.size(); i++) {
                if (i) o += ",";
                std::string n = longId(ov[i]);
                js_quote(o, utf8_to_u16(n.data(), n.size()));
            }
            o += "],\"props\":";
            if (s->hasProps) {
                std::string pj;
                props_json(pj, s->props);
                js_quote(o, utf8_to_u16(pj.data(), pj.size()));
            } else {
                o += "null";
            }
            o += "}";
            return true;
        };
        mt.walkAllSegments(mt.root, f);
        o += "]";
        return o;
    }

    // SnapshotV1.extractSync (snapshotV1.ts:151-247) + emit (:85-149); blobs in tree-entry order
    std::vector<std::string> snapshotBlobs(uint32_t chunkSize) {
        int minSeq = mt.cw.minSeq, currentSeq = mt.cw.currentSeq;
        std::vector<std::string> segJson;
        std::vector<int> segLen;
        // coalescing candidate: owned copy (clone + append never mutates the tree)
        std::unique_ptr<Segment> prevClone;
        Segment* prev = nullptr;
        auto pushSeg = [&](Segment* s) {
            if (!s) return;
            std::string j;
            segment_json(j, s);
            segJson.push_back(j);
            segLen.push_back(s->len);
        };
        auto f = [&](Segment* s) {
            if (s->seq == UnassignedSequenceNumber || (s->removed && s->removedSeq <= minSeq)) return true;
            if (s->seq <= minSeq && (!s->removed || s->removedSeq == UnassignedSequenceNumber)) {
                if (!prev) {
                    prev = s;
                } else if (canAppend(prev, s) && matchProperties(prev, s)) {
                    auto c = std::make_unique<Segment>(*prev);
                    appendSeg(c.get(), s);
                    prevClone = std::move(c);
                    prev = prevClone.get();
                } else {
                    pushSeg(prev);
                    prevClone.reset();
                    prev = s;
                }
            } else {
                pushSeg(prev);
                prevClone.reset();
                prev = nullptr;
                std::string raw = "{\"json\":";
                segment_json(raw, s);
                if (s->seq > minSeq) {
                    raw += ",\"seq\":" + js_number(s->seq) + ",\"client\":";
                    std::string c = longId(s->clientId);
                    js_quote(raw, utf8_to_u16(c.data(), c.size()));
                }
                if (s->removed) {
                    raw += ",\"removedSeq\":" + js_number(s->removedSeq) + ",\"removedClient\":";
                    std::string c = longId(s->removedClientId);
                    js_quote(raw, utf8_to_u16(c.data(), c.size()));
                }
                raw += "}";
                segJson.push_back(raw);
                segLen.push_back(s->len);
            }
            return true;
        };
        mt.walkAllSegments(mt.root, f);
        pushSeg(prev);

        // emit: greedy chunks (getSeqLengthSegs :57-79)
        struct Chunk { size_t start, count; long long length; };
        std::vector<Chunk> chunks;
        size_t total = 0;
        long long totalLen = 0;
        do {
            Chunk c{total, 0, 0};
            while (c.length < (long long)chunkSize && c.start + c.count < segJson.size()) {
                c.length += segLen[c.start + c.count];
                c.count++;
            }
            chunks.push_back(c);
            total += c.count;
            totalLen += c.length;
        } while (total < segJson.size());
        auto chunkJson = [&](const Chunk& c, bool header) {
            std::string o = "{\"version\":\"1\",\"segmentCount\":" + std::to_string(c.count) +
                            ",\"length\":" + std::to_string(c.length) + ",\"segments\":[";
            for (size_t i = 0; i < c.count; i++) {
                if (i) o += ",";
                o += segJson[c.start + i];
            }
            o += "],\"startIndex\":" + std::to_string(c.start);
            if (header) {
                o += ",\"headerMetadata\":{\"minSequenceNumber\":" + js_number(minSeq) +
                     ",\"sequenceNumber\":" + js_number(currentSeq) + ",\"orderedChunkMetadata\":[{\"id\":\"header\"}";
                for (size_t i = 1; i < chunks.size(); i++) o += ",{\"id\":\"body_" + std::to_string(i - 1) + "\"}";
                o += "],\"totalLength\":" + std::to_string(totalLen) +
                     ",\"totalSegmentCount\":" + std::to_string(total) + "}";
            }
            o += "}";
            return o;
        };
        std::vector<std::string> blobs;
        for (size_t i = 0; i < chunks.size(); i++) blobs.push_back(chunkJson(chunks[i], i == 0));
        return blobs;
    }

    std::string snapshotTree(uint32_t chunkSize) {
        auto blobs = snapshotBlobs(chunkSize);
        std::string o = "{\"entries\":[";
        for (size_t i = 0; i < blobs.size(); i++) {
            if (i) o += ",";
            std::string path = i == 0 ? "header" : "body_" + std::to_string(i - 1);
            o += "{\"mode\":\"100644\",\"path\":\"" + path + "\",\"type\":\"Blob\",\"value\":{\"contents\":";
            js_quote(o, utf8_to_u16(blobs[i].data(), blobs[i].size()));
            o += ",\"encoding\":\"utf-8\"}}";
        }
        o += "],\"id\":null}";
        return o;
    }

    // SnapshotLegacy.extractSync (snapshotlegacy.ts:184-238) + emit (:103-182) through
    // serializeAsMinSupportedVersion (snapshotChunks.ts:75-111): the view at minSeq (segments inserted
    // at or below minSeq and not removed at or below it) coalesced, a header chunk of at least
    // chunkSize characters, one body chunk with the rest, and the catch-up messages above minSeq
    // (sequence.ts:584-595: messagesSinceMSNChange trimmed, minimumSequenceNumber set to minSeq).
    // Returns (path, contents) in tree-entry order.
    std::vector<std::pair<std::string, std::string>> snapshotLegacyBlobs(uint32_t chunkSize, const std::string& catchName) {
        const int minSeq = mt.cw.minSeq;
        std::vector<std::string> segJson;
        std::vector<long long> segLen;
        std::unique_ptr<Segment> prevClone;
        Segment* prev = nullptr;
        auto pushSeg = [&](Segment* x) {
            std::string j;
            segment_json(j, x);
            segJson.push_back(j);
            segLen.push_back(x->len);
        };
        auto f = [&](Segment* x) {
            if (x->seq != UnassignedSequenceNumber && x->seq <= minSeq &&
                (!x->removed || x->removedSeq == UnassignedSequenceNumber || x->removedSeq > minSeq)) {
                if (prev && canAppend(prev, x) && matchProperties(prev, x)) {
                    auto c = std::make_unique<Segment>(*prev);
                    appendSeg(c.get(), x);
                    prevClone = std::move(c);
                    prev = prevClone.get();
                } else {
                    if (prev) pushSeg(prev);
                    prevClone.reset();
                    prev = x;
                }
            }
            return true;
        };
        mt.walkAllSegments(mt.root, f);
        if (prev) pushSeg(prev);
        long long total = 0;  // segmentsTotalLength, fixed up to the segments' sum (:228-236)
        for (long long l : segLen) total += l;
        const size_t n = segJson.size();
        // getSeqLengthSegs (:73-98)
        auto chunk = [&](long long approx, size_t start, size_t& count, long long& length) {
            count = 0;
            length = 0;
            while (length < approx && start + count < n) length += segLen[start + count++];
        };
        auto chunkJson = [&](size_t start, size_t count, long long length, bool header) {
            std::string o = "{\"chunkStartSegmentIndex\":" + std::to_string(start) +
                            ",\"chunkSegmentCount\":" + std::to_string(count) +
                            ",\"chunkLengthChars\":" + std::to_string(length) +
                            ",\"totalLengthChars\":" + std::to_string(total) +
                            ",\"totalSegmentCount\":" + std::to_string(n) +
                            ",\"chunkSequenceNumber\":" + js_number(minSeq) + ",\"segmentTexts\":[";
            for (size_t i = 0; i < count; i++) {
                if (i) o += ",";
                o += segJson[start + i];
            }
            o += "]";
            if (header) {  // buildHeaderMetadataForLegecyChunk (snapshotChunks.ts:178-199)
                o += ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}";
                if (length < total) o += ",{\"id\":\"body\"}";
                o += "],\"sequenceNumber\":" + js_number(minSeq) + ",\"totalLength\":" + std::to_string(total) +
                     ",\"totalSegmentCount\":" + std::to_string(n) + "}";
            }
            o += "}";
            return o;
        };
        std::vector<std::pair<std::string, std::string>> blobs;
        size_t c1 = 0;
        long long l1 = 0;
        chunk(chunkSize, 0, c1, l1);
        blobs.emplace_back("header", chunkJson(0, c1, l1, true));
        if (c1 < n) {
            size_t c2 = 0;
            long long l2 = 0;
            chunk(total, c1, c2, l2);
            blobs.emplace_back("body", chunkJson(c1, c2, l2, false));
        }
        std::string cu = "[";
        bool first = true;
        for (auto& m : catchup) {
            if (num(m->o, u"sequenceNumber") <= minSeq) continue;
            JV c = *m;
            c.o.set(u"minimumSequenceNumber", jnum(minSeq));
            if (!first) cu += ",";
            first = false;
            js_stringify(cu, c);
        }
        cu += "]";
        blobs.emplace_back(catchName, cu);
        return blobs;
    }
    std::string snapshotLegacyTree(uint32_t chunkSize, const std::string& catchName) {
        std::string o = "{\"entries\":[";
        bool firstE = true;
        for (auto& b : snapshotLegacyBlobs(chunkSize, catchName)) {
            if (!firstE) o += ",";
            firstE = false;
            o += "{\"mode\":\"100644\",\"path\":";
            js_quote(o, utf8_to_u16(b.first.data(), b.first.size()));
            o += ",\"type\":\"Blob\",\"value\":{\"contents\":";
            js_quote(o, utf8_to_u16(b.second.data(), b.second.size()));
            o += ",\"encoding\":\"utf-8\"}}";
        }
        o += "],\"id\":null}";
        return o;
    }

    uint64_t checksum(uint32_t chunkSize) {
        uint64_t h = 0xcbf29ce484222325ull;
        std::string t = u16_to_utf8(text());
        h = fnv1a(h, t.data(), t.size());
        for (auto& b : snapshotBlobs(chunkSize)) {
            uint8_t z = 0;
            h = fnv1a(h, &z, 1);
            h = fnv1a(h, b.data(), b.size());
        }
        return h;
    }
};

}  // namespace orc

using orc::Doc;

static char* dupstr(const std::string& s) {
    char* p = (char*)malloc(s.size() + 1);
    memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    return p;
}

namespace orc {
static std::string vector_tree(Doc* d, uint32_t chunk) {
    std::string ht = "[";
    for (size_t i = 0; i < d->handles.size(); i++) ht += (i ? "," : "") + std::to_string(d->handles[i]);
    ht += "]";
    return "{\"entries\":[{\"mode\":\"040000\",\"path\":\"segments\",\"type\":\"Tree\",\"value\":" +
           d->snapshotTree(chunk ? chunk : 10000) +
           "},{\"mode\":\"100644\",\"path\":\"handleTable\",\"type\":\"Blob\",\"value\":"
           "{\"contents\":\"" + ht + "\",\"encoding\":\"utf-8\"}}],\"id\":null}";
}

// ---- SharedMatrix (matrix.ts): both PermutationVectors, the HandleTables and the cells
// SparseArray2D (sparsearray2d.ts:57-235: root indexed by the Morton key of the high 16 bits, then four
// 256-entry tiles by the bytes of the low key), restated with an explicit tile tree.
static uint32_t interlace16(uint32_t x) {  // x8ToInterlacedX16 (sparsearray2d.ts:15-23), 16 bits
    uint32_t r = 0;
    for (int b = 0; b < 16; b++) r |= ((x >> b) & 1u) << (2 * b);
    return r;
}
struct Tile {  // new Array(256).fill(undefined)
    std::unique_ptr<Tile> sub[256];
    JVP val[256];
    bool has[256] = {};
};
struct Matrix {
    Doc rows, cols;
    std::vector<std::unique_ptr<Tile>> root{};  // [undefined]
    size_t rootLen = 1;
    std::string error;
    int status = 0;
    explicit Matrix(const char* obs) : rows(obs), cols(obs) {
        rows.permutation = cols.permutation = true;
        root.resize(1);
        rows.mt.onUnlink = [this](Segment* s) { recycled(rows, s, true); };
        cols.mt.onUnlink = [this](Segment* s) { recycled(cols, s, false); };
    }
    static uint32_t r0(uint32_t row) { return interlace16(row) << 1; }
    static uint32_t c0(uint32_t col) { return interlace16(col); }
    Tile* level(std::unique_ptr<Tile>& t) {  // getLevel (:220-226)
        if (!t) t.reset(new Tile());
        return t.get();
    }
    void setCell(uint32_t row, uint32_t col, JVP v) {  // :89-98
        const uint32_t hi = r0(row >> 16) | c0(col >> 16), lo = r0(row & 0xFFFF) | c0(col & 0xFFFF);
        if (hi >= root.size()) root.resize(hi + 1);
        rootLen = std::max<size_t>(rootLen, hi + 1);
        Tile* t = level(root[hi]);
        t = level(t->sub[lo >> 24]);
        t = level(t->sub[(lo >> 16) & 0xFF]);
        t = level(t->sub[(lo >> 8) & 0xFF]);
        t->val[lo & 0xFF] = v;
        t->has[lo & 0xFF] = (bool)v;
    }
    // clearRows / clearCols (:167-218): every tile of the row (col) in every populated top-level tile
    void clearLine(uint32_t h, bool isRow) {
        for (uint32_t other = 0; other < 0x10000; other++) {
            const uint32_t hi = isRow ? (r0(h >> 16) | c0(other)) : (c0(h >> 16) | r0(other));
            if (hi >= root.size() || !root[hi]) continue;
            const uint32_t lo = isRow ? r0(h & 0xFFFF) : c0(h & 0xFFFF);
            std::function<void(Tile*, int)> walk = [&](Tile* t, int depth) {
                const uint32_t bits = (lo >> (24 - 8 * depth)) & 0xFF;
                for (uint32_t k = 0; k < 16; k++) {
                    const uint32_t key = bits | (isRow ? c0(k) : r0(k));
                    if (depth == 3) {
                        t->val[key] = nullptr;
                        t->has[key] = false;
                    } else if (t->sub[key]) {
                        walk(t->sub[key].get(), depth + 1);
                    }
                }
            };
            walk(root[hi].get(), 0);
        }
    }
    // PermutationVector.onMaintenance UNLINK (permutationvector.ts:357-382) -> handlesRecycledCallback
    // (matrix.ts:626-640), then HandleTable.free of each handle
    void recycled(Doc& v, Segment* s, bool isRow) {
        if (!s->perm || s->start < 1) return;
        for (int i = 0; i < s->len; i++) clearLine((uint32_t)(s->start + i), isRow);
        for (int i = 0; i < s->len; i++) v.freeHandle(s->start + i);
    }
    // SharedMatrix.processCore (matrix.ts:548-605), observer (every message remote)
    void applyMsg(const JV& m) {
        if (status) return;
        const JObj& o = m.o;
        JVP c = o.get(u"contents");
        JVP t = c && c->t == JV::Obj ? c->o.get(u"target") : nullptr;
        if (t) {
            if (t->t == JV::Str && t->s == u"rows") rows.applyMsg(m);
            else if (t->t == JV::Str && t->s == u"cols") cols.applyMsg(m);
            if (rows.status || cols.status) {
                status = rows.status ? rows.status : cols.status;
                error = rows.status ? rows.error : cols.error;
            }
            return;
        }
        JVP ty = o.get(u"type");
        if (!c || c->t != JV::Obj || !ty || ty->t != JV::Str || ty->s != u"op") return;
        try {
            if (Doc::num(c->o, u"type") != 2) throw EngineError(MTE_DOC_UNSUPPORTED, "matrix op without target");
            JVP cid = o.get(u"clientId");
            const std::string name = cid && cid->t == JV::Str ? u16_to_utf8(cid->s) : "";
            const int refSeq = Doc::num(o, u"referenceSequenceNumber");
            const int row = Doc::num(c->o, u"row"), col = Doc::num(c->o, u"col");
            const int ar = rows.adjustPosition(row, refSeq, rows.getOrAddShortClientId(name));
            if (ar < 0) return;
            const int ac = cols.adjustPosition(col, refSeq, cols.getOrAddShortClientId(name));
            if (ac < 0) return;
            const int rh = rows.getAllocatedHandle(ar);
            const int ch = cols.getAllocatedHandle(ac);
            if (rh < 1 || ch < 1) throw EngineError(MTE_DOC_UNSUPPORTED, "invalid handle");
            JVP v = c->o.get(u"value");
            setCell((uint32_t)rh, (uint32_t)ch, v ? v : std::make_shared<JV>());
        } catch (EngineError& e) {
            status = e.code;
            error = e.what();
        }
    }
    // SharedMatrix.loadCore (matrix.ts:528-546): each PermutationVector.load (permutationvector.ts:
    // 284-294: HandleTable.load of the "handleTable" blob, then the merge-tree summary under "segments"),
    // then SparseArray2D.load of the cells blob's first element (sparsearray2d.ts:232-235:
    // nullToUndefined, so every tile of the snapshot exists again, emptied where it held null);
    // `pending` holds only unACKed local writes, none for an observer.
    void loadTile(std::unique_ptr<Tile>& t, const JV& a, int depth) {
        t.reset(new Tile());
        for (size_t i = 0; i < a.a.size() && i < 256; i++) {
            const JVP& x = a.a[i];
            if (!x || x->t == JV::Null) continue;
            if (depth < 3) {
                if (x->t != JV::Arr) throw EngineError(MTE_DOC_UNSUPPORTED, "cells tile is not an array");
                loadTile(t->sub[i], *x, depth + 1);
            } else {
                t->val[i] = x;
                t->has[i] = true;
            }
        }
    }
    void loadSummary(const JV& tree) {
        try {
            Doc* vs[2] = {&rows, &cols};
            const char16_t* paths[2] = {u"rows", u"cols"};
            for (int i = 0; i < 2; i++) {
                JVP e = Doc::treeEntry(tree, paths[i]);
                JVP vt = e && e->t == JV::Obj ? e->o.get(u"value") : nullptr;
                if (!vt) throw EngineError(MTE_DOC_UNSUPPORTED, "matrix summary without a vector");
                JVP he = Doc::treeEntry(*vt, u"handleTable");
                const std::string ht = Doc::blobText(he ? he->o.get(u"value") : nullptr, "handleTable blob missing");
                JVP hv = parse(ht.data(), ht.size());
                if (hv->t != JV::Arr || hv->a.empty()) throw EngineError(MTE_DOC_UNSUPPORTED, "handleTable is not an array");
                vs[i]->handles.clear();
                for (auto& h : hv->a) vs[i]->handles.push_back(h && h->t == JV::Num ? (int)h->n : 0);
                JVP se = Doc::treeEntry(*vt, u"segments");
                JVP st = se && se->t == JV::Obj ? se->o.get(u"value") : nullptr;
                if (!st) throw EngineError(MTE_DOC_UNSUPPORTED, "vector summary without segments");
                vs[i]->loadSnapshot(*st);
                if (vs[i]->status) {
                    status = vs[i]->status;
                    error = vs[i]->error;
                    return;
                }
            }
            JVP ce = Doc::treeEntry(tree, u"cells");
            const std::string ct = Doc::blobText(ce ? ce->o.get(u"value") : nullptr, "cells blob missing");
            JVP cv = parse(ct.data(), ct.size());
            if (cv->t != JV::Arr || cv->a.empty() || !cv->a[0] || cv->a[0]->t != JV::Arr)
                throw EngineError(MTE_DOC_UNSUPPORTED, "cells blob is not [cells, pending]");
            const JV& r = *cv->a[0];
            root.clear();
            root.resize(std::max<size_t>(1, r.a.size()));
            rootLen = std::max<size_t>(1, r.a.size());
            for (size_t k = 0; k < r.a.size(); k++)
                if (r.a[k] && r.a[k]->t == JV::Arr) loadTile(root[k], *r.a[k], 0);
        } catch (EngineError& e) {
            status = e.code;
            error = e.what();
        }
    }
    std::string cellsJson() {  // JSON.stringify([cells.snapshot(), pending.snapshot()])
        std::string o = "[[";
        std::function<void(const Tile*, int)> tile = [&](const Tile* t, int depth) {
            o += "[";
            for (int i = 0; i < 256; i++) {
                if (i) o += ",";
                if (depth < 3) {
                    if (t->sub[i]) tile(t->sub[i].get(), depth + 1);
                    else o += "null";
                } else if (t->has[i] && t->val[i]) {
                    js_stringify(o, *t->val[i]);
                } else {
                    o += "null";
                }
            }
            o += "]";
        };
        for (size_t k = 0; k < rootLen; k++) {
            if (k) o += ",";
            if (k < root.size() && root[k]) tile(root[k].get(), 0);
            else o += "null";
        }
        return o + "],[null]]";
    }
    std::string tree(uint32_t chunk) {  // snapshotCore (matrix.ts:405-433)
        std::string cells;
        js_quote(cells, utf8_to_u16(cellsJson().c_str(), cellsJson().size()));
        return "{\"entries\":[{\"mode\":\"040000\",\"path\":\"rows\",\"type\":\"Tree\",\"value\":" +
               vector_tree(&rows, chunk) +
               "},{\"mode\":\"040000\",\"path\":\"cols\",\"type\":\"Tree\",\"value\":" + vector_tree(&cols, chunk) +
               "},{\"mode\":\"100644\",\"path\":\"cells\",\"type\":\"Blob\",\"value\":{\"contents\":" + cells +
               ",\"encoding\":\"utf-8\"}}],\"id\":null}";
    }
};
}  // namespace orc
using orc::Matrix;

extern "C" {

Doc* orc_new(const char* observer) { return new Doc(observer); }
void orc_free(Doc* d) { delete d; }
void orc_str_free(char* p) { free(p); }

// Apply a JSON array of ISequencedDocumentMessage (or one message object).
int orc_apply_json(Doc* d, const char* json, size_t len) {
    try {
        orc::JVP v = orc::parse(json, len);
        if (v->t == orc::JV::Arr) {
            for (auto& m : v->a) d->applyMsg(*m);
        } else {
            d->applyMsg(*v);
        }
    } catch (std::exception& e) {
        d->status = MTE_DOC_UNSUPPORTED;
        d->error = e.what();
        return -1;
    }
    return d->status;
}

// SharedMatrix.processCore (matrix.ts:548-560) for one of its PermutationVectors: the messages whose
// contents target it go to its applyMsg; cell ops ("set", no target) allocate row / col handles
// (getAllocatedHandle, permutationvector.ts:174-193), which this restatement does not model.
int orc_apply_matrix_json(Doc* d, const char* json, size_t len, const char* target) {
    d->permutation = true;
    try {
        orc::JVP v = orc::parse(json, len);
        const orc::u16s tgt = orc::utf8_to_u16(target, strlen(target));
        for (auto& m : v->a) {
            if (d->status) break;
            orc::JVP c = m->t == orc::JV::Obj ? m->o.get(u"contents") : nullptr;
            orc::JVP t = c && c->t == orc::JV::Obj ? c->o.get(u"target") : nullptr;
            if (!t) {
                if (c && c->t == orc::JV::Obj) {
                    d->status = MTE_DOC_UNSUPPORTED;
                    d->error = "matrix cell ops (handle allocation) are out of scope";
                    break;
                }
                continue;
            }
            if (t->t == orc::JV::Str && t->s == tgt) d->applyMsg(*m);
        }
    } catch (std::exception& e) {
        d->status = MTE_DOC_UNSUPPORTED;
        d->error = e.what();
        return -1;
    }
    return d->status;
}
// PermutationVector.snapshot (permutationvector.ts:260-273): the merge-tree SnapshotV1 under
// "segments" and the handle table ([1] until a handle is allocated) as a blob.
char* orc_snapshot_vector_json(Doc* d, uint32_t chunk) { return dupstr(vector_tree(d, chunk)); }

Matrix* orc_matrix_new(const char* observer) { return new Matrix(observer); }
void orc_matrix_free(Matrix* m) { delete m; }
int orc_matrix_apply_json(Matrix* m, const char* json, size_t len) {
    try {
        orc::JVP v = orc::parse(json, len);
        if (v->t != orc::JV::Arr) return m->status = MTE_DOC_UNSUPPORTED;
        for (auto& x : v->a) m->applyMsg(*x);
    } catch (std::exception& e) {
        m->status = MTE_DOC_UNSUPPORTED;
        m->error = e.what();
    }
    return m->status;
}
Doc* orc_matrix_vector(Matrix* m, int which) { return which ? &m->cols : &m->rows; }
// SharedMatrix.loadCore (matrix.ts:528-546) from its summary ITree JSON; the matrix must be fresh
int orc_matrix_load_summary(Matrix* m, const char* json, size_t len) {
    try {
        orc::JVP v = orc::parse(json, len);
        m->loadSummary(*v);
    } catch (std::exception& e) {
        m->status = MTE_DOC_UNSUPPORTED;
        m->error = e.what();
    }
    return m->status;
}
char* orc_matrix_snapshot_json(Matrix* m, uint32_t chunk) { return dupstr(m->tree(chunk)); }

// Resume from a summary ITree JSON (SnapshotLoader); the doc must be fresh (observer set).
int orc_load_summary(Doc* d, const char* json, size_t len) { return d->loadSnapshotJson(json, len); }

int orc_apply_batch(Doc* d, const mte_batch* b, uint32_t doc) {
    d->applyBatch(b, doc);
    return d->status;
}

static orc::JObj parse_props(const char* props_json) {
    orc::JObj o;
    if (props_json) {
        orc::JVP v = orc::parse(props_json, strlen(props_json));
        if (v->t == orc::JV::Obj) o = v->o;
    }
    return o;
}

int orc_local_insert_text(Doc* d, int pos, const char* text, const char* props_json) {
    try {
        orc::Segment* s = d->mt.newSegment();
        s->text = orc::utf8_to_u16(text, strlen(text));
        s->len = (int)s->text.size();
        if (props_json) orc::MergeTree::addProperties(s, parse_props(props_json), false);
        d->localInsert(pos, s);
    } catch (orc::EngineError& e) {
        d->status = e.code;
        d->error = e.what();
        return e.code;
    }
    return 0;
}

int orc_local_insert_marker(Doc* d, int pos, int refType, const char* props_json) {
    try {
        orc::Segment* s = d->mt.newSegment();
        s->marker = true;
        s->refType = refType;
        s->len = 1;
        if (props_json) orc::MergeTree::addProperties(s, parse_props(props_json), false);
        d->localInsert(pos, s);
    } catch (orc::EngineError& e) {
        d->status = e.code;
        d->error = e.what();
        return e.code;
    }
    return 0;
}

int orc_local_remove(Doc* d, int start, int end) {
    d->mt.markRangeRemoved(start, end, d->mt.cw.currentSeq, d->mt.cw.clientId, orc::UniversalSequenceNumber);
    return 0;
}

int orc_local_annotate(Doc* d, int start, int end, const char* props_json) {
    d->mt.annotateRange(start, end, parse_props(props_json), false, d->mt.cw.currentSeq, d->mt.cw.clientId,
                        orc::UniversalSequenceNumber);
    return 0;
}

int orc_get_length(Doc* d) { return d->mt.getLength(d->mt.cw.currentSeq, d->mt.cw.clientId); }
int orc_get_length_at(Doc* d, int refSeq, int shortClientId) { return d->mt.getLength(refSeq, shortClientId); }

char* orc_text(Doc* d) { return dupstr(orc::u16_to_utf8(d->text())); }
char* orc_segments_json(Doc* d) { return dupstr(d->segmentsJson()); }
char* orc_snapshot_json(Doc* d, uint32_t chunk) { return dupstr(d->snapshotTree(chunk ? chunk : 10000)); }
uint64_t orc_checksum(Doc* d, uint32_t chunk) { return d->checksum(chunk ? chunk : 10000); }
// Legacy-format merge-tree summary (SnapshotLegacy, the format the reference emits unless
// newMergeTreeSnapshotFormat is set): the ITree JSON, catch-up blob named catch_name.
char* orc_snapshot_legacy_json(Doc* d, uint32_t chunk, const char* catch_name) {
    return dupstr(d->snapshotLegacyTree(chunk ? chunk : 10000, catch_name && *catch_name ? catch_name : "catchupOps"));
}
uint64_t orc_ops_applied(Doc* d) { return d->opsApplied; }

int orc_status(Doc* d, char* msg, size_t cap, long long* failing_seq) {
    if (msg && cap) {
        snprintf(msg, cap, "%s", d->error.c_str());
    }
    if (failing_seq) *failing_seq = d->failingSeq;
    return d->status;
}

int orc_stats(Doc* d, int* leaves, int* removed, int* height) {
    *leaves = *removed = *height = 0;
    d->mt.stats(d->mt.root, *leaves, *removed, *height);
    return 0;
}

// CPU baseline over a sample: replay the listed documents of a batch (in list order, dynamic queue)
// on `threads` threads; returns ops applied. checksums/statuses may be NULL.
uint64_t orc_replay_list(const mte_batch* b, const uint32_t* docs, uint32_t n, int threads, uint64_t* checksums,
                         int32_t* statuses, int with_snapshot) {
    std::atomic<uint32_t> next{0};
    std::atomic<uint64_t> ops{0};
    auto work = [&]() {
        uint64_t local = 0;
        for (uint32_t i; (i = next.fetch_add(1)) < n;) {
            const uint32_t d = docs[i];
            uint32_t c0 = b->doc_client_offsets[d];
            std::string obs(b->client_names + b->client_name_offsets[c0], b->client_names + b->client_name_offsets[c0 + 1]);
            Doc doc(obs.c_str());
            doc.applyBatch(b, d);
            local += doc.opsApplied;
            if (checksums) checksums[i] = with_snapshot ? doc.checksum(10000) : 0;
            if (statuses) statuses[i] = doc.status;
        }
        ops += local;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < std::max(1, threads); i++) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    return ops.load();
}

// CPU baseline / bulk parity: replay docs [d0, d1) of a batch on `threads` threads. Writes one
// checksum (text + SnapshotV1 blobs) and status per doc; returns ops applied.
uint64_t orc_replay_batch(const mte_batch* b, uint32_t d0, uint32_t d1, int threads, const char* observer,
                          uint64_t* checksums, int32_t* statuses, int with_snapshot) {
    std::atomic<uint32_t> next{d0};
    std::atomic<uint64_t> ops{0};
    auto work = [&]() {
        uint64_t local = 0;
        while (true) {
            uint32_t d = next.fetch_add(1);
            if (d >= d1) break;
            uint32_t c0 = b->doc_client_offsets[d];
            std::string obs(b->client_names + b->client_name_offsets[c0],
                            b->client_names + b->client_name_offsets[c0 + 1]);
            Doc doc(observer ? observer : obs.c_str());
            doc.applyBatch(b, d);
            local += doc.opsApplied;
            if (checksums) checksums[d - d0] = with_snapshot ? doc.checksum(10000) : 0;
            if (statuses) statuses[d - d0] = doc.status;
        }
        ops += local;
    };
    if (threads <= 1) {
        work();
    } else {
        std::vector<std::thread> ts;
        for (int i = 0; i < threads; i++) ts.emplace_back(work);
        for (auto& t : ts) t.join();
    }
    return ops.load();
}

// Synthetic log of one document (the GPU generator restated, Doc::generate), replayed into `d`
// (a fresh document with an observer). ops_out: n_ops records or NULL; pay_out: the inserted text
// (at most 8 units per op) or NULL, *pay_len its length.
int orc_generate(Doc* d, uint32_t kind, uint32_t gid, uint64_t n_ops, uint32_t n_clients, uint64_t seed,
                 mte_op* ops_out, uint16_t* pay_out, uint64_t* pay_len) {
    std::vector<uint16_t> pay;
    d->generate(kind, gid, n_ops, n_clients, seed, ops_out, pay_out || pay_len ? &pay : nullptr);
    if (pay_out) memcpy(pay_out, pay.data(), pay.size() * 2);
    if (pay_len) *pay_len = pay.size();
    return d->status;
}

// Generate + replay documents gids[0..n) on `threads` threads: checksum and status per document.
uint64_t orc_generate_batch(uint32_t kind, const uint32_t* gids, const uint64_t* n_ops, uint32_t n, uint32_t n_clients,
                            uint64_t seed, int threads, uint64_t* checksums, int32_t* statuses) {
    std::atomic<uint32_t> next{0};
    std::atomic<uint64_t> ops{0};
    auto work = [&]() {
        uint64_t local = 0;
        for (uint32_t i; (i = next.fetch_add(1)) < n;) {
            Doc doc("__observer__");
            doc.generate(kind, gids[i], n_ops[i], n_clients, seed, nullptr, nullptr);
            local += doc.opsApplied;
            if (checksums) checksums[i] = doc.checksum(10000);
            if (statuses) statuses[i] = doc.status;
        }
        ops += local;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < std::max(1, threads); i++) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    return ops.load();
}

}  // extern "C"
