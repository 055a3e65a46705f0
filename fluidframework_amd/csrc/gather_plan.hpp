// gather_plan.hpp — the host-side arithmetic of mte_gather_summaries (mte_host.cpp): RCCL's
// all-gather moves equal-sized blocks, so every rank sends its summary records padded to the largest
// rank's count, and the gathered blocks are concatenated back in rank order without the padding.
// Header-only and free of HIP/RCCL types, so the CPU suite checks it with a fake all-gather
// (tests/native/gather_test.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace mte {

struct GatherPlan {
    uint64_t stride;  // records per rank block (the largest count, at least 1: RCCL takes no empty block)
    uint64_t total;   // records after concatenation
};

inline GatherPlan gather_plan(const uint64_t* counts, int world) {
    GatherPlan g{1, 0};
    for (int q = 0; q < world; q++) {
        if (counts[q] > g.stride) g.stride = counts[q];
        g.total += counts[q];
    }
    return g;
}

// This rank's send block: its n records followed by zero padding up to g.stride records.
template <class T>
inline void gather_pack(const T* mine, uint64_t n, const GatherPlan& g, T* send) {
    if (n) memcpy(send, mine, n * sizeof(T));
    if (g.stride > n) memset(send + n, 0, (g.stride - n) * sizeof(T));
}

// The all-gathered blocks (world x g.stride records, rank order) without the padding.
template <class T>
inline void gather_concat(const T* flat, const uint64_t* counts, int world, const GatherPlan& g, T* out) {
    size_t k = 0;
    for (int q = 0; q < world; q++)
        for (uint64_t i = 0; i < counts[q]; i++) out[k++] = flat[(size_t)q * g.stride + i];
}

}  // namespace mte
