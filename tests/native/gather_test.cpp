// TEST INFRASTRUCTURE ONLY: mte_gather_summaries' count / pad / concatenate arithmetic
// (fluidframework_amd/csrc/gather_plan.hpp) driven through a fake all-gather, so the CPU suite covers
// the multi-rank path's host logic (unequal and empty ranks) without RCCL or a GPU
// (tests/test_gather_plan.py).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../fluidframework_amd/csrc/gather_plan.hpp"
#include "../../include/mte.h"

using namespace mte;

extern "C" {

// counts[q] records on rank q; returns 0 when every rank's gathered output is every rank's records in
// rank order, else a nonzero code naming the first failed check.
int gather_selftest(const uint64_t* counts, int world) {
    std::vector<std::vector<mte_doc_summary>> mine((size_t)world);
    for (int q = 0; q < world; q++) {
        mine[q].resize(counts[q]);
        for (uint64_t i = 0; i < counts[q]; i++) {
            memset(&mine[q][i], 0, sizeof(mte_doc_summary));
            mine[q][i].doc_id = (uint32_t)(q * 100000 + i);
            mine[q][i].checksum = 0x9E3779B97F4A7C15ull * (q + 1) + i;
            mine[q][i].ops = (uint32_t)i + 1;
        }
    }
    // every rank computes the same plan from the all-gathered counts
    const GatherPlan g = gather_plan(counts, world);
    uint64_t expect_total = 0;
    for (int q = 0; q < world; q++) expect_total += counts[q];
    if (g.total != expect_total) return 1;
    if (g.stride < 1) return 2;
    for (int q = 0; q < world; q++)
        if (counts[q] > g.stride) return 3;
    // the fake all-gather: rank q's padded block lands at block q of every rank's receive buffer
    std::vector<mte_doc_summary> flat(g.stride * (size_t)world);
    for (int q = 0; q < world; q++) {
        std::vector<mte_doc_summary> blk(g.stride);
        memset(blk.data(), 0xAB, blk.size() * sizeof(mte_doc_summary));  // padding must be overwritten
        gather_pack(mine[q].data(), counts[q], g, blk.data());
        for (uint64_t i = counts[q]; i < g.stride; i++) {
            const unsigned char* b = (const unsigned char*)&blk[i];
            for (size_t k = 0; k < sizeof(mte_doc_summary); k++)
                if (b[k]) return 4;  // zero padding
        }
        memcpy(&flat[(size_t)q * g.stride], blk.data(), g.stride * sizeof(mte_doc_summary));
    }
    std::vector<mte_doc_summary> out(g.total + 1);
    memset(out.data(), 0, out.size() * sizeof(mte_doc_summary));
    gather_concat(flat.data(), counts, world, g, out.data());
    size_t k = 0;
    for (int q = 0; q < world; q++)
        for (uint64_t i = 0; i < counts[q]; i++, k++)
            if (memcmp(&out[k], &mine[q][i], sizeof(mte_doc_summary))) return 5;
    const unsigned char* tail = (const unsigned char*)&out[g.total];
    for (size_t b = 0; b < sizeof(mte_doc_summary); b++)
        if (tail[b]) return 6;  // nothing written past the total
    return 0;
}
}
