// Issue cost of the instruction kinds a lone replay wave is made of (gfx950), one wave per CU,
// measured with s_memtime around REPS repetitions of a hand-written block (inline asm, so the
// compiler cannot reorder or fold it). Prints cycles per instruction of each block.
// Build: hipcc --offload-arch=gfx950 -O3 issue.hip -o issue
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
#define R4(x) x x x x

struct Test {
    const char* name;
    int n;  // instructions per block
};
#define N_TESTS 18
__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memtime(); }

__global__ __launch_bounds__(64) void k(uint64_t* out, int reps, uint32_t seed) {
    uint64_t t[N_TESTS + 1];
    int ti = 0;
    uint32_t a = threadIdx.x + seed, b = a * 3, c = a * 5, d = a * 7, e = a + 11, f = a + 13, g = a + 17, h = a + 19;
    uint32_t sa = seed, sb = seed + 1, sc = seed + 2, sd = seed + 3;
    __builtin_amdgcn_s_setprio(3);
    t[ti++] = now();
    // 0) 64 independent v_add_u32 (8 accumulators)
    for (int i = 0; i < reps; i++)
        asm volatile(R8("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                        "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                     : "v"(a));
    t[ti++] = now();
    // 1) 64 dependent v_add_u32
    for (int i = 0; i < reps; i++) asm volatile(R8(R8("v_add_u32 %0, %0, %1\n")) : "+v"(a) : "v"(b));
    t[ti++] = now();
    // 2) 64 independent s_add_u32
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n")) : "+s"(sa), "+s"(sb) :: "scc");
    t[ti++] = now();
    // 3) 32 v_add + 32 s_add interleaved (does SALU hide under VALU?)
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("v_add_u32 %0, %0, %3\n s_add_u32 %1, %1, 3\n v_add_u32 %2, %2, %3\n s_add_u32 %4, %4, 3\n"))
                     : "+v"(a), "+s"(sa), "+v"(b), "+v"(c), "+s"(sb)
                     :
                     : "scc");
    t[ti++] = now();
    // 4) 64 v_readlane_b32 (independent)
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("v_readlane_b32 %0, %4, 5\n v_readlane_b32 %1, %4, 9\n")) R8(R4("")) "s_add_u32 %2, %0, %1\n s_add_u32 %3, %3, %2\n"
                     : "=s"(sc), "=s"(sd), "=s"(sa), "+s"(sb)
                     : "v"(a)
                     : "scc");
    t[ti++] = now();
    // 5) 64 v_writelane_b32
    for (int i = 0; i < reps; i++) asm volatile(R8(R4("v_writelane_b32 %0, %2, 5\n v_writelane_b32 %1, %2, 9\n")) : "+v"(a), "+v"(b) : "s"(sb));
    t[ti++] = now();
    // 6) 64 v_cmp_lt_u32 -> SGPR pairs (independent)
    {
        uint64_t m0, m1;
        for (int i = 0; i < reps; i++)
            asm volatile(R8(R4("v_cmp_lt_u32 %0, %2, %3\n v_cmp_lt_u32 %1, %3, %2\n")) : "=s"(m0), "=s"(m1) : "v"(a), "v"(b));
        sa += (uint32_t)(m0 ^ m1);
    }
    t[ti++] = now();
    // 7) 64 v_cndmask_b32 with an SGPR-pair mask
    {
        uint64_t m = 0x5555555555555555ull ^ seed;
        for (int i = 0; i < reps; i++)
            asm volatile(R8(R4("v_cndmask_b32 %0, %0, %2, %3\n v_cndmask_b32 %1, %1, %2, %3\n")) : "+v"(a), "+v"(b) : "v"(c), "s"(m));
    }
    t[ti++] = now();
    // 8) one 6-step dependent DPP scan (v_add_u32_dpp + s_nop 1), 12 instructions
    for (int i = 0; i < reps; i++)
        asm volatile(R8(
                         "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n"
                         "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n"
                         "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n"
                         "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n"
                         "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n s_nop 1\n"
                         "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n s_nop 1\n")
                     : "+v"(a));
    t[ti++] = now();
    // 9) two interleaved DPP scans, no nops (24 instructions per block of 12 pairs)
    for (int i = 0; i < reps; i++)
        asm volatile(R4(
                         "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_add_u32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_add_u32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_add_u32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_add_u32_dpp %2, %2, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                     : "+v"(a), "+v"(b), "+v"(c));
    t[ti++] = now();
    // 10) v_cmp -> s_cbranch_vccz (not taken), dependent on the previous VALU, 16 pairs
    for (int i = 0; i < reps; i++)
        asm volatile(R8("v_add_u32 %0, %0, %1\n v_cmp_gt_u32 vcc, %0, %1\n s_cbranch_vccz 1f\n 1:\n"
                        "v_add_u32 %0, %0, %1\n v_cmp_gt_u32 vcc, %0, %1\n s_cbranch_vccz 1f\n 1:\n")
                     : "+v"(a)
                     : "v"(b)
                     : "vcc");
    t[ti++] = now();
    // 11) 32 ds_bpermute_b32 (independent) then one wait
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("ds_bpermute_b32 %0, %2, %1\n")) "s_waitcnt lgkmcnt(0)\n" : "=v"(c), "+v"(b) : "v"(d));
    t[ti++] = now();
    // 12) dependent ds_bpermute chain, 8
    for (int i = 0; i < reps; i++)
        asm volatile(R8("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)\n") : "+v"(c) : "v"(d));
    t[ti++] = now();
    // 13) v_readlane -> s_add -> v_add chain (VALU->SALU->VALU), 8 triples
    for (int i = 0; i < reps; i++)
        asm volatile(R8("v_readlane_b32 %1, %0, 3\n s_add_u32 %1, %1, 1\n v_add_u32 %0, %1, %0\n") : "+v"(a), "=s"(sa) :: "scc");
    t[ti++] = now();
    // 14) SALU -> scc branch, 32 pairs
    for (int i = 0; i < reps; i++) asm volatile(R8(R4("s_add_u32 %0, %0, 1\n s_cbranch_scc1 1f\n 1:\n")) : "+s"(sb) :: "scc");
    t[ti++] = now();
    // 15) 16 ds_read_b128 (independent) + one wait
    {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        __shared__ u4 buf[512];
        const uint32_t addr = (threadIdx.x * 16) & 4095;
        u4 v0, v1;
        for (int i = 0; i < reps; i++)
            asm volatile(R8("ds_read_b128 %0, %2\n ds_read_b128 %1, %2 offset:1024\n") "s_waitcnt lgkmcnt(0)\n"
                         : "=v"(v0), "=v"(v1)
                         : "v"(addr));
        a += v0.x + v1.y;
        if (seed == 12345) buf[threadIdx.x] = v0;
    }
    t[ti++] = now();
    // 16) v_mov_b32 64 independent
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("v_mov_b32 %0, %2\n v_mov_b32 %1, %2\n")) : "=v"(e), "=v"(f) : "v"(g));
    t[ti++] = now();
    // 17) v_readfirstlane 64
    for (int i = 0; i < reps; i++)
        asm volatile(R8(R4("v_readfirstlane_b32 %0, %2\n v_readfirstlane_b32 %1, %2\n")) : "=s"(sc), "=s"(sd) : "v"(a));
    t[ti++] = now();
    if (threadIdx.x == 0) {
        uint64_t* o = out + blockIdx.x * (N_TESTS + 1);
        for (int i = 0; i < N_TESTS; i++) o[i] = t[i + 1] - t[i];
        o[N_TESTS] = a + b + c + d + e + f + g + h + sa + sb + sc + sd;
    }
}

int main() {
    const Test tests[N_TESTS] = {{"v_add indep", 64},      {"v_add dep", 64},        {"s_add indep", 64},
                                 {"v_add/s_add mix", 128}, {"v_readlane", 64},       {"v_writelane", 64},
                                 {"v_cmp->sgpr", 64},      {"v_cndmask", 64},        {"dpp scan+nop (12)", 96},
                                 {"3 dpp chains", 24},     {"v_cmp->cbranch (x3)", 48}, {"ds_bpermute x32+wait", 32},
                                 {"ds_bpermute dep", 8},   {"rl->salu->valu (x3)", 24}, {"salu->scc br (x2)", 64},
                                 {"ds_read_b128 x16+wait", 16}, {"v_mov", 64},       {"v_readfirstlane", 64}};
    uint64_t* d;
    const int nb = 8, reps = 2000;
    hipMalloc(&d, nb * (N_TESTS + 1) * 8);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d, reps, (uint32_t)rep);
        hipDeviceSynchronize();
    }
    uint64_t h[nb * (N_TESTS + 1)];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int i = 0; i < N_TESTS; i++) {
        double s = 0;
        for (int b = 0; b < nb; b++) s += (double)h[b * (N_TESTS + 1) + i];
        s /= nb * (double)reps;
        printf("%-24s %8.1f cycles/block  %6.2f cycles/instr\n", tests[i].name, s, s / tests[i].n);
    }
    return 0;
}
