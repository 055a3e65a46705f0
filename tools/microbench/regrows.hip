// Register-resident rows for the lone critical wave (VERDICT r05 "Experiment A"): what one access to
// a whole 8-field row costs when the row index is only known at run time, in each place a row could
// live. One wave per CU at s_setprio 3 (the critical wave's situation), s_memtime around ITERS
// dependent accesses: each iteration's row index comes from the previous access's data, as in the
// engine (resolve -> the hit row -> its edit).
//   lds      : 2 x ds_read_b128 of the row (the engine's ldrow) + wait
//   va_dyn   : the row's 8 fields as 8 compiler-managed VA<8> arrays (ext_vector_type, dynamic index:
//              the compiler's s_set_gpr_idx_on / v_mov / s_set_gpr_idx_off per field)
//   idx_asm  : the same 64 VGPRs (v[192:255], reserved by clobbers) read with ONE s_set_gpr_idx_on,
//              8 v_mov, one s_set_gpr_idx_off (hand-written)
//   agpr_idx : rows in a[0:63], s_set_gpr_idx_on + 8 v_accvgpr_read (is AGPR indexing honoured?
//              checked against the expected values)
//   agpr_st  : 8 v_accvgpr_read of a static row (no index), the floor of an AGPR row read
//   lds_w    : the row write: 2 x ds_write_b128 (no wait needed: LDS is in order)
//   va_wr    : the row write into the 8 VA<8> arrays (dynamic index)
// Build: hipcc --offload-arch=gfx950 -O3 regrows.hip -o regrows
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 v8 __attribute__((ext_vector_type(8)));

#define N_T 7

__global__ __launch_bounds__(64) void k(u64* out, u32* chk, int iters, u32 seed, u32 do_agpr) {
    __shared__ uint4 lds[2 * 8 * 64];
    const u32 L = threadIdx.x;
    u64 t[N_T + 1];
    int ti = 0;
    // row r, field f of lane L holds (r * 8 + f) * 3 + L + seed; the next row index is (sum & 7)
    for (u32 r = 0; r < 8; r++) {
        lds[r * 64 + L] = make_uint4((r * 8 + 0) * 3 + L + seed, (r * 8 + 1) * 3 + L + seed, (r * 8 + 2) * 3 + L + seed,
                                     (r * 8 + 3) * 3 + L + seed);
        lds[512 + r * 64 + L] = make_uint4((r * 8 + 4) * 3 + L + seed, (r * 8 + 5) * 3 + L + seed,
                                           (r * 8 + 6) * 3 + L + seed, (r * 8 + 7) * 3 + L + seed);
    }
    __syncthreads();
    v8 F[8];
#pragma unroll
    for (int f = 0; f < 8; f++)
#pragma unroll
        for (int r = 0; r < 8; r++) F[f][r] = (r * 8 + f) * 3 + L + seed;
    // the hand-written copies: v[192:255] = row r field f at v[192 + f * 8 + r]; a[0:63] likewise
#pragma unroll
    for (int f = 0; f < 8; f++)
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 x = (r * 8 + f) * 3 + L + seed;
            asm volatile("v_mov_b32 v[%1], %0" ::"v"(x), "i"(192 + f * 8 + r) : "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199",
                         "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213",
                         "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227",
                         "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241",
                         "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
            asm volatile("v_accvgpr_write_b32 a[%1], %0" ::"v"(x), "i"(f * 8 + r) : "a0", "a63");
        }
    __builtin_amdgcn_s_setprio(3);
    u32 acc = 0, r = 0;
    t[ti++] = __builtin_amdgcn_s_memtime();
    // lds
    for (int i = 0; i < iters; i++) {
        const uint4 a = lds[r * 64 + L], b = lds[512 + r * 64 + L];
        const u32 s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
        r = __builtin_amdgcn_readfirstlane(s) & 7u;
        acc += s;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // va_dyn
    for (int i = 0; i < iters; i++) {
        u32 s = 0;
#pragma unroll
        for (int f = 0; f < 8; f++) s += F[f][r];
        r = __builtin_amdgcn_readfirstlane(s) & 7u;
        acc += s;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // idx_asm
    for (int i = 0; i < iters; i++) {
        u32 f0, f1, f2, f3, f4, f5, f6, f7;
        asm volatile(
            "s_set_gpr_idx_on %8, gpr_idx(SRC0)\n"
            "v_mov_b32 %0, v192\n v_mov_b32 %1, v200\n v_mov_b32 %2, v208\n v_mov_b32 %3, v216\n"
            "v_mov_b32 %4, v224\n v_mov_b32 %5, v232\n v_mov_b32 %6, v240\n v_mov_b32 %7, v248\n"
            "s_set_gpr_idx_off\n"
            : "=v"(f0), "=v"(f1), "=v"(f2), "=v"(f3), "=v"(f4), "=v"(f5), "=v"(f6), "=v"(f7)
            : "s"(r));
        const u32 s = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
        r = __builtin_amdgcn_readfirstlane(s) & 7u;
        acc += s;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    u32 agpr_sum = 0;
    // agpr_idx (one checked access first; a separate launch, in case the indexed AGPR read is refused)
    if (do_agpr) {
        u32 f0, f1, f2, f3, f4, f5, f6, f7;
        const u32 rr = seed & 7u;
        asm volatile(
            "s_set_gpr_idx_on %8, gpr_idx(SRC0)\n"
            "v_accvgpr_read_b32 %0, a0\n v_accvgpr_read_b32 %1, a8\n v_accvgpr_read_b32 %2, a16\n v_accvgpr_read_b32 %3, a24\n"
            "v_accvgpr_read_b32 %4, a32\n v_accvgpr_read_b32 %5, a40\n v_accvgpr_read_b32 %6, a48\n v_accvgpr_read_b32 %7, a56\n"
            "s_set_gpr_idx_off\n"
            : "=v"(f0), "=v"(f1), "=v"(f2), "=v"(f3), "=v"(f4), "=v"(f5), "=v"(f6), "=v"(f7)
            : "s"(rr));
        agpr_sum = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
    }
    for (int i = 0; i < (do_agpr ? iters : 0); i++) {
        u32 f0, f1, f2, f3, f4, f5, f6, f7;
        asm volatile(
            "s_set_gpr_idx_on %8, gpr_idx(SRC0)\n"
            "v_accvgpr_read_b32 %0, a0\n v_accvgpr_read_b32 %1, a8\n v_accvgpr_read_b32 %2, a16\n v_accvgpr_read_b32 %3, a24\n"
            "v_accvgpr_read_b32 %4, a32\n v_accvgpr_read_b32 %5, a40\n v_accvgpr_read_b32 %6, a48\n v_accvgpr_read_b32 %7, a56\n"
            "s_set_gpr_idx_off\n"
            : "=v"(f0), "=v"(f1), "=v"(f2), "=v"(f3), "=v"(f4), "=v"(f5), "=v"(f6), "=v"(f7)
            : "s"(r));
        const u32 s = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
        r = __builtin_amdgcn_readfirstlane(s) & 7u;
        acc += s;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // agpr_st
    for (int i = 0; i < iters; i++) {
        u32 f0, f1, f2, f3, f4, f5, f6, f7;
        asm volatile(
            "v_accvgpr_read_b32 %0, a1\n v_accvgpr_read_b32 %1, a9\n v_accvgpr_read_b32 %2, a17\n v_accvgpr_read_b32 %3, a25\n"
            "v_accvgpr_read_b32 %4, a33\n v_accvgpr_read_b32 %5, a41\n v_accvgpr_read_b32 %6, a49\n v_accvgpr_read_b32 %7, a57\n"
            : "=v"(f0), "=v"(f1), "=v"(f2), "=v"(f3), "=v"(f4), "=v"(f5), "=v"(f6), "=v"(f7)
            : "s"(r));
        const u32 s = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
        r = __builtin_amdgcn_readfirstlane(s) & 7u;
        acc += s;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // lds_w: write the row r then read one field of row (r + 1) & 7 to pick the next index
    for (int i = 0; i < iters; i++) {
        lds[r * 64 + L] = make_uint4(acc, acc + 1, acc + 2, acc + 3);
        lds[512 + r * 64 + L] = make_uint4(acc + 4, acc + 5, acc + 6, acc + 7);
        r = __builtin_amdgcn_readfirstlane(acc * 5u + (u32)i) & 7u;
        acc += r;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // va_wr
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int f = 0; f < 8; f++) F[f][r] = acc + f;
        r = __builtin_amdgcn_readfirstlane(acc * 5u + (u32)i) & 7u;
        acc += r;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    u32 keep = 0;
#pragma unroll
    for (int f = 0; f < 8; f++)
#pragma unroll
        for (int rr = 0; rr < 8; rr++) keep += F[f][rr];
    if (L == 0) {
        u64* o = out + blockIdx.x * (N_T + 1);
        for (int i = 0; i < N_T; i++) o[i] = t[i + 1] - t[i];
        o[N_T] = acc + keep + lds[(acc & 7) * 64].x;
    }
    // the AGPR index check: the expected sum of row (seed & 7)
    u32 want = 0;
    for (u32 f = 0; f < 8; f++) want += ((seed & 7u) * 8 + f) * 3 + L + seed;
    chk[blockIdx.x * 64 + L] = agpr_sum == want ? 1u : 0u;
}

int main(int argc, char** argv) {
    const u32 do_agpr = argc > 1 ? 1u : 0u;
    const char* names[N_T] = {"lds row read", "va_dyn row read", "idx_asm row read", "agpr_idx row read",
                              "agpr static row read", "lds row write", "va_dyn row write"};
    const int nb = 8, iters = 4000;
    u64* d;
    u32* c;
    hipMalloc(&d, nb * (N_T + 1) * 8);
    hipMalloc(&c, nb * 64 * 4);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d, c, iters, (u32)(rep * 5 + 3), do_agpr);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 1;
        }
    }
    u64 h[nb * (N_T + 1)];
    u32 hc[nb * 64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
    for (int i = 0; i < N_T; i++) {
        double s = 0;
        for (int b = 0; b < nb; b++) s += (double)h[b * (N_T + 1) + i];
        printf("%-22s %8.1f cycles per dependent access\n", names[i], s / (nb * (double)iters));
    }
    int ok = 0;
    for (int i = 0; i < nb * 64; i++) ok += hc[i];
    if (do_agpr) printf("AGPR gpr_idx reads the indexed row: %s (%d of %d lanes)\n", ok == nb * 64 ? "yes" : "NO", ok, nb * 64);
    return 0;
}
