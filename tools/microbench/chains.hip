// Latency of the dependent instruction chains a lone replay wave is made of (gfx950), measured with
// s_memtime by ONE wave per CU (the solo kernel's situation). Each loop iteration depends on the
// previous one. Build: hipcc --offload-arch=gfx950 -O3 chains.hip -o chains
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_TESTS 12
__global__ __launch_bounds__(64) void k(uint32_t* out, int iters, uint32_t seed) {
    __shared__ uint4 lds4[2048];
    uint32_t* lds = (uint32_t*)lds4;
    const uint32_t L = threadIdx.x;
    for (uint32_t i = L; i < 8192; i += 64) lds[i] = (i * 7 + 13 + seed) & 1023;
    __syncthreads();
    uint64_t t[N_TESTS + 1];
    uint32_t acc = 0;
    int ti = 0;
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 0) VALU compare -> uniform branch (v_cmp + s_cbranch on vcc), value carried in a VGPR
    {
        uint32_t v = L + seed;
        for (int i = 0; i < iters; i++) {
            if (__builtin_amdgcn_readfirstlane(v) > 100000u) v += 3;
            v = v * 3 + 1;
        }
        acc += v;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 1) readfirstlane -> SALU -> back to VALU
    {
        uint32_t v = L + seed;
        for (int i = 0; i < iters; i++) {
            uint32_t s = __builtin_amdgcn_readfirstlane(v);
            v = v + (s & 7) + 1;
        }
        acc += v;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 2) readlane with a lane index produced by the previous readlane (pointer chase in registers)
    {
        uint32_t arr = (L * 37 + seed) & 63, k = 0;
        for (int i = 0; i < iters; i++) k = __builtin_amdgcn_readlane(arr, k);
        acc += k;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 3) ballot + ctz + readlane (no memory)
    {
        uint32_t v = (L * 13 + seed) & 63, y = 0;
        for (int i = 0; i < iters; i++) {
            uint64_t m = __ballot(((v + y) & 63) > 31);
            uint32_t j = m ? (uint32_t)__builtin_ctzll(m) : 0;
            y = __builtin_amdgcn_readlane(v, j) + 1;
        }
        acc += y;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 4) dependent ds_read_b32, per-lane address
    {
        uint32_t x = L;
        for (int i = 0; i < iters; i++) x = lds[(x + L) & 1023];
        acc += x;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 5) ds_read_b32 at a uniform address + readfirstlane (scalar pointer chase through LDS)
    {
        uint32_t x = 0;
        for (int i = 0; i < iters; i++) x = __builtin_amdgcn_readfirstlane(lds[x & 1023]);
        acc += x;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 6) ds_read_b128 uniform address, 4 readfirstlanes
    {
        uint32_t x = 0;
        for (int i = 0; i < iters; i++) {
            uint4 q = lds4[x & 1023];
            x = __builtin_amdgcn_readfirstlane(q.x) + __builtin_amdgcn_readfirstlane(q.y) +
                __builtin_amdgcn_readfirstlane(q.z) + __builtin_amdgcn_readfirstlane(q.w);
        }
        acc += x;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 7) ds_bpermute chain
    {
        uint32_t x = (L * 5 + seed) & 63;
        for (int i = 0; i < iters; i++) x = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)(x + L)) & 63;
        acc += x;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 8) lane-0 ds_write then all-lane ds_read of the same word (uniform hand-off)
    {
        uint32_t q = 0;
        for (int i = 0; i < iters; i++) {
            if (L == 0) lds[100] = q + 1;
            __builtin_amdgcn_wave_barrier();
            q = lds[100];
        }
        acc += q;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 9) all-lane ds_write of a uniform value to one word, then read (no exec masking)
    {
        uint32_t q = 0;
        for (int i = 0; i < iters; i++) {
            lds[101] = q + 1;
            __builtin_amdgcn_wave_barrier();
            q = __builtin_amdgcn_readfirstlane(lds[101]);
        }
        acc += q;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 10) 6-step DPP inclusive scan + readlane 63, dependent
    {
        uint32_t z = L;
        for (int i = 0; i < iters; i++) {
            uint32_t a = z, b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x111, 0xf, 0xf, false); a += b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x112, 0xf, 0xf, false); a += b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x114, 0xf, 0xf, false); a += b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x118, 0xf, 0xf, false); a += b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x142, 0xa, 0xf, false); a += b;
            b = __builtin_amdgcn_update_dpp(0u, a, 0x143, 0xc, 0xf, false); a += b;
            z = __builtin_amdgcn_readlane(a, 63) + L;
        }
        acc += z;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    // 11) 20 independent VALU ops per iteration (issue rate of a lone wave)
    {
        uint32_t a = L, b = L + 1, c = L + 2, d = L + 3;
        for (int i = 0; i < iters; i++) {
#pragma unroll
            for (int r = 0; r < 5; r++) {
                a = a * 3 + b;
                b = b ^ (c + 7);
                c = c + (d >> 1);
                d = d * 5 + a;
            }
        }
        acc += a + b + c + d;
    }
    t[ti++] = __builtin_amdgcn_s_memtime();
    if (L == 0) {
        uint32_t* o = out + blockIdx.x * (N_TESTS + 1);
        for (int i = 0; i < N_TESTS; i++) o[i] = (uint32_t)(t[i + 1] - t[i]);
        o[N_TESTS] = acc;
    }
}

int main() {
    const char* names[N_TESTS] = {"valu->branch", "readfirstlane->salu->valu", "readlane chase", "ballot+ctz+readlane",
                                  "ds_read chain", "ds_read+readfirstlane", "ds_read_b128+4 rfl", "bpermute chain",
                                  "lane0 store->load", "all-lane store->load", "dpp scan+readlane", "20 indep VALU"};
    uint32_t* d;
    hipMalloc(&d, 256 * (N_TESTS + 1) * 4);
    const int iters = 4096;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k, dim3(256), dim3(64), 0, 0, d, iters, (uint32_t)rep);
        hipDeviceSynchronize();
    }
    uint32_t h[256 * (N_TESTS + 1)];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int i = 0; i < N_TESTS; i++) {
        double s = 0;
        for (int b = 0; b < 256; b++) s += h[b * (N_TESTS + 1) + i];
        printf("%-28s %8.1f cycles/iter\n", names[i], s / (256.0 * iters));
    }
    return 0;
}
