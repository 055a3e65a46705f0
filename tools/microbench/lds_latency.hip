// Microbenchmarks of the latency chains the replay engine is built from (gfx950), measured with
// s_memtime inside one wave: dependent ds_read, ds_read + ballot + readlane, DPP scan, heap-style
// serial LDS walk. Launch with W waves per workgroup, one workgroup per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(1024) void k(uint32_t* out, int iters) {
    __shared__ uint32_t lds[16384];
    const uint32_t t = threadIdx.x, L = t & 63, w = t >> 6;
    for (uint32_t i = t; i < 16384; i += blockDim.x) lds[i] = (i * 7 + 13) & 1023;
    __syncthreads();
    uint32_t base = w * 1024;
    // 1) dependent ds_read_b32 chain (same address across lanes)
    uint32_t x = L & 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) x = lds[base + (x & 1023)];
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    // 2) ds_read (per lane) + ballot + ctz + readlane chain
    uint32_t y = 0;
    for (int i = 0; i < iters; i++) {
        uint32_t v = lds[base + ((y + L) & 1023)];
        uint64_t m = __ballot(v > 500);
        uint32_t j = m ? (uint32_t)__builtin_ctzll(m) : 0;
        y = __builtin_amdgcn_readlane(v, j);
    }
    uint64_t t2 = __builtin_amdgcn_s_memtime();
    // 3) full wave scan (6 DPP) + readlane, dependent
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
    uint64_t t3 = __builtin_amdgcn_s_memtime();
    // 4) lane-0 store then all-lane load of the same word (hand-off through LDS)
    uint32_t q = 0;
    for (int i = 0; i < iters; i++) {
        if (L == 0) lds[base + 5] = q + 1;
        __builtin_amdgcn_wave_barrier();
        q = lds[base + 5];
    }
    uint64_t t4 = __builtin_amdgcn_s_memtime();
    if (L == 0) {
        uint32_t* o = out + (blockIdx.x * 16 + w) * 8;
        o[0] = (uint32_t)(t1 - t0);
        o[1] = (uint32_t)(t2 - t1);
        o[2] = (uint32_t)(t3 - t2);
        o[3] = (uint32_t)(t4 - t3);
        o[4] = x + y + z + q;
    }
}

int main() {
    uint32_t* d;
    hipMalloc(&d, 256 * 16 * 8 * 4);
    const int iters = 4096;
    for (int W : {1, 2, 4, 8, 16}) {
        hipLaunchKernelGGL(k, dim3(256), dim3(64 * W), 0, 0, d, iters);
        hipDeviceSynchronize();
        uint32_t h[256 * 16 * 8];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        double s[4] = {0, 0, 0, 0};
        for (int b = 0; b < 256; b++)
            for (int w = 0; w < W; w++)
                for (int i = 0; i < 4; i++) s[i] += h[(b * 16 + w) * 8 + i];
        printf("waves/CU=%2d  cycles/iter: ds_read chain %.1f | read+ballot+readlane %.1f | dpp scan %.1f | lane0 store->load %.1f\n",
               W, s[0] / (256.0 * W * iters), s[1] / (256.0 * W * iters), s[2] / (256.0 * W * iters), s[3] / (256.0 * W * iters));
    }
    return 0;
}
