// HBM stream microbenchmark (the measured peak beside the 8 TB/s spec, BASELINE.md / SURVEY §8(d)):
// float4 copy, read-only sum and write-only fill over buffers far larger than the 256 MiB MALL, one
// launch of 8 waves per CU x 4 workgroups per CU, grid-stride. Bytes moved / kernel time (HIP events),
// best of 10 launches after a warm-up.
// Build: hipcc --offload-arch=gfx950 -O3 stream.hip -o stream ; run: ./stream [GiB per buffer]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(512) void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ __launch_bounds__(512) void k_read(const float4* __restrict__ a, float* __restrict__ out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[threadIdx.x] = s;  // never true for the fill below: keeps the loads
}
__global__ __launch_bounds__(512) void k_fill(float4* __restrict__ b, size_t n, float x) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_float4(x, x, x, x);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const size_t bytes = (size_t)(gib * (1ull << 30));
    const size_t n = bytes / sizeof(float4);
    float4 *a, *b;
    float* o;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&o, 4096));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const dim3 grid(cus * 4), blk(512);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill, grid, blk, 0, 0, a, n, 1.0f);
    hipLaunchKernelGGL(k_fill, grid, blk, 0, 0, b, n, 2.0f);
    CHECK(hipDeviceSynchronize());
    const char* names[3] = {"copy (read + write)", "read", "write"};
    const double moved[3] = {2.0 * bytes, (double)bytes, (double)bytes};
    printf("{\"buffer_gib\": %.2f, \"cus\": %d, \"grid\": %u", gib, cus, grid.x);
    for (int t = 0; t < 3; t++) {
        float best = 1e30f;
        for (int r = 0; r < 11; r++) {
            CHECK(hipEventRecord(e0, 0));
            if (t == 0) hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n);
            else if (t == 1) hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, o, n);
            else hipLaunchKernelGGL(k_fill, grid, blk, 0, 0, b, n, 3.0f);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;  // (launch 0 warms up)
        }
        printf(", \"%s_GBps\": %.1f", names[t], moved[t] / (best * 1e-3) / 1e9);
    }
    printf("}\n");
    return 0;
}
