// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the replay engine uses, on known
// byte counts (MI355X_MICROARCH.md: FETCH_SIZE is ~1/2 of the bytes of 16-B-per-lane streams; other
// widths uncalibrated). Each kernel touches a 1 GiB buffer exactly once (well past the 256 MiB
// Infinity Cache), one launch each; run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
// (separate passes) and divide the bytes by the counter (KiB) x 1024.
// Build: hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t BYTES = 1ull << 30;

// one dword per lane, 256 B per wave instruction (the op-record chunk loads of k_solo)
__global__ void k_read_dword(const uint32_t* p, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
    if (acc == 0x12345678u) sink[0] = acc;
}
// 16 B per lane (k_lds / k_hbmq op-record ring loads)
__global__ void k_read_x4(const uint4* p, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
// 2 B per lane, coalesced (UTF-16 text copies)
// (the sink test must be reachable: an xor of u16 values never reaches 0x12345678, and the
// compiler dropped the whole loop of an earlier version -- FETCH_SIZE 0)
__global__ void k_read_u16(const uint16_t* p, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
    if (acc == 0x1234u) sink[0] = acc;
}
// one dword per lane stores (row output, scratch)
__global__ void k_write_dword(uint32_t* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (uint32_t)i;
}
// 16 B per lane stores
__global__ void k_write_x4(uint4* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    void *a = nullptr, *b = nullptr;
    uint32_t* sink = nullptr;
    if (hipMalloc(&a, BYTES) || hipMalloc(&b, BYTES) || hipMalloc(&sink, 64)) return 1;
    hipMemset(a, 1, BYTES);
    hipDeviceSynchronize();
    const dim3 g(1024 * 8), t(256);
    k_read_dword<<<g, t>>>((const uint32_t*)a, BYTES / 4, sink);
    k_read_x4<<<g, t>>>((const uint4*)a, BYTES / 16, sink);
    k_read_u16<<<g, t>>>((const uint16_t*)a, BYTES / 2, sink);
    k_write_dword<<<g, t>>>((uint32_t*)b, BYTES / 4);
    k_write_x4<<<g, t>>>((uint4*)b, BYTES / 16);
    hipDeviceSynchronize();
    printf("each kernel touches %zu bytes once\n", BYTES);
    return 0;
}
