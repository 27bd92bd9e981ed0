// tools/fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE (and the TCC request counters it
// is derived from) on access patterns of known byte count, as MI355X_MICROARCH.md §HBM asks
// before an absolute is trusted ("other access widths are uncalibrated").  Each kernel reads
// a known number of bytes; tools/fetch_calib.sh profiles one dispatch of each and divides.
//   stream16  : 16 B per lane, coalesced, once over a 1 GiB buffer (the guide's pattern)
//   randN_T   : N-byte aligned chunks (N = 32 / 64 / 128: 2 / 4 / 8 dwordx4 loads by one lane)
//               at hashed positions in a T-byte table (64 MiB: resident in the 256 MiB
//               Infinity Cache; 1 GiB: not)
//   ring32    : each lane reads 32 B of its own 2.5 KB ring per iteration (the RNG window read
//               of the fused kernels: lanes 2,500 B apart, the offset advancing by 32 B)
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16, x *= 0x7feb352du, x ^= x >> 15, x *= 0x846ca68bu, x ^= x >> 16;
    return x;
}

__global__ void k_stream16(const f4v* __restrict__ a, size_t n, float* sink) {
    f4v acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += a[i];
    if (acc.x == 1234.5f) sink[0] = acc.y + acc.z + acc.w;
}

template <int W>   // W = f4 loads per chunk (chunk = 16 W bytes)
__global__ void k_rand(const f4v* __restrict__ t, uint32_t chunk_mask, uint32_t reads, float* sink) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    f4v acc = {0, 0, 0, 0};
    uint32_t h = mix(gid * 0x9e3779b9u + 0x1234567u);
    for (uint32_t r = 0; r < reads; ++r) {
        h = mix(h + r);
        const f4v* c = t + (size_t)(h & chunk_mask) * W;
#pragma unroll
        for (int w = 0; w < W; ++w) acc += c[w];
    }
    if (acc.x == 1234.5f) sink[0] = acc.y + acc.z + acc.w;
}

__global__ void k_ring32(const f4v* __restrict__ ring, uint32_t ring_f4, uint32_t iters, float* sink) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const f4v* r = ring + (size_t)gid * ring_f4;
    f4v acc = {0, 0, 0, 0};
    for (uint32_t i = 0; i < iters; ++i) {
        const uint32_t o = (2 * i) % ring_f4;
        acc += r[o] + r[o + 1];
    }
    if (acc.x == 1234.5f) sink[0] = acc.y + acc.z + acc.w;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
    const size_t GiB = 1ull << 30, MiB = 1ull << 20;
    f4v* big;
    float* sink;
    CK(hipMalloc(&big, GiB));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(big, 0, GiB));
    const int threads = 256, blocks = 8192;                 // 2 M lanes
    const uint32_t lanes = threads * blocks, reads = 64;     // 128 M chunk reads per kernel
    // 1) stream16 over 1 GiB
    hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(threads), 0, 0, big, GiB / 16, sink);
    printf("{\"kernel\": \"k_stream16\", \"bytes\": %zu}\n", GiB);
    // 2) random chunks in 64 MiB and 1 GiB tables
    for (size_t T : {64 * MiB, GiB}) {
        hipLaunchKernelGGL(k_rand<2>, dim3(blocks), dim3(threads), 0, 0, big, (uint32_t)(T / 32 - 1), reads, sink);
        printf("{\"kernel\": \"k_rand<2>\", \"table\": %zu, \"bytes\": %zu}\n", T, (size_t)lanes * reads * 32);
        hipLaunchKernelGGL(k_rand<4>, dim3(blocks), dim3(threads), 0, 0, big, (uint32_t)(T / 64 - 1), reads, sink);
        printf("{\"kernel\": \"k_rand<4>\", \"table\": %zu, \"bytes\": %zu}\n", T, (size_t)lanes * reads * 64);
        hipLaunchKernelGGL(k_rand<8>, dim3(blocks), dim3(threads), 0, 0, big, (uint32_t)(T / 128 - 1), reads, sink);
        printf("{\"kernel\": \"k_rand<8>\", \"table\": %zu, \"bytes\": %zu}\n", T, (size_t)lanes * reads * 128);
    }
    // 3) per-lane rings of 625 f4 (10,000 B: > the 2,496 B of a kRing window so no two lanes
    //    share a line); 2 M lanes x 10 KB = 20 GB would not fit: 98,304 lanes (983 MB)
    const uint32_t ring_f4 = 625, rlanes = 98304, iters = 256;
    hipLaunchKernelGGL(k_ring32, dim3(rlanes / threads), dim3(threads), 0, 0, big, ring_f4, iters, sink);
    printf("{\"kernel\": \"k_ring32\", \"lanes\": %u, \"bytes\": %zu}\n", rlanes, (size_t)rlanes * iters * 32);
    CK(hipDeviceSynchronize());
    CK(hipFree(big));
    CK(hipFree(sink));
    return 0;
}
