// Memory-system calibration for the check path's access pattern (tooling, not part of the engine).
//
// The check kernel is a chain of dependent random reads: a 16-B row header, a 4-B id-table slot,
// 4-B edges.  This program measures, on an 8 GiB buffer (far beyond the 256 MiB Infinity Cache):
//   stream16   coalesced 16 B/lane streaming read of 4 GiB (the guide's FETCH_SIZE reference case)
//   gatherW    one random W-byte read per lane (W = 4, 16, 64, 128), 2^26 reads per launch, with
//              addresses from a hash (no index array), so FETCH_SIZE / reads = bytes counted per
//              random access, and reads / time = the random-access rate the chip sustains
//   chainW     the same reads as dependent chains (each address depends on the previous value),
//              as the DFS issues them: per-lane latency-bound throughput at full occupancy
// Run plain for timings, and under `rocprofv3 --pmc FETCH_SIZE` for the counter calibration.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// one random W-byte read per work item; lines = buffer size / 128
template <int W>
__global__ void gather(const uint32_t* __restrict__ a, uint64_t lines, uint64_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t line = mix64(i * 0x9E3779B97F4A7C15ull + 1) % lines;
        const uint32_t* p = a + line * 32;
        if constexpr (W == 4) {
            acc ^= p[0];
        } else {
#pragma unroll
            for (int k = 0; k < W / 16; ++k) {
                uint4 v = reinterpret_cast<const uint4*>(p)[k];
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// dependent chains: each lane does `hops` reads, the next address derived from the value read
template <int W>
__global__ void chain(const uint32_t* __restrict__ a, uint64_t lines, uint32_t hops, uint32_t* sink) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t x = mix64(t + 7);
    uint32_t acc = 0;
    for (uint32_t h = 0; h < hops; ++h) {
        const uint64_t line = mix64(x) % lines;
        const uint32_t* p = a + line * 32;
        uint32_t v;
        if constexpr (W == 4) {
            v = p[0];
        } else {
            v = 0;
#pragma unroll
            for (int k = 0; k < W / 16; ++k) {
                uint4 q = reinterpret_cast<const uint4*>(p)[k];
                v ^= q.x ^ q.y ^ q.z ^ q.w;
            }
        }
        x += v + 1;
        acc ^= v;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = 8ull << 30;
    const uint64_t lines = bytes / 128;
    uint32_t* a;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto timed = [&](const char* name, double units, const char* unit, double bytes_alg, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-10s %8.3f ms  %8.2f G%s/s  %8.1f GB/s (algorithmic)\n", name, ms, units / ms / 1e6, unit,
               bytes_alg / ms / 1e6);
        fflush(stdout);
    };
    const uint64_t ns = (4ull << 30) / 16;
    timed("stream16", (double)ns * 16, "B", (double)ns * 16,
          [&] { hipLaunchKernelGGL(stream16, dim3(cus * 32), dim3(256), 0, 0, (const uint4*)a, ns, sink); });
    const uint64_t n = 1ull << 26;
    const dim3 g(cus * 32), b(256);
    timed("gather4", n, "reads", n * 4.0, [&] { hipLaunchKernelGGL(gather<4>, g, b, 0, 0, a, lines, n, sink); });
    timed("gather16", n, "reads", n * 16.0, [&] { hipLaunchKernelGGL(gather<16>, g, b, 0, 0, a, lines, n, sink); });
    timed("gather64", n, "reads", n * 64.0, [&] { hipLaunchKernelGGL(gather<64>, g, b, 0, 0, a, lines, n, sink); });
    timed("gather128", n, "reads", n * 128.0, [&] { hipLaunchKernelGGL(gather<128>, g, b, 0, 0, a, lines, n, sink); });
    // chains: b = 256-lane blocks per CU (b=8: 8 waves per SIMD), 64 hops per lane
    const uint32_t hops = 64;
    for (int wps : {2, 4, 8, 16}) {
        const dim3 gc(cus * wps), bc(256);
        const double reads = (double)cus * wps * 256 * hops;
        char nm[32];
        snprintf(nm, sizeof nm, "chain4/b%d", wps);
        timed(nm, reads, "reads", reads * 4, [&] { hipLaunchKernelGGL(chain<4>, gc, bc, 0, 0, a, lines, hops, sink); });
        snprintf(nm, sizeof nm, "chain16/b%d", wps);
        timed(nm, reads, "reads", reads * 16, [&] { hipLaunchKernelGGL(chain<16>, gc, bc, 0, 0, a, lines, hops, sink); });
    }
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
