// Probe for a streaming check launch: can a kernel that holds every CU see chunks land that a copy
// stream moves in behind it, and read them without stale cache lines?
//   1. the data buffer is filled with 0xFF and a first kernel reads all of it (its lines sit in the
//      XCDs' L2, as a previous batch's would);
//   2. a kernel at full occupancy spins (bounded: 500 ms of wall clock) on per-chunk ready words;
//   3. the copy stream moves the chunks in and marks each ready with hipStreamWriteValue32 (mode 0)
//      or a 4-B H2D copy of a pinned word (mode 1);
//   4. each wave sums its slice of a ready chunk twice: plain loads and system-scope loads.
// Prints whether every wave saw every chunk, both sums against the host's, and when each chunk was
// first seen.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/dev/stream_probe tools/dev/stream_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define OK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            return 2;                                                                            \
        }                                                                                        \
    } while (0)

constexpr uint32_t CHUNKS = 8;
uint64_t CHUNK_WORDS = 64u << 10;                // 256 KB per chunk by default: the buffer fits one XCD's L2

__global__ void __launch_bounds__(256) touch(const uint32_t* data, uint64_t chunk_words, unsigned long long* sink) {
    // every XCD (workgroup b runs on XCD b % 8) reads every line of the buffer
    const uint32_t xcd_blocks = gridDim.x / 8;
    const uint32_t t = (blockIdx.x / 8) * blockDim.x + threadIdx.x;
    unsigned long long s = 0;
    for (uint64_t i = t; i < CHUNKS * chunk_words; i += (uint64_t)xcd_blocks * blockDim.x) s += data[i];
    if (s == 42) atomicAdd(sink, s);
}

__global__ void __launch_bounds__(256) spin(const uint32_t* ready, const uint32_t* data, uint64_t chunk_words,
                                            unsigned long long* sums, unsigned long long* sums_sys, uint32_t* seen_at,
                                            uint32_t* timeouts) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t waves = (gridDim.x * blockDim.x) >> 6;
    const uint64_t t0 = wall_clock64();
    for (uint32_t c = 0; c < CHUNKS; ++c) {
        bool ok = false;
        for (;;) {
            if (__hip_atomic_load(ready + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                ok = true;
                break;
            }
            if (wall_clock64() - t0 > 50000000ull) break;   // 100 MHz: 500 ms
            __builtin_amdgcn_s_sleep(8);
        }
        if (!ok) {
            if (lane == 0) atomicAdd(timeouts, 1u);
            return;
        }
        if (lane == 0) atomicMin(seen_at + c, (uint32_t)((wall_clock64() - t0) / 100u));   // us
        unsigned long long s = 0, s2 = 0;
        const uint32_t* d = data + c * chunk_words;
        for (uint64_t i = (uint64_t)wave * 64 + lane; i < chunk_words; i += (uint64_t)waves * 64) {
            s += d[i];
            s2 += __hip_atomic_load(d + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        atomicAdd(sums + c, s);
        atomicAdd(sums_sys + c, s2);
    }
}

// mode: 0 = hipStreamWriteValue32 marks, 1 = 4-B H2D copies of a pinned word; eighths: the spinning
// grid's share of the resident blocks (8 = every slot)
int run(int mode, int eighths) {
    int cus = 0, per_cu = 0;
    OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, spin, 256, 0));
    const uint32_t blocks = (uint32_t)std::max(8, cus * per_cu * eighths / 8);
    uint32_t *h_data = nullptr, *h_one = nullptr;
    OK(hipHostMalloc((void**)&h_data, CHUNKS * CHUNK_WORDS * 4, hipHostMallocDefault));
    OK(hipHostMalloc((void**)&h_one, 4, hipHostMallocDefault));
    *h_one = 1;
    std::vector<unsigned long long> want(CHUNKS, 0);
    for (uint64_t i = 0; i < CHUNKS * CHUNK_WORDS; ++i) {
        h_data[i] = (uint32_t)(i * 2654435761u) >> 8;
        want[i / CHUNK_WORDS] += h_data[i];
    }
    uint32_t *ready, *data, *seen, *tmo;
    unsigned long long *sums, *sums_sys, *sink;
    OK(hipMalloc(&ready, CHUNKS * 4));
    OK(hipMalloc(&data, CHUNKS * CHUNK_WORDS * 4));
    OK(hipMalloc(&sums, CHUNKS * 8));
    OK(hipMalloc(&sums_sys, CHUNKS * 8));
    OK(hipMalloc(&sink, 8));
    OK(hipMalloc(&seen, CHUNKS * 4));
    OK(hipMalloc(&tmo, 4));
    OK(hipMemset(ready, 0, CHUNKS * 4));
    OK(hipMemset(data, 0xFF, CHUNKS * CHUNK_WORDS * 4));   // stale contents a bad read would show
    OK(hipMemset(sums, 0, CHUNKS * 8));
    OK(hipMemset(sums_sys, 0, CHUNKS * 8));
    OK(hipMemset(seen, 0xFF, CHUNKS * 4));
    OK(hipMemset(tmo, 0, 4));
    OK(hipDeviceSynchronize());
    hipStream_t ks, cs;
    OK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    OK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipLaunchKernelGGL(touch, dim3(2048), dim3(256), 0, ks, data, CHUNK_WORDS, sink);
    OK(hipGetLastError());
    OK(hipStreamSynchronize(ks));
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin, dim3(blocks), dim3(256), 0, ks, ready, data, CHUNK_WORDS, sums, sums_sys, seen, tmo);
    OK(hipGetLastError());
    for (uint32_t c = 0; c < CHUNKS; ++c) {
        OK(hipMemcpyAsync(data + c * CHUNK_WORDS, h_data + c * CHUNK_WORDS, CHUNK_WORDS * 4, hipMemcpyHostToDevice, cs));
        if (mode == 0) OK(hipStreamWriteValue32(cs, ready + c, 1u, 0));
        else OK(hipMemcpyAsync(ready + c, h_one, 4, hipMemcpyHostToDevice, cs));
    }
    OK(hipStreamSynchronize(cs));
    const double copy_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    OK(hipStreamSynchronize(ks));
    const double all_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::vector<unsigned long long> got(CHUNKS), got_sys(CHUNKS);
    std::vector<uint32_t> at(CHUNKS);
    uint32_t t = 0;
    OK(hipMemcpy(got.data(), sums, CHUNKS * 8, hipMemcpyDeviceToHost));
    OK(hipMemcpy(got_sys.data(), sums_sys, CHUNKS * 8, hipMemcpyDeviceToHost));
    OK(hipMemcpy(at.data(), seen, CHUNKS * 4, hipMemcpyDeviceToHost));
    OK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
    printf("mode %d (%s), %llu KB chunks, %u blocks (%d/8 of the resident slots): copies done %.2f ms, kernel done "
           "%.2f ms, waves timed out %u\n", mode, mode == 0 ? "hipStreamWriteValue32" : "4-B H2D flag copy",
           (unsigned long long)(CHUNK_WORDS * 4 / 1024), blocks, eighths, copy_ms, all_ms, t);
    int bad = 0;
    for (uint32_t c = 0; c < CHUNKS; ++c) {
        printf("  chunk %u first seen at %u us, plain-load sum %s, system-scope sum %s\n", c, at[c],
               got[c] == want[c] ? "ok" : "WRONG", got_sys[c] == want[c] ? "ok" : "WRONG");
        bad += (got[c] != want[c]) + (got_sys[c] != want[c]);
    }
    (void)hipFree(ready);
    (void)hipFree(data);
    (void)hipFree(sums);
    (void)hipFree(sums_sys);
    (void)hipFree(sink);
    (void)hipFree(seen);
    (void)hipFree(tmo);
    (void)hipHostFree(h_data);
    (void)hipHostFree(h_one);
    (void)hipStreamDestroy(ks);
    (void)hipStreamDestroy(cs);
    return (t || bad) ? 1 : 0;
}

int main(int argc, char** argv) {
    // args: [chunk KB]; runs both modes at full, 7/8 and 1/2 of the resident slots
    if (argc > 1) CHUNK_WORDS = (uint64_t)atoll(argv[1]) * 256;
    int rc = 0;
    for (int eighths : {8, 7, 4})
        for (int m = 0; m < 2; ++m) {
            const int r = run(m, eighths);
            if (r == 2) return 2;
            rc |= r;
        }
    return rc;
}
