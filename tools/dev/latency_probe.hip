// Probe: what one dependent global access costs a lone lane on an otherwise idle MI355X, and why the
// deep check's and the expand's serial chains pay ~3-5 us per access ("What's weak" 2-3).
//
// A chain of K lines, each visited once in random order (cold: a 1-GiB sweep evicts L2 and the
// Infinity Cache first), is chased by one lane; every step's time is taken with s_memrealtime
// (100 MHz) and s_memtime (shader clock).  Modes:
//   chase      the bare pointer chase over a footprint F (the lines spread over F)
//   visit      + a dependent probe of a second table (V bytes), as a visited-map probe follows a header
//   store      + a store into a staging region every step (vmcnt counts stores too: the next load's
//              wait includes the store's completion)
//   instr      + N dependent VALU/SALU instructions per step (a state machine's work between accesses)
//   again      the same lines right after (their lines cached, the TLB warm)
//   load       the chase while 8 waves per SIMD on every CU chase their own chains (a busy chip)
// Allocations: hipMalloc (default), or hipExtMallocWithFlags(hipDeviceMallocContiguous), or the
// footprint as 64-MiB pieces from separate hipMalloc calls (fragmented).
// Prints one line per configuration: median / p10 / p90 ns per step and cycles per step.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dev/latency_probe tools/dev/latency_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define OK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

constexpr uint64_t LINE = 128;
constexpr int STEPS = 4096;

// the chain: word at line i holds the byte address of the next line (0 ends it)
__global__ void scatter_chain(const uint64_t* __restrict__ addr, uint32_t k) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) *reinterpret_cast<uint64_t*>(addr[i]) = i + 1 < k ? addr[i + 1] : 0;
}

__global__ void sweep(uint64_t* __restrict__ p, uint64_t words, unsigned long long* sink) {
    uint64_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 0x1234567) atomicAdd(sink, s);
}

__device__ inline uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }
__device__ inline uint64_t ct() { return __builtin_amdgcn_s_memtime(); }

// one lane chases; mode bits: 1 visit probe, 2 store, 4 instr.  Step times go to LDS (a global store
// per step would count in vmcnt and be waited for with the next load), copied out at the end.
__global__ void __launch_bounds__(64) chase(uint64_t start, int mode, const uint64_t* __restrict__ vis, uint64_t vis_mask,
                                            uint64_t* __restrict__ stage, int instr, uint32_t* __restrict__ ns_out,
                                            uint32_t* __restrict__ cyc_out, unsigned long long* sink) {
    __shared__ uint32_t s_ns[STEPS], s_cyc[STEPS];
    int n = 0;
    if (threadIdx.x == 0) {
        uint64_t p = start, acc = 0;
        for (int i = 0; i < STEPS && p; ++i) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const uint64_t t0 = rt(), c0 = ct();
            uint64_t nx = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
            if (mode & 1) {
                const uint64_t h = (nx * 0x9E3779B97F4A7C15ull) >> 17;
                const uint64_t v = __builtin_nontemporal_load(vis + (h & vis_mask));
                nx |= v & 0x8000000000000000ull;               // dependent on the probe, never set
            }
            if (mode & 2) stage[i * 16] = nx;
            if (mode & 4) {
                uint32_t x = (uint32_t)nx;
                for (int j = 0; j < instr; ++j) x = x * 1664525u + 1013904223u;
                acc += x;
                nx |= (uint64_t)(x & 0u);
            }
            p = nx;
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // the step's loads (and store) done
            const uint64_t t1 = rt(), c1 = ct();
            s_ns[i] = (uint32_t)((t1 - t0) * 10);
            s_cyc[i] = (uint32_t)(c1 - c0);
            n = i + 1;
        }
        if (acc == 42) atomicAdd(sink, acc);
    }
    n = __shfl(n, 0);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 64) {
        ns_out[i] = s_ns[i];
        cyc_out[i] = s_cyc[i];
    }
}

__global__ void put_links(const uint64_t* pr, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *reinterpret_cast<uint64_t*>(pr[2 * i]) = pr[2 * i + 1];
}

// background: every lane of many waves chases its own chain endlessly until `stop` (bounded steps)
__global__ void __launch_bounds__(256) busy(const uint64_t* __restrict__ starts, uint32_t n_starts, int steps,
                                            unsigned long long* sink) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t p = starts[t % n_starts], s = 0;
    for (int i = 0; i < steps && p; ++i) {
        p = *reinterpret_cast<const uint64_t*>(p);
        s += p;
    }
    if (s == 1) atomicAdd(sink, s);
}

struct Buf {
    std::vector<void*> pieces;
    std::vector<uint64_t> base;           // device address of each piece
    uint64_t piece = 0;
    void free() {
        for (void* p : pieces) (void)hipFree(p);
        pieces.clear();
        base.clear();
    }
};

Buf alloc(uint64_t bytes, const std::string& how) {
    Buf b;
    if (how == "frag") {
        b.piece = 64ull << 20;
        for (uint64_t o = 0; o < bytes; o += b.piece) {
            void* p = nullptr;
            OK(hipMalloc(&p, b.piece));
            b.pieces.push_back(p);
            b.base.push_back((uint64_t)p);
        }
    } else {
        void* p = nullptr;
        if (how == "contig")
            OK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous));
        else
            OK(hipMalloc(&p, bytes));
        b.piece = bytes;
        b.pieces.push_back(p);
        b.base.push_back((uint64_t)p);
    }
    return b;
}

uint64_t at(const Buf& b, uint64_t off) { return b.base[off / b.piece] + off % b.piece; }

// K distinct random lines of [0, bytes) (K <= lines), in random order; `shift` picks the other lines
// of the same 2-MiB pages for the warm pass
std::vector<uint64_t> chain(const Buf& b, uint64_t bytes, uint32_t k, uint64_t seed, uint64_t line_add) {
    std::mt19937_64 rng(seed);
    const uint64_t lines = bytes / LINE;
    std::vector<uint64_t> a;
    a.reserve(k);
    std::vector<uint64_t> pick;
    if (lines <= 4ull * k) {
        std::vector<uint64_t> all(lines);
        for (uint64_t i = 0; i < lines; ++i) all[i] = i;
        std::shuffle(all.begin(), all.end(), rng);
        pick.assign(all.begin(), all.begin() + std::min<uint64_t>(k, lines));
    } else {
        std::vector<uint64_t> s;
        while (s.size() < k) {
            s.push_back(rng() % lines);
            if (s.size() == k) {
                std::sort(s.begin(), s.end());
                s.erase(std::unique(s.begin(), s.end()), s.end());
            }
        }
        std::shuffle(s.begin(), s.end(), rng);
        pick = s;
    }
    for (uint64_t l : pick) a.push_back(at(b, ((l + line_add) % lines) * LINE));
    return a;
}

struct Stat {
    double med, p10, p90, cyc;
};

Stat stats(std::vector<uint32_t> ns, std::vector<uint32_t> cyc, int n) {
    ns.resize(n);
    cyc.resize(n);
    std::sort(ns.begin(), ns.end());
    std::sort(cyc.begin(), cyc.end());
    return {(double)ns[n / 2], (double)ns[n / 10], (double)ns[n * 9 / 10], (double)cyc[n / 2]};
}

int main(int argc, char** argv) {
    OK(hipSetDevice(0));
    unsigned long long* sink;
    OK(hipMalloc(&sink, 8));
    uint64_t* evict;
    const uint64_t evict_bytes = 1ull << 30;
    OK(hipMalloc(&evict, evict_bytes));
    OK(hipMemset(evict, 1, evict_bytes));
    uint32_t *d_ns, *d_cyc;
    OK(hipMalloc(&d_ns, STEPS * 4));
    OK(hipMalloc(&d_cyc, STEPS * 4));
    uint64_t* d_addr;
    OK(hipMalloc(&d_addr, STEPS * 8ull));
    uint64_t* stage;
    OK(hipMalloc(&stage, STEPS * 16 * 8ull + 4096));
    const uint64_t vis_bytes = 512ull << 20;
    uint64_t* vis;
    OK(hipMalloc(&vis, vis_bytes));
    OK(hipMemset(vis, 0, vis_bytes));
    std::vector<uint32_t> ns(STEPS), cyc(STEPS);

    auto run = [&](const char* name, const Buf& b, uint64_t bytes, int mode, int instr, uint64_t vmask, int line_add,
                   bool load, bool reuse) {
        std::vector<uint64_t> a = chain(b, bytes, STEPS, 1234 + bytes / LINE, line_add);
        const uint32_t k = (uint32_t)a.size();
        OK(hipMemcpy(d_addr, a.data(), k * 8ull, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(scatter_chain, dim3((k + 255) / 256), dim3(256), 0, 0, d_addr, k);
        OK(hipDeviceSynchronize());
        // background chains for "load": 64 per lane's worth of other lines
        uint64_t* d_bg = nullptr;
        std::vector<uint64_t> bg;
        if (load) {
            bg = chain(b, bytes, 65536, 99 + bytes / LINE, 7);
            // chains of 16 lines each: link bg[j] -> bg[j+1] within groups, written on the host side as pairs
            std::vector<uint64_t> starts;
            std::vector<uint64_t> link(bg.size());
            for (size_t j = 0; j < bg.size(); ++j) link[j] = (j % 16 == 15) ? bg[j - 15] : bg[j + 1];  // cycles of 16
            for (size_t j = 0; j < bg.size(); j += 16) starts.push_back(bg[j]);
            uint64_t* d_pairs;
            OK(hipMalloc(&d_pairs, bg.size() * 16));
            std::vector<uint64_t> pr;
            for (size_t j = 0; j < bg.size(); ++j) {
                pr.push_back(bg[j]);
                pr.push_back(link[j]);
            }
            OK(hipMemcpy(d_pairs, pr.data(), pr.size() * 8, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(put_links, dim3((bg.size() + 255) / 256), dim3(256), 0, 0, d_pairs, (uint32_t)bg.size());
            OK(hipDeviceSynchronize());
            OK(hipFree(d_pairs));
            OK(hipMalloc(&d_bg, starts.size() * 8));
            OK(hipMemcpy(d_bg, starts.data(), starts.size() * 8, hipMemcpyHostToDevice));
            bg.assign(starts.begin(), starts.end());
        }
        if (!reuse) {
            hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0, evict, evict_bytes / 8, sink);
            OK(hipDeviceSynchronize());
        }
        hipStream_t s2 = nullptr;
        if (load) {
            OK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
            hipLaunchKernelGGL(busy, dim3(1792), dim3(256), 0, s2, d_bg, (uint32_t)bg.size(), 20000, sink);
        }
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, a[0], mode, vis, vmask, stage, instr, d_ns, d_cyc, sink);
        OK(hipDeviceSynchronize());
        if (s2) OK(hipStreamDestroy(s2));
        if (d_bg) OK(hipFree(d_bg));
        OK(hipMemcpy(ns.data(), d_ns, STEPS * 4, hipMemcpyDeviceToHost));
        OK(hipMemcpy(cyc.data(), d_cyc, STEPS * 4, hipMemcpyDeviceToHost));
        const Stat s = stats(ns, cyc, (int)k - 1);
        printf("%-34s F=%9.3f GiB  ns/step med %6.0f p10 %6.0f p90 %6.0f  cycles/step med %6.0f\n", name,
               bytes / double(1ull << 30), s.med, s.p10, s.p90, s.cyc);
        fflush(stdout);
    };

    const std::string which = argc > 1 ? argv[1] : "all";
    const uint64_t GiB = 1ull << 30;
    if (which == "busy") {
        // the loaded regime only: does the allocation (page / fragment size) decide a miss's cost when
        // every CU chases its own chains over the same footprint?
        for (const char* how : {"malloc", "contig"})
            for (uint64_t F : std::vector<uint64_t>{512ull << 20, 2 * GiB, 8 * GiB, 32 * GiB}) {
                Buf b = alloc(F, how);
                const std::string h(how);
                run((h + " chase").c_str(), b, F, 0, 0, 0, 0, false, false);
                run((h + " chase, chip busy").c_str(), b, F, 0, 0, 0, 0, true, false);
                b.free();
            }
        return 0;
    }
    const std::vector<uint64_t> sizes = {2ull << 20, 64ull << 20, 512ull << 20, 2 * GiB, 8 * GiB, 32 * GiB};
    for (const char* how : {"malloc", "contig", "frag"}) {
        if (which != "all" && which != how) continue;
        for (uint64_t F : sizes) {
            if (std::string(how) == "frag" && F < (128ull << 20)) continue;
            void* probe = nullptr;
            if (std::string(how) == "contig" && hipExtMallocWithFlags(&probe, F, hipDeviceMallocContiguous) != hipSuccess) {
                printf("%-34s F=%9.3f GiB  contiguous allocation refused\n", how, F / double(GiB));
                (void)hipGetLastError();
                continue;
            }
            if (probe) OK(hipFree(probe));
            Buf b = alloc(F, how);
            const std::string h(how);
            run((h + " chase").c_str(), b, F, 0, 0, 0, 0, false, false);
            run((h + " chase, same lines again").c_str(), b, F, 0, 0, 0, 0, false, true);
            if (h == "malloc" && (F == 512ull << 20 || F == 8 * GiB)) {
                run("malloc chase + visit (512 MiB table)", b, F, 1, 0, vis_bytes / 8 - 1, 0, false, false);
                run("malloc chase + visit (4 KiB table)", b, F, 1, 0, 511, 0, false, false);
                run("malloc chase + store", b, F, 2, 0, 0, 0, false, false);
                run("malloc chase + 64 dependent ops", b, F, 4, 64, 0, 0, false, false);
                run("malloc chase + 512 dependent ops", b, F, 4, 512, 0, 0, false, false);
                run("malloc chase, chip busy", b, F, 0, 0, 0, 0, true, false);
            }
            b.free();
        }
    }
    return 0;
}
