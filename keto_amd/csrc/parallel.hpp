// Host-side parallel building blocks of the snapshot builder (snapshot.cpp): a dynamic parallel
// for, a parallel sample sort (the reference ORDER BY over 10^8-10^9 tuples), and a
// 64-bit string hash for sharded interning.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string_view>
#include <thread>
#include <vector>

namespace keto {

// Builder threads: KETO_BUILD_THREADS, else the hardware's, at most 16 (the GPU box's CPU share).
inline unsigned build_threads() {
    if (const char* e = getenv("KETO_BUILD_THREADS")) return (unsigned)std::max(1, atoi(e));
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Inputs below this many items take the sequential paths (KETO_BUILD_PAR_MIN: tests force the
// parallel ones on small tables).
inline uint64_t par_min() {
    if (const char* e = getenv("KETO_BUILD_PAR_MIN")) return (uint64_t)std::max(1ll, atoll(e));
    return 1ull << 15;
}

// f(begin, end, thread) over [0, n) in chunks handed out dynamically.
template <class F>
void par_chunks(uint64_t n, unsigned threads, uint64_t chunk, F f) {
    if (threads <= 1 || n <= chunk) {
        if (n) f(0, n, 0u);
        return;
    }
    std::atomic<uint64_t> next{0};
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            for (;;) {
                const uint64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                f(b, std::min(n, b + chunk), t);
            }
        });
    for (auto& x : ts) x.join();
}

// f(t) on threads t = 0 .. threads-1
template <class F>
void par_threads(unsigned threads, F f) {
    std::vector<std::thread> ts;
    for (unsigned t = 1; t < threads; ++t) ts.emplace_back([&, t] { f(t); });
    f(0u);
    for (auto& x : ts) x.join();
}

// Sample sort: splitters from a regular sample, per-thread bucket counts, a stable scatter, then
// every bucket sorted on its own.  `less` must be a strict weak order; equal elements may come out
// in any order (the builder's comparators are total orders).
template <class T, class Less>
void parallel_sort(std::vector<T>& v, Less less, unsigned threads) {
    const uint64_t n = v.size();
    if (threads <= 1 || n < par_min()) {
        std::sort(v.begin(), v.end(), less);
        return;
    }
    const uint32_t B = threads * 16;                        // buckets
    const uint64_t ns = std::min<uint64_t>(n, (uint64_t)B * 64);
    std::vector<T> sample(ns);
    for (uint64_t i = 0; i < ns; ++i) sample[i] = v[(uint64_t)((unsigned __int128)i * n / ns)];
    std::sort(sample.begin(), sample.end(), less);
    std::vector<T> split(B - 1);
    for (uint32_t b = 1; b < B; ++b) split[b - 1] = sample[(uint64_t)b * ns / B];
    std::vector<uint16_t> bucket(n);
    std::vector<uint64_t> cnt((uint64_t)threads * B, 0);
    auto slice = [&](unsigned t, uint64_t& lo, uint64_t& hi) {
        lo = (uint64_t)((unsigned __int128)t * n / threads);
        hi = (uint64_t)((unsigned __int128)(t + 1) * n / threads);
    };
    par_threads(threads, [&](unsigned t) {
        uint64_t lo, hi;
        slice(t, lo, hi);
        uint64_t* c = cnt.data() + (uint64_t)t * B;
        for (uint64_t i = lo; i < hi; ++i) {
            const uint32_t b = (uint32_t)(std::upper_bound(split.begin(), split.end(), v[i], less) - split.begin());
            bucket[i] = (uint16_t)b;
            ++c[b];
        }
    });
    std::vector<uint64_t> start(B + 1, 0), off((uint64_t)threads * B);
    {
        uint64_t acc = 0;
        for (uint32_t b = 0; b < B; ++b) {
            start[b] = acc;
            for (unsigned t = 0; t < threads; ++t) {
                off[(uint64_t)t * B + b] = acc;
                acc += cnt[(uint64_t)t * B + b];
            }
        }
        start[B] = acc;
    }
    std::vector<T> out(n);
    par_threads(threads, [&](unsigned t) {
        uint64_t lo, hi;
        slice(t, lo, hi);
        uint64_t* o = off.data() + (uint64_t)t * B;
        for (uint64_t i = lo; i < hi; ++i) out[o[bucket[i]]++] = v[i];
    });
    std::vector<uint16_t>().swap(bucket);
    par_chunks(B, threads, 1, [&](uint64_t b0, uint64_t b1, unsigned) {
        for (uint64_t b = b0; b < b1; ++b) std::sort(out.begin() + start[b], out.begin() + start[b + 1], less);
    });
    v.swap(out);
}

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

inline uint64_t load64(const char* p) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    return w;
}
inline uint32_t load32(const char* p) {
    uint32_t w;
    std::memcpy(&w, p, 4);
    return w;
}

// 64-bit hash of a byte string.  Short strings (the usual identifiers) take no loop and no
// variable-length copy: 1..3 bytes are read as first / middle / last byte, 4..8 as two overlapping
// 32-bit words, 9..16 as two overlapping 64-bit words -- together they cover every byte, so two
// strings of one length that differ anywhere differ in the mixed words.
inline uint64_t hash_bytes(std::string_view s, uint64_t seed = 0x9E3779B97F4A7C15ull) {
    const char* p = s.data();
    const size_t n = s.size();
    uint64_t h = seed ^ (n * 0xC2B2AE3D27D4EB4Full);
    uint64_t a, b;
    if (n <= 16) {
        if (n >= 8) {
            a = load64(p);
            b = load64(p + n - 8);
        } else if (n >= 4) {
            a = load32(p);
            b = load32(p + n - 4);
        } else if (n > 0) {
            a = (uint64_t)(uint8_t)p[0] | (uint64_t)(uint8_t)p[n / 2] << 8 | (uint64_t)(uint8_t)p[n - 1] << 16;
            b = 0;
        } else {
            a = b = 0;
        }
        return mix64(mix64(h ^ a) * 0x9E3779B97F4A7C15ull ^ b);
    }
    size_t i = 0;
    for (; i + 8 < n; i += 8) h = mix64(h ^ load64(p + i)) * 0x9E3779B97F4A7C15ull;
    return mix64(h ^ load64(p + n - 8));
}

}  // namespace keto
