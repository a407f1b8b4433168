// Request routing for edge-partitioned snapshots (keto_route_rows_device / keto_unroute_device).
//
// A partitioned batch travels between parts as row-id requests grouped by destination part
// (the owner of the top-level row, repo:keto_amd/multi.py route_device).  Grouping is a stable
// counting sort with at most 64 buckets, so it is three passes over the batch instead of a
// general sort:
//   route_count   one wave per tile of 2048 requests: gathers the owner of each row (int16 table),
//                 keeps the destination as one byte per request and counts the tile's requests
//                 per bucket with wave ballots (lane b holds bucket b);
//   route_scan    one workgroup: exclusive scan of the bucket-major (bucket, tile) counts, so the
//                 tiles of one bucket follow each other in batch order;
//   route_scatter each wave re-reads its tile's destinations, ranks every request inside its
//                 64-request chunk with a ballot + mbcnt per bucket, and writes the request and its
//                 origin index at the bucket's running offset.
// Traffic per request: 16 B request read twice, one 2-B owner gather, 1 B destination written
// and read, 16 B + 4 B written.  Nothing here calls into the snapshot: the owner table is the
// output of keto_row_owner uploaded once.
#include <hip/hip_runtime.h>

#include "snapshot.hpp"

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

namespace keto {
namespace {

constexpr uint32_t RT_CHUNKS = 32;                  // 64-request chunks per wave tile
constexpr uint32_t RT_TILE = 64 * RT_CHUNKS;
constexpr uint32_t RT_WAVES = 4;                    // waves per workgroup
constexpr uint32_t RT_SCAN_THREADS = 1024;
constexpr uint8_t RT_NONE = 0xFF;

struct RouteWork {
    uint8_t* dest;
    uint32_t* hist;                                 // [n_parts][n_tiles], scanned in place
    uint32_t* starts;                               // [n_parts + 1]
};

uint32_t n_tiles_of(uint32_t n) { return (n + RT_TILE - 1) / RT_TILE; }

uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

uint64_t work_bytes(uint32_t n, uint32_t n_parts) {
    return align256(n) + align256((uint64_t)n_parts * n_tiles_of(n) * 4) + align256(((uint64_t)n_parts + 1) * 4);
}

RouteWork carve(void* base, uint32_t n, uint32_t n_parts) {
    uint8_t* p = static_cast<uint8_t*>(base);
    RouteWork w;
    w.dest = p;
    p += align256(n);
    w.hist = reinterpret_cast<uint32_t*>(p);
    p += align256((uint64_t)n_parts * n_tiles_of(n) * 4);
    w.starts = reinterpret_cast<uint32_t*>(p);
    return w;
}

__device__ inline uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ void __launch_bounds__(64 * RT_WAVES) route_count(const keto_check_ids* __restrict__ reqs, uint32_t n,
                                                             const int16_t* __restrict__ owner, uint32_t n_rows,
                                                             uint32_t self, uint32_t n_parts, uint32_t n_tiles,
                                                             uint8_t* __restrict__ dest, uint32_t* __restrict__ hist) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x * RT_WAVES + (threadIdx.x >> 6);
    if (tile >= n_tiles) return;                   // whole wave
    uint32_t cnt = 0;                              // lane b: requests of this tile bound for part b
    for (uint32_t c = 0; c < RT_CHUNKS; ++c) {
        const uint32_t i = tile * RT_TILE + c * 64 + lane;
        uint32_t d = RT_NONE;
        if (i < n) {
            const uint32_t row = reqs[i].row;
            d = self;
            if (row < n_rows) {
                const int o = owner[row];
                if (o >= 0 && (uint32_t)o < n_parts) d = (uint32_t)o;
            }
            dest[i] = (uint8_t)d;
        }
        for (uint32_t b = 0; b < n_parts; ++b) {
            const uint64_t m = __ballot(d == b);
            if (lane == b) cnt += (uint32_t)__popcll(m);
        }
    }
    if (lane < n_parts) hist[(uint64_t)lane * n_tiles + tile] = cnt;
}

__global__ void __launch_bounds__(RT_SCAN_THREADS) route_scan(uint32_t* __restrict__ hist, uint32_t n_parts,
                                                              uint32_t n_tiles, uint32_t n, uint32_t* __restrict__ starts) {
    __shared__ uint32_t part_sum[RT_SCAN_THREADS];
    const uint64_t e = (uint64_t)n_parts * n_tiles;
    const uint64_t per = (e + RT_SCAN_THREADS - 1) / RT_SCAN_THREADS;
    const uint64_t lo = min<uint64_t>(e, threadIdx.x * per), hi = min<uint64_t>(e, lo + per);
    uint32_t s = 0;
    for (uint64_t k = lo; k < hi; ++k) s += hist[k];
    part_sum[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < RT_SCAN_THREADS; off <<= 1) {     // inclusive Hillis-Steele scan
        const uint32_t v = threadIdx.x >= off ? part_sum[threadIdx.x - off] : 0u;
        __syncthreads();
        part_sum[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part_sum[threadIdx.x] - s;
    for (uint64_t k = lo; k < hi; ++k) {
        const uint32_t v = hist[k];
        hist[k] = run;
        if (k % n_tiles == 0) starts[k / n_tiles] = run;
        run += v;
    }
    if (threadIdx.x == 0) starts[n_parts] = n;
}

__global__ void __launch_bounds__(64 * RT_WAVES) route_scatter(const keto_check_ids* __restrict__ reqs, uint32_t n,
                                                               uint32_t n_parts, uint32_t n_tiles,
                                                               const uint8_t* __restrict__ dest,
                                                               const uint32_t* __restrict__ hist,
                                                               keto_check_ids* __restrict__ send,
                                                               uint32_t* __restrict__ order) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x * RT_WAVES + (threadIdx.x >> 6);
    if (tile >= n_tiles) return;
    uint32_t base = lane < n_parts ? hist[(uint64_t)lane * n_tiles + tile] : 0u;   // lane b: next slot of part b
    for (uint32_t c = 0; c < RT_CHUNKS; ++c) {
        const uint32_t i = tile * RT_TILE + c * 64 + lane;
        const uint32_t d = i < n ? dest[i] : RT_NONE;
        uint32_t pos = 0;
        for (uint32_t b = 0; b < n_parts; ++b) {
            const uint64_t m = __ballot(d == b);
            const uint32_t at = __shfl(base, (int)b);
            if (d == b) pos = at + lanes_below(m);
            if (lane == b) base += (uint32_t)__popcll(m);
        }
        if (i < n) {
            send[pos] = reqs[i];
            order[pos] = i;
        }
    }
}

__global__ void unroute(const uint8_t* __restrict__ back, const uint32_t* __restrict__ order, uint32_t n,
                        uint8_t* __restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[order[j]] = back[j];
}

}  // namespace

uint64_t route_work_bytes(uint32_t n, uint32_t n_parts) { return work_bytes(n, n_parts); }

void route_rows(const keto_check_ids* d_reqs, uint32_t n, const int16_t* d_owner, uint32_t n_rows, uint32_t self_part,
                uint32_t n_parts, void* d_work, uint64_t work_len, keto_check_ids* d_send, uint32_t* d_order,
                uint32_t* counts_out, void* stream) {
    if (n_parts == 0 || n_parts > 64 || self_part >= n_parts) throw Error{KETO_E_INVALID, "bad part count"};
    if (work_len < work_bytes(n, n_parts)) throw Error{KETO_E_INVALID, "route workspace too small (keto_route_work_bytes)"};
    auto st = static_cast<hipStream_t>(stream);
    if (n == 0) {
        for (uint32_t b = 0; b < n_parts; ++b) counts_out[b] = 0;
        return;
    }
    const RouteWork w = carve(d_work, n, n_parts);
    const uint32_t tiles = n_tiles_of(n);
    const dim3 grid((tiles + RT_WAVES - 1) / RT_WAVES), block(64 * RT_WAVES);
    hipLaunchKernelGGL(route_count, grid, block, 0, st, d_reqs, n, d_owner, n_rows, self_part, n_parts, tiles, w.dest,
                       w.hist);
    hipLaunchKernelGGL(route_scan, dim3(1), dim3(RT_SCAN_THREADS), 0, st, w.hist, n_parts, tiles, n, w.starts);
    hipLaunchKernelGGL(route_scatter, grid, block, 0, st, d_reqs, n, n_parts, tiles, w.dest, w.hist, d_send, d_order);
    HIP_OK(hipGetLastError());
    uint32_t starts[65];
    HIP_OK(hipMemcpyAsync(starts, w.starts, ((size_t)n_parts + 1) * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (uint32_t b = 0; b < n_parts; ++b) counts_out[b] = starts[b + 1] - starts[b];
}

__global__ void __launch_bounds__(256) scatter_ids_kernel(keto_check_ids* __restrict__ d, const uint32_t* __restrict__ idx,
                                                          const keto_check_ids* __restrict__ vals, uint32_t m) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) d[idx[k]] = vals[k];
}

void scatter_ids(keto_check_ids* d, const uint32_t* d_idx, const keto_check_ids* d_vals, uint32_t m, void* stream) {
    if (!m) return;
    hipLaunchKernelGGL(scatter_ids_kernel, dim3((m + 255) / 256), dim3(256), 0, (hipStream_t)stream, d, d_idx, d_vals, m);
    HIP_OK(hipGetLastError());
}

// The local transport's exchange into one rank (comm.cpp LocalTransport::alltoallv): every peer's
// segment for this rank copied by one launch instead of one runtime copy (a blit kernel) per peer.
// Segments are copied in 16-B words when source, destination and length allow, else in 4-B words,
// else bytes.
__global__ void __launch_bounds__(256) copy_segments_kernel(CopySegments s) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t k = 0; k < s.n; ++k) {
        const uint8_t* src = static_cast<const uint8_t*>(s.src[k]);
        uint8_t* dst = static_cast<uint8_t*>(s.dst[k]);
        const uint64_t b = s.bytes[k];
        const uint64_t al = (uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst | b;
        if ((al & 15u) == 0) {
            for (uint64_t i = tid; i < b / 16; i += stride)
                reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        } else if ((al & 3u) == 0) {
            for (uint64_t i = tid; i < b / 4; i += stride)
                reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
        } else {
            for (uint64_t i = tid; i < b; i += stride) dst[i] = src[i];
        }
    }
}

void copy_segments(const CopySegments& s, void* stream) {
    uint64_t total = 0;
    for (uint32_t k = 0; k < s.n; ++k) total += s.bytes[k];
    if (total == 0) return;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(total / (256 * 64), 1), 2048);
    hipLaunchKernelGGL(copy_segments_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, s);
    HIP_OK(hipGetLastError());
}

void unroute_rows(const uint8_t* d_back, const uint32_t* d_order, uint32_t n, uint8_t* d_out, void* stream) {
    if (n == 0) return;
    hipLaunchKernelGGL(unroute, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), d_back, d_order,
                       n, d_out);
    HIP_OK(hipGetLastError());
}

}  // namespace keto
