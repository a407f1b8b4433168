// Check requests resolved on the GPU: the role of whereQuery (internal/persistence/sql/
// relationtuples.go:178-198) for every request of a batch, on the device, against the snapshot's
// string and row indexes uploaded once per version -- instead of on host threads (resolve.cpp),
// where a request costs ~6 dependent host-memory misses (16.7M requests: 175-195 ms on 16 EPYC
// threads, profiles/r03d_resolve.log).
//
// The batch comes packed (keto_check_batch_packed, include/keto_mi355x.h): every request's
// strings back to back in one buffer -- the Go batcher already copies a batch's strings into one C
// arena -- and a 24-B record per request with their offset and lengths.  The library copies both to
// the device, and one thread per request:
//   namespace name -> config namespace id      (a compare over the few configured names)
//   object, relation, subject id -> string ids (the host's open-addressing string index, same hash
//                                               and 16-B slots: length + first 11 bytes verify a
//                                               short string in the slot; a longer one compares its
//                                               bytes; strings a write added: a second table)
//   (namespace, object, relation) -> row id    (the real-row index; empty rows subject sets point
//                                               at and rows a write added: a second table)
//   subject set -> its row id (the target), flags
// exactly as Snapshot::resolve_query / resolve_general do; the row-id requests then go through
// device_check_rows (row ids -> handles, the check).  A request with an empty namespace, object or
// relation (a wildcard query, also in its subject set) is left to the host path (check_named: it
// may need a batch-local row); so is a field longer than 65535 bytes, which the record cannot
// hold (the caller passes those through keto_check_batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

namespace {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

struct RBuf {                      // grow-only device buffer
    void* p = nullptr;
    uint64_t cap = 0;
    RBuf() = default;
    RBuf(const RBuf&) = delete;
    RBuf& operator=(const RBuf&) = delete;
    template <class T>
    T* get(uint64_t n) {
        const uint64_t want = std::max<uint64_t>(64, n * sizeof(T));
        if (want > cap) {
            release();
            const uint64_t c = std::max<uint64_t>(want, cap + cap / 4);
            const hipError_t e = hipMalloc(&p, c);
            if (e != hipSuccess) {
                p = nullptr;
                throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
            }
            cap = c;
        }
        return static_cast<T*>(p);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    ~RBuf() { release(); }
};

using StrSlot = Snapshot::StrSlot;
using RowSlot = Snapshot::RowSlot;
constexpr uint32_t INLINE = sizeof(StrSlot::b);
constexpr uint32_t NO_BAD = 0xFFFFFFFFu;           // no request outside the blob
constexpr uint32_t NO_UNIT_R = 0xFFFFFFFFu;        // the row -> handle map's "not on this part" (engine.hip NO_UNIT)
constexpr uint8_t ST_HOST = 0xFF;                   // resolved on the host (wildcards)

// ---- hashing, mirrored bit for bit from parallel.hpp (hash_bytes, mix64) and resolve.cpp (row_hash)
__device__ inline uint64_t d_mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ inline uint64_t d_load(const uint8_t* p, int n) {        // n little-endian bytes
    uint64_t w = 0;
    for (int i = 0; i < n; ++i) w |= (uint64_t)p[i] << (8 * i);
    return w;
}
__device__ inline uint64_t d_hash_bytes(const uint8_t* p, uint32_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xC2B2AE3D27D4EB4Full);
    uint64_t a, b;
    if (n <= 16) {
        if (n >= 8) {
            a = d_load(p, 8);
            b = d_load(p + n - 8, 8);
        } else if (n >= 4) {
            a = d_load(p, 4);
            b = d_load(p + n - 4, 4);
        } else if (n > 0) {
            a = (uint64_t)p[0] | (uint64_t)p[n / 2] << 8 | (uint64_t)p[n - 1] << 16;
            b = 0;
        } else {
            a = b = 0;
        }
        return d_mix64(d_mix64(h ^ a) * 0x9E3779B97F4A7C15ull ^ b);
    }
    uint32_t i = 0;
    for (; i + 8 < n; i += 8) h = d_mix64(h ^ d_load(p + i, 8)) * 0x9E3779B97F4A7C15ull;
    return d_mix64(h ^ d_load(p + n - 8, 8));
}
__host__ __device__ inline uint64_t row_hash_hd(int64_t ns, uint32_t obj, uint32_t rel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return d_mix64((uint64_t)ns * 0x9E3779B97F4A7C15ull ^ d_mix64(((uint64_t)obj << 32) | rel));
#else
    return mix64((uint64_t)ns * 0x9E3779B97F4A7C15ull ^ mix64(((uint64_t)obj << 32) | rel));
#endif
}

struct StrIndex {                  // an open-addressing string table and the bytes behind it
    const StrSlot* slot;
    uint64_t mask;                 // 0 with slot == nullptr: empty
    const uint8_t* bytes;          // the table's strings back to back (id order)
    const uint64_t* off;           // string id - id0 -> offset in bytes
    uint64_t id0;                  // the table's first string id
};
struct RowIndex {
    const RowSlot* slot;
    uint64_t mask;
};
struct ResolveDev {
    StrIndex base, added;          // the build's strings; strings writes added (after the build's)
    RowIndex real, extra;          // the build's real rows; empty rows and rows writes added
    const uint8_t* ns_bytes;       // configured namespace names back to back (config order)
    const uint64_t* ns_off;
    const int32_t* ns_id;
    uint32_t n_ns;
};

__device__ inline bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}
__device__ int64_t find_str_dev(const StrIndex& T, const uint8_t* s, uint32_t n, uint64_t h) {
    if (!T.slot) return -1;
    const uint8_t n8 = (uint8_t)min(n, 255u);
    for (uint64_t j = h & T.mask;; j = (j + 1) & T.mask) {
        const StrSlot x = T.slot[j];
        if (!x.id1) return -1;
        if (x.n != n8) continue;
        if (!bytes_eq(reinterpret_cast<const uint8_t*>(x.b), s, min(n, INLINE))) continue;
        if (n <= INLINE) return x.id1 - 1;
        const uint64_t b = T.off[x.id1 - 1 - T.id0], e = T.off[x.id1 - T.id0];
        if (e - b == n && bytes_eq(T.bytes + b, s, n)) return x.id1 - 1;
    }
}
__device__ inline int64_t lookup_str_dev(const ResolveDev& R, const uint8_t* s, uint32_t n) {
    const uint64_t h = d_hash_bytes(s, n);
    const int64_t id = find_str_dev(R.base, s, n, h);
    return id >= 0 ? id : find_str_dev(R.added, s, n, h);
}
__device__ int64_t find_row_dev(const RowIndex& T, int32_t ns, uint32_t obj, uint32_t rel) {
    if (!T.slot) return -1;
    for (uint64_t j = row_hash_hd(ns, obj, rel) & T.mask;; j = (j + 1) & T.mask) {
        const RowSlot x = T.slot[j];
        if (!x.row1) return -1;
        if (x.ns == ns && x.obj == obj && x.rel == rel) return x.row1 - 1;
    }
}
__device__ inline int ns_index_dev(const ResolveDev& R, const uint8_t* s, uint32_t n) {
    for (uint32_t c = 0; c < R.n_ns; ++c) {
        const uint64_t b = R.ns_off[c], e = R.ns_off[c + 1];
        if (e - b == n && bytes_eq(R.ns_bytes + b, s, n)) return (int)c;
    }
    return -1;
}
// RelationQuery (namespace, object, relation), every field set -> row id; -1 none, -2 unknown namespace
__device__ int64_t query_row_dev(const ResolveDev& R, const uint8_t* f, uint32_t l_ns, uint32_t l_obj, uint32_t l_rel) {
    const int c = ns_index_dev(R, f, l_ns);
    if (c < 0) return -2;                                                  // ErrNotFound
    const int64_t o = lookup_str_dev(R, f + l_ns, l_obj);
    if (o < 0) return -1;                                                  // no row can match an unknown string
    const int64_t r = lookup_str_dev(R, f + l_ns + l_obj, l_rel);
    if (r < 0) return -1;
    const int32_t ns = R.ns_id[c];
    const int64_t row = find_row_dev(R.real, ns, (uint32_t)o, (uint32_t)r);
    return row >= 0 ? row : find_row_dev(R.extra, ns, (uint32_t)o, (uint32_t)r);
}

// cnt[0]: the first request whose fields lie outside the blob (atomicMin; NO_BAD = none) -- its fields
// are not read; cnt[1]: how many requests the host resolves (wildcard queries).  Both were host loops
// over every record before (~20 ms of a 16.7M-request batch's 40.7 ms, profiles/r05ap_*).  Requests
// [i0, i0 + n); the bytes [lo, hi) of the blob are on the device so far (a pipelined batch uploads it
// piece by piece): a request with a field outside them is counted in cnt[2] and left for a second
// pass once the whole blob is there.
//
// CLK (KETO_RESOLVE_CLOCKS, tooling): each request's lane records wall_clock64() (100 MHz) at its
// start, after its record load, after its row query and after its subject lookup into clk[4 i ..].
// XL (the batches in flight): rows and subject-set targets come out as handles through the device's
// row id -> handle map (rows_to_handles' rule), a row this part does not hold counted in cnt[3]
template <bool CLK = false, bool XL = false>
__global__ void __launch_bounds__(256) resolve_packed(ResolveDev R, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                      uint64_t lo, uint64_t hi, const keto_check_packed* __restrict__ q,
                                                      uint32_t i0, uint32_t n, keto_check_ids* __restrict__ out,
                                                      uint8_t* __restrict__ status, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ clk = nullptr,
                                                      const uint32_t* __restrict__ row_handle = nullptr, uint32_t n_rows = 0) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t i = i0 + k;
    uint64_t c0 = 0, c1 = 0, c2 = 0;
    if constexpr (CLK) c0 = wall_clock64();
    const keto_check_packed p = q[i];
    if constexpr (CLK) {
        asm volatile("" ::"v"(p.off), "v"(p.max_depth) : "memory");        // (the record is in)
        c1 = wall_clock64();
    }
    const uint8_t* f = blob + p.off;
    keto_check_ids r{KETO_NO_ROW, KETO_NO_TARGET, 0u, p.max_depth};
    uint8_t st = KETO_CHECK_OK;
    const bool set = p.kind != 0;
    const uint64_t len = (uint64_t)p.len[0] + p.len[1] + p.len[2] + p.len[3] + (set ? (uint64_t)p.len[4] + p.len[5] : 0);
    if ((uint64_t)p.off + len > blob_len) {
        atomicMin(cnt, i);
        st = ST_HOST;                                                      // (the batch fails)
    } else if (p.off < lo || (uint64_t)p.off + len > hi) {
        atomicAdd(cnt + 2, 1u);                                            // (the batch is resolved again)
    } else if (!p.len[0] || !p.len[1] || !p.len[2] || (set && (!p.len[3] || !p.len[4] || !p.len[5]))) {
        st = ST_HOST;                                                      // a wildcard query: the host
        atomicAdd(cnt + 1, 1u);
    } else {
        const int64_t row = query_row_dev(R, f, p.len[0], p.len[1], p.len[2]);
        if constexpr (CLK) {
            asm volatile("" ::"v"((uint32_t)row) : "memory");
            c2 = wall_clock64();
        }
        if (row == -2) st = KETO_CHECK_UNKNOWN_NAMESPACE;
        else if (row >= 0) r.row = (uint32_t)row;
        const uint8_t* g = f + p.len[0] + p.len[1] + p.len[2];
        if (!set) {
            const int64_t sid = lookup_str_dev(R, g, p.len[3]);
            if (sid >= 0) r.target = (uint32_t)sid;
        } else {
            const int64_t t = query_row_dev(R, g, p.len[3], p.len[4], p.len[5]);
            if (t >= 0) {
                r.target = (uint32_t)t;                                    // row-id form: translated below
                r.flags = 1;
            }
        }
    }
    if constexpr (XL) {
        if (r.row != KETO_NO_ROW) {
            const uint32_t h = r.row < n_rows ? row_handle[r.row] : NO_UNIT_R;
            if (h == NO_UNIT_R) atomicAdd(cnt + 3, 1u);
            r.row = h == NO_UNIT_R ? KETO_NO_ROW : h;
        }
        if ((r.flags & 1u) && r.target != KETO_NO_TARGET) {
            const uint32_t h = r.target < n_rows ? row_handle[r.target] : NO_UNIT_R;
            r.target = h == NO_UNIT_R ? KETO_NO_TARGET : h;
        }
    }
    out[i] = r;
    status[i] = st;
    if constexpr (CLK) {
        asm volatile("" ::"v"(r.target) : "memory");
        const uint64_t c3 = wall_clock64();
        clk[4ull * i] = (uint32_t)c0;
        clk[4ull * i + 1] = (uint32_t)(c1 - c0);
        clk[4ull * i + 2] = c2 ? (uint32_t)(c2 - c1) : 0u;
        clk[4ull * i + 3] = c2 ? (uint32_t)(c3 - c2) : 0u;
    }
}

// decisions > 1 (KETO_UNDECIDED from the check) become "not allowed" with an undecided status, as
// keto_check_batch reports them; requests the host resolves are left to it
__global__ void __launch_bounds__(256) fold_undecided(uint8_t* __restrict__ allowed, uint8_t* __restrict__ status,
                                                      uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || status[i] == ST_HOST || allowed[i] <= 1) return;
    allowed[i] = 0;
    if (status[i] == KETO_CHECK_OK) status[i] = KETO_CHECK_UNDECIDED;
}

// fold_undecided for a batch in flight; its first thread also readies the slot's other counter block
// for the slot's next batch ({NO_BAD, 0, ...}: that block's batch has completed)
__global__ void __launch_bounds__(256) fold_and_reset(uint8_t* __restrict__ allowed, uint8_t* __restrict__ status,
                                                      uint32_t n, uint32_t* __restrict__ next_cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        next_cnt[0] = NO_BAD;
        for (int k = 1; k < 8; ++k) next_cnt[k] = 0;
    }
    if (i >= n || status[i] == ST_HOST || allowed[i] <= 1) return;
    allowed[i] = 0;
    if (status[i] == KETO_CHECK_OK) status[i] = KETO_CHECK_UNDECIDED;
}

template <class T>
T* upload(RBuf& b, const T* src, uint64_t n, hipStream_t st) {
    T* d = b.get<T>(std::max<uint64_t>(n, 1));
    if (n) HIP_OK(hipMemcpyAsync(d, src, n * sizeof(T), hipMemcpyHostToDevice, st));
    return d;
}

}  // namespace

// A packed batch in flight (device_check_packed_async): its own stream, device buffers and pinned
// output staging, so that one batch's upload and resolution run while another's check does.
struct PSlot {
    int device = 0;
    hipStream_t st = nullptr;
    hipEvent_t ready = nullptr, done = nullptr;   // resolved (the check may start) / checked
    RBuf blob, reqs, ids, out;     // out: decisions | statuses | two blocks of 8 counter words
    uint64_t out_n = 0;            // the batch size out is laid out for
    uint32_t par = 0;              // the counter block of the next batch
    bool clean[2] = {false, false};   // that block holds {NO_BAD, 0, ...}
    uint8_t* host = nullptr;       // pinned: the copy of out
    uint64_t host_cap = 0;
    ~PSlot() {
        (void)hipSetDevice(device);
        if (st) (void)hipStreamSynchronize(st);
        if (host) (void)hipHostFree(host);
        if (ready) (void)hipEventDestroy(ready);
        if (done) (void)hipEventDestroy(done);
        if (st) (void)hipStreamDestroy(st);
    }
};

// The device copies of the indexes (per snapshot version) and the per-call buffers.
struct RDevState {
    int device = 0;
    uint64_t version = ~0ull;
    bool base_ready = false;       // the build's string and row indexes and the namespaces (fixed after the build)
    std::mutex mu;                 // the tables' refresh; a large (or fallback) batch holds it throughout
    hipStream_t stream = nullptr;
    hipStream_t copy = nullptr;    // a pipelined batch's uploads
    std::vector<hipEvent_t> ev;    // piece k's bytes are on the device
    RBuf str_slots, str_bytes, str_off, add_slots, add_bytes, add_off, row_slots, extra_slots, ns_bytes, ns_off, ns_id;
    ResolveDev view{};
    RBuf blob, reqs, ids, status, dec, cnt, clk;
    std::mutex slot_mu;            // the batches in flight (KETO_PACKED_SLOTS)
    std::condition_variable slot_cv;
    std::vector<std::unique_ptr<PSlot>> slots;
    std::vector<uint8_t> slot_busy;
    ~RDevState() {
        (void)hipSetDevice(device);
        slots.clear();
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        if (copy) (void)hipStreamDestroy(copy);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

void RDevStateDeleter::operator()(RDevState* r) const { delete r; }

namespace {

// an open-addressing table over (hash, fill) pairs, the host's layout and probing (resolve.cpp)
template <class Slot, class Fill>
std::vector<Slot> build_table(uint64_t n, uint64_t& mask, Fill fill) {
    uint64_t cap = 16;
    while (cap < n + n / 3 + 1) cap <<= 1;                               // load <= 3/4
    std::vector<Slot> t(cap);
    std::memset(t.data(), 0, cap * sizeof(Slot));
    mask = cap - 1;
    fill(t);
    return t;
}

// The state is created once per snapshot under a process-wide mutex: concurrent packed batches hold
// only the snapshot's shared lock, and two of them must not both create (and free) it.
RDevState& rdev_get(Snapshot& S, int device) {
    static std::mutex create_mu;
    std::lock_guard<std::mutex> lk(create_mu);
    if (!S.rdev) {
        std::unique_ptr<RDevState, RDevStateDeleter> r(new RDevState);
        r->device = device;
        HIP_OK(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
        HIP_OK(hipStreamCreateWithFlags(&r->copy, hipStreamNonBlocking));
        S.rdev = std::move(r);
    }
    return *S.rdev;
}

// Brings R's tables to the snapshot's version.  The caller holds R.mu, so no packed batch's kernel
// reads a table while it is rebuilt (the grow-only buffers free their old storage when they grow).
void rdev_refresh(Snapshot& S, RDevState& R) {
    if (R.version == S.version) return;
    hipStream_t st = R.stream;
    ResolveDev v = R.view;
    // the build's strings (strs[0, n_sorted_strs): the host index covers exactly them), its real rows
    // and the namespaces never change after the build: uploaded once per snapshot.  A write adds
    // strings and rows to the small second tables, rebuilt per version.
    if (!R.base_ready) {
        S.ensure_index();
        v.base.slot = upload(R.str_slots, static_cast<const StrSlot*>(S.str_idx.p), S.str_mask + 1, st);
        v.base.mask = S.str_mask;
        v.base.id0 = 0;
        const uint64_t ns = S.n_sorted_strs;
        std::vector<uint64_t> off(ns + 1, 0);
        for (uint64_t i = 0; i < ns; ++i) off[i + 1] = off[i] + S.strs[i].size();
        std::vector<uint8_t> bytes(std::max<uint64_t>(1, off[ns]));
        par_chunks(ns, ns >= par_min() ? build_threads() : 1u, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i)
                if (!S.strs[i].empty()) std::memcpy(bytes.data() + off[i], S.strs[i].data(), S.strs[i].size());
        });
        v.base.bytes = upload(R.str_bytes, bytes.data(), bytes.size(), st);
        v.base.off = upload(R.str_off, off.data(), off.size(), st);
        v.real.slot = upload(R.row_slots, static_cast<const RowSlot*>(S.row_idx.p), S.row_mask + 1, st);
        v.real.mask = S.row_mask;
        const uint32_t nn = (uint32_t)S.ns_names.size();
        std::vector<uint64_t> noff(nn + 1, 0);
        std::string nbytes;
        for (uint32_t c = 0; c < nn; ++c) {
            nbytes += S.ns_names[c];
            noff[c + 1] = nbytes.size();
        }
        v.ns_bytes = upload(R.ns_bytes, reinterpret_cast<const uint8_t*>(nbytes.data()), nbytes.size(), st);
        v.ns_off = upload(R.ns_off, noff.data(), noff.size(), st);
        v.ns_id = upload(R.ns_id, S.ns_ids.data(), S.ns_ids.size(), st);
        v.n_ns = nn;
        HIP_OK(hipStreamSynchronize(st));
        R.base_ready = true;
    }
    // strings writes added: ids n_sorted_strs and up, their own table and bytes
    v.added = StrIndex{nullptr, 0, nullptr, nullptr, S.n_sorted_strs};
    if (!S.added_str.empty()) {
        const uint64_t id0 = S.n_sorted_strs, na = S.strs.size() - id0;
        std::vector<uint64_t> off(na + 1, 0);
        for (uint64_t i = 0; i < na; ++i) off[i + 1] = off[i] + S.strs[id0 + i].size();
        std::vector<uint8_t> bytes(std::max<uint64_t>(1, off[na]));
        for (uint64_t i = 0; i < na; ++i)
            if (!S.strs[id0 + i].empty()) std::memcpy(bytes.data() + off[i], S.strs[id0 + i].data(), S.strs[id0 + i].size());
        uint64_t mask = 0;
        auto t = build_table<StrSlot>(S.added_str.size(), mask, [&](std::vector<StrSlot>& tab) {
            const uint64_t m = tab.size() - 1;
            for (const auto& kv : S.added_str) {
                const std::string& s = kv.first;
                for (uint64_t j = hash_bytes(s) & m;; j = (j + 1) & m) {
                    if (tab[j].id1) continue;
                    tab[j].id1 = kv.second + 1;
                    tab[j].n = (uint8_t)std::min<size_t>(s.size(), 255);
                    std::memcpy(tab[j].b, s.data(), std::min<size_t>(s.size(), INLINE));
                    break;
                }
            }
        });
        v.added.slot = upload(R.add_slots, t.data(), t.size(), st);
        v.added.mask = mask;
        v.added.bytes = upload(R.add_bytes, bytes.data(), bytes.size(), st);
        v.added.off = upload(R.add_off, off.data(), off.size(), st);
        HIP_OK(hipStreamSynchronize(st));
    }
    // every other row a query can name (empty rows subject sets point at, rows writes added; not the
    // wildcard rows): a second table
    v.extra = RowIndex{nullptr, 0};
    {
        std::vector<std::pair<RowKey, uint32_t>> rows;
        for (const auto& kv : S.row_of)
            if (kv.first.ns != ANY_NS && kv.first.obj != ANY && kv.first.rel != ANY && kv.first.ns >= INT32_MIN &&
                kv.first.ns <= INT32_MAX)
                rows.push_back(kv);
        if (!rows.empty()) {
            uint64_t mask = 0;
            auto t = build_table<RowSlot>(rows.size(), mask, [&](std::vector<RowSlot>& tab) {
                const uint64_t m = tab.size() - 1;
                for (const auto& kv : rows) {
                    const RowKey& k = kv.first;
                    for (uint64_t j = row_hash_hd(k.ns, k.obj, k.rel) & m;; j = (j + 1) & m) {
                        if (tab[j].row1) continue;
                        tab[j] = RowSlot{(int32_t)k.ns, k.obj, k.rel, kv.second + 1};
                        break;
                    }
                }
            });
            v.extra.slot = upload(R.extra_slots, t.data(), t.size(), st);
            v.extra.mask = mask;
            HIP_OK(hipStreamSynchronize(st));
        }
    }
    R.view = v;
    R.version = S.version;
}

}  // namespace

namespace {
// requests per piece of a pipelined packed batch (KETO_PACKED_CHUNK; 0 = one piece)
uint64_t packed_chunk() {
    const char* e = getenv("KETO_PACKED_CHUNK");
    return e ? (uint64_t)std::max(0ll, atoll(e)) : (1ull << 21);
}

// packed batches a snapshot keeps in flight at once (KETO_PACKED_SLOTS, default 2; 0 = one batch at
// a time through the synchronous path)
uint32_t packed_slots() {
    const char* e = getenv("KETO_PACKED_SLOTS");
    return e ? (uint32_t)std::min(16, std::max(0, atoi(e))) : 2u;
}

// A batch of one piece on an unpartitioned snapshot, with max-depth <= 9, and no host round trip
// before its results: a free slot takes it; its upload and its resolution -- straight to the handle
// form through the device's row -> handle map -- run on the slot's stream (no lock: other slots'
// batches may be resolving or checking meanwhile), its tier-0 check is enqueued behind them under the
// device lock (device_check_rows_async, one of two check streams), and the decisions, statuses and
// every counter come home in one copy.  Only then are the counters looked at: a request outside the
// blob fails the call before the outputs are written, as on the synchronous path; a batch some of
// whose requests tier 0 hands up (rare at max-depth <= 9: none in the 1B graph's 16.7M) returns
// false, and the caller checks it again synchronously through every tier.  The slot's counters are
// two blocks used in turn: each batch's last kernel readies the other one, so no batch starts with
// memsets.
bool device_check_packed_async(Snapshot& S, RDevState& R, const uint8_t* blob, uint64_t blob_len,
                               const keto_check_packed* reqs, uint32_t n, int32_t gmd, uint8_t* allowed, uint8_t* status,
                               std::vector<uint32_t>& host) {
    ResolveDev view;
    {
        std::lock_guard<std::mutex> lk(R.mu);
        rdev_refresh(S, R);
        view = R.view;
    }
    const uint32_t* row_handle = device_row_handle_map(S);
    PSlot* P = nullptr;
    uint32_t si = 0;
    {
        std::unique_lock<std::mutex> lk(R.slot_mu);
        const uint32_t want = packed_slots();
        while (R.slots.size() < want) {
            R.slots.emplace_back(new PSlot);
            R.slot_busy.push_back(0);
        }
        R.slot_cv.wait(lk, [&] {
            for (si = 0; si < want; ++si)
                if (!R.slot_busy[si]) return true;
            return false;
        });
        R.slot_busy[si] = 1;
        P = R.slots[si].get();
    }
    struct Free {                    // the slot's work drained (no copy from the caller outlives the call), then freed
        RDevState& R;
        PSlot* P;
        uint32_t si;
        bool checking = false;       // a check reading the slot's buffers is enqueued on the device's stream
        ~Free() {
            if (checking) (void)hipEventSynchronize(P->done);
            if (P->st) (void)hipStreamSynchronize(P->st);
            {
                std::lock_guard<std::mutex> lk(R.slot_mu);
                R.slot_busy[si] = 0;
            }
            R.slot_cv.notify_one();
        }
    } free_slot{R, P, si};
    P->device = R.device;
    if (!P->st) {
        HIP_OK(hipStreamCreateWithFlags(&P->st, hipStreamNonBlocking));
        HIP_OK(hipEventCreateWithFlags(&P->ready, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&P->done, hipEventDisableTiming));
    }
    // out: decisions at 0, statuses at n, the counter blocks 16-B aligned after them
    const uint64_t coff = (2ull * n + 15) & ~15ull, obytes = coff + 64;
    if (P->host_cap < obytes) {
        if (P->host) (void)hipHostFree(P->host);
        P->host = nullptr;
        P->host_cap = 0;
        const uint64_t c = std::max<uint64_t>(obytes + obytes / 4, 1 << 20);
        const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&P->host), c, hipHostMallocDefault);
        if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e)};
        P->host_cap = c;
    }
    hipStream_t st = P->st;
    uint8_t* d_blob = P->blob.get<uint8_t>(std::max<uint64_t>(blob_len, 1));
    keto_check_packed* d_q = P->reqs.get<keto_check_packed>(std::max<uint32_t>(n, 1));
    keto_check_ids* d_x = P->ids.get<keto_check_ids>(n);
    if (P->out_n != n) {                      // the counter blocks move with n: both need setting up
        P->out_n = n;
        P->clean[0] = P->clean[1] = false;
    }
    uint8_t* d_out = P->out.get<uint8_t>(obytes);
    uint8_t* d_dec = d_out;
    uint8_t* d_st = d_out + n;
    const uint32_t par = P->par;
    uint32_t* d_cnt = reinterpret_cast<uint32_t*>(d_out + coff) + 8 * par;   // resolve: bad, host, order, misrouted |
    uint32_t* d_next = reinterpret_cast<uint32_t*>(d_out + coff) + 8 * (par ^ 1u);   // tier-0 overflows
    if (!P->clean[par]) {
        HIP_OK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_cnt), NO_BAD, 1, st));
        HIP_OK(hipMemsetAsync(d_cnt + 1, 0, 7 * sizeof(uint32_t), st));
    }
    P->clean[par] = false;
    P->par = par ^ 1u;
    if (blob_len) HIP_OK(hipMemcpyAsync(d_blob, blob, blob_len, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_q, reqs, (uint64_t)n * sizeof(keto_check_packed), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL((resolve_packed<false, true>), dim3((n + 255) / 256), dim3(256), 0, st, view, d_blob, blob_len, 0ull,
                       blob_len, d_q, 0u, n, d_x, d_st, d_cnt, nullptr, row_handle, S.n_rows());
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(P->ready, st));
    if (!device_check_rows_async(S, d_x, n, gmd, d_dec, d_cnt + 4, P->ready, P->done)) return false;
    free_slot.checking = true;
    HIP_OK(hipStreamWaitEvent(st, P->done, 0));
    hipLaunchKernelGGL(fold_and_reset, dim3((n + 255) / 256), dim3(256), 0, st, d_dec, d_st, n, d_next);
    HIP_OK(hipGetLastError());
    uint8_t* h = P->host;
    HIP_OK(hipMemcpyAsync(h, d_out, coff + 8 * (par + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    P->clean[par ^ 1u] = true;
    const uint32_t* hc = reinterpret_cast<const uint32_t*>(h + coff) + 8 * par;
    lock_trace("packed async: copied back");
    if (hc[0] != NO_BAD) throw Error{KETO_E_INVALID, "request " + std::to_string(hc[0]) + "'s fields lie outside the blob"};
    static const bool force_sync = getenv("KETO_TEST_PACKED_FALLBACK") != nullptr;   // test hook
    if (hc[4] || hc[3] || force_sync) return false;   // the next tiers needed (or a misrouted row): the synchronous path
    std::memcpy(allowed, h, n);
    std::memcpy(status, h + n, n);
    if (hc[1])                                   // the wildcard queries: the host's
        for (uint32_t i = 0; i < n && host.size() < hc[1]; ++i)
            if (status[i] == ST_HOST) host.push_back(i);
    return true;
}
}  // namespace

// A batch of 2 pieces or more on an unpartitioned snapshot is pipelined: the blob and the records go
// up in pieces on R.copy while the compute stream resolves and checks each piece once its bytes are
// there, so the resolution and the check hide under the upload, which is the floor (821 MB of a
// 16.7M-request batch: 14.5 ms of its 21.6 ms unpipelined, profiles/r05aq_string_form_trace.txt).
// Piece k's blob window comes from the records at the piece boundaries, exact for a batch packed in
// request order (the Go batcher's and the generator's); a request whose fields lie outside its window
// is counted by resolve_packed, and then the whole batch is resolved and checked again over the whole
// blob.  The bounds error is raised before anything is written to the outputs, as unpipelined;
// (a partitioned snapshot is never pipelined: its misrouted-row error must not precede it).
void device_check_packed(Snapshot& S, const uint8_t* blob, uint64_t blob_len, const keto_check_packed* reqs, uint32_t n,
                         int32_t gmd, uint8_t* allowed, uint8_t* status, std::vector<uint32_t>& host) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    const DevView dv = device_view(S);
    HIP_OK(hipSetDevice(dv.device));
    RDevState& R = rdev_get(S, dv.device);
    static const bool clocks = getenv("KETO_RESOLVE_CLOCKS") != nullptr;  // tooling: per-step clocks
    {
        const uint64_t chunk = packed_chunk();
        const bool one_piece = !(chunk && S.n_parts == 1 && n >= 2 * chunk);
        if (n && one_piece && S.n_parts == 1 && !clocks && packed_slots() > 0 && std::min<int32_t>(gmd, 65535) <= 9 &&
            device_check_packed_async(S, R, blob, blob_len, reqs, n, gmd, allowed, status, host))
            return;
        host.clear();
    }
    lock_trace("packed: waiting for R.mu");
    std::lock_guard<std::mutex> lk(R.mu);                                   // held through the last copy
    lock_trace("packed: R.mu");
    rdev_refresh(S, R);
    lock_trace("packed: refreshed");
    hipStream_t st = R.stream, cs = R.copy;
    struct Drain {                       // no copy from the caller's memory outlives the call
        hipStream_t a, b;
        ~Drain() {
            (void)hipStreamSynchronize(a);
            (void)hipStreamSynchronize(b);
        }
    } drain{cs, st};
    const uint64_t chunk = packed_chunk();
    uint32_t K = 1;
    if (chunk && S.n_parts == 1 && n >= 2 * chunk) K = (uint32_t)std::min<uint64_t>(64, (n + chunk - 1) / chunk);
    std::vector<uint32_t> cb(K + 1);
    std::vector<uint64_t> wb(K + 1);
    for (uint32_t k = 0; k <= K; ++k) cb[k] = (uint32_t)((uint64_t)n * k / K);
    wb[0] = 0;
    wb[K] = blob_len;
    for (uint32_t k = 1; k < K; ++k) wb[k] = std::min<uint64_t>(blob_len, std::max<uint64_t>(wb[k - 1], reqs[cb[k]].off));
    uint8_t* d_blob = R.blob.get<uint8_t>(std::max<uint64_t>(blob_len, 1));
    keto_check_packed* d_q = R.reqs.get<keto_check_packed>(std::max<uint32_t>(n, 1));
    keto_check_ids* d_ids = R.ids.get<keto_check_ids>(n);
    uint8_t* d_st = R.status.get<uint8_t>(n);
    uint8_t* d_dec = R.dec.get<uint8_t>(n);
    uint32_t* d_cnt = R.cnt.get<uint32_t>(3);
    while (R.ev.size() < K) {
        hipEvent_t e;
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        R.ev.push_back(e);
    }
    if (K > 1) HIP_OK(hipEventRecord(R.ev[0], st));                        // (the buffers are free: the last
    for (uint32_t k = 0; k < K; ++k) {                                     //  call's work on st is done)
        if (k == 0 && K > 1) HIP_OK(hipStreamWaitEvent(cs, R.ev[0], 0));
        hipStream_t s = K > 1 ? cs : st;
        if (wb[k + 1] > wb[k])
            HIP_OK(hipMemcpyAsync(d_blob + wb[k], blob + wb[k], wb[k + 1] - wb[k], hipMemcpyHostToDevice, s));
        if (cb[k + 1] > cb[k])
            HIP_OK(hipMemcpyAsync(d_q + cb[k], reqs + cb[k], (uint64_t)(cb[k + 1] - cb[k]) * sizeof(keto_check_packed),
                                  hipMemcpyHostToDevice, s));
        if (K > 1) HIP_OK(hipEventRecord(R.ev[k], cs));
    }
    auto reset = [&] {
        HIP_OK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_cnt), NO_BAD, 1, st));
        HIP_OK(hipMemsetAsync(d_cnt + 1, 0, 2 * sizeof(uint32_t), st));
    };
    uint32_t* d_clk = clocks && K == 1 ? R.clk.get<uint32_t>(4ull * n) : nullptr;
    auto resolve = [&](uint32_t i0, uint32_t m, uint64_t hi) {
        if (!m) return;
        if (d_clk && i0 == 0 && m == n)
            hipLaunchKernelGGL(resolve_packed<true>, dim3((m + 255) / 256), dim3(256), 0, st, R.view, d_blob, blob_len, 0ull,
                               hi, d_q, i0, m, d_ids, d_st, d_cnt, d_clk);
        else
            hipLaunchKernelGGL(resolve_packed<false>, dim3((m + 255) / 256), dim3(256), 0, st, R.view, d_blob, blob_len, 0ull,
                               hi, d_q, i0, m, d_ids, d_st, d_cnt, nullptr);
        HIP_OK(hipGetLastError());
    };
    uint32_t cnt[3] = {NO_BAD, 0u, 0u};
    auto read_cnt = [&] {
        HIP_OK(hipMemcpyAsync(cnt, d_cnt, sizeof cnt, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
    };
    reset();
    if (K == 1) {
        resolve(0, n, blob_len);
        read_cnt();                                                        // (before the check, as the host loop was)
        if (cnt[0] != NO_BAD)
            throw Error{KETO_E_INVALID, "request " + std::to_string(cnt[0]) + "'s fields lie outside the blob"};
        device_check_rows(S, d_ids, n, gmd, d_dec, st, S.n_parts == 1);                    // row ids -> handles, the check
    } else {
        for (uint32_t k = 0; k < K; ++k) {
            HIP_OK(hipStreamWaitEvent(st, R.ev[k], 0));
            resolve(cb[k], cb[k + 1] - cb[k], wb[k + 1]);
            device_check_rows(S, d_ids + cb[k], cb[k + 1] - cb[k], gmd, d_dec + cb[k], st, true);
        }
        read_cnt();
        if (cnt[0] != NO_BAD)
            throw Error{KETO_E_INVALID, "request " + std::to_string(cnt[0]) + "'s fields lie outside the blob"};
        if (cnt[2]) {                                                      // not packed in request order
            reset();
            resolve(0, n, blob_len);
            read_cnt();
            device_check_rows(S, d_ids, n, gmd, d_dec, st, S.n_parts == 1);
        }
    }
    lock_trace("packed: checked");
    hipLaunchKernelGGL(fold_undecided, dim3((n + 255) / 256), dim3(256), 0, st, d_dec, d_st, n);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(allowed, d_dec, n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    lock_trace("packed: copied back");
    if (d_clk) {                                   // tooling: percentiles of the per-step clocks (us)
        std::vector<uint32_t> c(4ull * n);
        HIP_OK(hipMemcpy(c.data(), d_clk, c.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        uint32_t t0 = c[0];
        for (uint32_t i = 0; i < n; ++i) t0 = (int32_t)(c[4ull * i] - t0) < 0 ? c[4ull * i] : t0;
        std::string line = "[resolve clocks] n " + std::to_string(n);
        const char* names[4] = {"start", "record", "row_query", "subject"};
        for (int k = 0; k < 4; ++k) {
            std::vector<double> v(n);
            for (uint32_t i = 0; i < n; ++i) v[i] = (k ? c[4ull * i + k] : c[4ull * i] - t0) / 100.0;
            std::sort(v.begin(), v.end());
            char b[160];
            snprintf(b, sizeof b, " | %s p50 %.2f p90 %.2f p99 %.2f max %.2f", names[k], v[n / 2], v[n * 9 / 10],
                     v[(uint64_t)n * 99 / 100], v[n - 1]);
            line += b;
        }
        fprintf(stderr, "%s\n", line.c_str());
    }
    if (cnt[1])                                                            // the wildcard queries: the host's
        for (uint32_t i = 0; i < n && host.size() < cnt[1]; ++i)
            if (status[i] == ST_HOST) host.push_back(i);
}

// A packed batch resolved on the device into the row-id form the routed path sends between parts
// (keto_check_batch_routed_packed, comm.cpp): the snapshot's device indexes as for
// keto_check_batch_packed, the requests' row ids and subject targets into d_out (n entries), their
// statuses into status_out (host).  Requests the device leaves to the host (wildcard queries) are
// listed in host_idx, with d_out holding {no row, no target} for them.  A request whose fields lie
// outside the blob fails the call (KETO_E_INVALID) before anything is written to status_out.
void device_resolve_packed_rows(Snapshot& S, const uint8_t* blob, uint64_t blob_len, const keto_check_packed* reqs,
                                uint32_t n, keto_check_ids* d_out, uint8_t* status_out, std::vector<uint32_t>& host_idx,
                                void* stream) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    host_idx.clear();
    if (!n) return;
    const DevView dv = device_view(S);
    HIP_OK(hipSetDevice(dv.device));
    RDevState& R = rdev_get(S, dv.device);
    std::lock_guard<std::mutex> lk(R.mu);
    rdev_refresh(S, R);
    hipStream_t st = (hipStream_t)stream;
    uint8_t* d_blob = R.blob.get<uint8_t>(std::max<uint64_t>(blob_len, 1));
    keto_check_packed* d_q = R.reqs.get<keto_check_packed>(n);
    uint8_t* d_st = R.status.get<uint8_t>(n);
    uint32_t* d_cnt = R.cnt.get<uint32_t>(4);
    if (blob_len) HIP_OK(hipMemcpyAsync(d_blob, blob, blob_len, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_q, reqs, (uint64_t)n * sizeof(keto_check_packed), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_cnt), NO_BAD, 1, st));
    HIP_OK(hipMemsetAsync(d_cnt + 1, 0, 3 * sizeof(uint32_t), st));
    hipLaunchKernelGGL(resolve_packed<false>, dim3((n + 255) / 256), dim3(256), 0, st, R.view, d_blob, blob_len, 0ull,
                       blob_len, d_q, 0u, n, d_out, d_st, d_cnt, nullptr);
    HIP_OK(hipGetLastError());
    uint32_t cnt[3] = {NO_BAD, 0u, 0u};
    std::vector<uint8_t> stv(n);
    HIP_OK(hipMemcpyAsync(cnt, d_cnt, sizeof cnt, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(stv.data(), d_st, n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (cnt[0] != NO_BAD) throw Error{KETO_E_INVALID, "request " + std::to_string(cnt[0]) + "'s fields lie outside the blob"};
    std::memcpy(status_out, stv.data(), n);
    if (cnt[1])
        for (uint32_t i = 0; i < n && host_idx.size() < cnt[1]; ++i)
            if (stv[i] == ST_HOST) host_idx.push_back(i);
}

void rdev_release(Snapshot& S) { S.rdev.reset(); }

}  // namespace keto
