// MI355X (gfx950) device engine for batched check and expand.
//
// Kernels
//   check_kernel   exact, order-faithful, depth-bounded DFS per request as a per-lane state machine
//                  over a persistent grid.  Reproduces check.(*Engine).SubjectIsAllowed /
//                  checkOneIndirectionFurther / subjectIsAllowed (internal/check/engine.go:36-123),
//                  including the first-encounter visited map keyed by Subject.String()
//                  (internal/x/graph/graph_utils.go:13-35) that is fresh for every top-level tuple
//                  and shared below it.
//   expand_kernel  the same traversal for expand.(*Engine).BuildTree (internal/expand/engine.go:
//                  33-102): one visited map per tree, counted first (FILL=false), then written in
//                  pre-order (FILL=true).
//
// Data: the snapshot is one u32 arena per device (layout in snapshot.hpp).  A row visit reads the
// row's 16-B header, which sits right in front of its edges, so the header line usually also holds
// the subject sets and a short id region.  A requested subject id is looked up in the row's
// id window (binary search, <= WINDOW_WORDS edges) or in the bucketed id table stored
// in front of the header: an id never changes the visited map unless its key collides, so only
// membership matters, which is what makes looking it up (instead of walking to it) exact.
// Visited maps keep their first REG_VIDS visit ids in registers and spill into a per-lane,
// epoch-tagged table in HBM; a table filling past 1/2 aborts the request, which is re-run on a
// tier with larger tables; the last tier is sized so it cannot overflow.  No request leaves the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <unordered_map>
#include <unordered_set>
#include <thread>
#include <vector>

#include "snapshot.hpp"

namespace keto {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

#ifndef KETO_CHECK_WAVES
// check_kernel: 5 waves per SIMD (84 VGPRs).  At 7 (72 VGPRs) the kernel spilled 28-40 B per lane to
// scratch inside the walk loop, and config #3's tier 0 took 158 ms against 124 ms at 5
// (profiles/r03m_config3_waves.log); it is the deep tier and the overflow tiers, where lanes wait on
// one long chain, so fewer resident lanes cost nothing.
#define KETO_CHECK_WAVES 5
#endif

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr int RES_FALSE = 0, RES_TRUE = 1, RES_OVERFLOW = 2;
constexpr int EXP_TREE = 0, EXP_NIL = 1, EXP_ERROR = 2, EXP_OVERFLOW = 3;
// (internal) the walk met a row another part owns with no copy in the call's overlay yet: the
// migrating part copies the rows it recorded and runs the count pass again
constexpr int EXP_RETRY = 4;

struct DevSnap {
    const uint32_t* arena;    // main arena (u32 words; tier 0 adds 2^32 words for segment 1)
    const uint64_t* coll;     // (edge value << 32) | visit id ; empty = ~0
    uint32_t coll_mask;       // 0 = no collisions
    uint32_t n_units;         // handles of the main arena are < n_units (DirectVisited's class base)
    uint32_t root_g;          // wide arenas: root handles past 2^31 count 16 << root_g bytes (hword)
};

struct DevOverlay {           // batch-local wildcard rows (top-level / root only)
    const uint32_t* arena;
    uint32_t base;            // handles >= base live in this arena (unit = handle - base)
    // expand on a migrating part: rows another part owns, copied into this arena for the call.  A
    // stub (HDR_REMOTE) is looked up here by its handle -> the handle of its copy (key << 32 | value,
    // ~0 = empty); NULL = no copies
    const uint64_t* rmap = nullptr;
    uint32_t rmask = 0;
};

__host__ __device__ inline uint32_t mix32(uint32_t k) {
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}
// the copy of a remote row (rmap), or NONE32
__device__ inline uint32_t rmap_find(const DevOverlay& ov, uint32_t h) {
    if (!ov.rmap) return 0xFFFFFFFFu;
    uint32_t i = mix32(h) & ov.rmask;
    for (;;) {
        const uint64_t e = ov.rmap[i];
        if (e == ~0ull) return 0xFFFFFFFFu;
        if ((uint32_t)(e >> 32) == h) return (uint32_t)e;
        i = (i + 1) & ov.rmask;
    }
}

__device__ inline uint32_t coll_lookup(const DevSnap& s, uint32_t key) {
    if (s.coll_mask == 0) return NONE32;
    uint32_t i = mix32(key) & s.coll_mask;
    for (;;) {
        uint64_t e = s.coll[i];
        if (e == ~0ull) return NONE32;
        if ((uint32_t)(e >> 32) == key) return (uint32_t)e;
        i = (i + 1) & s.coll_mask;
    }
}

struct RowView {
    const uint32_t* a;        // arena holding the row
    uint64_t beg;             // word index of the first edge
    uint32_t n_sets, n_ids;   // effective counts (ROW_SEQ: n_sets = all edges, in order)
    uint32_t hlog2;           // id table size (0 = none), table ends at beg - HDR_WORDS
    bool poison, poison0;     // some page / the first page fails toInternal (expand)
    bool seq;
    bool closure;             // a closure filter precedes the header (the id table precedes that)
    bool remote = false;      // a stub: the row lives on another part (migrating partition)
};

__device__ inline RowView load_row(const DevSnap& s, const DevOverlay& ov, uint32_t h) {
    RowView rv;
    uint64_t w;
    if (h >= ov.base) {
        rv.a = ov.arena;
        w = (uint64_t)(h - ov.base) * HDR_WORDS;
    } else {
        rv.a = s.arena;
        w = hword(h, s.root_g);
    }
    uint4 v = *reinterpret_cast<const uint4*>(rv.a + w);
    while (v.z & HDR_FWD) {                        // a row a write moved (delta.cpp): its current place
        w = hword(v.x, s.root_g);
        v = *reinterpret_cast<const uint4*>(rv.a + w);
    }
    rv.beg = w + HDR_WORDS;
    rv.n_sets = v.x;
    rv.n_ids = v.y;
    rv.seq = (v.z & HDR_SEQ) != 0;
    rv.hlog2 = (v.z >> 8) & 31u;
    rv.poison = (v.z & HDR_POISON) != 0;
    rv.poison0 = (v.z & HDR_POISON0) != 0;
    rv.closure = (v.z & HDR_CLOSURE) != 0;
    rv.remote = (v.z & HDR_REMOTE) != 0;
    return rv;
}

// Algorithmic-work counters (bench.py's roofline): compiled out of the production kernels.
template <bool ON>
struct Work {
    __device__ inline void row() {}
    __device__ inline void edge() {}
    __device__ inline void idread(uint32_t) {}
    __device__ inline void vprobe() {}
    __device__ inline void vinsert() {}
    __device__ inline void item() {}
    __device__ inline void request() {}
    __device__ inline void header(const void*) {}
    __device__ inline void edge_at(const void*) {}
    __device__ inline void id_at(const void*, bool) {}
    __device__ inline void push() {}
    __device__ inline void pop() {}
    __device__ inline void leaf(bool, uint32_t) {}
    __device__ inline void pruned() {}
    __device__ inline void simt(int) {}
};
template <>
struct Work<true> {
    // 0 rows, 1 set edges, 2 id words, 3 visited HBM probes, 4 visited inserts, 5 top-level items,
    // line touches (a 128-B line different from the lane's previous access in that stream):
    // 6 requests, 7 row headers, 8 edges, 9 id table, 10 id search, 11 frame pushes, 12 frame pops
    uint64_t c[16] = {};
    uint64_t edge_line = ~0ull, id_line = ~0ull;
    __device__ inline void row() { ++c[0]; }
    __device__ inline void edge() { ++c[1]; }
    __device__ inline void idread(uint32_t k) { c[2] += k; }
    __device__ inline void vprobe() { ++c[3]; }
    __device__ inline void vinsert() { ++c[4]; }
    __device__ inline void item() { ++c[5]; }
    __device__ inline void request() { ++c[6]; }
    __device__ inline void header(const void* p) {
        ++c[7];
        edge_line = id_line = (uint64_t)p >> 7;
    }
    __device__ inline void edge_at(const void* p) {
        const uint64_t l = (uint64_t)p >> 7;
        if (l != edge_line) ++c[8];
        edge_line = l;
    }
    __device__ inline void id_at(const void* p, bool table) {
        const uint64_t l = (uint64_t)p >> 7;
        if (l != id_line) ++c[table ? 9 : 10];
        id_line = l;
    }
    __device__ inline void push() { ++c[11]; }
    __device__ inline void pop() { ++c[12]; }
    // 13 leaf rows entered (no subject sets), 14 of them without the requested id; 15 subject
    // sets skipped by their closure filter
    __device__ inline void leaf(bool miss, uint32_t) {
        ++c[13];
        if (miss) ++c[14];
    }
    __device__ inline void pruned() { ++c[15]; }
    // SIMT profile (work slots 16..23, KETO_SIMT_PROF): even k = wave-level count of event k/2
    // (once per wave, by its first active lane), odd k = lane-level count of it
    uint32_t s[8] = {};
    __device__ inline void simt(int k) {
        const uint64_t m = __ballot(1);
        if ((threadIdx.x & 63u) == (uint32_t)__ffsll((unsigned long long)m) - 1u) ++s[2 * k];
        ++s[2 * k + 1];
    }
};
// ------------------------------------------------------------------ visited maps
// Probe sequence of the hashed maps: 32-B buckets of four entries (epoch << 32 | visit id), read
// with two 16-B loads from one line, bucket after bucket; the entries of a bucket are taken in
// order.  Entries are never removed, so an id is always found before the first empty entry of its
// sequence.  A deep search's map lives mostly here (tens of thousands of ids at depth 32), so a
// test is one line round trip instead of a dependent chain of 8-B probes.  Returns 1 if vid is
// present; else 0 and *slot = the first empty entry.
__device__ inline int probe_bucketed(const uint64_t* tab, uint32_t mask, uint32_t epoch, uint32_t vid, uint32_t* slot) {
    uint32_t i = mix32(vid) & mask & ~3u;
    for (;;) {
        const uint4 a = *reinterpret_cast<const uint4*>(tab + i);
        const uint4 b = *reinterpret_cast<const uint4*>(tab + i + 2);
        const uint32_t lo[4] = {a.x, a.z, b.x, b.z}, hi[4] = {a.y, a.w, b.y, b.w};
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            if (hi[k] != epoch) {
                *slot = i + k;
                return 0;
            }
            if (lo[k] == vid) return 1;
        }
        i = (i + 4) & mask;
    }
}

struct Visited {
    uint64_t* tab;
    uint32_t mask;
    uint32_t epoch;
    uint32_t count;
    __device__ inline void fresh() {
        if (epoch >= 0xFFFFFFFEu) {        // epoch wrap: clear this lane's table once
            for (uint32_t i = 0; i <= mask; ++i) tab[i] = 0;
            epoch = 0;
        }
        ++epoch;
        count = 0;
    }
    // 0 = newly added, 1 = already present, 2 = table too full (request must move up a tier)
    template <class W>
    __device__ inline int test_add(uint32_t vid, W& w) {
        const uint64_t want = ((uint64_t)epoch << 32) | vid;
        if (mask >= 3) {                   // tables of >= 4 entries (every tier's): bucketed
            uint32_t at = 0;
            w.vprobe();
            if (probe_bucketed(tab, mask, epoch, vid, &at)) return 1;
            if ((++count) * 2u > mask + 1u) return 2;
            tab[at] = want;
            w.vinsert();
            return 0;
        }
        uint32_t i = mix32(vid) & mask;
        for (;;) {
            uint64_t e = tab[i];
            w.vprobe();
            if ((uint32_t)(e >> 32) != epoch) {
                if ((++count) * 2u > mask + 1u) return 2;
                tab[i] = want;
                w.vinsert();
                return 0;
            }
            if (e == want) return 1;
            i = (i + 1) & mask;
        }
    }
    // read-only membership (a borrowing map's earlier ids)
    __device__ inline bool has(uint32_t vid) const {
        if (mask >= 3) {
            uint32_t at = 0;
            return probe_bucketed(tab, mask, epoch, vid, &at) == 1;
        }
        const uint64_t want = ((uint64_t)epoch << 32) | vid;
        for (uint32_t i = mix32(vid) & mask;; i = (i + 1) & mask) {
            const uint64_t e = tab[i];
            if ((uint32_t)(e >> 32) != epoch) return false;
            if (e == want) return true;
        }
    }
    __device__ inline void release() {}
};

// Tier 2 (the few requests whose maps outgrow every hashed table): one 16-bit epoch per possible
// visit id (main-arena handle or collision class), indexed directly.  A test is one 2-B load with
// no probe chain, over 2 B per arena unit instead of a hash table of 2^(log2(2 x rows) + 1) 8-B
// entries; a fresh map is one increment, and the table is cleared once every 65535 maps.
struct DirectVisited {
    uint64_t* tab;       // the lane's tier-2 table (mask + 1 words), used as uint16_t[4 (mask + 1)]
    uint32_t mask;
    uint32_t epoch;
    uint32_t count;
    uint32_t base;       // n_units: collision class c has index base + c
    // visit ids are main-arena handles (< n_units; set edges never point into a batch overlay)
    // or VID_CLASS | class; both map to one dense index below 4 (mask + 1)
    __device__ inline uint32_t index(uint32_t vid) const { return (vid & VID_CLASS) ? base + (vid & ~VID_CLASS) : vid; }
    __device__ inline void fresh() {
        epoch = (epoch & 0xFFFFu) + 1u;
        if (epoch == 0x10000u) {                   // epoch wrap: clear this lane's table once
            uint64_t* t = tab;
            for (uint64_t i = 0; i <= (uint64_t)mask; ++i) t[i] = 0;
            epoch = 1;
        }
        count = 0;
    }
    template <class W>
    __device__ inline int test_add(uint32_t vid, W& w) {
        uint16_t* t = reinterpret_cast<uint16_t*>(tab) + index(vid);
        w.vprobe();
        if (*t == (uint16_t)epoch) return 1;
        *t = (uint16_t)epoch;
        w.vinsert();
        return 0;
    }
    __device__ inline void release() {}
};

// Tiers 0 and 1 of deep batches: a hashed map (Visited) that, when it outgrows the lane's table,
// borrows a bigger table of the NEXT tier for the rest of the request instead of sending the
// request up a tier, where it would restart from scratch and run after every request of this tier:
// tier 0 borrows one of tier 1's hashed tables (Visited, DIRECT = false), tier 1 one of tier 2's
// direct tables (DirectVisited, DIRECT = true).  The lane's own table keeps the map's earlier ids
// (read-only from then on); new ids go to the borrowed table.  The next tier runs after this one
// on the same stream and its lanes own the same tables, so a table's epoch lives in the next
// tier's slot_epoch and is handed over on release.  With every table borrowed, or the borrowed
// one full too, the request moves up a tier as before.
template <bool DIRECT>
struct PromoVisited {
    uint64_t* tab;       // hashed: the lane's tier-1 table
    uint32_t mask;
    uint32_t epoch;
    uint32_t count;
    uint32_t base;       // n_units (DirectVisited::index)
    uint64_t* pool;      // tier 2's tables, pool_n x (pool_mask + 1) words
    uint32_t pool_mask, pool_n;
    uint32_t* pool_epoch;
    uint32_t* pool_busy; // bitmap of borrowed tables
    int d;               // borrowed table, -1 = none
    uint32_t depoch;     // its epoch for the current map
    uint32_t dcount;     // ids in it (hashed tables)
    uint32_t hint;       // first bitmap word to try
    bool live;           // the hashed table holds ids of the current map
    using BT = typename std::conditional<DIRECT, DirectVisited, Visited>::type;
    __device__ inline Visited hashed() { return Visited{tab, mask, epoch, count}; }
    __device__ inline BT borrowed() {
        uint64_t* const t = pool + (uint64_t)d * (pool_mask + 1ull);
        if constexpr (DIRECT) return DirectVisited{t, pool_mask, depoch, dcount, base};
        else return Visited{t, pool_mask, depoch, dcount};
    }
    __device__ inline void fresh() {
        Visited H = hashed();
        H.fresh();
        epoch = H.epoch;
        count = H.count;
        if (d >= 0) {
            BT B = borrowed();
            B.fresh();
            depoch = B.epoch;
            dcount = B.count;
            live = false;
        }
    }
    __device__ inline bool borrow() {
        const uint32_t nw = (pool_n + 31u) / 32u;
        for (uint32_t k = 0; k < nw; ++k) {
            const uint32_t wi = (hint + k) % nw;
            const uint32_t valid = pool_n - wi * 32u >= 32u ? NONE32 : (1u << (pool_n - wi * 32u)) - 1u;
            uint32_t cur = __hip_atomic_load(pool_busy + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (~cur & valid) {
                const uint32_t b = __ffs(~cur & valid) - 1u;
                const uint32_t old = atomicOr(pool_busy + wi, 1u << b);
                if (!(old & (1u << b))) {
                    __threadfence();                 // acquire: the last owner's epoch and marks
                    d = (int)(wi * 32u + b);
                    depoch = pool_epoch[d];
                    dcount = 0;
                    BT B = borrowed();
                    B.fresh();                       // a new map on the borrowed table
                    depoch = B.epoch;
                    dcount = B.count;
                    return true;
                }
                cur = old | (1u << b);
            }
        }
        return false;
    }
    __device__ inline void release() {
        if (d < 0) return;
        pool_epoch[d] = depoch;
        __threadfence();                             // release: marks and epoch before the bit
        atomicAnd(pool_busy + (d >> 5), ~(1u << (d & 31)));
        d = -1;
    }
    template <class W>
    __device__ inline int test_add(uint32_t vid, W& w) {
        if (d < 0) {
            Visited H = hashed();
            const int t = H.test_add(vid, w);
            epoch = H.epoch;
            count = H.count;
            if (t != 2 || pool_n == 0 || !borrow()) return t;
            live = true;                             // vid is in neither table: add it below
        } else if (live) {
            w.vprobe();                              // earlier ids of this map (table <= half full)
            if (hashed().has(vid)) return 1;
        }
        BT B = borrowed();
        const int t = B.test_add(vid, w);
        depoch = B.epoch;
        dcount = B.count;
        return t;
    }
};

// The first REG_VIDS visit ids of a map live in registers; a map that grows past them spills into
// the lane's HBM table.  Typical check items mark a handful of subject sets.
#ifndef KETO_REG_VIDS
#define KETO_REG_VIDS 8
#endif
constexpr int REG_VIDS = KETO_REG_VIDS;
// ...then the next LDS_VIDS in a per-lane LDS column ([slot][lane], conflict-free), then HBM.
#ifndef KETO_LDS_VIDS
#define KETO_LDS_VIDS 8
#endif
constexpr int LDS_VIDS = KETO_LDS_VIDS;
constexpr int LDS_STRIDE = 256;          // lanes per block
// A visited map of one lane: the first REG_VIDS ids in registers, the next LV in the lane's LDS
// column, and only the ids beyond those in the lane's HBM table (started fresh on the first
// overflow), so a test probes HBM only when a map has outgrown registers + LDS.  A 64-bit filter of
// hashed ids answers "new" for most tests of a small map with no scan; a scan reads the LDS slots
// with independent loads (one LDS round trip, not one per slot).
template <int LV, class VT = Visited, int RV = REG_VIDS, int STRIDE = LDS_STRIDE>
struct VisitedRS {
    uint32_t r[RV > 0 ? RV : 1];
    uint32_t n;          // ids held in r + lds; RV + LV + 1 = the HBM table holds the rest
    uint32_t f0, f1;     // filter of the ids in r + lds: bit (vid * 0x9E3779B1) >> 26
    uint32_t* lds;       // this lane's LDS column (stride STRIDE), or nullptr
    VT V;
    __device__ inline void fresh() {
        n = 0;
        f0 = f1 = 0;
    }
    template <class W>
    __device__ inline int test_add(uint32_t vid, W& w) {
        const uint32_t lcap = lds ? (uint32_t)LV : 0u;
        // a map past registers + LDS lives wholly in the table (its first ids were copied there at
        // the overflow), so a deep search's test is one table probe: the register compares and the
        // serial LDS scan cost a long chain ~0.5 us per step (tools/dev/chain_probe.py)
        if (n > (uint32_t)RV + lcap) return V.test_add(vid, w);
        const uint32_t b = (vid * 0x9E3779B1u) >> 26;
        const uint32_t bit = 1u << (b & 31u);
        if (((b < 32 ? f0 : f1) & bit) != 0) {             // the filter cannot rule vid out: scan
            const uint32_t m = min(n, (uint32_t)RV + lcap);
            bool hit = false;
#pragma unroll
            for (int i = 0; i < RV; ++i) hit |= ((uint32_t)i < m) & (r[i] == vid);
            // the LDS slots in groups of four independent loads (one LDS round trip per group), up to
            // the map's size: a map of a few ids reads one group, not all LV slots
            static_assert(LV % 4 == 0, "LDS slots come in groups of four");
            for (uint32_t i0 = 0; lcap && (uint32_t)RV + i0 < m && !hit; i0 += 4) {
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) hit |= ((uint32_t)RV + i0 + k < m) & (lds[(i0 + k) * STRIDE] == vid);
            }
            if (hit) return 1;
        }
        if (b < 32) f0 |= bit;
        else f1 |= bit;
        if (n < (uint32_t)RV) {
#pragma unroll
            for (int i = 0; i < RV; ++i)
                if ((uint32_t)i == n) r[i] = vid;
            ++n;
            return 0;
        }
        if (n < (uint32_t)RV + lcap) {
            lds[(n - RV) * STRIDE] = vid;
            ++n;
            return 0;
        }
        // first overflow of this map: the table takes every id so far (all distinct), then vid
        V.fresh();
        ++n;
#pragma unroll
        for (int i = 0; i < RV; ++i)
            if (V.test_add(r[i], w) == 2) return 2;
        for (uint32_t i = 0; i < lcap; ++i)
            if (V.test_add(lds[i * STRIDE], w) == 2) return 2;
        return V.test_add(vid, w);
    }
};

struct Frame {
    uint64_t pos;      // word index of the next edge
    uint32_t left;
    uint16_t k;        // remaining depth of the row
    uint16_t fl;       // FR_* flags
};
constexpr uint16_t FR_SEQ = 1, FR_TOP = 2, FR_OV = 4;
constexpr uint16_t FR_WV = 8;   // the frame's edge block (tier 0: window) holds the block of `pos`

template <int N>
struct LocalStack {
    Frame f[N];
    __device__ inline Frame& operator[](int i) { return f[i]; }
    __device__ inline void save(int i, const Frame& x) { f[i] = x; }
    __device__ inline Frame load(int i) { return f[i]; }
    __device__ static constexpr int cap() { return N; }
};
struct GlobalStack {
    Frame* f;           // this lane's frames
    int n;
    __device__ inline Frame& operator[](int i) { return f[i]; }
    __device__ inline void save(int i, const Frame& x) { f[i] = x; }
    __device__ inline Frame load(int i) { return f[i]; }
    __device__ inline int cap() const { return n; }
};
// Saved check frames in a per-lane LDS column ([frame][lane], 8 B each): the word position and
// the edges left, with the frame flags in the top bits of `left`.  A frame's remaining depth is
// not stored: a parent's is always its child's + 1 (the caller restores it).  Check only: a row
// with >= 2^29 edges left cannot be saved here and sends its request up a tier (LFULL).
constexpr uint32_t LDS_LEFT_MAX = (1u << 29) - 1u;
template <int N>
struct LdsStack {
    uint2* col;         // this lane's column: col[i * LDS_STRIDE]
    __device__ inline bool fits(const Frame& x) const { return x.left <= LDS_LEFT_MAX; }
    __device__ inline void save(int i, const Frame& x) {
        col[i * LDS_STRIDE] = make_uint2((uint32_t)x.pos, x.left | ((uint32_t)x.fl << 29));
    }
    __device__ inline Frame load(int i) {
        const uint2 v = col[i * LDS_STRIDE];
        return Frame{v.x, v.y & LDS_LEFT_MAX, 0, (uint16_t)(v.y >> 29)};
    }
    __device__ static constexpr int cap() { return N; }
};
template <class S>
struct is_lds_stack : std::false_type {
    static constexpr int frames = 1;
};
template <int N>
struct is_lds_stack<LdsStack<N>> : std::true_type {
    static constexpr int frames = N;
};

struct TierArgs {
    uint64_t* vtab;          // n_slots * (mask+1) entries
    uint32_t mask;
    uint32_t* slot_epoch;    // n_slots
    Frame* gstack;           // n_slots * gstack_n (GlobalStack tiers only)
    int gstack_n;
    const uint32_t* in_list; // NULL = all requests [0, n)
    const uint32_t* in_count;
    uint32_t* out_list;      // overflowed requests
    uint32_t* out_count;
    // tiers 0 / 1 of deep batches: the next tier's tables, borrowed on overflow (PromoVisited)
    uint64_t* pool;
    uint32_t pool_mask, pool_n;
    uint32_t* pool_epoch;
    uint32_t* pool_busy;
    // tier-0 wave kernel: dyn bits 0..15 > 0 hand out request runs of that many requests once a
    // lane's static first run (its share of dyn bits 16..18 eighths of the XCD's range) is done,
    // from 2^(dyn bits 20..23) heads per XCD (heads[32 (xcd H + h)], one line each) that deal the
    // XCD's runs out interleaved (head h: runs h, h + H, ...); 0 = static runs only
    uint32_t* heads;
    uint32_t dyn;
    // tier-0 wave kernel: walk at most this many window edges / pops per loop iteration (>= 1;
    // ~0u = until the lane needs a global access); a lane stopped early goes on next iteration
    // without one
    uint32_t walk_cap;
    // COUNT kernels: per-request loop iterations (the serial chain length of a request's search),
    // added over the tiers that ran it; NULL = not recorded
    uint32_t* steps;
    // check_kernel: requests with flags bit KETO_ITEM_FLAG are top-level items (reach.hip) when set;
    // item_owner[w] = the request of work request w, item_acc[request] bit 0 = some item of it is
    // allowed (set by the lane that finds it; the request's other items stop when they see it)
    uint32_t items;
    const uint32_t* item_owner;
    uint32_t* item_acc;
    // check_kernel: non-NULL = requests handed out one at a time from this counter after each lane's
    // first (a lane never holds a run of long searches back to back); NULL = contiguous runs
    uint32_t* next;
    // streamed host batch (tier-0 wave kernel, STREAM): 8-B keto_check_pair requests by row id that
    // land in chunks of 2^chunk_log2 behind the running launch; ready[c] != 0 once chunk c has
    // landed (written in copy order, so it also vouches for every earlier chunk).  Row ids become
    // handles through row_handle (n_rows entries, NO_UNIT: another part's root row, counted in
    // *misrouted); a lane that waits more than wait_ticks (100 MHz) for a chunk sets *stalled and
    // stops, and the caller checks the batch again without streaming
    const keto_check_pair* pairs;
    const uint32_t* ready;
    uint32_t chunk_log2;
    const uint32_t* row_handle;
    uint32_t n_rows;
    int32_t pair_depth;
    uint32_t* misrouted;
    uint32_t* stalled;
    uint64_t wait_ticks;
};

// ------------------------------------------------------------------ check
// T_NEVER: a subject-set request's target past 2^31 units is a root row (snapshot.hpp SEG_SHIFT):
// no tuple has it as subject, and no edge could hold its handle.  Its target is clamped to EDGE_VAL,
// whose set-edge value EDGE_SET | EDGE_VAL no edge has (targets lie below EDGE_VAL), so the search
// runs as the reference's does and never matches: false.
__device__ inline uint32_t win_at(const uint4& w, uint32_t i) {
    const uint32_t lo = (i & 1u) ? w.y : w.x;              // two-level select: no branches
    const uint32_t hi = (i & 1u) ? w.w : w.z;
    return (i & 2u) ? hi : lo;
}
__device__ inline bool has4(const uint4& v, uint32_t t) { return v.x == t || v.y == t || v.z == t || v.w == t; }

// Saved frames of check_kernel carry the 16-B edge block of their position (when the frame had it),
// so the walk resumes after a pop without reloading it.  GlobalStack tiers give each lane
// 2 x frames entries (frame, block, frame, block, ...); LocalStack tiers keep both in scratch.
template <class Stack>
struct CheckStack;
template <int N>
struct CheckStack<LocalStack<N>> {
    Frame f[N];
    uint4 b[N];
    __device__ inline CheckStack(const TierArgs&, uint32_t) {}
    __device__ static constexpr int cap() { return N; }
    __device__ inline void save(int i, const Frame& x, const uint4& blk) {
        f[i] = x;
        b[i] = blk;
    }
    __device__ inline Frame load(int i, uint4& blk) {
        blk = b[i];
        return f[i];
    }
};
template <>
struct CheckStack<GlobalStack> {
    uint4* p;           // this lane's frames: p[2i] = frame i, p[2i + 1] = its edge block
    int n;
    __device__ inline CheckStack(const TierArgs& ta, uint32_t slot)
        : p(reinterpret_cast<uint4*>(ta.gstack + (uint64_t)slot * ta.gstack_n)), n(ta.gstack_n / 2) {}
    __device__ inline int cap() const { return n; }
    __device__ inline void save(int i, const Frame& x, const uint4& blk) {
        reinterpret_cast<Frame*>(p)[2 * i] = x;
        p[2 * i + 1] = blk;
    }
    __device__ inline Frame load(int i, uint4& blk) {
        const uint4 a = p[2 * i];
        blk = p[2 * i + 1];
        return Frame{(uint64_t)a.x | ((uint64_t)a.y << 32), a.z, (uint16_t)(a.w & 0xFFFFu), (uint16_t)(a.w >> 16)};
    }
};

// Batched SubjectIsAllowed (internal/check/engine.go:36-123) as a per-lane state machine; the
// deep-request tier 0 (max-depth > 9) and the overflow tiers 1 and 2 of every depth.  A lane owns
// one request at a time; each loop iteration does ONE of
//   (a) fetch the lane's next request, or
//   (b) pop a finished row, or
//   (c) one edge of the current row: the top-level row (FR_TOP) starts a fresh visited map per
//       subject set (the shadowed ctx at engine.go:48), deeper rows test-and-set it
//       (graph_utils.go:13-35), in ORDER BY order,
// then, if (a) or (c) produced one, enters a row.  Long searches here are latency-bound chains of
// dependent accesses, so the kernel keeps them short: a row's header comes with its window (the
// first 16-B edge block) and, for a subject set, the requested id's closure-filter word, all from
// one line; that load is issued for a candidate child BEFORE its visited test, so the header and
// the HBM visited probe are in flight together; edges are read a 16-B block at a time and saved
// frames keep their block; the header bloom filter rules most absent ids out without the id table.
// Only a subject set reached with remaining depth >= 2 is entered (engine.go:65-69,88-91).
// check_kernel's visited map: KETO_CK_RV ids in registers, KETO_CK_LV in the lane's LDS column
#ifndef KETO_CK_RV
#define KETO_CK_RV REG_VIDS
#endif
#ifndef KETO_CK_LV
#define KETO_CK_LV LDS_VIDS
#endif
template <class Stack, bool COUNT, int TIER>
__global__ void __launch_bounds__(256, KETO_CHECK_WAVES) check_kernel(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q,
                                                    uint32_t n, int gmd, uint8_t* __restrict__ allowed, TierArgs ta,
                                                    unsigned long long* __restrict__ work) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    __shared__ uint32_t lds_vis[(KETO_CK_LV > 0 ? KETO_CK_LV : 1) * LDS_STRIDE];
    VisitedRS<KETO_CK_LV, typename std::conditional<TIER == 2, DirectVisited, PromoVisited<TIER == 1>>::type, KETO_CK_RV> V;
    V.fresh();
    V.lds = KETO_CK_LV > 0 ? lds_vis + threadIdx.x : nullptr;
    V.V.tab = ta.vtab + (uint64_t)slot * (ta.mask + 1u);
    V.V.mask = ta.mask;
    V.V.epoch = ta.slot_epoch[slot];
    V.V.count = 0;
    if constexpr (TIER == 2) V.V.base = min(s.n_units, EDGE_VAL);   // set visit ids are targets' handles (< 2^31)
    if constexpr (TIER < 2) {
        V.V.base = min(s.n_units, EDGE_VAL);   // set visit ids are targets' handles (< 2^31)
        V.V.hint = slot;
        V.V.dcount = 0;
        V.V.pool = ta.pool;
        V.V.pool_mask = ta.pool_mask;
        V.V.pool_n = ta.pool_n;
        V.V.pool_epoch = ta.pool_epoch;
        V.V.pool_busy = ta.pool_busy;
        V.V.d = -1;
        V.V.depoch = 0;
        V.V.live = false;
    }
    CheckStack<Stack> st(ta, slot);
    Work<COUNT> w;
    const uint32_t total = ta.in_list ? *ta.in_count : n;
    // each lane owns a contiguous run of requests, so consecutive fetches share request lines; with
    // ta.next, its first request and then one request per grab.  Fewer requests than lanes (the
    // overflow tiers: the longest searches) are spread one per `spread` lanes, so that they do not
    // share waves: a wave waits on its slowest lane every iteration, and 64 long searches in one
    // wave ran at 3.6 us per iteration against 1.7 us alone (profiles/r03de_deep_exp.log)
    const uint32_t per = ta.next ? 1u : (total + stride - 1) / stride;
    const uint32_t spread = (!ta.next && total > 0 && total < stride) ? stride / total : 1u;
    uint32_t j = slot % spread ? total : (slot / spread) * per;
    uint32_t j_end = min(total, j + per);
    bool busy = false;           // a request is in flight on this lane
    uint32_t qi = 0, T = 0;
    bool tset = false;
    uint32_t cwb = 0;            // T's closure-filter word << 5 | bit
    Frame cur{0, 0, 0, 0};
    uint32_t it = 0;                // iterations of the current request (COUNT: ta.steps)
    uint32_t own = NONE32;          // items: the request the current work request belongs to
    uint32_t poll = 0;              // items: iterations since the request's decision was last looked at
    const uint32_t* ce = s.arena;   // arena of the current frame
    uint4 blk = make_uint4(0, 0, 0, 0);
    uint64_t blk_at = ~0ull;        // word index of the 16-B edge block held in blk
    int sp = 0;
    for (;;) {
        uint32_t enter = NONE32;     // row handle to enter this iteration
        uint16_t enter_k = 0, enter_fl = 0;
        uint4 h0 = make_uint4(0, 0, 0, 0), h1 = make_uint4(0, 0, 0, 0);   // its header and window
        uint32_t cbw = NONE32;       // its closure-filter word of T (subject sets only)
        const uint32_t* ea = s.arena;   // its arena
        int res = -1;                // >= 0: request decided (RES_*)
        if constexpr (COUNT) ++it;
        if (!busy) {
            if (j >= j_end) {
                if (!ta.next) break;
                // the wave's lanes that need a request now take consecutive ones with one atomic
                const uint64_t want = __ballot(1);
                const uint32_t lane = threadIdx.x & 63u;
                const uint32_t leader = (uint32_t)__ffsll((unsigned long long)want) - 1u;
                uint32_t got = 0;
                if (lane == leader) got = atomicAdd(ta.next, (uint32_t)__popcll(want));
                got = __shfl(got, (int)leader);
                j = stride + got + (uint32_t)__popcll(want & ((1ull << lane) - 1ull));
                if (j >= total) break;
                j_end = j + 1;
            }
            qi = ta.in_list ? ta.in_list[j] : j;
            ++j;
            const keto_check_ids qq = q[qi];
            w.request();
            int d = qq.max_depth;
            if (d <= 0 || gmd < d) d = gmd;                       // engine.go:118-120
            if (qq.row == KETO_NO_ROW || d <= 0 || qq.target == KETO_NO_TARGET) {
                allowed[qi] = 0;
                continue;
            }
            busy = true;
            if constexpr (COUNT) it = 1;
            tset = (qq.flags & 1u) != 0;
            T = (qq.flags & 1u) ? min(qq.target, EDGE_VAL) : qq.target;   // see T_NEVER
            {
                uint32_t cwd, cbit;
                closure_bit(T, cwd, cbit);
                cwb = cwd << 5 | cbit;
            }
            sp = 0;
            enter = qq.row;
            enter_k = (uint16_t)d;
            enter_fl = FR_TOP;
            own = ta.item_owner ? ta.item_owner[qi] : NONE32;
            poll = 0;
            if (ta.items && (qq.flags & KETO_ITEM_FLAG)) {
                // a top-level item (reach.hip): the request row's subject set `row`, entered at the
                // item's depth with the fresh map of its top-level tuple, which holds the set itself
                // (engine.go:47-48 with the shadowed ctx; the item's root is not ROW_SEQ, so its visit
                // id is its handle)
                enter_fl = 0;
                V.fresh();
                w.item();
                (void)V.test_add(qq.row, w);
            }
            uint64_t hw;
            if (enter >= ov.base) {
                ea = ov.arena;
                hw = (uint64_t)(enter - ov.base) * HDR_WORDS;
            } else {
                hw = hword(enter, s.root_g);
            }
            h0 = *reinterpret_cast<const uint4*>(ea + hw);
            h1 = *reinterpret_cast<const uint4*>(ea + hw + HDR_WORDS);
        } else if (own != NONE32 && ++poll >= 256u) {
            // another item of this request allowed it (engine.go:73-75 returns there): this item's
            // decision no longer matters, stop its search
            poll = 0;
            if (__hip_atomic_load(ta.item_acc + own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u) res = RES_FALSE;
        } else if (cur.left == 0) {                               // row exhausted: pop
            if (--sp == 0) {
                res = RES_FALSE;
            } else {
                cur = st.load(sp - 1, blk);                       // with its own remaining depth
                blk_at = (cur.fl & FR_WV) ? (cur.pos & ~3ull) : ~0ull;
                w.pop();
                ce = (cur.fl & FR_OV) ? ov.arena : s.arena;
            }
        } else {
            const uint64_t bw = cur.pos & ~3ull;
            if (bw != blk_at) {                                   // next 16-B block of the row
                blk = *reinterpret_cast<const uint4*>(ce + bw);
                blk_at = bw;
                w.edge_at(ce + bw);
            }
            const uint32_t e = win_at(blk, (uint32_t)cur.pos & 3u);
            const uint32_t tval = tset ? (EDGE_SET | T) : T;
            ++cur.pos;
            --cur.left;
            w.edge();
            if (e & EDGE_SET) {
                const uint32_t child = e & EDGE_VAL;
                uint32_t vid = child;
                if (cur.fl & FR_SEQ) {
                    uint32_t c = coll_lookup(s, e);
                    if (c != NONE32) vid = c;
                }
                // a child that would be entered if new: its header, window and filter word are
                // loaded now, in flight together with the visited probe below
                if (cur.k >= 2 && !(tset && e == tval)) {
                    const uint64_t hw = (uint64_t)child * HDR_WORDS;
                    h0 = *reinterpret_cast<const uint4*>(s.arena + hw);
                    h1 = *reinterpret_cast<const uint4*>(s.arena + hw + HDR_WORDS);
                    if (!tset) cbw = s.arena[hw - CB_WORDS + (cwb >> 5)];     // every set target has a filter
                }
                if (cur.fl & FR_TOP) {                            // fresh map per top-level tuple
                    V.fresh();
                    w.item();
                }
                const int t = V.test_add(vid, w);
                if (t == 2) res = RES_OVERFLOW;
                else if (t == 0) {
                    if (tset && e == tval) res = RES_TRUE;        // engine.go:54-57
                    else if (cur.k >= 2) {                        // remaining depth after the hop >= 1
                        enter = child;
                        enter_k = cur.k - 1;
                        enter_fl = 0;
                    }
                }
            } else {                                              // subject id in an ordered row
                int t = 0;
                if (!(cur.fl & FR_TOP)) {
                    uint32_t c = coll_lookup(s, e);
                    if (c != NONE32) t = V.test_add(c, w);
                }
                if (t == 2) res = RES_OVERFLOW;
                else if (t == 0 && !tset && e == tval) res = RES_TRUE;
            }
        }
        if (enter != NONE32) {
            // a forward at the row's identity (delta.cpp): prune with the identity's filter below, then
            // read the row where it lives now
            const bool pruned_cb = (h0.z & HDR_CLOSURE) != 0;
            uint32_t at = enter;
            while (h0.z & HDR_FWD) {
                at = h0.x;
                h0 = *reinterpret_cast<const uint4*>(ea + hword(at, s.root_g));
                h1 = *reinterpret_cast<const uint4*>(ea + hword(at, s.root_g) + HDR_WORDS);
            }
            const uint32_t n_sets = h0.x, n_ids = h0.y;
            const bool seq = (h0.z & HDR_SEQ) != 0;
            const uint32_t hl = (h0.z >> 8) & 31u;
            const bool cb = pruned_cb;
            const bool tcb = (h0.z & HDR_CLOSURE) != 0;       // the id table sits below a filter
            const uint64_t beg = (at >= ov.base ? (uint64_t)(at - ov.base) * HDR_WORDS : hword(at, s.root_g)) + HDR_WORDS;
            w.row();
            w.header(ea + beg - HDR_WORDS);
            if (cb && !tset && !(enter_fl & FR_TOP) && !((cbw >> (cwb & 31u)) & 1u)) {
                enter = NONE32;                                   // T is not below this set: skip it
                w.pruned();
            } else if (!seq && !tset && n_ids > 0) {              // is the requested id in the row?
                bool hit = false;
                if (hl == 0) {                                    // all ids are in the window
#pragma unroll
                    for (uint32_t i = 0; i < WINDOW_WORDS; ++i)
                        hit |= (i >= n_sets) & (i < n_sets + n_ids) & (win_at(h1, i) == T);
                    w.idread(n_ids);
                } else {
                    uint32_t b1, b2;
                    bloom_bits(T, b1, b2);
                    if (bloom_has(h0.z, h0.w, b1) && bloom_has(h0.z, h0.w, b2)) {
                        const uint32_t nb = (1u << hl) / BUCKET_WORDS;
                        const uint64_t tb = beg - HDR_WORDS - (tcb ? CB_WORDS : 0u) - (1ull << hl);
                        for (uint32_t b = mix32(T) & (nb - 1);; b = (b + 1) & (nb - 1)) {
                            const uint4 v = *reinterpret_cast<const uint4*>(ea + tb + (uint64_t)b * BUCKET_WORDS);
                            w.idread(BUCKET_WORDS);
                            w.id_at(ea + tb + (uint64_t)b * BUCKET_WORDS, true);
                            if (has4(v, T)) {
                                hit = true;
                                break;
                            }
                            if (has4(v, NONE32)) break;
                        }
                    }
                }
                if (hit) res = RES_TRUE;
            }
            // the parent is saved only if it has edges left (saved frames: st[0 .. sp-1)); an
            // exhausted one is replaced, and the child returns straight to the grandparent
            const bool save = sp > 0 && cur.left > 0;
            if (enter != NONE32 && res < 0 && save && sp > st.cap()) res = RES_OVERFLOW;
            if (enter != NONE32 && res < 0) {
                if (save) {
                    Frame sv = cur;
                    sv.fl = (blk_at == (cur.pos & ~3ull)) ? (uint16_t)(cur.fl | FR_WV) : (uint16_t)(cur.fl & ~FR_WV);
                    st.save(sp - 1, sv, blk);
                    w.push();
                }
                cur = Frame{beg, n_sets, enter_k,
                            (uint16_t)(enter_fl | (seq ? FR_SEQ : 0) | (ea != s.arena ? FR_OV : 0))};
                ce = ea;
                blk = h1;
                blk_at = beg;
                if (save || sp == 0) ++sp;
            }
        }
        if (res >= 0) {
            if constexpr (COUNT) {
                if (ta.steps) ta.steps[qi] += it;
            }
            if (res == RES_OVERFLOW) {
                uint32_t at = atomicAdd(ta.out_count, 1u);
                ta.out_list[at] = qi;
            } else {
                allowed[qi] = (uint8_t)res;
                if (res == RES_TRUE && own != NONE32) atomicOr(ta.item_acc + own, 1u);
            }
            V.V.release();                                        // a borrowed tier-2 table (tier 1)
            busy = false;
        }
    }
    ta.slot_epoch[slot] = V.V.epoch;
    if constexpr (COUNT) {
        for (int i = 0; i < 16; ++i) atomicAdd(work + i, (unsigned long long)w.c[i]);
    }
}

// ------------------------------------------------------------------ check, tier 0
// The same traversal as check_kernel, restructured so that every loop iteration issues at most
// ONE global access per lane, and every lane issues it from the same instruction: a row's header
// together with its window of the first four edge words (2 x 16 B from one 32-B slot that never
// straddles a line), one 16-B bucket of a row's id table, or the next 16-B block of a long row's
// edges.  The lane's next request is prefetched alongside (into LDS), so starting a request costs
// no iteration.  Everything else -- walking the window, the visited maps, saving and restoring
// frames -- runs on registers and LDS, so a wave waits once per iteration with all of its lanes'
// accesses in flight together.  The header's bloom filter rules most absent ids out without the
// table.  Saved frames (position, edges left | depth | flags, optionally the unread window) live
// in LDS; a frame with no edges left is not saved (the child returns straight to the grandparent).
// A request needing more than F saved frames, or a row with more than WF_LEFT_MAX edges left when
// saved, overflows to the next tier (check_kernel).  Lane control state is one packed word.
constexpr uint32_t P_REQ = 0, P_HDR = 1, P_IDQ = 2, P_EDGE = 3, P_WALK = 4;
constexpr uint32_t WF_LEFT_MAX = (1u << 18) - 1u;   // saved lkf = left | skip << 18 | k << 22 | seg << 26 | fl << 28
// control word: phase 0..2 | k 3..7 | fl 8..11 | sp 12..15 | have 16 | nq 17 | tset 18 | hl 19..23 | nq2 24
// | cb 25 (the current row has a closure filter, so its id table starts CB_WORDS further down)
// | seg 26, 31 (bits 0 and 1 of the current row's arena segment: positions are 32-bit words within
//   a segment)
// | skip 27..30 (window slot i's subject set is ruled out by the row's child signatures; cleared
//   when the walk leaves the row's first block)
constexpr uint32_t C_PH = 0, C_K = 3, C_FL = 8, C_SP = 12, C_HL = 19, C_MK = 27;
constexpr uint32_t C_HAVE = 1u << 16, C_NQ = 1u << 17, C_TSET = 1u << 18, C_NQ2 = 1u << 24, C_CB = 1u << 25;
constexpr uint32_t C_SEG = 1u << 26, C_SEG2 = 1u << 31, C_MKS = 15u << C_MK;
// saved frame word: left 0..17 | skip 18..21 | k 22..25 (tier 0 runs max-depth <= 9) | seg 26..27 | fl 28..31
__device__ inline uint32_t bf(uint32_t c, uint32_t off, uint32_t wd) { return (c >> off) & ((1u << wd) - 1u); }
__device__ inline uint32_t c_seg(uint32_t c) { return ((c >> 26) & 1u) | ((c >> 30) & 2u); }
__device__ inline uint32_t c_with_seg(uint32_t c, uint32_t seg) {
    return (c & ~(C_SEG | C_SEG2)) | ((seg & 1u) << 26) | ((seg & 2u) << 30);
}
__device__ inline uint32_t bf_set(uint32_t c, uint32_t off, uint32_t wd, uint32_t v) {
    const uint32_t m = ((1u << wd) - 1u) << off;
    return (c & ~m) | ((v << off) & m);
}

// request prefetch slots per lane of the tier-0 kernels (2: the next pair; 1: the next request only,
// 4 KB less LDS per block -- room for a 7th wave per SIMD at 20 KB -- measured slower at 6 and at 7
// waves, 2.81 / 2.61-2.65 ms against 2.49-2.54, profiles/r06l_tier0_one_prefetch_slot_rejected.log)
#ifndef KETO_NQ_SLOTS
#define KETO_NQ_SLOTS 2
#endif

// requests j and j + 1 (if in the run) straight into the wave's LDS prefetch slots (global_load_lds:
// no VGPR destination; lane L's 16 B land at wave_base + 16 L, i.e. lds_nq[tid] and
// lds_nq[LDS_STRIDE + tid]); retired by the iteration's vmcnt(0)
__device__ inline void prefetch_pair(const keto_check_ids* q, uint32_t j, uint32_t j_end, uint4* wave_base) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(q + j), reinterpret_cast<void*>(wave_base), 16, 0, 0);
    if (j + 1u < j_end)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(q + j + 1u),
                                         reinterpret_cast<void*>(wave_base + LDS_STRIDE), 16, 0, 0);
}

// visited map of a tier-0 lane.  A 64-bit filter of hashed ids answers "new" for most tests with
// no scan; ids are kept newest-first in RV registers (inserting shifts the oldest out), then the
// lane's LDS column (LV slots), then the lane's HBM table (started fresh on the first overflow).
template <int RV, int LV>
struct LaneVisited {
    uint32_t r[RV];
    uint32_t f0, f1;             // filter bits 0..31, 32..63
    uint32_t n, epoch, count;
    __device__ inline void fresh() {
        n = 0;
        f0 = f1 = 0;
#pragma unroll
        for (int i = 0; i < RV; ++i) r[i] = NONE32;          // no visit id is NONE32: no count test
    }
    template <class W>
    __device__ inline int test_add(uint32_t vid, uint32_t* lds, uint64_t* tab, uint32_t mask, W& w) {
        const uint32_t b = (vid * 0x9E3779B1u) >> 26;
        const uint32_t bit = 1u << (b & 31u);
        const bool maybe = ((b < 32 ? f0 : f1) & bit) != 0;
        if (maybe) {                                         // the filter cannot rule it out: scan
            const uint32_t m = min(n, (uint32_t)(RV + LV));
            bool hit = false;
#pragma unroll
            for (int i = 0; i < RV; ++i) hit |= r[i] == vid;
            for (uint32_t i = RV; i < m && !hit; ++i) hit = lds[(i - RV) * LDS_STRIDE] == vid;
            if (hit) return 1;
            if (n > (uint32_t)(RV + LV)) {                   // the rest is in the HBM table
                Visited H{tab, mask, epoch, count};
                const int t = H.test_add(vid, w);
                epoch = H.epoch;
                count = H.count;
                return t;
            }
        }
        if (b < 32) f0 |= bit;
        else f1 |= bit;
        // insert newest-first; the oldest register entry moves out to LDS / HBM
        const uint32_t out = r[RV - 1];
#pragma unroll
        for (int i = RV - 1; i > 0; --i) r[i] = r[i - 1];
        r[0] = vid;
        ++n;
        if (n <= (uint32_t)RV) return 0;
        if (n <= (uint32_t)(RV + LV)) {
            lds[(n - 1 - RV) * LDS_STRIDE] = out;
            return 0;
        }
        Visited H{tab, mask, epoch, count};
        if (n == (uint32_t)(RV + LV) + 1u) H.fresh();       // first overflow of this map
        const int t = H.test_add(out, w);                   // `out` cannot be present yet
        epoch = H.epoch;
        count = H.count;
        return t == 2 ? 2 : 0;
    }
};

// waves per SIMD the wave kernels are compiled for (__launch_bounds__' second argument).  6, not 8:
// at 8 the compiler squeezed tier 0 into 64 VGPRs with spills and extra moves; at 6 it may use up
// to 80, and the 16.7M batch on the 1B graph runs 2.48 ms against 2.55 ms (8 + 8 visit ids) and
// 2.99 ms (4 + 16) on one box (profiles/r04aj_wave_waves.log)
#ifndef KETO_WAVE_WAVES
#define KETO_WAVE_WAVES 6
#endif

// streamed batches: wait (bounded) until chunk word `p` says the chunk has landed.  Relaxed is
// enough: the requests are only read after the word's value came back (program order), and the
// launch started with caches holding none of this batch's lines (tools/dev/stream_probe.hip)
__device__ inline bool chunk_wait(const uint32_t* p, uint64_t ticks) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return true;
    const uint64_t t0 = wall_clock64();
    for (;;) {
        __builtin_amdgcn_s_sleep(2);
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return true;
        if (wall_clock64() - t0 > ticks) return false;
    }
}

#ifndef KETO_STREAM_CPOL
#define KETO_STREAM_CPOL 0            // cache policy of the streamed request loads
#endif
constexpr uint32_t P_XLT = 5;          // streamed: the request's row id (and set target) -> handles

// WIDE: an arena past 64 GiB (snapshot.hpp hword).  Root rows may lie in any of its up to 18
// segments, targets only in segments 0 and 1; only a search's top frame is ever a root row, so the
// segment field of the control word and of saved frames keeps 0 and 1 as they are and 2 for "the
// lane's root segment", held in one register (rseg) set when the request's row is entered.
template <int F, bool WIN, int LV, int RV, bool COUNT, bool STREAM, bool WIDE = false>
__device__ __forceinline__ void
    check_wave_body(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                    uint8_t* __restrict__ allowed, TierArgs ta, unsigned long long* __restrict__ work) {
    const uint32_t tid = threadIdx.x;
    const uint32_t slot = blockIdx.x * blockDim.x + tid;
    const uint32_t stride = gridDim.x * blockDim.x;
    __shared__ uint32_t lds_vis[(LV > 0 ? LV : 1) * LDS_STRIDE];
    __shared__ uint2 sf_pk[F * LDS_STRIDE];
    __shared__ uint4 sf_win[(WIN ? F : 1) * LDS_STRIDE];
    // the lane's prefetched requests (STREAM: one slot holds a pair of 8-B requests)
    __shared__ uint4 lds_nq[(STREAM ? 1 : KETO_NQ_SLOTS) * LDS_STRIDE];
    uint32_t* const vcol = lds_vis + tid;
    LaneVisited<RV, LV> V;
    V.fresh();
    V.epoch = ta.slot_epoch[slot];
    V.count = 0;
    Work<COUNT> w;
    // each lane works through contiguous runs of requests (multiples of 4 long, 4-aligned):
    // requests are fetched two at a time and decisions are stored four at a time.  Static mode: one
    // run per lane.  Dynamic mode (ta.dyn): the batch is split into 8 per-XCD ranges (workgroup b
    // runs on XCD b % 8); a lane's first run covers its share of part of its XCD's range, then it takes
    // runs of ta.dyn requests from its XCD's head (one returning atomic per wave and grab), so lanes
    // that drew long searches do not hold up the end of the launch
    // Streamed batches (STREAM): dynamic runs only, dealt interleaved over the XCDs (run g of the
    // batch goes to XCD g % 8) so that every XCD works near the front where the chunks have landed
    const uint32_t R = ta.dyn & 0xFFFFu;
    uint32_t j, j_end, xe = n, dyn_base = 0;
    uint32_t* head = nullptr;
    bool whole_groups = true;                                  // runs are 4-aligned multiples of 4
    uint32_t known = 0;                                        // STREAM: chunks [0, known) have landed
    if (STREAM) {
        const uint32_t nx = min(8u, gridDim.x);
        j = j_end = 0;
        head = ta.heads + 32u * ((blockIdx.x % nx) << ((ta.dyn >> 20) & 15u));
    } else if (R == 0) {
        // batches under 4 requests per lane: runs of 1-3 requests (every lane busy; decisions are
        // then stored byte by byte); otherwise runs rounded up to a multiple of 4
        uint32_t per = (n + stride - 1) / stride;
        if (per >= 4u) per = (per + 3u) & ~3u;
        whole_groups = (per & 3u) == 0;
        j = min(n, slot * per);                                // next request to start
        j_end = min(n, j + per);
    } else {
        const uint32_t nx = min(8u, gridDim.x);                // ranges: one per XCD that has workgroups
        const uint32_t xcd = blockIdx.x % nx;
        const uint32_t lanes_x = (gridDim.x - xcd + nx - 1u) / nx * blockDim.x;
        const uint32_t lx = (blockIdx.x / nx) * blockDim.x + tid;
        const uint32_t xs = (uint32_t)(((uint64_t)n * xcd / nx) & ~3ull);
        xe = xcd == nx - 1u ? n : (uint32_t)(((uint64_t)n * (xcd + 1u) / nx) & ~3ull);
        const uint32_t r0 = (uint32_t)((uint64_t)(xe - xs) * ((ta.dyn >> 16) & 7u) / 8u / lanes_x) & ~3u;
        j = min(xe, xs + lx * r0);
        j_end = min(xe, j + r0);
        dyn_base = xs + lanes_x * r0;
        head = ta.heads + 32u * (xcd << ((ta.dyn >> 20) & 15u));
    }
    const bool packed = ((uintptr_t)allowed & 3u) == 0 && whole_groups;
    uint32_t acc = 0;                                          // decisions of the current group of 4

    uint32_t c = P_REQ;                                        // control word
    uint32_t T = 0;                                            // requested subject
    uint32_t pos = 0, left = 0;                                // current frame (k, fl in c)
    uint4 win = make_uint4(0, 0, 0, 0);
    uint32_t eh = 0;                                           // row to enter (P_HDR) / bucket (P_IDQ)
    uint32_t rseg = 0;                                         // WIDE: the segment of the request's row
    // record request qi's decision: whole groups of 4 are stored as one word, a run's partial last
    // group byte by byte
    auto decide = [&](uint32_t qi, uint32_t r) {
        if (!packed || (qi | 3u) >= j_end) {
            allowed[qi] = (uint8_t)r;
            return;
        }
        acc |= r << ((qi & 3u) * 8u);
        if ((qi & 3u) == 3u) {
            *reinterpret_cast<uint32_t*>(allowed + (qi & ~3u)) = acc;
            acc = 0;
        }
    };
    // start the lane's next request from its LDS prefetch slots (no iteration spent on fetching
    // it); requests that need no traversal are decided on the spot.  Leaves the phase at P_HDR, or
    // at P_REQ when no prefetched request is left (the next iteration fetches one or the lane ends)
    auto start_next = [&]() {
        while (c & C_NQ) {
            const uint4 nq = lds_nq[tid];
            const uint32_t qi = j++;
            uint32_t keep = 0;                                    // the pair's second request moves up
            if constexpr (STREAM) {
                // {row id, subject} x 2; the batch's request depth; P_XLT looks the handles up
                if (c & C_NQ2) {
                    lds_nq[tid] = make_uint4(nq.z, nq.w, 0u, 0u);
                    keep = C_NQ;
                }
                int d = ta.pair_depth;
                if (d <= 0 || gmd < d) d = gmd;                   // engine.go:118-120
                if (nq.x == KETO_NO_ROW || d <= 0 || nq.y == KETO_NO_TARGET) {
                    decide(qi, 0);
                    c = keep;
                    continue;
                }
                T = nq.y;                                         // bit 31: a subject set's row id
                eh = nq.x;
                c = P_XLT | ((uint32_t)d << C_K) | ((nq.y & EDGE_SET) ? C_TSET : 0u) | keep;
                return;
            }
            if constexpr (KETO_NQ_SLOTS == 2) {
                if (c & C_NQ2) {
                    lds_nq[tid] = lds_nq[LDS_STRIDE + tid];
                    keep = C_NQ;
                }
            }
            int d = (int)nq.w;
            if (d <= 0 || gmd < d) d = gmd;                       // engine.go:118-120
            if (nq.x == KETO_NO_ROW || d <= 0 || nq.y == KETO_NO_TARGET) {
                decide(qi, 0);
                c = keep;
                continue;
            }
            T = (nq.z & 1u) ? min(nq.y, EDGE_VAL) : nq.y;   // see T_NEVER
            eh = nq.x;
            c = P_HDR | ((uint32_t)d << C_K) | ((nq.z & 1u) ? C_TSET : 0u) | keep;   // sp 0, no frame
            return;
        }
        c = (c & ~7u) | P_REQ;
    };
    for (;;) {
        const uint32_t ph = bf(c, C_PH, 3);
        if (ph == P_REQ && j >= j_end) {
            if (R == 0) break;
            // the lanes that finished their run take the next runs of their XCD's range together:
            // from the wave's home head first, then (that head dealt out) from the XCD's others
            const uint32_t hl2 = (ta.dyn >> 20) & 15u, H = 1u << hl2;
            uint32_t h = ((blockIdx.x / min(8u, gridDim.x)) * (blockDim.x >> 6) + (tid >> 6)) & (H - 1u);
            bool got = false;
            for (uint32_t t = 0; t < H; ++t, h = (h + 1u) & (H - 1u)) {
                const uint64_t m = __ballot(1);
                const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
                uint32_t base = 0;
                if ((tid & 63u) == leader) base = atomicAdd(head + 32u * h, (uint32_t)__popcll(m));
                base = __shfl(base, (int)leader);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                const uint64_t run = ((uint64_t)(base + below) << hl2) + h;
                const uint64_t st = STREAM ? (run * min(8u, gridDim.x) + blockIdx.x % min(8u, gridDim.x)) * R
                                           : (uint64_t)dyn_base + run * R;
                if (st < xe) {
                    j = (uint32_t)st;
                    j_end = (uint32_t)min<uint64_t>(xe, st + R);
                    got = true;
                    break;
                }
            }
            if (!got) break;
            if constexpr (STREAM) {
                // the run's chunk (runs never straddle one) must have landed
                const uint32_t ck = j >> ta.chunk_log2;
                if (ck >= known) {
                    if (!chunk_wait(ta.ready + ck, ta.wait_ticks)) {
                        atomicAdd(ta.stalled, 1u);                 // (counted: keto_batch_timing)
                        break;
                    }
                    known = ck + 1u;
                }
            }
        }
        w.simt(0);
        // ---- the iteration's global accesses: one per lane (selected without branches), plus the
        // next request pair's prefetch
        const bool hdr = ph == P_HDR;
        const bool in_ov = hdr ? eh >= ov.base : (bf(c, C_FL, 4) & FR_OV) != 0;
        uint32_t seg, hdr_w;                                      // a header's segment and word in it
        if constexpr (WIDE) {
            const uint64_t hw = hword(eh, s.root_g);
            const uint32_t f = c_seg(c);
            seg = in_ov ? 0u : hdr ? (uint32_t)(hw >> 32) : f == 2u ? rseg : f;
            hdr_w = in_ov ? (eh - ov.base) * HDR_WORDS : (uint32_t)hw;
        } else {
            seg = in_ov ? 0u : hdr ? (eh >> SEG_SHIFT) : c_seg(c);
            hdr_w = 0;                                            // (the narrow form below, as before)
        }
        const uint32_t* const ar = (in_ov ? ov.arena : s.arena) + ((uint64_t)seg << 32);
        const uint32_t hl = bf(c, C_HL, 5);
        const uint32_t word = hdr ? (WIDE ? hdr_w : (in_ov ? eh - ov.base : eh & SEG_MASK) * HDR_WORDS)
                                  : ph == P_IDQ ? pos - HDR_WORDS - ((c & C_CB) ? CB_WORDS : 0u) - (1u << hl) +
                                                      eh * BUCKET_WORDS
                                                : (pos & ~3u);
        const uint4* const a0 = reinterpret_cast<const uint4*>(ar + word);
        // entering a subject set (always a row some set points at, so it has a closure filter):
        // the filter word of T, from the line the header comes in with
        const bool cbq = hdr && (c & (C_HAVE | C_TSET)) == C_HAVE;
        uint32_t cwd, cbit;
        closure_bit(T, cwd, cbit);
        if (hdr) w.header(a0);
        else if (ph == P_IDQ) {
            w.idread(BUCKET_WORDS);
            w.id_at(a0, true);
        } else if (ph == P_EDGE) {
            w.edge_at(a0);
        }
        if (!(c & C_NQ) && j < j_end) {                           // prefetch the next pair
            if constexpr (STREAM) {
                // requests j, j + 1 (j is even: runs are 4-aligned) in one 16-B load
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ta.pairs + j),
                                                 reinterpret_cast<void*>(lds_nq + (__builtin_amdgcn_readfirstlane(tid) & ~63u)),
                                                 16, 0, KETO_STREAM_CPOL);
            } else if constexpr (KETO_NQ_SLOTS == 1) {
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(q + j),
                                                 reinterpret_cast<void*>(lds_nq + (__builtin_amdgcn_readfirstlane(tid) & ~63u)),
                                                 16, 0, 0);
            } else {
                // (the wave's LDS base from a scalar: a vector copy of it was spilled to scratch)
                prefetch_pair(q, j, j_end, lds_nq + (__builtin_amdgcn_readfirstlane(tid) & ~63u));
            }
            c |= C_NQ | ((STREAM || KETO_NQ_SLOTS == 2) && j + 1u < j_end ? C_NQ2 : 0u);
            w.request();
        }
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        uint32_t cbw = NONE32, sgw = NONE32;
        uint32_t xr = NO_UNIT, xt = NO_UNIT;                      // STREAM, P_XLT: the handles
        if constexpr (STREAM) {
            if (ph == P_XLT) {
                if (eh < ta.n_rows) xr = ta.row_handle[eh];
                if ((c & C_TSET) && (T & EDGE_VAL) < ta.n_rows) xt = ta.row_handle[T & EDGE_VAL];
            }
        }
        if (ph != P_REQ && ph != P_WALK && (!STREAM || ph != P_XLT)) v0 = a0[0];
        if (hdr) v1 = a0[1];
        if (cbq) {
            // T's closure-filter word and T's child-signature word (both in the header's line)
            cbw = reinterpret_cast<const uint32_t*>(a0)[(int)cwd - (int)CB_WORDS];
            sgw = reinterpret_cast<const uint32_t*>(a0)[(int)((cbit & 15u) >> 3) - (int)SIG_WORDS];
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), seen by the compiler's waitcnt pass; also retires the LDS-direct prefetch
        if (ph == P_REQ) {
            start_next();
            continue;
        }
        if constexpr (STREAM) {
            if (ph == P_XLT) {                                    // as pairs_to_handles
                const uint32_t qi = j - 1;
                bool drop = false;
                if (xr == NO_UNIT) {                              // another part's root row
                    atomicAdd(ta.misrouted, 1u);
                    drop = true;
                } else if (c & C_TSET) {
                    drop = xt >= EDGE_VAL;                        // no tuple has it as subject (NO_UNIT too)
                    T = xt;
                }
                if (drop) {
                    decide(qi, 0);
                    start_next();
                } else {
                    eh = xr;
                    c = bf_set(c, C_PH, 3, P_HDR);
                }
                continue;
            }
        }
        w.simt(1);
        int res = -1;
        const bool tset = (c & C_TSET) != 0;
        if (ph == P_HDR && cbq && (v0.z & HDR_CLOSURE) && !((cbw >> cbit) & 1u)) {
            // T is not below this subject set: skip it, the parent's walk goes on (the set stays
            // marked visited, as in the reference; see HDR_CLOSURE)
            w.row();
            w.pruned();
            c = bf_set(c, C_PH, 3, P_WALK);
        } else if (ph == P_HDR && (v0.z & HDR_FWD)) {
            // the row's identity header forwards to where a write moved the row (delta.cpp): load
            // it there next iteration (the prune above used the identity's filter)
            eh = v0.x;
        } else if (ph == P_HDR) {
            // entering a row (engine.go:82-114): save the parent if it still has edges
            w.row();
            w.simt(3);
            const bool have = (c & C_HAVE) != 0;
            if (have && left > 0) {
                const uint32_t sp = bf(c, C_SP, 4);
                if (sp == F || left > WF_LEFT_MAX) {
                    res = RES_OVERFLOW;
                } else {
                    const uint32_t fl0 = bf(c, C_FL, 4);
                    uint32_t fl = fl0, px = pos;
                    if constexpr (!WIN) {
                        // one edge left and it is in the window: save the edge itself (WV marks
                        // it), so the pop needs no reload; otherwise the pop reloads the block
                        if (left == 1 && (fl0 & FR_WV)) px = win_at(win, pos & 3u);
                        else fl = fl0 & ~(uint32_t)FR_WV;
                    }
                    // the window's skip bits go with it (a saved single edge: its own, as slot 0)
                    const uint32_t mk = !WIN && (fl & FR_WV) && left == 1 ? (c >> (C_MK + (pos & 3u))) & 1u : bf(c, C_MK, 4);
                    sf_pk[sp * LDS_STRIDE + tid] =
                        make_uint2(px, left | (mk << 18) | (bf(c, C_K, 5) << 22) | (c_seg(c) << 26) | (fl << 28));
                    if constexpr (WIN) sf_win[sp * LDS_STRIDE + tid] = win;
                    c = bf_set(c, C_SP, 4, sp + 1);
                    w.push();
                }
            }
            if (res < 0) {
                const bool is_ov = eh >= ov.base;
                const bool seq = (v0.z & HDR_SEQ) != 0;
                const uint32_t hl = (v0.z >> 8) & 31u;
                const uint32_t k = have ? bf(c, C_K, 5) - 1u : bf(c, C_K, 5);
                const uint32_t fl = (have ? 0u : (uint32_t)FR_TOP) | (seq ? FR_SEQ : 0u) | (is_ov ? FR_OV : 0u) | FR_WV;
                left = v0.x;
                win = v1;
                c = bf_set(bf_set(bf_set(bf_set(c, C_K, 5, k), C_FL, 4, fl), C_HL, 5, hl), C_PH, 3, P_WALK) | C_HAVE;
                c = (v0.z & HDR_CLOSURE) ? (c | C_CB) : (c & ~C_CB);
                if constexpr (WIDE) {
                    // (seg / hdr_w are this iteration's header: eh has not changed since)
                    pos = hdr_w + HDR_WORDS;
                    if (seg >= 2u) rseg = seg;
                    c = c_with_seg(c, min(seg, 2u));
                } else {
                    pos = (is_ov ? eh - ov.base : eh & SEG_MASK) * HDR_WORDS + HDR_WORDS;
                    c = c_with_seg(c, is_ov ? 0u : eh >> SEG_SHIFT);
                }
                // window slots whose subject set cannot reach T (child signatures, read entering a
                // subject set; never for a subject-set request)
                const uint32_t skip = (have && !tset && (v0.z & HDR_CLOSURE)) ? ~(sgw >> ((cbit & 7u) * 4u)) & 15u : 0u;
                c = (c & ~C_MKS) | (skip << C_MK);
                const uint32_t n_sets = v0.x, n_ids = v0.y;
                if constexpr (COUNT) {
                    if (!seq && n_sets == 0 && !tset) {
                        bool in = false;
                        if (hl == 0) {
                            for (uint32_t i = 0; i < WINDOW_WORDS; ++i) in |= (i < n_ids) & (win_at(win, i) == T);
                        } else {
                            const uint32_t nb = (1u << hl) / BUCKET_WORDS;
                            const uint32_t* tab = ar + pos - HDR_WORDS -
                                                  ((v0.z & HDR_CLOSURE) ? CB_WORDS : 0u) - (1u << hl);
                            for (uint32_t b = mix32(T) & (nb - 1);; b = (b + 1) & (nb - 1)) {
                                const uint4 v = *reinterpret_cast<const uint4*>(tab + b * BUCKET_WORDS);
                                if (has4(v, T)) { in = true; break; }
                                if (has4(v, NONE32)) break;
                            }
                        }
                        w.leaf(!in, n_ids);
                    }
                }
                if (!seq && !tset && n_ids > 0) {                 // is the requested id in the row?
                    if (hl == 0) {                                // all ids are in the window
                        bool hit = false;
#pragma unroll
                        for (uint32_t i = 0; i < WINDOW_WORDS; ++i)
                            hit |= (i >= n_sets) & (i < n_sets + n_ids) & (win_at(win, i) == T);
                        w.idread(n_ids);
                        if (hit) res = RES_TRUE;
                    } else {
                        uint32_t b1, b2;
                        bloom_bits(T, b1, b2);
                        if (bloom_has(v0.z, v0.w, b1) && bloom_has(v0.z, v0.w, b2)) {
                            eh = mix32(T) & ((1u << hl) / BUCKET_WORDS - 1u);   // probe the table
                            c = bf_set(c, C_PH, 3, P_IDQ);
                        }
                    }
                }
            }
        } else if (ph == P_IDQ) {
            if (has4(v0, T)) res = RES_TRUE;
            else if (has4(v0, NONE32)) c = bf_set(c, C_PH, 3, P_WALK);
            else eh = (eh + 1u) & ((1u << bf(c, C_HL, 5)) / BUCKET_WORDS - 1u);
        } else if (ph == P_EDGE) {
            win = v0;
            c = bf_set(c, C_PH, 3, P_WALK) | ((uint32_t)FR_WV << C_FL);
        }
        // ---- walk the window (registers, LDS; HBM only for visited spills and collisions)
        for (uint32_t trip = 0; res < 0 && bf(c, C_PH, 3) == P_WALK; ++trip) {
            if (trip == ta.walk_cap) break;                       // go on next iteration
            w.simt(2);
            if (left == 0) {                                      // row exhausted: pop
                uint32_t sp = bf(c, C_SP, 4);
                if (sp == 0) {
                    res = RES_FALSE;
                    break;
                }
                --sp;
                const uint2 pk = sf_pk[sp * LDS_STRIDE + tid];
                if constexpr (WIN) {
                    win = sf_win[sp * LDS_STRIDE + tid];
                    pos = pk.x;
                } else if ((pk.y >> 28) & FR_WV) {               // a saved single edge
                    win = make_uint4(pk.x, pk.x, pk.x, pk.x);
                    pos = 0;
                } else {
                    pos = pk.x;
                }
                left = pk.y & WF_LEFT_MAX;
                c = bf_set(bf_set(bf_set(bf_set(c, C_SP, 4, sp), C_K, 5, (pk.y >> 22) & 15u), C_FL, 4, pk.y >> 28), C_MK,
                           4, pk.y >> 18);
                c = c_with_seg(c, (pk.y >> 26) & 3u);
                w.pop();
                continue;
            }
            const uint32_t fl = bf(c, C_FL, 4);
            if (!(fl & FR_WV)) {
                c = bf_set(c, C_PH, 3, P_EDGE);
                break;
            }
            const uint32_t e = win_at(win, pos & 3u);
            const bool skip = (c >> (C_MK + (pos & 3u))) & 1u;
            ++pos;
            --left;
            if ((pos & 3u) == 0) c &= ~(((uint32_t)FR_WV << C_FL) | C_MKS);
            w.edge();
            const uint32_t tval = tset ? (EDGE_SET | T) : T;
            if (e & EDGE_SET) {
                uint32_t vid = e & EDGE_VAL;
                if (fl & FR_SEQ) {
                    const uint32_t cv = coll_lookup(s, e);
                    if (cv != NONE32) vid = cv;
                }
                if (fl & FR_TOP) {                                // fresh map per top-level tuple
                    V.fresh();
                    w.item();
                }
                const int t = V.test_add(vid, vcol, ta.vtab + (uint64_t)slot * (ta.mask + 1u), ta.mask, w);
                if (t == 2) res = RES_OVERFLOW;
                else if (t == 0) {
                    if (tset && e == tval) res = RES_TRUE;        // engine.go:54-57
                    else if (bf(c, C_K, 5) >= 2) {                // remaining depth after the hop >= 1
                        if (skip) {
                            w.pruned();                           // its closure filter rules T out
                        } else {
                            eh = e & EDGE_VAL;
                            c = bf_set(c, C_PH, 3, P_HDR);
                        }
                    }
                }
            } else {                                              // subject id in an ordered row
                int t = 0;
                if (!(fl & FR_TOP)) {
                    const uint32_t cv = coll_lookup(s, e);
                    if (cv != NONE32) t = V.test_add(cv, vcol, ta.vtab + (uint64_t)slot * (ta.mask + 1u), ta.mask, w);
                }
                if (t == 2) res = RES_OVERFLOW;
                else if (t == 0 && !tset && e == tval) res = RES_TRUE;
            }
        }
        if (res >= 0) {
            const uint32_t qi = j - 1;
            if (res == RES_OVERFLOW) {                            // decided by the next tier
                const uint32_t at = atomicAdd(ta.out_count, 1u);
                ta.out_list[at] = qi;
                decide(qi, 0);
            } else {
                decide(qi, (uint32_t)res);
            }
            start_next();
        }
    }
    ta.slot_epoch[slot] = V.epoch;
    if constexpr (COUNT) {
        for (int i = 0; i < 16; ++i) atomicAdd(work + i, (unsigned long long)w.c[i]);
        for (int i = 0; i < 8; ++i) atomicAdd(work + 16 + i, (unsigned long long)w.s[i]);
    }
}
template <int F, bool WIN, int LV, int RV, bool COUNT, bool STREAM = false>
__global__ void __launch_bounds__(256, KETO_WAVE_WAVES)
    check_wave_kernel(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                      uint8_t* __restrict__ allowed, TierArgs ta, unsigned long long* __restrict__ work) {
    check_wave_body<F, WIN, LV, RV, COUNT, STREAM>(s, ov, q, n, gmd, allowed, ta, work);
}
// the same walk compiled for 8 waves per SIMD (64 VGPRs), for batches of fewer than 16 requests per
// lane: there the lanes a launch holds matter more than the instructions per iteration (config #2,
// 1M requests: 0.149 ms against 0.160-0.164 ms at 6 waves, profiles/r04al_small_batch_waves.log)
template <int F, int LV, int RV>
__global__ void __launch_bounds__(256, 8)
    check_wave_kernel_w8(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                         uint8_t* __restrict__ allowed, TierArgs ta, unsigned long long* __restrict__ work) {
    check_wave_body<F, false, LV, RV, false, false>(s, ov, q, n, gmd, allowed, ta, work);
}
// tier 0 of a wide arena (past 64 GiB): the default geometry, root rows in any segment
template <int F, bool STREAM>
__global__ void __launch_bounds__(256, KETO_WAVE_WAVES)
    check_wave_kernel_wide(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                           uint8_t* __restrict__ allowed, TierArgs ta, unsigned long long* __restrict__ work) {
    check_wave_body<F, false, 8, 8, false, STREAM, true>(s, ov, q, n, gmd, allowed, ta, work);
}

// ------------------------------------------------------------------ check, deep requests
// Tier 0 for global max-depth 10..64 (config #3: nested groups, depth 32, cycles).  The same design
// as check_wave_kernel -- a per-lane state machine over a persistent grid in which every loop
// iteration issues at most one global access per lane, from one instruction for the whole wave --
// extended to the two things deep searches do all the time and the shallow kernel does inline:
//   * saved frames live in HBM ([frame][lane], 8 B each, coalesced across the wave); a pop is its
//     own phase (P_POP: the frame load is the iteration's access);
//   * visited maps outgrow registers + LDS after a few dozen sets, so their HBM hash-table probes are
//     a phase too (P_VIS: one probe per iteration, test-and-insert).
// A lane whose map needs another probe, or whose row needs another id-table bucket, takes another
// iteration while the other lanes of its wave go on: no lane waits for another lane's probe chain,
// which is what bounded the inline check_kernel (an iteration there waited for the longest chain of
// 64 lanes: 5-6 us per step for the long searches in a full wave, 1.9 us alone,
// profiles/r02h_deep_experiments.log).  A map that fills its table moves the request to tier 1
// (check_kernel with larger / borrowed tables), as does a search deeper than DF saved frames.
constexpr uint32_t P_POP = 5, P_VIS = 6;
// control word: phase 0..2 | k 3..9 | fl 10..13 | sp 14..19 | have 20 | nq 21 | tset 22 | hl 23..27 |
// nq2 28 | cb 29 | seg 30 | match 31 (the pending visited test decides the request when it is new)
constexpr uint32_t D_K = 3, D_FL = 10, D_SP = 14, D_HL = 23;
constexpr uint32_t D_HAVE = 1u << 20, D_NQ = 1u << 21, D_TSET = 1u << 22, D_NQ2 = 1u << 28, D_CB = 1u << 29;
constexpr uint32_t D_SEG = 1u << 30, D_MATCH = 1u << 31;
// saved frame: x = position (word within its segment) or the saved single edge (FR_WV);
// y = left 0..19 | k 20..26 | seg 27 | fl 28..31
constexpr uint32_t DF_LEFT_MAX = (1u << 20) - 1u;
constexpr int DF = 63;                                     // saved frames: max-depth <= 64

template <int RV, int LV, bool COUNT>
__global__ void __launch_bounds__(256, KETO_WAVE_WAVES)
    deep_wave_kernel(DevSnap s, DevOverlay ov, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                     uint8_t* __restrict__ allowed, TierArgs ta, unsigned long long* __restrict__ work) {
    const uint32_t tid = threadIdx.x;
    const uint32_t slot = blockIdx.x * blockDim.x + tid;
    const uint32_t stride = gridDim.x * blockDim.x;
    __shared__ uint32_t lds_vis[(LV > 0 ? LV : 1) * LDS_STRIDE];
    __shared__ uint4 lds_nq[2 * LDS_STRIDE];                   // the lane's prefetched request pair
    uint32_t* const vcol = lds_vis + tid;
    uint2* const frames = reinterpret_cast<uint2*>(ta.gstack) + slot;   // frame f at frames[f * stride]
    uint64_t* const tab = ta.vtab + (uint64_t)slot * (ta.mask + 1u);
    Work<COUNT> w;
    // visited map: the first RV ids in registers, the next LV in the lane's LDS column, the rest in
    // the lane's epoch-tagged HBM table (probed by P_VIS); a 64-bit filter of all of them
    uint32_t vr[RV];
    uint32_t vf0 = 0, vf1 = 0, vn = 0, vcount = 0;
    uint32_t epoch = ta.slot_epoch[slot];
    auto vfresh = [&]() {
        vn = 0;
        vf0 = vf1 = 0;
#pragma unroll
        for (int i = 0; i < RV; ++i) vr[i] = NONE32;
        if (epoch >= 0xFFFFFFFEu) {                            // epoch wrap: clear this lane's table once
            for (uint32_t i = 0; i <= ta.mask; ++i) tab[i] = 0;
            epoch = 0;
        }
        ++epoch;
        vcount = 0;
    };
    vfresh();
    // runs of requests: as check_wave_kernel (static runs, or per-XCD dynamic runs)
    const uint32_t R = ta.dyn & 0xFFFFu;
    uint32_t j, j_end, xe = n, dyn_base = 0;
    uint32_t* head = nullptr;
    bool whole_groups = true;
    if (R == 0) {
        uint32_t per = (n + stride - 1) / stride;
        if (per >= 4u) per = (per + 3u) & ~3u;
        whole_groups = (per & 3u) == 0;
        j = min(n, slot * per);
        j_end = min(n, j + per);
    } else {
        const uint32_t nx = min(8u, gridDim.x);
        const uint32_t xcd = blockIdx.x % nx;
        const uint32_t lanes_x = (gridDim.x - xcd + nx - 1u) / nx * blockDim.x;
        const uint32_t lx = (blockIdx.x / nx) * blockDim.x + tid;
        const uint32_t xs = (uint32_t)(((uint64_t)n * xcd / nx) & ~3ull);
        xe = xcd == nx - 1u ? n : (uint32_t)(((uint64_t)n * (xcd + 1u) / nx) & ~3ull);
        const uint32_t r0 = (uint32_t)((uint64_t)(xe - xs) * ((ta.dyn >> 16) & 7u) / 8u / lanes_x) & ~3u;
        j = min(xe, xs + lx * r0);
        j_end = min(xe, j + r0);
        dyn_base = xs + lanes_x * r0;
        head = ta.heads + 32u * xcd;
    }
    const bool packed = ((uintptr_t)allowed & 3u) == 0 && whole_groups && (R & 3u) == 0;
    uint32_t acc = 0;

    uint32_t c = P_REQ;
    // top-level items (reach.hip, ta.items): the request a work request belongs to (its other items
    // stop when one is allowed, polled every 256 iterations), and "the next header is the item's own
    // set", entered below the top level with a map that already holds it (engine.go:47-48)
    uint32_t own = NONE32, poll = 0;
    bool item_entry = false;
    uint32_t T = 0;
    uint32_t pos = 0, left = 0;
    uint4 win = make_uint4(0, 0, 0, 0);
    uint32_t eh = 0;                                           // row to enter / bucket / pending child
    uint32_t vv = 0, pi = 0;                                   // pending visited test: id, probe slot
    uint32_t it = 0;                                           // COUNT: iterations of the request
    auto decide = [&](uint32_t qi, uint32_t r) {
        if (!packed || (qi | 3u) >= j_end) {
            allowed[qi] = (uint8_t)r;
            return;
        }
        acc |= r << ((qi & 3u) * 8u);
        if ((qi & 3u) == 3u) {
            *reinterpret_cast<uint32_t*>(allowed + (qi & ~3u)) = acc;
            acc = 0;
        }
    };
    auto start_next = [&]() {
        while (c & D_NQ) {
            const uint4 nq = lds_nq[tid];
            const uint32_t qi = j++;
            uint32_t keep = 0;
            if (c & D_NQ2) {
                lds_nq[tid] = lds_nq[LDS_STRIDE + tid];
                keep = D_NQ;
            }
            int d = (int)nq.w;
            if (d <= 0 || gmd < d) d = gmd;                       // engine.go:118-120
            if (nq.x == KETO_NO_ROW || d <= 0 || nq.y == KETO_NO_TARGET) {
                decide(qi, 0);
                c = keep;
                continue;
            }
            T = (nq.z & 1u) ? min(nq.y, EDGE_VAL) : nq.y;   // see T_NEVER
            eh = nq.x;
            if constexpr (COUNT) it = 0;
            c = P_HDR | ((uint32_t)d << D_K) | ((nq.z & 1u) ? D_TSET : 0u) | keep;
            own = ta.item_owner ? ta.item_owner[qi] : NONE32;
            poll = 0;
            item_entry = ta.items && (nq.z & KETO_ITEM_FLAG);
            if (item_entry) {
                // the item's set, entered at its depth with the fresh map of its top-level tuple, which
                // holds the set itself (its root is not ROW_SEQ: its visit id is its handle)
                vfresh();
                const uint32_t b = (eh * 0x9E3779B1u) >> 26;       // vtest's insert into a fresh map
                if (b < 32) vf0 |= 1u << b;
                else vf1 |= 1u << (b & 31u);
                vr[0] = eh;
                vn = 1;
                w.item();
            }
            return;
        }
        c = (c & ~7u) | P_REQ;
    };
    // a visited test the registers / LDS decide: 1 visited, 0 new (inserted), -1 the HBM table must
    // be probed (P_VIS; vv set, the first probe slot in pi)
    auto vtest = [&](uint32_t vid) -> int {
        const uint32_t b = (vid * 0x9E3779B1u) >> 26;
        const uint32_t bit = 1u << (b & 31u);
        const bool maybe = ((b < 32 ? vf0 : vf1) & bit) != 0;
        if (maybe) {
            const uint32_t m = min(vn, (uint32_t)(RV + LV));
            bool hit = false;
#pragma unroll
            for (int i = 0; i < RV; ++i) hit |= vr[i] == vid;
            for (uint32_t i = RV; i < m && !hit; ++i) hit = vcol[(i - RV) * LDS_STRIDE] == vid;
            if (hit) return 1;
        }
        if (b < 32) vf0 |= bit;
        else vf1 |= bit;
        if (vn < (uint32_t)RV) {
#pragma unroll
            for (int i = 0; i < RV; ++i)
                if ((uint32_t)i == vn) vr[i] = vid;
            ++vn;
            return 0;
        }
        if (vn < (uint32_t)(RV + LV)) {
            vcol[(vn - RV) * LDS_STRIDE] = vid;
            ++vn;
            return 0;
        }
        if (!maybe && vn == (uint32_t)(RV + LV)) {
            // (the filter ruled it out, but the table may be needed for the insert)
        }
        vv = vid;
        pi = mix32(vid) & ta.mask;
        return -1;
    };
    for (;;) {
        uint32_t ph = bf(c, C_PH, 3);
        if (ph == P_REQ && j >= j_end) {
            if (R == 0) break;
            const uint64_t m = __ballot(1);
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
            uint32_t base = 0;
            if ((tid & 63u) == leader) base = atomicAdd(head, (uint32_t)__popcll(m));
            base = __shfl(base, (int)leader);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint64_t st = (uint64_t)dyn_base + (uint64_t)(base + below) * R;
            if (st >= xe) break;
            j = (uint32_t)st;
            j_end = (uint32_t)min<uint64_t>(xe, st + R);
        }
        if constexpr (COUNT) ++it;
        // ---- the iteration's global access (one per lane) and the next request pair's prefetch
        const bool hdr = ph == P_HDR;
        const bool in_ov = hdr ? eh >= ov.base : (bf(c, D_FL, 4) & FR_OV) != 0;
        const bool hi = hdr ? ((eh >> SEG_SHIFT) & 1u) != 0 : (c & D_SEG) != 0;
        const uint32_t* const ar = (in_ov ? ov.arena : s.arena) + ((hi && !in_ov) ? (1ull << 32) : 0ull);
        const uint32_t hl = bf(c, D_HL, 5);
        const uint32_t sp = bf(c, D_SP, 6);
        const uint4* a0 = reinterpret_cast<const uint4*>(
            ar + (hdr ? (in_ov ? eh - ov.base : eh & SEG_MASK) * HDR_WORDS
                      : ph == P_IDQ ? pos - HDR_WORDS - ((c & D_CB) ? CB_WORDS : 0u) - (1u << hl) + eh * BUCKET_WORDS
                                    : (pos & ~3u)));
        const bool cbq = hdr && (c & (D_HAVE | D_TSET)) == D_HAVE;
        uint32_t cwd, cbit;
        closure_bit(T, cwd, cbit);
        if (hdr) w.header(a0);
        else if (ph == P_IDQ) w.id_at(a0, true);
        else if (ph == P_EDGE) w.edge_at(a0);
        if (!(c & D_NQ) && j < j_end) {
            prefetch_pair(q, j, j_end, lds_nq + (tid & ~63u));
            c |= D_NQ | (j + 1u < j_end ? D_NQ2 : 0u);
            w.request();
        }
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        uint2 fr = make_uint2(0, 0);
        uint64_t ve = 0;
        uint32_t cbw = NONE32;
        if (ph == P_POP) fr = frames[(uint64_t)(sp - 1u) * stride];
        else if (ph == P_VIS) ve = tab[pi];
        else if (ph != P_REQ) v0 = a0[0];
        if (hdr) v1 = a0[1];
        if (cbq) cbw = reinterpret_cast<const uint32_t*>(a0)[(int)cwd - (int)CB_WORDS];
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (visible to the compiler's waitcnt pass)
        if (ph == P_REQ) {
            start_next();
            continue;
        }
        int res = -1;
        const bool tset = (c & D_TSET) != 0;
        if (own != NONE32 && ++poll >= 256u) {
            // another item of this request allowed it (engine.go:73-75 returns there): stop
            poll = 0;
            if (__hip_atomic_load(ta.item_acc + own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u) res = RES_FALSE;
        }
        if (res >= 0) {
        } else if (ph == P_VIS) {
            // one probe of the HBM table: empty (another epoch) -> the id is new, insert it here
            w.vprobe();
            const uint64_t want = ((uint64_t)epoch << 32) | vv;
            if ((uint32_t)(ve >> 32) != epoch) {
                if ((++vcount) * 2u > ta.mask + 1u) {
                    res = RES_OVERFLOW;                        // the map outgrew the table: next tier
                } else {
                    tab[pi] = want;
                    w.vinsert();
                    if (c & D_MATCH) res = RES_TRUE;          // engine.go:54-57
                    else c = bf_set(c, C_PH, 3, eh != NONE32 ? P_HDR : P_WALK);
                }
            } else if (ve == want) {
                c = bf_set(c, C_PH, 3, P_WALK);               // visited: skip it
            } else {
                pi = (pi + 1u) & ta.mask;                     // next probe, next iteration
            }
            c &= ~(res < 0 && bf(c, C_PH, 3) != P_VIS ? D_MATCH : 0u);
        } else if (ph == P_POP) {
            const uint32_t nsp = sp - 1u;
            if ((fr.y >> 28) & FR_WV) {                        // a saved single edge
                win = make_uint4(fr.x, fr.x, fr.x, fr.x);
                pos = 0;
            } else {
                pos = fr.x;
            }
            left = fr.y & DF_LEFT_MAX;
            c = bf_set(bf_set(bf_set(c, D_SP, 6, nsp), D_K, 7, (fr.y >> 20) & 127u), D_FL, 4, fr.y >> 28);
            c = ((fr.y >> 27) & 1u) ? (c | D_SEG) : (c & ~D_SEG);
            c = bf_set(c, C_PH, 3, P_WALK);
            w.pop();
        } else if (ph == P_HDR && cbq && (v0.z & HDR_CLOSURE) && !((cbw >> cbit) & 1u)) {
            w.row();
            w.pruned();
            c = bf_set(c, C_PH, 3, P_WALK);                   // T is not below this set: skip it
        } else if (ph == P_HDR && (v0.z & HDR_FWD)) {
            eh = v0.x;                                        // a row a write moved (delta.cpp)
        } else if (ph == P_HDR) {
            w.row();
            const bool have = (c & D_HAVE) != 0;
            if (have && left > 0) {                           // save the parent (it has edges left)
                if (sp == (uint32_t)DF || left > DF_LEFT_MAX) {
                    res = RES_OVERFLOW;
                } else {
                    const uint32_t fl0 = bf(c, D_FL, 4);
                    uint32_t fl = fl0, px = pos;
                    if (left == 1 && (fl0 & FR_WV)) px = win_at(win, pos & 3u);
                    else fl = fl0 & ~(uint32_t)FR_WV;
                    frames[(uint64_t)sp * stride] =
                        make_uint2(px, left | (bf(c, D_K, 7) << 20) | ((c & D_SEG) ? (1u << 27) : 0u) | (fl << 28));
                    c = bf_set(c, D_SP, 6, sp + 1u);
                    w.push();
                }
            }
            if (res < 0) {
                const bool is_ov = eh >= ov.base;
                const bool seq = (v0.z & HDR_SEQ) != 0;
                const uint32_t hln = (v0.z >> 8) & 31u;
                const uint32_t k = have ? bf(c, D_K, 7) - 1u : bf(c, D_K, 7);
                const uint32_t fl = (have || item_entry ? 0u : (uint32_t)FR_TOP) | (seq ? FR_SEQ : 0u) | (is_ov ? FR_OV : 0u) | FR_WV;
                item_entry = false;
                pos = (is_ov ? eh - ov.base : eh & SEG_MASK) * HDR_WORDS + HDR_WORDS;
                left = v0.x;
                win = v1;
                c = bf_set(bf_set(bf_set(bf_set(c, D_K, 7, k), D_FL, 4, fl), D_HL, 5, hln), C_PH, 3, P_WALK) | D_HAVE;
                c = (v0.z & HDR_CLOSURE) ? (c | D_CB) : (c & ~D_CB);
                c = (!is_ov && ((eh >> SEG_SHIFT) & 1u)) ? (c | D_SEG) : (c & ~D_SEG);
                const uint32_t n_sets = v0.x, n_ids = v0.y;
                if (!seq && !tset && n_ids > 0) {             // is the requested id in the row?
                    if (hln == 0) {
                        bool hit = false;
#pragma unroll
                        for (uint32_t i = 0; i < WINDOW_WORDS; ++i)
                            hit |= (i >= n_sets) & (i < n_sets + n_ids) & (win_at(win, i) == T);
                        w.idread(n_ids);
                        if (hit) res = RES_TRUE;
                    } else {
                        uint32_t b1, b2;
                        bloom_bits(T, b1, b2);
                        if (bloom_has(v0.z, v0.w, b1) && bloom_has(v0.z, v0.w, b2)) {
                            eh = mix32(T) & ((1u << hln) / BUCKET_WORDS - 1u);
                            c = bf_set(c, C_PH, 3, P_IDQ);
                        }
                    }
                }
            }
        } else if (ph == P_IDQ) {
            w.idread(BUCKET_WORDS);
            if (has4(v0, T)) res = RES_TRUE;
            else if (has4(v0, NONE32)) c = bf_set(c, C_PH, 3, P_WALK);
            else eh = (eh + 1u) & ((1u << bf(c, D_HL, 5)) / BUCKET_WORDS - 1u);
        } else if (ph == P_EDGE) {
            win = v0;
            c = bf_set(c, C_PH, 3, P_WALK) | ((uint32_t)FR_WV << D_FL);
        }
        // ---- walk the window (registers, LDS); HBM probes, pops and reloads are phases
        while (res < 0 && bf(c, C_PH, 3) == P_WALK) {
            if (left == 0) {                                  // row exhausted: pop
                if (bf(c, D_SP, 6) == 0) {
                    res = RES_FALSE;
                    break;
                }
                c = bf_set(c, C_PH, 3, P_POP);
                break;
            }
            const uint32_t fl = bf(c, D_FL, 4);
            if (!(fl & FR_WV)) {
                c = bf_set(c, C_PH, 3, P_EDGE);
                break;
            }
            const uint32_t e = win_at(win, pos & 3u);
            ++pos;
            --left;
            if ((pos & 3u) == 0) c &= ~((uint32_t)FR_WV << D_FL);
            w.edge();
            const uint32_t tval = tset ? (EDGE_SET | T) : T;
            int t = 0;
            bool match = false;
            eh = NONE32;
            if (e & EDGE_SET) {
                uint32_t vid = e & EDGE_VAL;
                if (fl & FR_SEQ) {
                    const uint32_t cv = coll_lookup(s, e);
                    if (cv != NONE32) vid = cv;
                }
                if (fl & FR_TOP) {                            // fresh map per top-level tuple
                    vfresh();
                    w.item();
                }
                match = tset && e == tval;
                if (!match && bf(c, D_K, 7) >= 2) eh = e & EDGE_VAL;   // remaining depth after the hop >= 1
                t = vtest(vid);
            } else {                                          // subject id in an ordered row
                match = !tset && e == tval;
                if (!(fl & FR_TOP)) {
                    const uint32_t cv = coll_lookup(s, e);
                    if (cv != NONE32) t = vtest(cv);
                }
            }
            if (t < 0) {                                      // the HBM table decides: P_VIS
                c = bf_set(c, C_PH, 3, P_VIS) | (match ? D_MATCH : 0u);
                break;
            }
            if (t == 0) {
                if (match) res = RES_TRUE;                    // engine.go:54-57
                else if (eh != NONE32) c = bf_set(c, C_PH, 3, P_HDR);
            }
        }
        if (res >= 0) {
            const uint32_t qi = j - 1;
            if constexpr (COUNT) {
                if (ta.steps) ta.steps[qi] += it;
            }
            c &= ~D_MATCH;
            if (res == RES_OVERFLOW) {
                const uint32_t at = atomicAdd(ta.out_count, 1u);
                ta.out_list[at] = qi;
                decide(qi, 0);
            } else {
                decide(qi, (uint32_t)res);
                if (res == RES_TRUE && own != NONE32) atomicOr(ta.item_acc + own, 1u);
            }
            own = NONE32;
            start_next();
        }
    }
    ta.slot_epoch[slot] = epoch;
    if constexpr (COUNT) {
        for (int i = 0; i < 16; ++i) atomicAdd(work + i, (unsigned long long)w.c[i]);
    }
}

// ------------------------------------------------------------------ expand
// A row's run of subject ids (all leaves) is not copied by the traversing lane, one node per
// iteration while its wave waits, but queued and copied afterwards, coalesced (copy_lane_runs,
// copy_big_runs).  Each tier-0 lane queues into its own RUNS_PER_LANE entries (no atomics: a
// returning atomic per run, or per few runs, put a round trip on the traversal's critical path:
// the fill pass took twice the count pass's time, profiles/r03ex_expand_ab.txt); runs of at most
// ExpandOut::run_inline ids (KETO_EXPAND_RUN_INLINE, default 0), runs past a lane's entries and runs
// of later tiers are copied in place.
constexpr uint32_t RUN_INLINE_DEFAULT = 0;
constexpr uint32_t RUNS_PER_LANE = 32;
// a run longer than BIG_RUN ids goes to a shared queue instead, cut into BIG_RUN-id pieces that
// different waves copy (one atomic per big run: rare, and small next to the copy it saves).  256
// instead of 1024 made config #5's stage pass 178 -> 612 us (the queue's claims contend),
// profiles/r06zg_expand_big_run_256_rejected.log
#ifndef KETO_BIG_RUN
#define KETO_BIG_RUN 1024
#endif
constexpr uint32_t BIG_RUN = KETO_BIG_RUN;
struct CopyRun {
    const uint32_t* src;     // the ids
    keto_tree_node* dst;     // their leaf nodes
    uint64_t len;
};
struct ExpandOut {
    keto_tree_node* nodes;   // FILL only
    const uint64_t* offset;  // FILL only
    uint64_t* count;         // count pass: nodes per root
    uint8_t* status;
    CopyRun* runs;           // FILL, tier 0: the lanes' queued id runs (NULL = copy every run in place)
    uint32_t* lane_runs;     // runs queued per lane (RUNS_PER_LANE entries per lane at runs + lane * ..)
    uint32_t run_inline;
    CopyRun* big;            // pieces of runs longer than BIG_RUN | their count
    uint32_t* n_big;
    uint32_t big_cap;
    // staging (EXP_STAGE, tier 0 of the one-pass expand): each lane writes its roots' trees into its
    // own region of `stage` (stage_cap nodes, trees back to back) and records where (stage_pos, ~0 =
    // not staged: the tree did not fit, or a later tier decided it); a fill pass (EXP_FILL) then
    // skips the staged roots
    keto_tree_node* stage;
    uint64_t stage_cap;
    uint64_t* stage_pos;
    // a tree that outgrows its lane's region goes on in an overflow chunk (ovf_chunk nodes taken from
    // the pool at stage + ovf_base, *ovf_used of ovf_cap taken so far): its first split_at nodes stay
    // in the region, the rest follow in the chunk, and segs[k] records both (stage_pos = SPLIT_POS | k).
    // ovf_used = NULL: no overflow chunks (the tree is counted only and filled by the second pass)
    unsigned long long* ovf_used;
    uint64_t ovf_base, ovf_cap, ovf_chunk;
    struct StageSeg* segs;
    uint32_t* seg_n;
    uint32_t seg_cap;
    // the snapshot has no poisoned row: a subject set at remaining depth <= 1 is a leaf whatever its
    // row holds (engine.go:72-75; only a failing first page would make it an error), so its row is
    // not loaded
    uint32_t leaf_sets_blind;
    // entering a union, start the header loads of the subject sets in its window (the children it will
    // open) at once: global_load_lds into a per-wave scratch word (no register, no wait), so the
    // lines are in the caches when the walk reaches those children one after another
    uint32_t prefetch;
    // edges past the window read a 16-B block at a time (KETO_EXPAND_EDGE_BLOCKS=0: a word at a time)
    uint32_t edge_blocks;
    // tooling (KETO_EXPAND_CLOCKS=1): each root's walk time in wall-clock ticks (100 MHz), or NULL
    uint32_t* clocks;
    // expand on a migrating part: the handles of rows another part owns that a walk met without a
    // copy in the overlay (miss_cap entries, *n_miss recorded; the walk returns EXP_RETRY)
    uint32_t* miss = nullptr;
    uint32_t* n_miss = nullptr;
    uint32_t miss_cap = 0;
};
__device__ inline void record_miss(const ExpandOut& o, uint32_t h) {
    if (!o.n_miss) return;
    const uint32_t at = atomicAdd(o.n_miss, 1u);
    if (at < o.miss_cap) o.miss[at] = h;
}
// expand kernel modes: count the trees' nodes; write them at their offsets; write them to staging
constexpr int EXP_COUNT = 0, EXP_FILL = 1, EXP_STAGE = 2;
constexpr uint64_t NOT_STAGED = ~0ull;
constexpr uint64_t SPLIT_POS = 1ull << 62;     // stage_pos of a tree staged in two pieces: | its StageSeg
constexpr uint64_t NO_SPLIT = ~0ull;
// a staged tree in two pieces: nodes [0, split_at) at region, the rest at chunk (stage positions)
struct StageSeg {
    uint64_t region, chunk, split_at;
    uint32_t root, pad;
};
// a tree's overflow chunk while it is staged (expand_sm)
struct SplitState {
    uint64_t split_at = NO_SPLIT, chunk = 0;
    bool tried = false;
};

// cnt < cap: the node is written (cap = ~0 in a fill pass; a staged tree past its region is only
// counted, and filled again later)
__device__ inline void emit(keto_tree_node* out, uint64_t& cnt, bool fill, uint64_t cap, uint32_t subject, uint32_t info) {
    if (fill && cnt < cap) out[cnt] = keto_tree_node{subject, info};
    ++cnt;
}

// BuildTree for one root (engine.go:33-102).  root: row handle (root_flags bit0 = subject set) or
// a string id.  Set nodes are emitted with their row handle (the host maps handles to row ids).
template <bool FILL, class Stack, class VT>
__device__ int expand_one(const DevSnap& s, const DevOverlay& ov, uint32_t root, uint32_t root_flags,
                          uint32_t root_vid, int d, VT& V, keto_tree_node* out, uint64_t& cnt, uint64_t cap,
                          Stack& st, const ExpandOut& o, uint32_t& nr, uint64_t& qend, uint32_t* pf_lds) {
    if (!(root_flags & 1u)) {                               // SubjectID -> Leaf (:97-101)
        emit(out, cnt, FILL, cap, root, 0x80000000u);
        return EXP_TREE;
    }
    if (root == KETO_NO_ROW) return EXP_NIL;                // no tuples at all (:68-70)
    V.fresh();
    Work<false> nw;
    V.test_add(root_vid, nw);                               // :40-43 (root marked too)
    // the current frame lives in registers; a parent is saved on the stack only while it still
    // has edges (a child whose parent is exhausted returns straight to the grandparent)
    int sp = 0;
    Frame cur{0, 0, 0, 0};
    // the current frame's window: its first WINDOW_WORDS edge words, read with the header from the
    // same line (a main-arena row's header and window share one; the arena has slack at its end), so
    // the edges a row holds there cost no load of their own; wbeg = their first word (~0: none held,
    // e.g. after a pop)
    uint4 win = make_uint4(0, 0, 0, 0);
    uint64_t wbeg = ~0ull;
    // past the window, the current frame's edges are read a 16-B block at a time (rows are padded to
    // 16 B): one dependent load per four set edges instead of one per edge (ExpandOut::edge_blocks)
    uint4 blk = make_uint4(0, 0, 0, 0);
    uint64_t blk_at = ~0ull;
    // "open" a subject set at remaining depth k: NIL / ERROR / leaf written / union entered
    bool retry = false;
    auto open = [&](uint32_t h, int k) -> int {
        RowView rv;
        uint4 w4 = make_uint4(0, 0, 0, 0);
        // h names the set; hl is where its row is read: another part's row (a stub, migrating
        // partition) is read from its copy in the call's overlay, or recorded as missing
        uint32_t hl = h;
        for (int hop = 0;; ++hop) {
            if (hl >= ov.base) {
                rv = load_row(s, ov, hl);
            } else {
                uint64_t w = hword(hl, s.root_g);
                uint4 v = *reinterpret_cast<const uint4*>(s.arena + w);
                w4 = *reinterpret_cast<const uint4*>(s.arena + w + HDR_WORDS);
                while (v.z & HDR_FWD) {                     // a row a write moved (delta.cpp)
                    w = hword(v.x, s.root_g);
                    v = *reinterpret_cast<const uint4*>(s.arena + w);
                    w4 = *reinterpret_cast<const uint4*>(s.arena + w + HDR_WORDS);
                }
                rv.a = s.arena;
                rv.beg = w + HDR_WORDS;
                rv.n_sets = v.x;
                rv.n_ids = v.y;
                rv.seq = (v.z & HDR_SEQ) != 0;
                rv.hlog2 = (v.z >> 8) & 31u;
                rv.poison = (v.z & HDR_POISON) != 0;
                rv.poison0 = (v.z & HDR_POISON0) != 0;
                rv.closure = (v.z & HDR_CLOSURE) != 0;
                rv.remote = (v.z & HDR_REMOTE) != 0;
            }
            if (!rv.remote) break;
            const uint32_t to = rmap_find(ov, hl);
            if (to == NONE32 || to == hl || hop > 1) {
                record_miss(o, hl);
                return EXP_RETRY;
            }
            hl = to;
        }
        const uint32_t n_all = rv.n_sets + rv.n_ids;
        if (!rv.poison && n_all == 0) return EXP_NIL;
        if (rv.poison0) return EXP_ERROR;                   // the first page fails toInternal
        if (k <= 1) {                                       // :72-75
            emit(out, cnt, FILL, cap, EDGE_SET | h, 0x80000000u);
            return EXP_TREE;
        }
        if (rv.poison) return EXP_ERROR;                    // a later page fails
        if (cur.left > 0) {
            if (sp == st.cap()) return EXP_OVERFLOW;
            st[sp] = cur;
            ++sp;
        }
        emit(out, cnt, FILL, cap, EDGE_SET | h, n_all);
        cur = Frame{rv.beg, n_all, (uint16_t)k, (uint16_t)((rv.seq ? FR_SEQ : 0) | (rv.a != s.arena ? FR_OV : 0))};
        win = w4;
        wbeg = rv.a != s.arena ? ~0ull : rv.beg;
        blk_at = ~0ull;
        if (o.prefetch && wbeg != ~0ull && (k - 1 >= 2 || !o.leaf_sets_blind)) {
            // the window's subject sets (set edges always target main-arena rows)
#pragma unroll
            for (uint32_t j = 0; j < WINDOW_WORDS; ++j) {
                const uint32_t e = win_at(w4, j);
                if (j < n_all && (e & EDGE_SET))
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(s.arena + (uint64_t)(e & EDGE_VAL) * HDR_WORDS),
                                                     reinterpret_cast<void*>(pf_lds), 4, 0, 0);
            }
        }
        return EXP_TREE;
    };
    int r0 = open(root, d);
    if (r0 != EXP_TREE) return r0;
    for (;;) {
        if (cur.left == 0) {
            if (sp == 0) break;
            --sp;
            cur = st[sp];
            wbeg = ~0ull;
            blk_at = ~0ull;
            continue;
        }
        const uint32_t* const a = (cur.fl & FR_OV) ? ov.arena : s.arena;
        const uint64_t wo = cur.pos - wbeg;                 // (huge when no window is held)
        uint32_t e;
        if (wo < WINDOW_WORDS) {
            e = win_at(win, (uint32_t)wo);
        } else if (o.edge_blocks) {
            const uint64_t bw = cur.pos & ~3ull;
            if (bw != blk_at) {
                blk = *reinterpret_cast<const uint4*>(a + bw);
                blk_at = bw;
            }
            e = win_at(blk, (uint32_t)cur.pos & 3u);
        } else {
            e = a[cur.pos];
        }
        if (!(e & EDGE_SET) && !(cur.fl & FR_SEQ)) {
            // a normal row keeps its subject sets first: every edge left is a subject id, and each
            // is a leaf (:97-101) -- counted at once, copied in one pass
            if constexpr (FILL) {
                if (cnt + cur.left <= cap) {                // (a staged tree past its region: counted only)
                    bool queued = false;
                    if (cur.left > o.run_inline && o.runs) {
                        if (cur.left <= BIG_RUN && nr < RUNS_PER_LANE) {
                            o.runs[nr++] = CopyRun{a + cur.pos, out + cnt, cur.left};   // (o.runs: this lane's)
                            queued = true;
                        } else if (cur.left > BIG_RUN) {
                            // reserve the pieces only if all of them fit: a slot below the count
                            // is always written, so copy_big_runs never reads a stale entry
                            const uint32_t pieces = (cur.left + BIG_RUN - 1) / BIG_RUN;
                            uint32_t at = __hip_atomic_load(o.n_big, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            bool got = false;
                            while ((uint64_t)at + pieces <= o.big_cap) {
                                const uint32_t prev = atomicCAS(o.n_big, at, at + pieces);
                                if (prev == at) {
                                    got = true;
                                    break;
                                }
                                at = prev;
                            }
                            if (got) {
                                for (uint32_t k = 0; k < pieces; ++k)
                                    o.big[at + k] = CopyRun{a + cur.pos + (uint64_t)k * BIG_RUN, out + cnt + (uint64_t)k * BIG_RUN,
                                                            min(BIG_RUN, cur.left - k * BIG_RUN)};
                                queued = true;
                            }
                        }
                        if (queued) qend = max(qend, cnt + cur.left);   // (positions a later copy writes)
                    }
                    if (!queued) {
                        // eight loads in flight per round, then their stores
                        const uint32_t* src = a + cur.pos;
                        keto_tree_node* dst = out + cnt;
                        for (uint32_t i = 0; i < cur.left; i += 8) {
                            uint32_t v[8];
#pragma unroll
                            for (int j = 0; j < 8; ++j) v[j] = i + j < cur.left ? src[i + j] : 0u;
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (i + j < cur.left) dst[i + j] = keto_tree_node{v[j], 0x80000000u};
                        }
                    }
                }
            }
            cnt += cur.left;
            cur.left = 0;
            continue;
        }
        cur.pos++;
        cur.left--;
        if (!(e & EDGE_SET)) {
            emit(out, cnt, FILL, cap, e, 0x80000000u);     // subject id child -> Leaf
            continue;
        }
        const uint32_t c = e & EDGE_VAL;
        uint32_t vid = c;
        if (cur.fl & FR_SEQ) {
            uint32_t cv = coll_lookup(s, e);
            if (cv != NONE32) vid = cv;
        }
        const uint16_t k = cur.k - 1;
        int t = V.test_add(vid, nw);
        if (t == 2) return EXP_OVERFLOW;
        if (t == 1 || (k <= 1 && o.leaf_sets_blind)) {      // visited -> nil -> Leaf(set); or :72-75
            emit(out, cnt, FILL, cap, e, 0x80000000u);
            continue;
        }
        int r = open(c, k);
        if (r == EXP_RETRY) retry = true;                   // (a leaf for now: the walk goes on)
        if (r == EXP_NIL || r == EXP_RETRY) emit(out, cnt, FILL, cap, e, 0x80000000u);
        else if (r != EXP_TREE) return r;
    }
    return retry ? EXP_RETRY : EXP_TREE;
}

// The same walk as expand_one, restructured like the tier-0 check kernel (round 4): each loop
// iteration issues ONE global access per lane, from one place in the loop -- a subject set's header
// and window (with the forward followed on the next iteration), or the next 16-B block of the
// current row's edges -- and the walk in between needs no memory: window and block edges, visited
// tests in registers / LDS, node stores, queued id runs, and the saved frames in LDS.  expand_one
// waited on each lane's loads where they occurred, so a wave of 64 trees paid one round trip per
// load of any of its lanes.  Measured on config #5 it takes the same time (profiles/r04o_expand_sm.txt):
// a wave lives as long as its slowest lane's chain of dependent accesses -- 25 per wave at the
// median, 39 at most (KETO_EXPAND_CLOCKS counts them) -- at ~4 us each with 1.5 waves per SIMD, so
// the pass is that chain's latency, not where the waits sit.  Kept: no scratch, fewer waits.
// SmFrames selects it (tier 0, max-depth <= SM_FRAMES); the visited map gets SM_LDS_VIDS LDS
// entries per lane (config #5's trees mark at most 25 sets; 16 made 4.5 % of them probe HBM).
struct SmFrames {};
constexpr int SM_FRAMES = 8;
constexpr int SM_LDS_VIDS = 24;

template <bool FILL, int COLS, class VT>
__device__ int expand_sm(const DevSnap& s, const DevOverlay& ov, uint32_t root, uint32_t root_flags,
                         uint32_t root_vid, int d, VT& V, keto_tree_node*& out, uint64_t& cnt, uint64_t& cap,
                         uint4* frames, const ExpandOut& o, uint32_t& nr, uint64_t& qend, uint32_t* pf_lds,
                         uint32_t& iters, SplitState& sg) {
    // k more nodes past the staging region: go on in an overflow chunk (once per tree; out is then
    // based so that out + cnt is the chunk's first node)
    auto room = [&](uint64_t k) {
        if constexpr (FILL) {
            if (cnt + k > cap && o.ovf_used && !sg.tried) {
                sg.tried = true;
                const uint64_t at = atomicAdd(o.ovf_used, (unsigned long long)o.ovf_chunk);
                if (at + o.ovf_chunk <= o.ovf_cap && k <= o.ovf_chunk) {
                    sg.split_at = cnt;
                    sg.chunk = o.ovf_base + at;
                    out = reinterpret_cast<keto_tree_node*>(reinterpret_cast<uintptr_t>(o.stage + sg.chunk) -
                                                            cnt * sizeof(keto_tree_node));
                    cap = cnt + o.ovf_chunk;
                }
            }
        }
    };
    if (!(root_flags & 1u)) {                               // SubjectID -> Leaf (:97-101)
        room(1);
        emit(out, cnt, FILL, cap, root, 0x80000000u);
        return EXP_TREE;
    }
    if (root == KETO_NO_ROW) return EXP_NIL;                // no tuples at all (:68-70)
    V.fresh();
    Work<false> nw;
    V.test_add(root_vid, nw);                               // :40-43 (root marked too)
    int sp = 0;
    Frame cur{0, 0, 0, 0};
    uint4 win = make_uint4(0, 0, 0, 0), blk = make_uint4(0, 0, 0, 0);
    uint64_t wbeg = ~0ull, blk_at = ~0ull;
    // the pending open: identity handle oh (what its node names), the handle its header is read at
    // (ol: a forward moves it), remaining depth od, and its edge in the parent (oe; NONE32 = the root)
    bool opening = true, retry = false;
    uint32_t oh = root, ol = root, oe = NONE32;
    int od = d;
    for (;;) {
        ++iters;
        // ---- the iteration's access
        uint4 v = make_uint4(0, 0, 0, 0), w4 = make_uint4(0, 0, 0, 0);
        const bool in_ov = ol >= ov.base;
        const uint32_t* const ha = in_ov ? ov.arena : s.arena;
        const uint64_t hw = in_ov ? (uint64_t)(ol - ov.base) * HDR_WORDS : hword(ol, s.root_g);
        if (opening) {
            v = *reinterpret_cast<const uint4*>(ha + hw);
            if (!in_ov) w4 = *reinterpret_cast<const uint4*>(ha + hw + HDR_WORDS);   // (the arena has slack)
        } else {
            const uint32_t* const a = (cur.fl & FR_OV) ? ov.arena : s.arena;
            blk_at = cur.pos & ~3ull;                       // (rows are padded to 16 B)
            blk = *reinterpret_cast<const uint4*>(a + blk_at);
        }
        if (opening) {
            if (v.z & HDR_FWD) {                            // a row a write moved (delta.cpp)
                ol = v.x;
                continue;
            }
            if (v.z & HDR_REMOTE) {                         // another part's row (migrating partition)
                const uint32_t to = rmap_find(ov, ol);
                if (to != NONE32 && to != ol) {             // its copy in the call's overlay
                    ol = to;
                    continue;
                }
                // no copy yet: recorded, and the walk goes on past it (a leaf for now) to find the
                // tree's other missing rows in this round; the tree is counted again next round
                record_miss(o, ol);
                if (oe == NONE32) return EXP_RETRY;
                retry = true;
                opening = false;
                room(1);
                emit(out, cnt, FILL, cap, oe, 0x80000000u);
                goto walk;
            }
            opening = false;
            const uint32_t n_all = v.x + v.y;
            const bool poison = (v.z & HDR_POISON) != 0, poison0 = (v.z & HDR_POISON0) != 0;
            if (!poison && n_all == 0) {                    // nil (:68-70)
                if (oe == NONE32) return EXP_NIL;
                room(1);
                emit(out, cnt, FILL, cap, oe, 0x80000000u);     // a nil child -> Leaf(set)
            } else if (poison0) {
                return EXP_ERROR;                           // the first page fails toInternal
            } else if (od <= 1) {                           // :72-75
                room(1);
                emit(out, cnt, FILL, cap, EDGE_SET | oh, 0x80000000u);
            } else if (poison) {
                return EXP_ERROR;                           // a later page fails
            } else {                                        // a union: enter it
                if (cur.left > 0) {
                    if (sp == SM_FRAMES) return EXP_OVERFLOW;
                    frames[sp * COLS] = make_uint4((uint32_t)cur.pos, (uint32_t)(cur.pos >> 32), cur.left,
                                                         (uint32_t)cur.k | ((uint32_t)cur.fl << 16));
                    ++sp;
                }
                room(1);
                emit(out, cnt, FILL, cap, EDGE_SET | oh, n_all);
                const uint64_t beg = hw + HDR_WORDS;
                cur = Frame{beg, n_all, (uint16_t)od, (uint16_t)(((v.z & HDR_SEQ) ? FR_SEQ : 0) | (in_ov ? FR_OV : 0))};
                win = w4;
                wbeg = in_ov ? ~0ull : beg;
                blk_at = ~0ull;
                if (o.prefetch && !in_ov && (od - 1 >= 2 || !o.leaf_sets_blind)) {
                    // the window's subject sets: their header lines start loading now (no register)
#pragma unroll
                    for (uint32_t j = 0; j < WINDOW_WORDS; ++j) {
                        const uint32_t e = win_at(w4, j);
                        if (j < n_all && (e & EDGE_SET))
                            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(s.arena + (uint64_t)(e & EDGE_VAL) * HDR_WORDS),
                                                             reinterpret_cast<void*>(pf_lds), 4, 0, 0);
                    }
                }
            }
        }
        // ---- walk until the next access is needed
    walk:
        for (;;) {
            if (cur.left == 0) {
                if (sp == 0) return retry ? EXP_RETRY : EXP_TREE;
                --sp;
                const uint4 f = frames[sp * COLS];
                cur = Frame{(uint64_t)f.x | ((uint64_t)f.y << 32), f.z, (uint16_t)(f.w & 0xFFFFu), (uint16_t)(f.w >> 16)};
                wbeg = ~0ull;
                blk_at = ~0ull;
                continue;
            }
            const uint64_t wo = cur.pos - wbeg;             // (huge when no window is held)
            uint32_t e;
            if (wo < WINDOW_WORDS) e = win_at(win, (uint32_t)wo);
            else if ((cur.pos & ~3ull) == blk_at) e = win_at(blk, (uint32_t)cur.pos & 3u);
            else break;                                     // next: this edge's block
            const uint32_t* const a = (cur.fl & FR_OV) ? ov.arena : s.arena;
            if (!(e & EDGE_SET) && !(cur.fl & FR_SEQ)) {
                // the rest of a normal row are subject ids, all leaves: queued (or copied) at once
                if constexpr (FILL) {
                    room(cur.left);
                    if (cnt + cur.left <= cap) {
                        bool queued = false;
                        if (cur.left > o.run_inline && o.runs) {
                            if (cur.left <= BIG_RUN && nr < RUNS_PER_LANE) {
                                o.runs[nr++] = CopyRun{a + cur.pos, out + cnt, cur.left};
                                queued = true;
                            } else if (cur.left > BIG_RUN) {
                                const uint32_t pieces = (cur.left + BIG_RUN - 1) / BIG_RUN;
                                uint32_t at = __hip_atomic_load(o.n_big, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                bool got = false;
                                while ((uint64_t)at + pieces <= o.big_cap) {
                                    const uint32_t prev = atomicCAS(o.n_big, at, at + pieces);
                                    if (prev == at) {
                                        got = true;
                                        break;
                                    }
                                    at = prev;
                                }
                                if (got) {
                                    for (uint32_t k = 0; k < pieces; ++k)
                                        o.big[at + k] = CopyRun{a + cur.pos + (uint64_t)k * BIG_RUN, out + cnt + (uint64_t)k * BIG_RUN,
                                                                min(BIG_RUN, cur.left - k * BIG_RUN)};
                                    queued = true;
                                }
                            }
                            if (queued) qend = max(qend, cnt + cur.left);
                        }
                        if (!queued) {
                            const uint32_t* src = a + cur.pos;
                            keto_tree_node* dst = out + cnt;
                            for (uint32_t i = 0; i < cur.left; i += 8) {
                                uint32_t x[8];
#pragma unroll
                                for (int j = 0; j < 8; ++j) x[j] = i + j < cur.left ? src[i + j] : 0u;
#pragma unroll
                                for (int j = 0; j < 8; ++j)
                                    if (i + j < cur.left) dst[i + j] = keto_tree_node{x[j], 0x80000000u};
                            }
                        }
                    }
                }
                cnt += cur.left;
                cur.left = 0;
                continue;
            }
            cur.pos++;
            cur.left--;
            if (!(e & EDGE_SET)) {
                room(1);
                emit(out, cnt, FILL, cap, e, 0x80000000u);     // subject id child -> Leaf
                continue;
            }
            const uint32_t c = e & EDGE_VAL;
            uint32_t vid = c;
            if (cur.fl & FR_SEQ) {
                const uint32_t cv = coll_lookup(s, e);
                if (cv != NONE32) vid = cv;
            }
            const int k = (int)cur.k - 1;
            const int t = V.test_add(vid, nw);
            if (t == 2) return EXP_OVERFLOW;
            if (t == 1 || (k <= 1 && o.leaf_sets_blind)) {  // visited -> nil -> Leaf(set); or :72-75
                room(1);
                emit(out, cnt, FILL, cap, e, 0x80000000u);
                continue;
            }
            opening = true;                                 // next: the child's header
            oh = ol = c;
            oe = e;
            od = k;
            break;
        }
    }
}

struct ExpandReq {
    uint32_t root;
    uint32_t flags;
    uint32_t vid;
    int32_t depth;
};

// SPREAD > 1 (tier 0 of expand_sm, KETO_EXPAND_SPREAD): only 64 / SPREAD lanes of each wave walk a
// tree, the rest exit at once, and the block's LDS columns are its active lanes' (256 / SPREAD): a
// wave's instruction stream is the union of fewer lanes' paths, and with less LDS per block more
// waves are resident to interleave their issue
template <int MODE, class Stack, int SPREAD = 1>
__global__ void __launch_bounds__(256) expand_kernel(DevSnap s, DevOverlay ov, const ExpandReq* __restrict__ q,
                                                     uint32_t n, int gmd, ExpandOut o, TierArgs ta) {
    constexpr bool FILL = MODE != EXP_COUNT, STAGE = MODE == EXP_STAGE;
    constexpr bool SM = std::is_same<Stack, SmFrames>::value;  // expand_sm (saved frames in LDS)
    constexpr int LV = SM ? SM_LDS_VIDS : LDS_VIDS;
    constexpr int ACT = 64 / SPREAD, COLS = 256 / SPREAD;     // active lanes per wave, per block
    static_assert(SPREAD == 1 || SM, "spread lanes: expand_sm only");
    if (SPREAD > 1 && (threadIdx.x & 63u) >= (uint32_t)ACT) return;
    const uint32_t col = SPREAD > 1 ? (threadIdx.x >> 6) * ACT + (threadIdx.x & 63u) : threadIdx.x;
    const uint32_t slot = blockIdx.x * COLS + col;
    const uint32_t stride = gridDim.x * COLS;
    // a tree's map: its first REG_VIDS + LV sets in registers and the lane's LDS column (one
    // tree at max-depth 5 marks a handful of sets), the rest in the lane's HBM table
    __shared__ uint32_t lds_vis[(LV > 0 ? LV : 1) * COLS];
    __shared__ uint32_t lds_pf[256];                          // the waves' prefetch scratch (never read)
    __shared__ uint4 lds_fr[SM ? SM_FRAMES * COLS : 1];       // SM: the lane's saved frames
    VisitedRS<LV, Visited, REG_VIDS, COLS> V;
    V.fresh();
    V.lds = LV > 0 ? lds_vis + col : nullptr;
    V.V.tab = ta.vtab + (uint64_t)slot * (ta.mask + 1u);
    V.V.mask = ta.mask;
    V.V.epoch = ta.slot_epoch[slot];
    V.V.count = 0;
    typename std::conditional<SM, LocalStack<1>, Stack>::type st;
    if constexpr (std::is_same<Stack, GlobalStack>::value) {
        st.f = ta.gstack + (uint64_t)slot * ta.gstack_n;
        st.n = ta.gstack_n;
    }
    const uint32_t total = ta.in_list ? *ta.in_count : n;
    const uint64_t stage0 = (uint64_t)slot * o.stage_cap;    // STAGE: this lane's region
    uint64_t used = 0;
    uint32_t nr = 0;                                          // this lane's queued runs
    if (FILL && o.runs) o.runs += (uint64_t)slot * RUNS_PER_LANE;
    for (uint32_t j = slot; j < total; j += stride) {
        const uint32_t i = ta.in_list ? ta.in_list[j] : j;
        // nil / error roots own no output; a staged tree is already written
        if (MODE == EXP_FILL && (o.status[i] != EXP_TREE || (o.stage_pos && o.stage_pos[i] != NOT_STAGED))) continue;
        const ExpandReq rq = q[i];
        int d = rq.depth;
        if (d <= 0 || gmd < d) d = gmd;
        uint64_t cnt = 0;
        keto_tree_node* out = !FILL ? nullptr : STAGE ? o.stage + stage0 + used : o.nodes + o.offset[i];
        uint64_t cap = STAGE ? o.stage_cap - used : ~0ull;
        SplitState sg;
        uint64_t qend = 0;
        const uint64_t t_tree = o.clocks ? wall_clock64() : 0;
        int r;
        uint32_t iters = 0;
        if constexpr (SM)
            r = expand_sm<FILL, COLS>(s, ov, rq.root, rq.flags, rq.vid, d, V, out, cnt, cap, lds_fr + col, o, nr, qend,
                                lds_pf + (threadIdx.x & ~63u), iters, sg);
        else
            r = expand_one<FILL>(s, ov, rq.root, rq.flags, rq.vid, d, V, out, cnt, cap, st, o, nr, qend,
                                 lds_pf + (threadIdx.x & ~63u));
        if (o.clocks) {
            o.clocks[i] = (uint32_t)(wall_clock64() - t_tree);
            o.clocks[n + i] = iters;                       // (expand_sm: its accesses)
        }
        const bool staged = STAGE && r == EXP_TREE && cnt <= cap;
        const bool split = sg.split_at != NO_SPLIT;
        // a tree not staged (too big, or left to the next tier) may have queued runs into the region:
        // that part stays dead, so the copies cannot land on the next tree (a split tree wrote the
        // region below its split only)
        if (STAGE && !staged) used += split ? sg.split_at : qend;
        if (r == EXP_OVERFLOW) {
            uint32_t at = atomicAdd(ta.out_count, 1u);
            ta.out_list[at] = i;
        } else if (MODE != EXP_FILL) {
            o.count[i] = r == EXP_TREE ? cnt : 0;
            o.status[i] = (uint8_t)r;
            if (staged && split) {
                const uint32_t k = atomicAdd(o.seg_n, 1u);
                // (one record per chunk taken, so k < seg_cap; a full list leaves the tree to pass 2)
                o.stage_pos[i] = k < o.seg_cap ? SPLIT_POS | k : NOT_STAGED;
                if (k < o.seg_cap) o.segs[k] = StageSeg{stage0 + used, sg.chunk, sg.split_at, i, 0u};
                used += sg.split_at;
            } else if (staged) {
                o.stage_pos[i] = stage0 + used;
                used += cnt;
            }
        }
    }
    if (FILL && o.runs) o.lane_runs[slot] = nr;
    ta.slot_epoch[slot] = V.V.epoch;
}

// The staged trees of the one-pass expand, copied to their offsets in the node arena: 16 lanes per
// root (four roots per wave, grid-stride), whose position and offsets are loaded together (a tree
// is ~37 nodes on average: a wave per root waited three dependent loads for one short copy).
// unit_row != NULL: set nodes' row handles become row ids on the way (handles_to_rows_direct's
// translation, fused: the translated staged trees need no pass of their own)
__global__ void __launch_bounds__(256) gather_staged(keto_tree_node* __restrict__ nodes,
                                                     const keto_tree_node* __restrict__ stage,
                                                     const uint64_t* __restrict__ stage_pos,
                                                     const uint64_t* __restrict__ offset, uint32_t n,
                                                     const uint32_t* __restrict__ unit_row, uint32_t ov_units_base,
                                                     uint64_t big) {
    const uint32_t gl = threadIdx.x & 15u;
    const uint32_t groups = gridDim.x * (blockDim.x >> 4);
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; i < n; i += groups) {
        const uint64_t sp = stage_pos[i], b = offset[i], e = offset[i + 1];
        // not staged, in two pieces, or bigger than `big` nodes: copy_stage_pieces, a wave per piece
        if (sp >= SPLIT_POS || e - b > big) continue;
        for (uint64_t k = gl; k < e - b; k += 16) {
            keto_tree_node v = stage[sp + k];
            if (unit_row && (v.subject & EDGE_SET) && (v.subject & EDGE_VAL) < ov_units_base)
                v.subject = EDGE_SET | unit_row[v.subject & EDGE_VAL];
            nodes[b + k] = v;
        }
    }
}

// The staged trees in two pieces (StageSeg), and the single-piece ones past the gather's size bound:
// each piece of at most GPIECE (512) nodes {source in the staging
// pool, destination in the node arena, length} copied by one wave, set handles turned into row ids on
// the way as in gather_staged (unit_row != NULL)
__global__ void __launch_bounds__(256) copy_stage_pieces(keto_tree_node* __restrict__ nodes,
                                                         const keto_tree_node* __restrict__ stage,
                                                         const uint64_t* __restrict__ pieces, uint32_t n_pieces,
                                                         const uint32_t* __restrict__ unit_row, uint32_t ov_units_base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < n_pieces; w += waves) {
        const uint64_t src = pieces[3 * w], dst = pieces[3 * w + 1], len = pieces[3 * w + 2];
        for (uint64_t k = lane; k < len; k += 64) {
            keto_tree_node v = stage[src + k];
            if (unit_row && (v.subject & EDGE_SET) && (v.subject & EDGE_VAL) < ov_units_base)
                v.subject = EDGE_SET | unit_row[v.subject & EDGE_VAL];
            nodes[dst + k] = v;
        }
    }
}

// The queued id runs of a fill pass.  A run queued twice (a root that overflowed a tier and was
// filled again on the next) is copied twice, to the same bytes.
//   copy_lane_runs: half a wave per tier-0 lane (one queue entry per thread: RUNS_PER_LANE = 32);
//     its runs' ids are laid end to end and the half-wave copies 32 of them per round (thread k:
//     flat position base + k, its run found by a search over the runs' exclusive prefix, read
//     across the half-wave)
//   copy_big_runs: a wave per BIG_RUN-id piece
static_assert(RUNS_PER_LANE == 32, "copy_lane_runs holds one queue entry per thread of a half-wave");
__global__ void __launch_bounds__(256) copy_lane_runs(const CopyRun* __restrict__ runs,
                                                      const uint32_t* __restrict__ lane_runs, uint32_t lanes) {
    constexpr int G = 32;
    const int t = (int)(threadIdx.x & (G - 1));
    const uint32_t groups = gridDim.x * (blockDim.x / G);
    for (uint32_t l = (blockIdx.x * blockDim.x + threadIdx.x) / G; l < lanes; l += groups) {
        const uint32_t m = lane_runs[l];
        if (m == 0) continue;
        CopyRun c{nullptr, nullptr, 0};
        if ((uint32_t)t < m) c = runs[(uint64_t)l * RUNS_PER_LANE + t];
        const uint32_t len = (uint32_t)t < m ? (uint32_t)c.len : 0u;
        uint32_t incl = len;
        for (int off = 1; off < G; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, G);
            if (t >= off) incl += y;
        }
        const uint32_t total = __shfl(incl, G - 1, G);
        const uint32_t excl = incl - len;
        const uint64_t src = (uint64_t)c.src, dst = (uint64_t)c.dst;
        // U ids per thread per round, their loads in flight together (a lane's runs of up to 32K ids
        // are copied in rounds of U x 32, not 32)
        constexpr int U = 4;
        for (uint32_t base = 0; base < total; base += U * G) {  // every thread takes part in the shuffles
            uint32_t val[U];
            keto_tree_node* dps[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t f = base + (uint32_t)(u * G + t);
                int j = 0;
                for (int step = G / 2; step > 0; step >>= 1) {
                    const uint32_t ev = __shfl(excl, j + step < G ? j + step : G - 1, G);
                    if ((uint32_t)(j + step) < m && ev <= f) j += step;
                }
                const uint32_t ej = __shfl(excl, j, G);
                const uint32_t slo = __shfl((uint32_t)src, j, G), shi = __shfl((uint32_t)(src >> 32), j, G);
                const uint32_t dlo = __shfl((uint32_t)dst, j, G), dhi = __shfl((uint32_t)(dst >> 32), j, G);
                dps[u] = nullptr;
                val[u] = 0;
                if (f < total) {
                    const uint32_t* sp = reinterpret_cast<const uint32_t*>(((uint64_t)shi << 32) | slo);
                    dps[u] = reinterpret_cast<keto_tree_node*>(((uint64_t)dhi << 32) | dlo) + (f - ej);
                    val[u] = sp[f - ej];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (dps[u]) *dps[u] = keto_tree_node{val[u], 0x80000000u};
        }
    }
}
__global__ void __launch_bounds__(256) copy_big_runs(const CopyRun* __restrict__ runs, const uint32_t* __restrict__ n_runs,
                                                     uint32_t cap) {
    const uint32_t n = min(*n_runs, cap);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += waves) {
        const CopyRun c = runs[r];
        uint64_t i = lane;
        for (; i + 192 < c.len; i += 256) {                  // four loads in flight per lane
            const uint32_t v0 = c.src[i], v1 = c.src[i + 64], v2 = c.src[i + 128], v3 = c.src[i + 192];
            c.dst[i] = keto_tree_node{v0, 0x80000000u};
            c.dst[i + 64] = keto_tree_node{v1, 0x80000000u};
            c.dst[i + 128] = keto_tree_node{v2, 0x80000000u};
            c.dst[i + 192] = keto_tree_node{v3, 0x80000000u};
        }
        for (; i < c.len; i += 64) c.dst[i] = keto_tree_node{c.src[i], 0x80000000u};
    }
}

// ------------------------------------------------------------------ host side
struct Tier {
    uint32_t n_slots = 0;
    uint32_t cap = 0;             // visited entries per slot (power of two)
    int gstack_n = 0;             // 0 = local stack
    uint64_t* vtab = nullptr;
    uint32_t* slot_epoch = nullptr;
    Frame* gstack = nullptr;
};

// The workspaces one check in flight uses: visited tables and frames per tier, overflow lists, tier
// counters, dynamic-run heads, borrowed-table bitmaps.  The pipelined host path keeps two, so the
// checks of consecutive chunks can overlap on two compute streams (one's tail, the other's start).
struct WorkSet {
    Tier tiers[3];
    uint32_t* lists = nullptr;    // 2 overflow lists, capacity list_cap each
    uint64_t list_cap = 0;
    uint32_t* counters = nullptr; // [0..3] tiers (cleared per batch), [4] misrouted
    uint32_t* heads = nullptr;    // tier-0 run heads (8 XCDs x up to 16 heads x 128 B)
    uint32_t* pool_busy = nullptr; // borrowed-table bitmaps: tier 2's tables (8 words), tier 1's
    uint64_t pool_words = 0;
};

// streams (and workspaces) of the packed batches checked without a host round trip: two checks of
// ~65K requests (a few hundred waves each, latency-bound) run side by side
constexpr int ASYNC_STREAMS = 2;

struct DeviceState {
    int device = 0;
    uint32_t* arena = nullptr;
    uint64_t arena_words = 0;     // allocated (the tail beyond S.n_units holds rows writes move)
    uint64_t* coll = nullptr;
    uint32_t coll_mask = 0;
    uint64_t bytes = 0;
    uint32_t vid_bound = 0;       // distinct visit ids that can exist (rows + collision classes)
    uint32_t n_units = 0;         // main-arena handles are < n_units
    uint32_t n_coll = 0;          // collision classes
    std::mutex mu;                // one batch at a time per snapshot (workspaces are shared)
    WorkSet ws[2 + ASYNC_STREAMS];   // check workspaces (ws[1]: the second compute stream of the pipeline;
                                     // ws[2 + k]: packed batches checked without a host round trip, astream[k])
    WorkSet ews;                  // expand workspaces
    uint32_t v1_lanes[16] = {};   // resident lanes of the tier-0 check kernel, per variant
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;    // the pipeline's second compute stream (ws[1])
    hipStream_t astream[ASYNC_STREAMS] = {};   // device_check_rows_async: the checks, dealt in turn (ws[2 + k])
    uint32_t amax[ASYNC_STREAMS] = {};         // the largest batch each has checked (its workspace's size)
    uint32_t anext = 0;
    hipEvent_t ev[6] = {};
    keto_batch_timing last{};
    uint32_t* row_handle = nullptr;   // row id -> handle (NO_UNIT: another part's root row), lazily
    uint32_t* layout_units = nullptr; // handles in arena order (increasing) and their rows, lazily:
    uint32_t* rows_by_unit = nullptr; //   expand output handle -> row id on the device
    uint32_t* unit_row = nullptr;     // handle -> row id, direct (handles below min(n_units, 2^31); lazily)
    uint64_t row_handle_cap = 0;      // entries allocated (a write patches the maps in place while its rows fit)
    uint64_t row_handle_rows = 0;     // entries written (rows below it hold their handle or NO_UNIT)
    uint64_t unit_row_cap = 0;
    // the closure rows of the last write (device_apply): the rows with a filter and subject sets
    // (closure_pass) and every row with a filter (sig_pass), kept while a write changes neither set
    uint32_t* cl_list = nullptr;
    uint32_t* cl_all = nullptr;
    uint32_t* cl_changed = nullptr;
    uint64_t cl_list_n = 0, cl_all_n = 0, cl_list_cap = 0, cl_all_cap = 0;
    std::vector<uint8_t> cl_in;       // per row: in cl_list
    bool cl_valid = false;
    void* ex_buf = nullptr;           // expand workspace (requests, counts, statuses, offsets)
    uint64_t ex_cap = 0;
    keto_tree_node* ex_nodes = nullptr;
    uint64_t ex_nodes_cap = 0;
    CopyRun* ex_runs = nullptr;       // the fill pass's queued id runs | their count (last 8 B)
    uint32_t ex_runs_cap = 0;
    CopyRun* ex_big = nullptr;        // pieces of long id runs | their count (last 8 B)
    uint32_t ex_big_cap = 0;
    keto_tree_node* ex_stage = nullptr;   // one-pass expand: the lanes' staging regions | overflow chunks
    uint64_t ex_stage_nodes = 0;
    uint8_t* ex_seg = nullptr;        // overflow chunks taken (8 B) | split trees (4 B + pad) | StageSeg list
    uint32_t ex_seg_cap = 0;
    uint64_t* ex_pieces = nullptr;    // copy_stage_pieces' {source, destination, length} triples
    uint64_t ex_pieces_cap = 0;
    hipEvent_t ex_ev[4] = {};         // copy_runs / gather timing (added to tier 0 of the batch timing)
    uint8_t* ap_buf = nullptr;        // a write's row images and their places, uploaded at once
    uint64_t ap_cap = 0;
    keto_check_ids* xlate = nullptr;  // requests translated from row ids to handles
    uint64_t xlate_cap = 0;
    // host-buffer calls (device_check_host): a pipeline of chunks over two device slots, H2D on
    // copy_in, the check on `stream`, D2H on copy_out; pinned staging when the caller's buffers
    // are pageable.  Kept across calls (no per-call allocation).
    hipStream_t copy_in = nullptr, copy_out = nullptr;
    keto_check_ids* slot_q[2] = {};   // raw requests of a chunk (handles or row ids)
    keto_check_ids* slot_x[2] = {};   // translated requests (row-id form)
    uint8_t* slot_a[2] = {};          // decisions of a chunk
    uint64_t slot_cap = 0;
    keto_check_ids* pin_q[2] = {};    // pinned staging (pageable callers)
    uint8_t* pin_a[2] = {};
    uint64_t pin_cap = 0;
    hipEvent_t pev[8] = {};           // pipeline events: in_done[2], kern_done[2], out_done[2]
    keto_check_ids* ps_q = nullptr;   // pipeline stash of tier-1 overflows (PipeStash), kept across calls
    uint32_t* ps_idx = nullptr;
    uint32_t* ps_count = nullptr;     // [0] stashed, [1] tier-1 requests
    uint64_t ps_cap = 0;
    std::vector<hipEvent_t> ps_ev;    // per chunk: 3 timing events
    // streamed host batches (device_check_stream): the whole batch's pairs, its chunks' ready words,
    // its decisions and the handle form of the requests tier 0 hands up
    keto_check_pair* st_pairs = nullptr;
    uint8_t* st_dec = nullptr;
    keto_check_ids* st_x = nullptr;
    uint32_t* st_ready = nullptr;
    uint64_t st_cap = 0;

    uint32_t root_g = 0;          // wide arenas (snapshot.hpp hword)
    DevSnap view() const { return DevSnap{arena, coll, coll_mask, n_units, root_g}; }
};

namespace {

template <class T>
T* dmalloc(uint64_t n, uint64_t& acc) {
    void* p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    acc += n * sizeof(T);
    // KETO_DEBUG_FILL=<u32>: every fresh allocation starts as that word (tests pick a plausible handle),
    // so a read of memory nothing wrote gives the same wrong answer on every run instead of by chance
    if (const char* f = getenv("KETO_DEBUG_FILL"); f && *f) {
        const uint64_t words = n * sizeof(T) / 4;
        if (words) HIP_OK(hipMemsetD32((hipDeviceptr_t)p, (int)strtoul(f, nullptr, 0), words));
        HIP_OK(hipDeviceSynchronize());
    }
    return (T*)p;
}

// a device buffer freed at scope exit
template <class T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(uint64_t n) {
        uint64_t acc = 0;
        p = dmalloc<T>(n, acc);
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

uint32_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return (uint32_t)std::min<uint64_t>(p, 1ull << 31);
}

void free_tier(Tier& t) {
    if (t.vtab) (void)hipFree(t.vtab);
    if (t.slot_epoch) (void)hipFree(t.slot_epoch);
    if (t.gstack) (void)hipFree(t.gstack);
    t = Tier{};
}

void ensure_tier(Tier* set, int level, uint32_t n_slots, uint32_t cap, int gstack_n) {
    Tier& t = set[level];
    // a workspace with at least as many slots of the same shape is reused (kernels index slots only
    // below their grid size), so batches of changing sizes do not reallocate
    if (t.n_slots >= n_slots && t.cap == cap && t.gstack_n == gstack_n && t.vtab) return;
    free_tier(t);
    uint64_t acc = 0;
    t.n_slots = n_slots;
    t.cap = cap;
    t.gstack_n = gstack_n;
    t.vtab = dmalloc<uint64_t>((uint64_t)n_slots * cap, acc);
    HIP_OK(hipMemset(t.vtab, 0, (uint64_t)n_slots * cap * sizeof(uint64_t)));
    t.slot_epoch = dmalloc<uint32_t>(n_slots, acc);
    std::vector<uint32_t> ones(n_slots, 1u);
    HIP_OK(hipMemcpy(t.slot_epoch, ones.data(), n_slots * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (gstack_n) t.gstack = dmalloc<Frame>((uint64_t)n_slots * gstack_n, acc);
}

void ensure_lists(WorkSet& W, uint64_t n) {
    if (W.list_cap >= n && W.lists) return;
    if (W.lists) (void)hipFree(W.lists);
    uint64_t acc = 0;
    if (!W.counters) W.counters = dmalloc<uint32_t>(8, acc);   // [0..3] tiers (cleared per batch), [4] misrouted
    W.list_cap = std::max<uint64_t>(n, 1024);
    W.lists = dmalloc<uint32_t>(2 * W.list_cap, acc);
}

int hw_slots() {
    // persistent grid sized to residency: 256 CUs x 28 waves (7 per SIMD at the kernel's register
    // budget) x 64 lanes; every lane owns one visited table.  KETO_SLOTS overrides (tuning, tests;
    // read on every batch).
    const char* e = getenv("KETO_SLOTS");
    int s = e ? atoi(e) : 256 * 28 * 64;
    s = (s + 255) / 256 * 256;
    return s < 256 ? 256 : s;
}

TierArgs tier_args(Tier& t, const uint32_t* in_list, const uint32_t* in_count, uint32_t* out_list,
                   uint32_t* out_count) {
    TierArgs a;
    a.vtab = t.vtab;
    a.mask = t.cap - 1;
    a.slot_epoch = t.slot_epoch;
    a.gstack = t.gstack;
    a.gstack_n = t.gstack_n;
    a.pool = nullptr;
    a.heads = nullptr;
    a.dyn = 0;
    a.walk_cap = 0xFFFFFFFFu;
    a.steps = nullptr;
    a.items = 0;
    a.item_owner = nullptr;
    a.item_acc = nullptr;
    a.next = nullptr;
    a.pool_mask = 0;
    a.pool_n = 0;
    a.pool_epoch = nullptr;
    a.pool_busy = nullptr;
    a.in_list = in_list;
    a.in_count = in_count;
    a.out_list = out_list;
    a.out_count = out_count;
    a.pairs = nullptr;
    a.ready = nullptr;
    a.chunk_log2 = 0;
    a.row_handle = nullptr;
    a.n_rows = 0;
    a.pair_depth = 0;
    a.misrouted = nullptr;
    a.stalled = nullptr;
    a.wait_ticks = 0;
    return a;
}

template <class F>
void host_parallel_for(uint64_t n, F f) {
    unsigned th = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 100000) th = 1;
    std::vector<std::thread> ts;
    const uint64_t chunk = (n + th - 1) / th;
    for (unsigned t = 0; t < th; ++t)
        ts.emplace_back([&, t] {
            uint64_t b = t * chunk, e = std::min(n, b + chunk);
            for (uint64_t i = b; i < e; ++i) f(i);
        });
    for (auto& x : ts) x.join();
}

// Write one row (table, closure filter seed, header, edges) into an arena at its handle.  The
// closure filter starts as the row's own ids (all bits for a ROW_SEQ row); closure_pass adds the
// closures of its subject sets on the device, then sig_pass its child signatures.
void put_row(uint32_t* arena, uint64_t hdr_word, const RowRec& rec, uint32_t pp, uint32_t hlog2, const uint32_t* edges,
             uint64_t n_stored, const std::vector<uint32_t>& unit_of_row, bool closure, uint64_t base = 0) {
    // `arena` holds the arena's words from `base` on
    uint64_t h = hdr_word - base;
    const bool seq = ((rec.hi_flags >> 8) & ROW_SEQ) != 0;
    arena[h + 0] = rec.n_sets;
    arena[h + 1] = rec.n_ids;
    uint32_t w2 = (seq ? HDR_SEQ : 0u) | (pp != NO_PAGE ? HDR_POISON : 0u) | (pp == 0 ? HDR_POISON0 : 0u) |
                  (closure ? HDR_CLOSURE : 0u) | (hlog2 << 8);
    if (closure) {
        uint32_t* cf = arena + h - CB_WORDS;
        for (uint32_t i = 0; i < CF_WORDS; ++i) cf[i] = seq ? NONE32 : 0u;
        for (uint32_t i = CF_WORDS; i < CB_WORDS; ++i) cf[i] = NONE32;   // signatures: sig_pass
        if (!seq)
            for (uint64_t i = 0; i < n_stored; ++i) {
                const uint32_t v = edges[i];
                if (v & EDGE_SET) continue;                     // subject sets: closure_pass
                if (v == EDGE_POISON) continue;
                uint32_t wd, bit;
                closure_bit(v, wd, bit);
                cf[wd] |= 1u << bit;
            }
    }
    uint32_t w3 = 0;
    if (hlog2) {
        for (uint32_t k = 0; k < rec.n_ids; ++k) {
            uint32_t b[2];
            bloom_bits(edges[rec.n_sets + k], b[0], b[1]);
            for (uint32_t x : b) {
                if (x < 32) w3 |= 1u << x;
                else w2 |= 1u << (x - 32 + 13);
            }
        }
    }
    arena[h + 2] = w2;
    arena[h + 3] = w3;
    uint32_t* e = arena + h + HDR_WORDS;
    for (uint64_t i = 0; i < n_stored; ++i) {
        uint32_t v = edges[i];
        if ((v & EDGE_SET) && v != EDGE_POISON) v = EDGE_SET | unit_of_row[v & EDGE_VAL];
        e[i] = v;
    }
    for (uint64_t i = n_stored; i < ((n_stored + 3) & ~3ull); ++i) e[i] = NONE32;
    if (hlog2) {
        const uint32_t nb = (1u << hlog2) / BUCKET_WORDS;
        uint32_t* tab = arena + h - (closure ? CB_WORDS : 0u) - (1ull << hlog2);
        for (uint32_t i = 0; i < (1u << hlog2); ++i) tab[i] = NONE32;
        for (uint32_t k = 0; k < rec.n_ids; ++k) {
            const uint32_t id = edges[rec.n_sets + k];
            for (uint32_t b = mix32(id) & (nb - 1);; b = (b + 1) & (nb - 1)) {
                uint32_t* q = tab + (uint64_t)b * BUCKET_WORDS;
                uint32_t i = 0;
                while (i < BUCKET_WORDS && q[i] != NONE32 && q[i] != id) ++i;
                if (i < BUCKET_WORDS) {
                    q[i] = id;
                    break;
                }
            }
        }
    }
}

// One round of closure propagation: each listed row ORs the closure filters of its subject sets
// into its own.  Filters only gain bits that are in the true closures, so rounds may overlap with
// one another's writes (reads of a half-updated filter are still subsets); a round that changes
// nothing means every filter is closed.  One lane per row.
__global__ void __launch_bounds__(256) closure_pass(uint32_t* __restrict__ arena, const uint32_t* __restrict__ rows,
                                                   uint32_t n, uint32_t* __restrict__ changed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = (uint64_t)rows[i] * HDR_WORDS;
    uint2* const cf = reinterpret_cast<uint2*>(arena + h - CB_WORDS);
    uint2 acc[CF_WORDS / 2];
#pragma unroll
    for (int k = 0; k < (int)(CF_WORDS / 2); ++k) acc[k] = cf[k];
    uint4 v = *reinterpret_cast<const uint4*>(arena + h);
    uint64_t hc = h;                                   // where the row's edges are (forwards: delta.cpp)
    while (v.z & HDR_FWD) {
        hc = (uint64_t)v.x * HDR_WORDS;
        v = *reinterpret_cast<const uint4*>(arena + hc);
    }
    const uint32_t n_sets = v.x;
    uint32_t more = 0;
    for (uint32_t e = 0; e < n_sets; ++e) {
        const uint32_t x = arena[hc + HDR_WORDS + e];
        if (!(x & EDGE_SET)) continue;
        const uint64_t ch = (uint64_t)(x & EDGE_VAL) * HDR_WORDS;
        const uint32_t cz = arena[ch + 2];
        if (!(cz & HDR_CLOSURE)) {                    // cannot happen: a set's target has a filter
            more = NONE32;
            continue;
        }
        const uint2* const cc = reinterpret_cast<const uint2*>(arena + ch - CB_WORDS);
#pragma unroll
        for (int k = 0; k < (int)(CF_WORDS / 2); ++k) {
            const uint2 y = cc[k];
            acc[k].x |= y.x;
            acc[k].y |= y.y;
        }
    }
    if (more) {
#pragma unroll
        for (int k = 0; k < (int)(CF_WORDS / 2); ++k) acc[k] = make_uint2(NONE32, NONE32);
    }
    bool diff = false;
#pragma unroll
    for (int k = 0; k < (int)(CF_WORDS / 2); ++k) {
        const uint2 o = cf[k];
        if (o.x != acc[k].x || o.y != acc[k].y) {
            cf[k] = acc[k];
            diff = true;
        }
    }
    if (diff) atomicAdd(changed, 1u);
}

__global__ void __launch_bounds__(256) closure_fill(uint32_t* __restrict__ arena, const uint32_t* __restrict__ rows,
                                                   uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* const cf = arena + (uint64_t)rows[i] * HDR_WORDS - CB_WORDS;
    for (uint32_t k = 0; k < CF_WORDS; ++k) cf[k] = NONE32;
}

// Child signatures of one closure row (see SIG_WORDS): the 16-bit OR-fold of the closure filter
// of each subject set in its window, stored transposed.  Runs once the filters are closed.  One
// lane per row; a forwarded row keeps none (its content is elsewhere, without a filter block), and a
// migrating part's stub has no edges (its owner holds the row).
__global__ void __launch_bounds__(256) sig_pass(uint32_t* __restrict__ arena, const uint32_t* __restrict__ rows,
                                               uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = (uint64_t)rows[i] * HDR_WORDS;
    const uint4 v = *reinterpret_cast<const uint4*>(arena + h);
    if ((v.z & (HDR_FWD | HDR_REMOTE)) || !(v.z & HDR_CLOSURE)) return;   // stubs: no edges here
    const uint4 win = *reinterpret_cast<const uint4*>(arena + h + HDR_WORDS);
    const uint32_t n_edges = (v.z & HDR_SEQ) ? v.x : v.x + v.y;
    uint32_t fold[4];
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t e = k == 0 ? win.x : k == 1 ? win.y : k == 2 ? win.z : win.w;
        fold[k] = 0xFFFFu;
        if (k >= n_edges || !(e & EDGE_SET) || e == EDGE_POISON) continue;
        const uint64_t ch = (uint64_t)(e & EDGE_VAL) * HDR_WORDS;
        if (!(arena[ch + 2] & HDR_CLOSURE)) continue;           // cannot happen: a set's target has a filter
        uint32_t f = 0;
        for (uint32_t w = 0; w < CF_WORDS; ++w) f |= arena[ch - CB_WORDS + w];
        fold[k] = (f | (f >> 16)) & 0xFFFFu;
    }
    uint32_t out[SIG_WORDS] = {0, 0};
    for (uint32_t b = 0; b < 16; ++b)
        for (uint32_t k = 0; k < 4; ++k) out[b >> 3] |= ((fold[k] >> b) & 1u) << ((b & 7u) * 4u + k);
    *reinterpret_cast<uint2*>(arena + h - SIG_WORDS) = make_uint2(out[0], out[1]);
}

// Close every row's closure filter on the device: rounds of closure_pass over the rows that have
// a filter and subject sets, until a round changes nothing.  A graph that has not converged after
// CLOSURE_MAX_ROUNDS rounds gets full filters (no pruning) instead.
constexpr int CLOSURE_MAX_ROUNDS = 2048;
// The rows of a snapshot with a closure block: `all` (stubs included) and `list`, those whose
// filter closure_pass recomputes (this part's rows with subject sets, not ROW_SEQ).
void closure_rows(const Snapshot& S, std::vector<uint32_t>& list, std::vector<uint32_t>& all) {
    for (uint32_t r = 0; r < S.n_rows(); ++r) {
        if (!S.row_cb[r] || !S.mapped(r)) continue;
        all.push_back(S.unit_of_row[r]);
        if (S.present(r) && S.rows[r].n_sets > 0 && !(S.row_flags(r) & ROW_SEQ)) list.push_back(S.unit_of_row[r]);
    }
}

// Rounds of closure_pass over `list` until one changes nothing (true), or CLOSURE_MAX_ROUNDS
// (false).  *changed_total (optional) gets the number of filter updates.
bool close_filters(uint32_t* d_arena, const std::vector<uint32_t>& list, uint64_t* changed_total) {
    if (list.empty()) return true;
    uint32_t *d_rows = nullptr, *d_changed = nullptr;
    HIP_OK(hipMalloc(&d_rows, list.size() * sizeof(uint32_t)));
    HIP_OK(hipMalloc(&d_changed, sizeof(uint32_t)));
    HIP_OK(hipMemcpy(d_rows, list.data(), list.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    const uint32_t n = (uint32_t)list.size();
    bool done = false;
    for (int round = 0; round < CLOSURE_MAX_ROUNDS && !done; ++round) {
        HIP_OK(hipMemset(d_changed, 0, sizeof(uint32_t)));
        hipLaunchKernelGGL(closure_pass, dim3((n + 255) / 256), dim3(256), 0, 0, d_arena, d_rows, n, d_changed);
        HIP_OK(hipGetLastError());
        uint32_t ch = 0;
        HIP_OK(hipMemcpy(&ch, d_changed, sizeof(uint32_t), hipMemcpyDeviceToHost));
        done = ch == 0;
        if (changed_total) *changed_total += ch;
    }
    (void)hipFree(d_rows);
    (void)hipFree(d_changed);
    return done;
}

// Full filters (no pruning) for the given closure rows, or child signatures from closed filters.
void finish_filters(uint32_t* d_arena, const std::vector<uint32_t>& all, bool converged) {
    if (all.empty()) return;
    uint32_t* d_rows = nullptr;
    HIP_OK(hipMalloc(&d_rows, all.size() * sizeof(uint32_t)));
    HIP_OK(hipMemcpy(d_rows, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    const uint32_t m = (uint32_t)all.size();
    if (!converged) {
        hipLaunchKernelGGL(closure_fill, dim3((m + 255) / 256), dim3(256), 0, 0, d_arena, d_rows, m);
        HIP_OK(hipGetLastError());
    }
    // child signatures of every closure row, from the closed filters
    hipLaunchKernelGGL(sig_pass, dim3((m + 255) / 256), dim3(256), 0, 0, d_arena, d_rows, m);
    HIP_OK(hipGetLastError());
    HIP_OK(hipDeviceSynchronize());
    (void)hipFree(d_rows);
}

// Close every row's closure filter on the device: rounds of closure_pass over the rows that have
// a filter and subject sets, until a round changes nothing.  A graph that has not converged after
// CLOSURE_MAX_ROUNDS rounds gets full filters (no pruning) instead.  A migrating part's stubs start
// empty and its filters are only partial until the parts' filter exchange has converged
// (part_close / part_closure_done), so the signatures wait for that.
void build_closures(const Snapshot& S, uint32_t* d_arena) {
    std::vector<uint32_t> list, all;
    closure_rows(S, list, all);
    if (all.empty()) return;
    const bool done = close_filters(d_arena, list, nullptr);
    if (S.part_mode == PART_MIGRATE && S.n_parts > 1) {
        if (!done) finish_filters(d_arena, all, false);
        HIP_OK(hipDeviceSynchronize());
        return;
    }
    finish_filters(d_arena, all, done);
}

}  // namespace

// The device's collision table: edge value (subject sets by handle) -> visit id of its class.
void upload_coll(Snapshot& S, DeviceState& D, uint64_t& acc) {
    if (D.coll) (void)hipFree(D.coll);
    D.coll = nullptr;
    D.coll_mask = 0;
    S.coll_dirty = false;
    if (S.coll.empty()) return;
    uint32_t cap = pow2_at_least(S.coll.size() * 2 + 2);
    std::vector<uint64_t> tab(cap, ~0ull);
    for (auto& kv : S.coll) {
        uint32_t key = kv.first;
        if (key & EDGE_SET) {
            if (!S.mapped(key & EDGE_VAL)) continue;     // another part's row (stubs are mapped)
            key = EDGE_SET | S.unit_of_row[key & EDGE_VAL];   // row -> handle
        }
        uint32_t vid = kv.second;
        uint32_t i = mix32(key) & (cap - 1);
        while (tab[i] != ~0ull) i = (i + 1) & (cap - 1);
        tab[i] = ((uint64_t)key << 32) | vid;
    }
    D.coll = dmalloc<uint64_t>(cap, acc);
    HIP_OK(hipMemcpy(D.coll, tab.data(), cap * sizeof(uint64_t), hipMemcpyHostToDevice));
    D.coll_mask = cap - 1;
}

void device_upload(Snapshot& S, int device) {
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) throw Error{KETO_E_HIP, "no HIP device"};
    if (device < 0 || device >= n_dev) throw Error{KETO_E_INVALID, "bad device ordinal"};
    HIP_OK(hipSetDevice(device));
    auto D = std::make_unique<DeviceState>();
    D->device = device;
    uint64_t acc = 0;
    const uint64_t words = S.n_words;
    if (words > ARENA_MAX_WORDS) throw Error{KETO_E_RANGE, "device arena exceeds 288 GiB"};
    // a split layout's reserve [tgt_tail, roots_at) is not built on the host: the targets below it
    // and the roots above it are two host pieces
    const bool split = S.tgt_end > 0;
    const uint64_t lo_words = split ? S.tgt_tail : words, hi_base = split ? S.roots_at : words;
    std::vector<uint32_t> arena(std::max<uint64_t>(lo_words, 4)), arena_hi(split ? words - hi_base : 0);
    const uint32_t R = S.n_rows();
    host_parallel_for(R, [&](uint64_t r) {
        if (!S.mapped((uint32_t)r)) return;                  // another part's row
        if (!S.present((uint32_t)r)) {                       // a stub (PART_MIGRATE): owner + its handle
            uint32_t* h = arena.data() + (uint64_t)S.unit_of_row[r] * HDR_WORDS;
            uint32_t* cf = h - CB_WORDS;
            for (uint32_t i = 0; i < CF_WORDS; ++i) cf[i] = 0u;                 // filled by the exchange
            for (uint32_t i = CF_WORDS; i < CB_WORDS; ++i) cf[i] = NONE32;
            h[0] = S.root_owner((uint32_t)r, S.n_parts);
            h[1] = S.g_handle[r];
            h[2] = HDR_REMOTE | HDR_CLOSURE;
            h[3] = 0;
            return;
        }
        const auto ed = S.row_edges((uint32_t)r);
        const bool hi = split && S.hdr_word(S.unit_of_row[r]) >= hi_base;
        put_row(hi ? arena_hi.data() : arena.data(), S.hdr_word(S.unit_of_row[r]), S.rows[r], S.row_pp[r], S.row_hlog2((uint32_t)r),
                ed.first, ed.second, S.unit_of_row, S.row_cb[r] != 0, hi ? hi_base : 0);
    });
    // room at the tail for rows writes move (keto_snapshot_apply; grown on demand)
    const uint64_t used = std::max<uint64_t>(words, 4);
    D->arena_words = std::min<uint64_t>(ARENA_MAX_WORDS, used + std::max<uint64_t>(used / 16, 1ull << 20));
    D->arena = dmalloc<uint32_t>(D->arena_words, acc);
    HIP_OK(hipMemcpy(D->arena, arena.data(), arena.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (split) {
        HIP_OK(hipMemcpy(D->arena + hi_base, arena_hi.data(), arena_hi.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        // the reserve's slots are read 32 B at a time like any header slot once writes fill them
        HIP_OK(hipMemset(D->arena + lo_words, 0, (hi_base - lo_words) * sizeof(uint32_t)));
    }
    build_closures(S, D->arena);
    S.mig_ready = !(S.part_mode == PART_MIGRATE && S.n_parts > 1);   // else after the filter exchange
    upload_coll(S, *D, acc);
    D->bytes = acc;
    // a map holds at most one id per row / collision class (+ an expand root outside the rows)
    D->vid_bound = (uint32_t)std::min<uint64_t>(0xFFFFFFF0ull, (uint64_t)S.n_rows() + S.n_coll_keys + 2);
    D->n_units = (uint32_t)S.n_units;
    D->root_g = S.root_g;
    D->n_coll = S.n_coll_keys;
    // the compute stream and the two copy streams; the pipeline's optional second compute stream is
    // created on first use (KETO_PIPE_STREAMS=2): a process gets few hardware queues
    // (GPU_MAX_HW_QUEUES, 4 by default) and streams beyond them share one, so an idle extra stream
    // could put a copy stream and the compute stream on one queue
    HIP_OK(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&D->copy_in, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&D->copy_out, hipStreamNonBlocking));
    for (auto& e : D->ev) HIP_OK(hipEventCreate(&e));
    for (auto& e : D->pev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    S.device = device;
    S.dev.reset(D.release());
}

DevView device_view(const Snapshot& S) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    const DeviceState& D = *S.dev;
    return DevView{D.arena, D.arena_words, D.coll, D.coll_mask, D.device, (void*)D.stream};
}

namespace {
// filters of the listed handles -> out (CF_WORDS words each)
__global__ void __launch_bounds__(256) filters_get(const uint32_t* __restrict__ arena, const uint32_t* __restrict__ units,
                                                   uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* cf = arena + (uint64_t)units[i] * HDR_WORDS - CB_WORDS;
    for (uint32_t k = 0; k < CF_WORDS; ++k) out[(uint64_t)i * CF_WORDS + k] = cf[k];
}
// OR the given filters into the listed stubs' filters; counts the stubs that gained bits
__global__ void __launch_bounds__(256) filters_or(uint32_t* __restrict__ arena, const uint32_t* __restrict__ units,
                                                  uint32_t n, const uint32_t* __restrict__ in, uint32_t* changed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* cf = arena + (uint64_t)units[i] * HDR_WORDS - CB_WORDS;
    bool diff = false;
    for (uint32_t k = 0; k < CF_WORDS; ++k) {
        const uint32_t o = cf[k], v = o | in[(uint64_t)i * CF_WORDS + k];
        if (v != o) {
            cf[k] = v;
            diff = true;
        }
    }
    if (diff) atomicAdd(changed, 1u);
}

std::vector<uint32_t> units_of(const Snapshot& S, const uint32_t* rows, uint64_t n, bool stubs) {
    std::vector<uint32_t> u(n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = rows[i];
        // reads (stubs = false) take this part's set targets and its stubs; writes only stubs
        if (r >= S.n_rows() || !S.mapped(r) || (stubs && S.present(r)) || !S.row_cb[r])
            throw Error{KETO_E_INVALID, "row " + std::to_string(r) + (stubs ? " is not a stub of this part"
                                                                           : " has no closure filter on this part")};
        u[i] = S.unit_of_row[r];
    }
    return u;
}
}  // namespace

void part_filters(Snapshot& S, const uint32_t* rows, uint64_t n, uint32_t* out) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    if (n == 0) return;
    const std::vector<uint32_t> u = units_of(S, rows, n, false);
    DevBuf<uint32_t> du(n), dout(n * CF_WORDS);
    HIP_OK(hipMemcpy(du.p, u.data(), n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(filters_get, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, D.arena, du.p, (uint32_t)n, dout.p);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(out, dout.p, n * CF_WORDS * 4, hipMemcpyDeviceToHost));
}

uint64_t part_close(Snapshot& S, const uint32_t* rows, uint64_t n, const uint32_t* filters) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    if (S.part_mode != PART_MIGRATE) throw Error{KETO_E_INVALID, "not a migrating part"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    uint64_t changed = 0;
    if (n) {
        const std::vector<uint32_t> u = units_of(S, rows, n, true);
        DevBuf<uint32_t> du(n), din(n * CF_WORDS), dch(1);
        HIP_OK(hipMemcpy(du.p, u.data(), n * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(din.p, filters, n * CF_WORDS * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemset(dch.p, 0, 4));
        hipLaunchKernelGGL(filters_or, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, D.arena, du.p, (uint32_t)n,
                           din.p, dch.p);
        HIP_OK(hipGetLastError());
        uint32_t c = 0;
        HIP_OK(hipMemcpy(&c, dch.p, 4, hipMemcpyDeviceToHost));
        changed += c;
    }
    std::vector<uint32_t> list, all;
    closure_rows(S, list, all);
    if (!close_filters(D.arena, list, &changed)) {
        finish_filters(D.arena, all, false);       // all ones from now on: the exchange ends here
    }
    return changed;
}

void part_closure_done(Snapshot& S, bool converged) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    std::vector<uint32_t> list, all;
    closure_rows(S, list, all);
    finish_filters(D.arena, all, converged);
    S.mig_ready = true;
}

namespace {
// A tail place for a row (the same line and segment rules as compute_layout): returns its header
// unit.  A subject-set target (cb) needs a handle below 2^31: in a split layout it goes into the
// target reserve, else to the tail while that is low enough; without room the caller must rebuild
// (compute_layout places it among the targets).  `low`: the new content of a target a write moved
// (its identity keeps the closure block) in a wide layout, whose tier 0 holds the segment of the
// search's top row only (check_wave_kernel_wide): it goes into the target reserve too.
uint32_t tail_place(Snapshot& S, uint32_t hlog2, bool cb, uint64_t n_edges, uint64_t& total_words, bool low = false) {
    const uint64_t table = hlog2 ? (1ull << hlog2) : 0;
    const uint64_t c = cb ? CB_WORDS : 0;
    if ((cb || low) && S.tgt_end) {
        const uint64_t w = arena_fit(S.tgt_tail, table, c, n_edges, total_words);
        if (w + total_words > S.tgt_end)
            throw Error{KETO_E_REBUILD, "the arena's reserve for new subject-set targets is full: rebuild the snapshot"};
        S.tgt_tail = w + total_words;
        return (uint32_t)((w + table + c) / HDR_WORDS);
    }
    const uint64_t w = arena_fit_g(S.n_words, table, c, n_edges, total_words, S.root_g);
    const uint64_t unit = handle_at_word(w + table + c, S.root_g);
    if (cb && unit >= (uint64_t)EDGE_VAL)
        throw Error{KETO_E_REBUILD, "a new subject-set target would lie past 2^31 16-byte units: rebuild the snapshot"};
    // past the narrow layout's 64 GiB, or out of handles: laid out afresh (wide, or a coarser root unit)
    if (w + total_words > (S.root_g ? ARENA_MAX_WORDS : NARROW_MAX_WORDS) || unit >= HANDLE_MAX - 0x1000u)
        throw Error{KETO_E_REBUILD, "the arena's tail is out of handles: rebuild the snapshot"};
    S.n_words = w + total_words;
    S.n_units = handle_end(S.n_words, S.root_g);
    return (uint32_t)unit;
}
}  // namespace

// Closure filters after a write (device_apply): rounds of closure_pass over the rows with a filter
// and subject sets until one changes nothing, then the child signatures of every row with a filter
// -- as build_closures, on the snapshot's stream, over row lists kept on the device from the last
// write: they are rebuilt only when this write gave a target row a new identity (fresh) or changed
// whether a row takes part (its first subject set, or its last, or the ordered path)
void apply_closures(Snapshot& S, DeviceState& D, bool fresh) {
    const uint32_t R = S.n_rows();
    // only rows some subject set points at carry a filter: a write that changed none of them (e.g.
    // tuples on documents, the root rows) leaves every filter and signature as it was.  (A re-close
    // over all closure rows found nothing to do and cost ~6.7 ms per such write on the 1B graph.)
    bool touched = fresh;
    for (uint32_t r : S.dirty)
        if (r < R && S.row_cb[r]) {
            touched = true;
            break;
        }
    if (!touched) return;
    auto in_list = [&](uint32_t r) {
        return S.row_cb[r] && S.present(r) && S.rows[r].n_sets > 0 && !(S.row_flags(r) & ROW_SEQ);
    };
    // rows past the lists' last build (rows writes added since) are in neither list until a check
    // here finds one that belongs: every added row is dirty in the write that adds it, so a write of
    // new root rows keeps the lists (rebuilding them scanned every row: 322 ms a write on the 1B graph,
    // profiles/r05ak_apply_1b_new_rows.log)
    bool valid = D.cl_valid && !fresh && D.cl_in.size() <= R;
    for (uint32_t r : S.dirty) {
        if (!valid) break;
        if (r >= R || (uint8_t)in_list(r) != (r < D.cl_in.size() ? D.cl_in[r] : 0u)) valid = false;
    }
    if (!valid) {
        std::vector<uint32_t> list, all;
        closure_rows(S, list, all);
        D.cl_in.assign(R, 0);
        for (uint32_t r = 0; r < R; ++r) D.cl_in[r] = S.mapped(r) ? (uint8_t)in_list(r) : 0;
        auto put = [&](uint32_t*& d, uint64_t& cap, const std::vector<uint32_t>& v) {
            if (v.size() > cap) {
                if (d) (void)hipFree(d);
                d = nullptr;
                cap = v.size() + v.size() / 8 + 1024;
                HIP_OK(hipMalloc(&d, cap * sizeof(uint32_t)));
            }
            if (!v.empty())
                HIP_OK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice, D.stream));
        };
        put(D.cl_list, D.cl_list_cap, list);
        put(D.cl_all, D.cl_all_cap, all);
        D.cl_list_n = list.size();
        D.cl_all_n = all.size();
        if (!D.cl_changed) HIP_OK(hipMalloc(&D.cl_changed, sizeof(uint32_t)));
        HIP_OK(hipStreamSynchronize(D.stream));
        D.cl_valid = true;
    }
    if (!D.cl_all_n) return;
    bool done = D.cl_list_n == 0;
    const uint32_t n = (uint32_t)D.cl_list_n, m = (uint32_t)D.cl_all_n;
    for (int round = 0; round < CLOSURE_MAX_ROUNDS && !done; ++round) {
        HIP_OK(hipMemsetAsync(D.cl_changed, 0, sizeof(uint32_t), D.stream));
        hipLaunchKernelGGL(closure_pass, dim3((n + 255) / 256), dim3(256), 0, D.stream, D.arena, D.cl_list, n, D.cl_changed);
        HIP_OK(hipGetLastError());
        uint32_t ch = 0;
        HIP_OK(hipMemcpyAsync(&ch, D.cl_changed, sizeof(uint32_t), hipMemcpyDeviceToHost, D.stream));
        HIP_OK(hipStreamSynchronize(D.stream));
        done = ch == 0;
    }
    if (!done) {
        hipLaunchKernelGGL(closure_fill, dim3((m + 255) / 256), dim3(256), 0, D.stream, D.arena, D.cl_all, m);
        HIP_OK(hipGetLastError());
    }
    hipLaunchKernelGGL(sig_pass, dim3((m + 255) / 256), dim3(256), 0, D.stream, D.arena, D.cl_all, m);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(D.stream));
}

// dst[pairs[2k]] = pairs[2k + 1]: the map entries a write changed
__global__ void __launch_bounds__(256) scatter_pairs(uint32_t* __restrict__ dst, const uint32_t* __restrict__ pairs,
                                                     uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) dst[pairs[2 * k]] = pairs[2 * k + 1];
}

// Patch the device arena after apply_writes (delta.cpp): every changed row is rewritten where it is
// if its new content fits there, else placed at the arena's tail with a forward at its identity
// handle (the handle subject sets hold; its closure filter stays in front of it).  New rows, and
// root rows that became subject-set targets (a target must have a closure filter in front of its
// identity header), get a new identity at the tail; an old identity keeps a forward for handles
// resolved before.  Closure filters are then re-closed on the device from their rows' own ids
// (filters of other rows only ever lose precision: a deleted id's bit may stay, never a needed one
// go missing).  Runs under the snapshot's device lock, between batches.
namespace {
// device_apply in place; false (nothing written to the device yet) when a new subject-set target
// finds no place below 2^31 units
// a write's row images into the arena, in order (one block: a later image wins where two meet, as
// the per-image copies did; seg: arena word, first word in img, words)
__global__ void __launch_bounds__(256) scatter_images(uint32_t* __restrict__ arena, const uint64_t* __restrict__ seg,
                                                      const uint32_t* __restrict__ img, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t to = seg[3 * i], from = seg[3 * i + 1], len = seg[3 * i + 2];
        for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) arena[to + k] = img[from + k];
        __syncthreads();
    }
}

bool apply_in_place(Snapshot& S) {
    DeviceState& D = *S.dev;
    lock_trace("apply: waiting for D.mu");
    std::lock_guard<std::mutex> lk(D.mu);
    lock_trace("apply: D.mu");
    HIP_OK(hipSetDevice(D.device));
    const bool trace = getenv("KETO_APPLY_TRACE") != nullptr;          // tooling: phase times
    auto t_lap = std::chrono::steady_clock::now();
    std::string laps;
    auto lap = [&](const char* what) {
        lock_trace(what);
        if (!trace) return;
        const auto t = std::chrono::steady_clock::now();
        char b[64];
        snprintf(b, sizeof b, " %s %.3f", what, std::chrono::duration<double, std::milli>(t - t_lap).count());
        laps += b;
        t_lap = t;
    };
    struct Write {
        uint64_t word;                    // first word of the image in the arena
        std::vector<uint32_t> img;
    };
    std::vector<Write> writes;
    auto image = [&](uint32_t r, uint32_t unit, bool cb) {
        const auto ed = S.row_edges(r);
        const uint32_t hl = S.row_hlog2(r);
        const uint64_t table = hl ? (1ull << hl) : 0, c = cb ? CB_WORDS : 0;
        Write w;
        w.word = S.hdr_word(unit) - table - c;
        w.img.assign(table + c + HDR_WORDS + ((ed.second + 3) & ~3ull), 0);
        // put_row writes relative to the header: lay it out in a scratch arena starting at word 0
        const uint32_t u0 = (uint32_t)((table + c + HDR_WORDS - 1) / HDR_WORDS);
        std::vector<uint32_t> scratch((uint64_t)u0 * HDR_WORDS + HDR_WORDS + ((ed.second + 3) & ~3ull) + 8, 0);
        put_row(scratch.data(), (uint64_t)u0 * HDR_WORDS, S.rows[r], S.row_pp[r], hl, ed.first, ed.second, S.unit_of_row, cb);
        const uint64_t from = (uint64_t)u0 * HDR_WORDS - table - c;
        std::copy(scratch.begin() + from, scratch.begin() + from + w.img.size(), w.img.begin());
        writes.push_back(std::move(w));
    };
    auto forward = [&](uint32_t at, uint32_t to, bool cb) {
        Write w;
        w.word = S.hdr_word(at);
        w.img = {to, 0u, HDR_FWD | (cb ? HDR_CLOSURE : 0u), 0u};
        writes.push_back(std::move(w));
    };
    // a part of an edge-partitioned snapshot (PART_SHARED) holds every row some subject set points at
    // and its own root rows: another part's root row has no place here, whatever a write did to it
    // (that part's apply writes it), and a root row that became a target joins every part
    const bool parted = S.n_parts > 1;
    auto elsewhere = [&](uint32_t r) { return parted && S.is_root[r] && S.root_owner(r, S.n_parts) != S.part; };
    // 1. new identities first: edges name targets by identity handle
    std::vector<std::pair<uint32_t, uint32_t>> moved;        // (row, old identity)
    std::vector<uint32_t> fresh;
    for (uint32_t r : S.dirty)
        if (S.unit_of_row[r] == NO_UNIT && !elsewhere(r)) fresh.push_back(r);
    for (uint32_t r : S.needs_cb) {
        if (S.unit_of_row[r] != NO_UNIT && !S.row_cb[r]) {
            moved.push_back({r, S.unit_of_row[r]});
            fresh.push_back(r);
        } else if (S.unit_of_row[r] == NO_UNIT) {
            fresh.push_back(r);                                   // another part's root row until now
        }
    }
    std::sort(fresh.begin(), fresh.end());
    fresh.erase(std::unique(fresh.begin(), fresh.end()), fresh.end());
    // a fresh row some subject set points at gets a closure block and a handle below 2^31 (a target);
    // one nothing points at yet (a new root row) goes to the tail like a root of the build, and
    // moves to a target's place once a set points at it (needs_cb)
    for (uint32_t r : fresh) {
        const bool tgt = !S.is_root[r];
        uint64_t tw = 0;
        uint32_t u = 0;
        try {
            u = tail_place(S, S.row_hlog2(r), tgt, S.row_edges(r).second, tw);
        } catch (const Error& e) {
            if (e.code == KETO_E_REBUILD) return false;
            throw;
        }
        S.unit_of_row[r] = u;
        S.row_cb[r] = tgt;
        S.row_place[r] = Snapshot::RowPlace{u, S.row_hlog2(r), (S.row_edges(r).second + 3) & ~3ull, tgt};
        S.layout_units.push_back(u);
        S.rows_by_unit.push_back(r);
    }
    // 2. every changed row's content (fresh is sorted: a write's work stays proportional to its rows,
    // not to the graph's -- a per-row flag array cost 25 ms per write at 155M rows)
    auto is_fresh = [&](uint32_t r) { return std::binary_search(fresh.begin(), fresh.end(), r); };
    std::vector<uint32_t> todo;
    for (uint32_t r : S.dirty)
        if (S.unit_of_row[r] != NO_UNIT) todo.push_back(r);    // (elsewhere: not on this part)
    for (uint32_t r : fresh) todo.push_back(r);
    std::sort(todo.begin(), todo.end());
    todo.erase(std::unique(todo.begin(), todo.end()), todo.end());
    for (uint32_t r : todo) {
        const uint32_t id = S.unit_of_row[r];
        const uint32_t hl = S.row_hlog2(r);
        const uint64_t cap = (S.row_edges(r).second + 3) & ~3ull;
        Snapshot::RowPlace& pl = S.row_place[r];
        if (is_fresh(r)) {
            image(r, id, S.row_cb[r] != 0);
        } else if (pl.hlog2 == hl && pl.edge_cap >= cap) {
            image(r, pl.unit, pl.cb);                         // fits where it is
            if (pl.unit != id && S.row_cb[r]) {               // a forwarded row: re-seed the identity filter
                Write w;
                w.word = S.hdr_word(id) - CB_WORDS;
                w.img.assign(CF_WORDS, 0);
                const auto ed = S.row_edges(r);
                const bool seq = (S.row_flags(r) & ROW_SEQ) != 0;
                for (auto& x : w.img) x = seq ? NONE32 : 0u;
                if (!seq)
                    for (uint64_t i = 0; i < ed.second; ++i)
                        if (!(ed.first[i] & EDGE_SET)) {
                            uint32_t wd, bit;
                            closure_bit(ed.first[i], wd, bit);
                            w.img[wd] |= 1u << bit;
                        }
                writes.push_back(std::move(w));
            }
        } else {
            uint64_t tw = 0;
            uint32_t u = 0;
            try {
                u = tail_place(S, hl, false, S.row_edges(r).second, tw, S.root_g && S.row_cb[r]);
            } catch (const Error& e) {
                if (e.code == KETO_E_REBUILD) return false;       // (nothing written to the device yet)
                throw;
            }
            pl = Snapshot::RowPlace{u, hl, cap, false};
            image(r, u, false);
            forward(id, u, S.row_cb[r] != 0);
            if (S.row_cb[r]) {                                // the identity's filter, re-seeded
                Write w;
                w.word = S.hdr_word(id) - CB_WORDS;
                w.img.assign(CF_WORDS, 0);
                const auto ed = S.row_edges(r);
                const bool seq = (S.row_flags(r) & ROW_SEQ) != 0;
                for (auto& x : w.img) x = seq ? NONE32 : 0u;
                if (!seq)
                    for (uint64_t i = 0; i < ed.second; ++i)
                        if (!(ed.first[i] & EDGE_SET)) {
                            uint32_t wd, bit;
                            closure_bit(ed.first[i], wd, bit);
                            w.img[wd] |= 1u << bit;
                        }
                writes.push_back(std::move(w));
            }
        }
    }
    for (auto& m : moved) forward(m.second, S.unit_of_row[m.first], false);   // stale top-level handles
    lap("images");
    // 3. room: grow the arena if the tail outgrew it (handles are word offsets: copied as is)
    const uint64_t need = S.n_words;
    if (need > D.arena_words) {
        // (slack past the last row: the kernels read a header's 32-B slot, window included)
        const uint64_t cap = std::min<uint64_t>(ARENA_MAX_WORDS, std::max<uint64_t>(need + 1024, D.arena_words + D.arena_words / 4));
        uint64_t acc = 0;
        uint32_t* na = dmalloc<uint32_t>(cap, acc);
        HIP_OK(hipMemcpy(na, D.arena, D.arena_words * sizeof(uint32_t), hipMemcpyDeviceToDevice));
        (void)hipFree(D.arena);
        D.bytes += (cap - D.arena_words) * sizeof(uint32_t);
        D.arena = na;
        D.arena_words = cap;
    }
    // every image in one upload, then one kernel writes them into the arena in order (one pageable
    // copy per image took ~4 us each: 0.42 ms of a 100-row write's exclusive part on the 1B graph)
    if (!writes.empty()) {
        uint64_t words = 0;
        for (const Write& w : writes) words += w.img.size();
        const uint64_t nw = writes.size(), need_b = words * 4 + nw * 24;
        if (D.ap_cap < need_b) {
            if (D.ap_buf) (void)hipFree(D.ap_buf);
            D.ap_buf = nullptr;
            D.ap_cap = 0;
            uint64_t acc = 0;
            const uint64_t c = std::max<uint64_t>(need_b + need_b / 2, 1 << 20);
            D.ap_buf = dmalloc<uint8_t>(c, acc);
            D.ap_cap = c;
        }
        std::vector<uint8_t> up(need_b);
        uint64_t* seg = reinterpret_cast<uint64_t*>(up.data());          // (arena word, first image word, words)
        uint32_t* img = reinterpret_cast<uint32_t*>(up.data() + nw * 24);
        uint64_t at = 0;
        for (uint64_t i = 0; i < nw; ++i) {
            const Write& w = writes[i];
            seg[3 * i] = w.word;
            seg[3 * i + 1] = at;
            seg[3 * i + 2] = w.img.size();
            std::memcpy(img + at, w.img.data(), w.img.size() * 4);
            at += w.img.size();
        }
        HIP_OK(hipMemcpyAsync(D.ap_buf, up.data(), need_b, hipMemcpyHostToDevice, D.stream));
        hipLaunchKernelGGL(scatter_images, dim3(1), dim3(256), 0, D.stream, D.arena,
                           reinterpret_cast<const uint64_t*>(D.ap_buf),
                           reinterpret_cast<const uint32_t*>(D.ap_buf + nw * 24), nw);
        HIP_OK(hipGetLastError());
    }
    HIP_OK(hipStreamSynchronize(D.stream));
    lap("copies");
    // 4. closure filters of every row with one (from their own ids up)
    // (a fresh root row carries no filter and is in no closure list: only fresh targets rebuild them)
    apply_closures(S, D, std::any_of(fresh.begin(), fresh.end(), [&](uint32_t r) { return S.row_cb[r] != 0; }));
    lap("closures");
    // 5. what the kernels and expand output read next: the collision table when a write added
    // classes or gave a classed row a new identity handle
    if (!moved.empty() && !S.coll.empty()) S.coll_dirty = true;
    if (S.coll_dirty) {
        uint64_t acc = 0;
        upload_coll(S, D, acc);
        D.bytes += acc;
    }
    D.n_coll = S.n_coll_keys;
    D.n_units = (uint32_t)S.n_units;
    D.vid_bound = (uint32_t)std::min<uint64_t>(0xFFFFFFF0ull, (uint64_t)S.n_rows() + S.n_coll_keys + 2);
    if (!moved.empty()) {
        // old identities are no longer row handles of expand output
        std::vector<uint32_t> lu, rbu;
        std::unordered_map<uint32_t, uint32_t> old_of;
        for (auto& m : moved) old_of[m.second] = m.first;
        for (size_t i = 0; i < S.layout_units.size(); ++i) {
            auto it = old_of.find(S.layout_units[i]);
            if (it != old_of.end() && S.rows_by_unit[i] == it->second) continue;
            lu.push_back(S.layout_units[i]);
            rbu.push_back(S.rows_by_unit[i]);
        }
        S.layout_units.swap(lu);
        S.rows_by_unit.swap(rbu);
    }
    // 6. the lazily built maps, each on its own: the rows with a fresh identity are patched into
    // whichever of them exists (row -> handle, handle -> row) while they fit; a map past its room is
    // dropped and rebuilt by the next batch that needs it.  (Both were dropped when either was missing:
    // with no expand since the build -- no handle -> row map -- every row-adding write made the next
    // check re-upload the whole row -> handle map, 1.2 GB and ~12 ms at the 1B graph,
    // profiles/r05am_apply_rows_lock_trace.log.)  An old identity keeps its stale entry: only top-level
    // handles resolved before the write reach it, through its forward.  Rows the write added that got
    // no handle here (another part's root rows) still need their NO_UNIT entry in the row -> handle
    // map: the map's slack past its rows is uninitialized
    const bool grew = D.row_handle && S.n_rows() > D.row_handle_rows;
    if (!fresh.empty() || grew) {
        const bool rh_ok = D.row_handle && S.n_rows() <= D.row_handle_cap &&
                           fresh.size() + (S.n_rows() - D.row_handle_rows) <= (1u << 20);
        const bool ur_ok = D.unit_row && std::min<uint64_t>(S.n_units, 1ull << 31) <= D.unit_row_cap &&
                           fresh.size() <= (1u << 20);
        if (D.row_handle && !rh_ok) {
            (void)hipFree(D.row_handle);
            D.row_handle = nullptr;
            D.row_handle_cap = D.row_handle_rows = 0;
        }
        if (D.unit_row && !ur_ok) {
            (void)hipFree(D.unit_row);
            D.unit_row = nullptr;
            D.unit_row_cap = 0;
        }
        // (row, handle) for row_handle: the fresh rows and every row the write added; (handle, row)
        // for unit_row: the fresh rows
        std::vector<uint32_t> rh, hr;
        for (uint32_t r : fresh) {
            if (rh_ok) {
                rh.push_back(r);
                rh.push_back(S.unit_of_row[r]);
            }
            if (ur_ok && S.unit_of_row[r] < D.unit_row_cap) {     // (a root past 2^31: never translated)
                hr.push_back(S.unit_of_row[r]);
                hr.push_back(r);
            }
        }
        if (rh_ok) {
            for (uint64_t r = D.row_handle_rows; r < S.n_rows(); ++r) {
                rh.push_back((uint32_t)r);
                rh.push_back(S.unit_of_row[r]);
            }
            D.row_handle_rows = S.n_rows();
        }
        if (!rh.empty() || !hr.empty()) {
            std::vector<uint32_t> pr(rh);
            pr.insert(pr.end(), hr.begin(), hr.end());
            uint32_t* d_pr = nullptr;
            HIP_OK(hipMalloc(&d_pr, pr.size() * sizeof(uint32_t)));
            HIP_OK(hipMemcpyAsync(d_pr, pr.data(), pr.size() * sizeof(uint32_t), hipMemcpyHostToDevice, D.stream));
            const uint32_t n1 = (uint32_t)(rh.size() / 2), n2 = (uint32_t)(hr.size() / 2);
            if (n1) hipLaunchKernelGGL(scatter_pairs, dim3((n1 + 255) / 256), dim3(256), 0, D.stream, D.row_handle, d_pr, n1);
            if (n2) hipLaunchKernelGGL(scatter_pairs, dim3((n2 + 255) / 256), dim3(256), 0, D.stream, D.unit_row, d_pr + rh.size(), n2);
            HIP_OK(hipGetLastError());
            HIP_OK(hipStreamSynchronize(D.stream));
            (void)hipFree(d_pr);
        }
        // the arena-order handle lists (expand output without the direct map): rebuilt when needed
        for (uint32_t** p : {&D.layout_units, &D.rows_by_unit})
            if (*p) {
                (void)hipFree(*p);
                *p = nullptr;
            }
    }
    lap("maps");
    if (trace) fprintf(stderr, "[apply] device phases (ms):%s\n", laps.c_str());
    S.dirty.clear();
    S.needs_cb.clear();
    return true;
}
}  // namespace

void device_apply(Snapshot& S) {
    if (!S.dev) return;
    // a migrating part (see apply_writes): its stubs name rows by their owners' handles, so it is laid
    // out afresh and uploaded, its filters stale until the next routed batch's exchange
    if (!(S.part_mode == PART_MIGRATE && S.n_parts > 1) && apply_in_place(S)) return;
    // a new subject-set target found no place below 2^31 units (the split layout's reserve is full,
    // or an unsplit arena's tail is past it): lay the arena out afresh, as a build would, and upload
    // it again (handles are per version)
    const int dev = S.dev->device;
    device_release(S);
    compute_layout(S);
    device_upload(S, dev);
    S.dirty.clear();
    S.needs_cb.clear();
}

void device_release(Snapshot& S) {
    if (!S.dev) return;
    DeviceState& D = *S.dev;
    (void)hipSetDevice(D.device);
    mig_release(S);
    S.proto.reset();
    S.reach.reset();
    rdev_release(S);
    for (auto& W : D.ws) {
        for (auto& t : W.tiers) free_tier(t);
        if (W.lists) (void)hipFree(W.lists);
        if (W.pool_busy) (void)hipFree(W.pool_busy);
        if (W.counters) (void)hipFree(W.counters);
        if (W.heads) (void)hipFree(W.heads);
    }
    for (auto& t : D.ews.tiers) free_tier(t);
    if (D.ews.lists) (void)hipFree(D.ews.lists);
    if (D.ews.pool_busy) (void)hipFree(D.ews.pool_busy);
    if (D.ews.counters) (void)hipFree(D.ews.counters);
    if (D.ews.heads) (void)hipFree(D.ews.heads);
    if (D.arena) (void)hipFree(D.arena);
    if (D.coll) (void)hipFree(D.coll);
    if (D.row_handle) (void)hipFree(D.row_handle);
    for (uint32_t* p : {D.cl_list, D.cl_all, D.cl_changed})
        if (p) (void)hipFree(p);
    if (D.layout_units) (void)hipFree(D.layout_units);
    if (D.unit_row) (void)hipFree(D.unit_row);
    if (D.rows_by_unit) (void)hipFree(D.rows_by_unit);
    if (D.ex_buf) (void)hipFree(D.ex_buf);
    if (D.ex_nodes) (void)hipFree(D.ex_nodes);
    if (D.ex_runs) (void)hipFree(D.ex_runs);
    if (D.ex_stage) (void)hipFree(D.ex_stage);
    if (D.ex_seg) (void)hipFree(D.ex_seg);
    if (D.ex_pieces) (void)hipFree(D.ex_pieces);
    if (D.ex_big) (void)hipFree(D.ex_big);
    for (hipEvent_t e : D.ex_ev)
        if (e) (void)hipEventDestroy(e);
    if (D.xlate) (void)hipFree(D.xlate);
    if (D.ap_buf) (void)hipFree(D.ap_buf);
    if (D.st_pairs) (void)hipFree(D.st_pairs);
    if (D.st_dec) (void)hipFree(D.st_dec);
    if (D.st_x) (void)hipFree(D.st_x);
    if (D.st_ready) (void)hipFree(D.st_ready);
    for (int i = 0; i < 2; ++i) {
        if (D.slot_q[i]) (void)hipFree(D.slot_q[i]);
        if (D.slot_x[i]) (void)hipFree(D.slot_x[i]);
        if (D.slot_a[i]) (void)hipFree(D.slot_a[i]);
        if (D.pin_q[i]) (void)hipHostFree(D.pin_q[i]);
        if (D.pin_a[i]) (void)hipHostFree(D.pin_a[i]);
    }
    if (D.stream) (void)hipStreamDestroy(D.stream);
    if (D.stream2) (void)hipStreamDestroy(D.stream2);
    for (hipStream_t& a : D.astream)
        if (a) (void)hipStreamDestroy(a);
    if (D.copy_in) (void)hipStreamDestroy(D.copy_in);
    if (D.copy_out) (void)hipStreamDestroy(D.copy_out);
    for (auto& e : D.ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : D.pev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : D.ps_ev) (void)hipEventDestroy(e);
    if (D.ps_q) (void)hipFree(D.ps_q);
    if (D.ps_idx) (void)hipFree(D.ps_idx);
    if (D.ps_count) (void)hipFree(D.ps_count);
    S.dev.reset();
}

uint64_t device_bytes(const Snapshot& S) { return S.dev ? S.dev->bytes : 0; }

keto_batch_timing device_last_timing(const Snapshot& S) { return S.dev ? S.dev->last : keto_batch_timing{}; }

Snapshot::~Snapshot() {
    if (dev) device_release(*this);
}

void DeviceStateDeleter::operator()(DeviceState* d) const { delete d; }

namespace {

// Tier plan: 0 = every lane of a full persistent grid, small tables; 1 = fewer lanes, large
// tables; 2 = a handful of lanes with tables that hold every visit id of the snapshot.
struct Plan {
    uint32_t slots[3];
    uint32_t cap[3];
    int frames[3];
    bool pool = false;   // tier 1 borrows tier 2's tables on overflow (deep batches)
};

Plan make_plan(const DeviceState& D, uint32_t n, int frames_needed) {
    Plan p;
    uint32_t full = pow2_at_least(2ull * D.vid_bound + 2);
    p.slots[0] = (uint32_t)std::min<uint64_t>((uint64_t)hw_slots(), ((uint64_t)n + 255) / 256 * 256);
    if (p.slots[0] == 0) p.slots[0] = 256;
    p.cap[0] = std::min<uint32_t>(256, full);
    if (const char* e = getenv("KETO_TEST_T0_CAP"))      // test hook: push shallow requests up the tiers
        p.cap[0] = std::min<uint32_t>(full, pow2_at_least((uint32_t)std::max(16, atoi(e))));
    p.slots[1] = (uint32_t)std::min<uint64_t>(4096, ((uint64_t)n + 255) / 256 * 256);
    p.cap[1] = std::min<uint32_t>(1u << 15, full);
    // tier 2: tables that hold every visit id of the snapshot, as many lanes as 8 GiB allows (>= 1)
    p.cap[2] = full;
    {
        const uint64_t per = (uint64_t)full * sizeof(uint64_t);
        uint64_t sl = std::max<uint64_t>(1, (8ull << 30) / per);
        uint32_t s2 = 1;
        while (s2 * 2 <= std::min<uint64_t>(sl, 256)) s2 *= 2;
        p.slots[2] = s2;
    }
    const int fr = std::max(1, frames_needed);
    p.frames[0] = fr <= 16 ? 0 : std::min(fr, 64);   // 0 = LocalStack; deeper paths overflow upward
    p.frames[1] = fr <= 16 ? 0 : std::min(fr, 256);
    p.frames[2] = std::min<int>(fr, (int)std::min<uint64_t>(D.vid_bound + 2ull, 1u << 20));
    if (p.frames[2] < 17) p.frames[2] = 17;
    return p;
}

// Requests (or expand roots) still on the final tier's overflow list: no tier could decide them
// within its limits.  They get a per-request status instead of failing the batch: check decisions
// become KETO_UNDECIDED, expand roots EXP_OVERFLOW with no nodes.
__global__ void __launch_bounds__(256) mark_undecided(uint8_t* __restrict__ dst, uint64_t* __restrict__ cnt,
                                                     const uint32_t* __restrict__ list, uint32_t n, uint8_t value) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = list[i];
    dst[k] = value;
    if (cnt) cnt[k] = 0;
}

struct Undecided {
    uint8_t* dst = nullptr;       // decisions / statuses
    uint64_t* cnt = nullptr;      // expand count pass: node counts zeroed
    uint8_t value = 0;
};

// Pipelined host batches (device_check_host) defer everything after tier 1: no host synchronization
// per chunk, so the next chunk's work is already queued when this one ends.  The chunk's tier-1
// overflows (requests that need tier 2) are copied to a batch-wide stash instead, and decided by a
// full check of the stash once every chunk is done.
struct PipeStash {
    // t0_only (device_check_rows_async): tier 0 alone; its overflow count goes to count[0] and the
    // workset's counters are left zero for the next batch (one small kernel, no memset, no events)
    bool t0_only = false;
    keto_check_ids* q = nullptr;   // device: stashed requests (handle form)
    uint32_t* idx = nullptr;       // device: their batch indices
    uint32_t* count = nullptr;     // device: how many
    uint64_t cap = 0;
    uint32_t base = 0;             // batch index of the current chunk's first request
    const keto_check_ids* dq = nullptr;   // the current chunk's requests
    std::vector<hipEvent_t> ev;    // per chunk: tier 0 start, tier 0 end, tier 1 end
    uint32_t chunk = 0;
};

__global__ void __launch_bounds__(256) stash_overflow(const keto_check_ids* __restrict__ q, const uint32_t* __restrict__ list,
                                                      const uint32_t* __restrict__ count, keto_check_ids* __restrict__ sq,
                                                      uint32_t* __restrict__ sidx, uint32_t* __restrict__ scount,
                                                      uint32_t base, uint64_t cap, const uint32_t* __restrict__ t1_count,
                                                      uint32_t* __restrict__ t1_total) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(t1_total, *t1_count);   // tier-1 requests (timing)
    const uint32_t m = *count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t at = atomicAdd(scount, 1u);
        if (at < cap) {
            sq[at] = q[list[i]];
            sidx[at] = base + list[i];
        }
    }
}

// the end of a t0_only batch: tier 0's overflow count out, the workset's tier counters zeroed
__global__ void t0_tail(uint32_t* __restrict__ counters, uint32_t* __restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = counters[0];
        for (int i = 0; i < 4; ++i) counters[i] = 0;
    }
}

// Runs tiers 0..2 over a batch of n; the batch's timing goes to D.last (added to it when
// `accumulate`, for the chunks of one host-buffer call).  With `stash`: tiers 0 and 1 only, no
// host synchronization, tier-1 overflows to the stash (the caller finishes the batch).
template <class Launch>
void run_tiers(DeviceState& D, WorkSet& W, uint32_t n, const Plan& p, hipStream_t st, Launch launch,
               const Undecided& und, bool accumulate = false, PipeStash* stash = nullptr) {
    Tier* set = W.tiers;
    ensure_lists(W, n);
    uint32_t* list0 = W.lists;
    uint32_t* list1 = W.lists + W.list_cap;
    uint32_t* c0 = W.counters;
    uint32_t* c1 = W.counters + 1;
    ensure_tier(set, 0, p.slots[0], p.cap[0], p.frames[0]);
    ensure_tier(set, 1, p.slots[1], p.cap[1], p.frames[1]);
    if (p.pool) {
        ensure_tier(set, 2, p.slots[2], p.cap[2], p.frames[2]);
        uint64_t acc = 0;
        const uint64_t words = 8 + ((uint64_t)set[1].n_slots + 31) / 32;   // tier 2's tables, then tier 1's
        if (W.pool_words < words) {
            if (W.pool_busy) (void)hipFree(W.pool_busy);
            W.pool_busy = dmalloc<uint32_t>(words, acc);
            W.pool_words = words;
        }
        HIP_OK(hipMemsetAsync(W.pool_busy, 0, words * sizeof(uint32_t), st));
    }
    if (stash && stash->t0_only) {
        launch(0, set[0], (const uint32_t*)nullptr, (const uint32_t*)nullptr, list0, c0, p.slots[0]);
        hipLaunchKernelGGL(t0_tail, dim3(1), dim3(64), 0, st, W.counters, stash->count);
        HIP_OK(hipGetLastError());
        return;
    }
    HIP_OK(hipMemsetAsync(W.counters, 0, 4 * sizeof(uint32_t), st));
    if (stash) {
        // deferred: tiers 0 and 1, then the tier-1 overflows into the stash; no synchronization
        hipEvent_t* e = stash->ev.data() + 3 * stash->chunk;
        HIP_OK(hipEventRecord(e[0], st));
        launch(0, set[0], (const uint32_t*)nullptr, (const uint32_t*)nullptr, list0, c0, p.slots[0]);
        HIP_OK(hipEventRecord(e[1], st));
        launch(1, set[1], list0, c0, list1, c1, p.slots[1]);
        HIP_OK(hipEventRecord(e[2], st));
        hipLaunchKernelGGL(stash_overflow, dim3(16), dim3(256), 0, st, stash->dq, list1, c1, stash->q, stash->idx,
                           stash->count, stash->base, stash->cap, c0, stash->count + 1);
        HIP_OK(hipGetLastError());
        return;
    }
    // tier 0 over all requests
    HIP_OK(hipEventRecord(D.ev[0], st));
    launch(0, set[0], (const uint32_t*)nullptr, (const uint32_t*)nullptr, list0, c0, p.slots[0]);
    HIP_OK(hipEventRecord(D.ev[1], st));
    // tier 1 over tier-0 overflows (count read on the device)
    launch(1, set[1], list0, c0, list1, c1, p.slots[1]);
    HIP_OK(hipEventRecord(D.ev[2], st));
    uint32_t cnt[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(cnt, c0, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    keto_batch_timing T{};
    T.requests[0] = n;
    T.requests[1] = cnt[0];
    T.requests[2] = cnt[1];
    HIP_OK(hipEventElapsedTime(&T.tier_ms[0], D.ev[0], D.ev[1]));
    HIP_OK(hipEventElapsedTime(&T.tier_ms[1], D.ev[1], D.ev[2]));
    if (cnt[1]) {
        ensure_tier(set, 2, p.slots[2], p.cap[2], p.frames[2]);
        HIP_OK(hipMemsetAsync(c0, 0, sizeof(uint32_t), st));
        HIP_OK(hipEventRecord(D.ev[3], st));
        launch(2, set[2], list1, c1, list0, c0, p.slots[2]);
        HIP_OK(hipEventRecord(D.ev[4], st));
        uint32_t still = 0;
        HIP_OK(hipMemcpyAsync(&still, c0, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipEventElapsedTime(&T.tier_ms[2], D.ev[3], D.ev[4]));
        if (still) {
            hipLaunchKernelGGL(mark_undecided, dim3((still + 255) / 256), dim3(256), 0, st, und.dst, und.cnt, list0, still,
                               und.value);
            HIP_OK(hipGetLastError());
            T.undecided = still;
        }
    }
    keto_batch_timing& L = D.last;
    if (!accumulate) {
        L = T;
        return;
    }
    for (int i = 0; i < 3; ++i) {
        L.tier_ms[i] += T.tier_ms[i];
        L.requests[i] += T.requests[i];
    }
    L.undecided += T.undecided;
}

// batch-local overlay arena on the device (freed when the batch returns)
struct OverlayBuf {
    DevOverlay v{nullptr, 0xFFFFFFFFu};
    void* p = nullptr;
    OverlayBuf(const Snapshot& S, const Overlay* ov) {
        if (!ov || ov->empty()) return;
        std::vector<uint32_t> arena(std::max<uint64_t>(ov->n_units * HDR_WORDS, 4));
        for (size_t i = 0; i < ov->rows.size(); ++i) {
            const RowRec& rec = ov->rows[i];
            const uint64_t b = (uint64_t)rec.edge_lo | ((uint64_t)(rec.hi_flags & 0xFFu) << 32);
            const uint64_t e = i + 1 < ov->rows.size()
                                   ? ((uint64_t)ov->rows[i + 1].edge_lo | ((uint64_t)(ov->rows[i + 1].hi_flags & 0xFFu) << 32))
                                   : ov->edges.size();
            put_row(arena.data(), (uint64_t)ov->unit[i] * HDR_WORDS, rec, ov->pp[i], 0, ov->edges.data() + b, e - b, S.unit_of_row, false);
        }
        uint64_t acc = 0;
        uint32_t* a = dmalloc<uint32_t>(arena.size(), acc);
        p = a;
        HIP_OK(hipMemcpy(a, arena.data(), arena.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        v = DevOverlay{a, (uint32_t)S.n_units};
    }
    ~OverlayBuf() {
        if (p) (void)hipFree(p);
    }
};

struct DevFree {
    std::vector<void*> p;
    ~DevFree() {
        for (void* q : p)
            if (q) (void)hipFree(q);
    }
};

// Expand on a migrating part (PART_MIGRATE, n_parts > 1): the part's arena holds its own rows, the
// replicated hot rows and a stub (HDR_REMOTE) for every other part's row one of them points at.  A
// tree that reaches another part's row needs that row's edges, and every part's host tables hold the
// whole graph, so the call copies such rows into its overlay arena: the count pass records the rows
// its walks met without a copy (ExpandOut::miss; the tree returns EXP_RETRY), they are copied in, and
// the pass runs again until no tree needs one.  A row keeps one identity (the handle its node and
// visit id carry): its stub's handle where this part has a stub, else an identity slot of the
// overlay (a REMOTE header, allocated on first sight).  rmap maps an identity to the handle of the
// row's copy.  Overlay layout: [the call's wildcard rows][identity slots][copies].
struct PullSet {
    const Snapshot& S;
    const Overlay* wild;
    uint64_t wild_units;
    std::vector<uint32_t> id_row;                    // identity slot k -> row
    std::unordered_map<uint32_t, uint32_t> ident;    // row -> identity handle (rows without a stub)
    std::vector<uint32_t> pulled;                    // rows copied into the overlay, in order
    std::unordered_set<uint32_t> have;
    DevFree bufs;                                    // this round's device copies
    PullSet(const Snapshot& s, const Overlay* w) : S(s), wild(w), wild_units(w && !w->empty() ? w->n_units : 0) {}
    uint32_t identity(uint32_t r) {
        if (S.mapped(r)) return S.unit_of_row[r];
        auto it = ident.find(r);
        if (it != ident.end()) return it->second;
        const uint64_t h = S.n_units + wild_units + id_row.size();
        if (h >= EDGE_VAL) throw Error{KETO_E_RANGE, "expand on a migrating part: identity handles past 2^31"};
        id_row.push_back(r);
        ident.emplace(r, (uint32_t)h);
        return (uint32_t)h;
    }
    uint32_t vid(uint32_t r) {                        // Snapshot::vid_of_row with identities
        if (!S.coll.empty()) {
            auto it = S.coll.find(EDGE_SET | r);
            if (it != S.coll.end()) return it->second;
        }
        return identity(r);
    }
    bool add(uint32_t r) {
        if (r >= S.n_rows() || S.present(r) || !have.insert(r).second) return false;
        pulled.push_back(r);
        return true;
    }
    int64_t row_of(uint32_t h) const {                // the row a recorded handle names
        if (h < S.n_units) return S.row_of_handle(h);
        const uint64_t k = (uint64_t)h - S.n_units;
        if (k < wild_units) return -1;
        return k - wild_units < id_row.size() ? (int64_t)id_row[k - wild_units] : -1;
    }
    // the overlay arena, rmap and (with collision classes) a collision table keyed by identities, on
    // the device for the next pass
    void build(DevOverlay& dov, DevSnap& sv, const DevSnap& base) {
        auto scan = [&](const uint32_t* ed, uint64_t m) {
            for (uint64_t i = 0; i < m; ++i)
                if ((ed[i] & EDGE_SET) && ed[i] != EDGE_POISON) (void)identity(ed[i] & EDGE_VAL);
        };
        auto wild_edges = [&](size_t i) {
            const RowRec& rec = wild->rows[i];
            const uint64_t b = (uint64_t)rec.edge_lo | ((uint64_t)(rec.hi_flags & 0xFFu) << 32);
            const uint64_t e = i + 1 < wild->rows.size()
                                   ? ((uint64_t)wild->rows[i + 1].edge_lo | ((uint64_t)(wild->rows[i + 1].hi_flags & 0xFFu) << 32))
                                   : wild->edges.size();
            return std::make_pair(wild->edges.data() + b, e - b);
        };
        const size_t n_wild = wild_units ? wild->rows.size() : 0;
        for (size_t i = 0; i < n_wild; ++i) {
            const auto ed = wild_edges(i);
            scan(ed.first, ed.second);
        }
        for (uint32_t r : pulled) {
            const auto ed = S.row_edges(r);
            scan(ed.first, ed.second);
        }
        const uint64_t slots_at = wild_units, copies_at = wild_units + id_row.size();
        std::vector<uint64_t> at(pulled.size());
        uint64_t units = copies_at;
        for (size_t k = 0; k < pulled.size(); ++k) {
            at[k] = units;
            units += 1 + (S.row_edges(pulled[k]).second + 3) / 4;
        }
        std::vector<uint32_t> arena(std::max<uint64_t>(units, 1) * HDR_WORDS, 0u);
        auto patch = [&](uint64_t unit, const uint32_t* ed, uint64_t m) {   // set edges -> identities
            uint32_t* e = arena.data() + unit * HDR_WORDS + HDR_WORDS;
            for (uint64_t i = 0; i < m; ++i)
                if ((ed[i] & EDGE_SET) && ed[i] != EDGE_POISON) e[i] = EDGE_SET | identity(ed[i] & EDGE_VAL);
        };
        for (size_t i = 0; i < n_wild; ++i) {
            const auto ed = wild_edges(i);
            put_row(arena.data(), (uint64_t)wild->unit[i] * HDR_WORDS, wild->rows[i], wild->pp[i], 0, ed.first, ed.second, S.unit_of_row, false);
            patch(wild->unit[i], ed.first, ed.second);
        }
        for (size_t k = 0; k < id_row.size(); ++k) arena[(slots_at + k) * HDR_WORDS + 2] = HDR_REMOTE;
        for (size_t k = 0; k < pulled.size(); ++k) {
            const uint32_t r = pulled[k];
            const auto ed = S.row_edges(r);
            put_row(arena.data(), (uint64_t)at[k] * HDR_WORDS, S.rows[r], S.row_pp[r], 0, ed.first, ed.second, S.unit_of_row, false);
            patch(at[k], ed.first, ed.second);
        }
        for (void* q : bufs.p)
            if (q) (void)hipFree(q);
        bufs.p.clear();
        uint64_t acc = 0;
        uint32_t* a = dmalloc<uint32_t>(arena.size(), acc);
        bufs.p.push_back(a);
        HIP_OK(hipMemcpy(a, arena.data(), arena.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        const uint32_t cap = pow2_at_least(pulled.size() * 2 + 2);
        std::vector<uint64_t> tab(cap, ~0ull);
        for (size_t k = 0; k < pulled.size(); ++k) {
            const uint32_t key = identity(pulled[k]);
            uint32_t i = mix32(key) & (cap - 1);
            while (tab[i] != ~0ull) i = (i + 1) & (cap - 1);
            tab[i] = ((uint64_t)key << 32) | (uint32_t)(S.n_units + at[k]);
        }
        uint64_t* rm = dmalloc<uint64_t>(cap, acc);
        bufs.p.push_back(rm);
        HIP_OK(hipMemcpy(rm, tab.data(), cap * sizeof(uint64_t), hipMemcpyHostToDevice));
        dov = DevOverlay{a, (uint32_t)S.n_units, rm, cap - 1};
        sv = base;
        if (!S.coll.empty() && !id_row.empty()) {
            // the device table keys classes by handles of mapped rows (upload_coll); the identity
            // slots' rows join it here
            const uint32_t cc = pow2_at_least(S.coll.size() * 2 + 2);
            std::vector<uint64_t> ct(cc, ~0ull);
            for (const auto& kv : S.coll) {
                uint32_t key = kv.first;
                if (key & EDGE_SET) {
                    const uint32_t r = key & EDGE_VAL;
                    if (S.mapped(r)) key = EDGE_SET | S.unit_of_row[r];
                    else if (auto it = ident.find(r); it != ident.end()) key = EDGE_SET | it->second;
                    else continue;
                }
                uint32_t i = mix32(key) & (cc - 1);
                while (ct[i] != ~0ull) i = (i + 1) & (cc - 1);
                ct[i] = ((uint64_t)key << 32) | kv.second;
            }
            uint64_t* c = dmalloc<uint64_t>(cc, acc);
            bufs.p.push_back(c);
            HIP_OK(hipMemcpy(c, ct.data(), cc * sizeof(uint64_t), hipMemcpyHostToDevice));
            sv.coll = c;
            sv.coll_mask = cc - 1;
        }
    }
};


}  // namespace

namespace {
using CheckKernelFn = void (*)(DevSnap, DevOverlay, const keto_check_ids*, uint32_t, int, uint8_t*, TierArgs,
                               unsigned long long*);
// tier-0 variants for max-depth <= 5 (4 saved frames): {LDS visit ids, register visit ids}; then the
// max-depth <= 9 kernel (8 frames).  KETO_T0 picks a variant (tuning).  The default is 3 (8 + 8
// visit ids): on one box, 2.53-2.55 ms per 16.7M batch on the 1B graph against 2.97-3.01 ms for
// variant 0 (4 + 16), the round-3 default, with identical decisions (profiles/r04ae_tier0_variants.log;
// it runs 6 waves per SIMD against 8: its LDS columns hold 8 ids).  Variant 7 (12 + 8) ties.
constexpr int T0_VARIANTS = 8;
constexpr uint32_t KETO_HEAD_WORDS = 8 * 16 * 32;
int t0_variant() {
    const char* e = getenv("KETO_T0");
    const int v = e ? atoi(e) : 3;
    return v >= 0 && v < T0_VARIANTS ? v : 3;
}
// request runs handed out per grab by the tier-0 wave kernel (TierArgs::dyn) for a batch of n
// requests over `lanes` lanes: runs of 4 after a static first quarter, dealt by 4 heads per XCD,
// used once every lane has at least 16 requests (with fewer, one static run per lane keeps more
// lanes busy).  On the 1B graph a lane holds only ~32 requests of a 16.7M batch, so runs of 32
// (the round-1 setting: 2.81-3.00 ms) left the launch's tail to a few lanes per wave (37 of 64
// lanes busy per wave-iteration); runs of 4 keep 56 busy (2.76-2.82 ms, profiles/r02m_dyn_heads.log,
// r02q_tune_sigs.log).  KETO_T0_DYN overrides the run size (0 = static runs), KETO_T0_DYN_STATIC
// the static eighths, KETO_T0_HEADS the heads per XCD, KETO_T0_DYN_FORCE=1 drops the batch-size
// condition (tests).
uint32_t t0_dyn(uint64_t n, uint64_t lanes) {
    const char* e = getenv("KETO_T0_DYN");
    const char* f = getenv("KETO_T0_DYN_STATIC");       // eighths of a range handed out statically
    const char* force = getenv("KETO_T0_DYN_FORCE");
    if (!(force && atoi(force) == 1) && n < 16 * lanes) return 0u;
    const char* hs = getenv("KETO_T0_HEADS");          // heads per XCD (a power of two, <= 16)
    const int v = e ? atoi(e) : 4;
    const int st = f ? std::min(7, std::max(0, atoi(f))) : 2;
    const int heads = hs ? std::min(16, atoi(hs)) : 4;
    uint32_t hl2 = 0;
    while ((1 << (hl2 + 1)) <= heads) ++hl2;
    return v > 0 ? (std::min<uint32_t>((uint32_t)v + 3u, 0xFFFCu) & ~3u) | ((uint32_t)st << 16) | (hl2 << 20) : 0u;
}
// streamed batches: runs of 4 (a power of two, so no run straddles a chunk), all of them dealt by
// the heads (no static part: a lane's static run could lie in the last chunk)
uint32_t t0_stream_dyn() {
    const char* hs = getenv("KETO_T0_HEADS");
    const int heads = hs ? std::min(16, atoi(hs)) : 4;
    uint32_t hl2 = 0;
    while ((1 << (hl2 + 1)) <= heads) ++hl2;
    return 4u | (hl2 << 20);
}
const char* t0_kernel_name(int var) {
    switch (var) {
        case 0: return "keto::check_wave_kernel<4, false, 4, 16, false, false>";
        case 1: return "keto::check_wave_kernel<4, false, 4, 8, false, false>";
        case 2: return "keto::check_wave_kernel<4, false, 12, 4, false, false>";
        case 3: return "keto::check_wave_kernel<4, false, 8, 8, false, false>";
        case 4: return "keto::check_wave_kernel<4, false, 8, 6, false, false>";
        case 5: return "keto::check_wave_kernel<4, false, 12, 6, false, false>";
        case 6: return "keto::check_wave_kernel<4, false, 6, 8, false, false>";
        case 7: return "keto::check_wave_kernel<4, true, 8, 8, false, false>";
        default: return "keto::check_wave_kernel<8, false, 8, 8, false, false>";
    }
}
CheckKernelFn t0_kernel(int var, bool count) {
    // <saved frames, save windows, LDS visit ids, register visit ids>
    switch (var) {
        case 0: return count ? check_wave_kernel<4, false, 4, 16, true> : check_wave_kernel<4, false, 4, 16, false>;
        case 1: return count ? check_wave_kernel<4, false, 4, 8, true> : check_wave_kernel<4, false, 4, 8, false>;
        case 2: return count ? check_wave_kernel<4, false, 12, 4, true> : check_wave_kernel<4, false, 12, 4, false>;
        case 3: return count ? check_wave_kernel<4, false, 8, 8, true> : check_wave_kernel<4, false, 8, 8, false>;
        case 4: return count ? check_wave_kernel<4, false, 8, 6, true> : check_wave_kernel<4, false, 8, 6, false>;
        case 5: return count ? check_wave_kernel<4, false, 12, 6, true> : check_wave_kernel<4, false, 12, 6, false>;
        case 6: return count ? check_wave_kernel<4, false, 6, 8, true> : check_wave_kernel<4, false, 6, 8, false>;
        case 7: return count ? check_wave_kernel<4, true, 8, 8, true> : check_wave_kernel<4, true, 8, 8, false>;
        default: return count ? check_wave_kernel<8, false, 8, 8, true> : check_wave_kernel<8, false, 8, 8, false>;
    }
}
// the streamed launch: the default variant's geometry (KETO_T0_STREAM=0: variant 0's)
bool t0_stream_v0() {
    const char* e = getenv("KETO_T0_STREAM");
    return e && atoi(e) == 0;
}
CheckKernelFn t0_stream_kernel() {
    return t0_stream_v0() ? check_wave_kernel<4, false, 4, 16, false, true> : check_wave_kernel<4, false, 8, 8, false, true>;
}
}  // namespace

// deep batches (global max-depth 10..64) take deep_wave_kernel as tier 0 only with KETO_DEEP_WAVE=1:
// on config #3 it lost to the inline check_kernel (366 + 231 ms vs 258 ms, the critical path is ~4
// dependent accesses per DFS step either way, and its 16K-entry maps overflow to tier 1 where the
// inline kernel borrows in place; profiles/r02j_deep_sweep.log)
bool deep_wave(int32_t gmd) {
    const char* e = getenv("KETO_DEEP_WAVE");
    return gmd - 1 <= DF && e && atoi(e) == 1;
}

const char* device_check_kernel_name(int32_t gmd) {
    const int fr = std::max(1, std::min<int32_t>(gmd, 65535) - 1);
    if (fr > 8 && deep_wave(gmd)) return "keto::deep_wave_kernel<8, 8, false>";
    if (fr > 8) return "keto::check_kernel<keto::GlobalStack, false, 0>";
    return t0_kernel_name(fr <= 4 ? t0_variant() : T0_VARIANTS);
}

namespace {

// A streamed host batch (device_check_stream): tier 0 reads the 8-B pairs as their chunks land; the
// requests it hands up are translated into `xlate` (at their batch index) for tiers 1 and 2
struct StreamSrc {
    const keto_check_pair* pairs = nullptr;
    const uint32_t* ready = nullptr;
    uint32_t chunk_log2 = 0;
    int32_t depth = 0;
    uint32_t* stalled = nullptr;
    uint64_t wait_ticks = 0;
    keto_check_ids* xlate = nullptr;
};

__device__ inline keto_check_ids pair_to_ids(const keto_check_pair p, int32_t depth, const uint32_t* __restrict__ table,
                                             uint32_t n_rows, bool& misrouted) {
    keto_check_ids q{KETO_NO_ROW, KETO_NO_TARGET, 0u, depth};
    misrouted = false;
    if (p.row != KETO_NO_ROW) {
        const uint32_t h = p.row < n_rows ? table[p.row] : NO_UNIT;
        misrouted = h == NO_UNIT;
        q.row = h == NO_UNIT ? KETO_NO_ROW : h;
    }
    if (p.subject != KETO_NO_TARGET) {
        if (p.subject & EDGE_SET) {
            const uint32_t r = p.subject & EDGE_VAL;
            const uint32_t h = r < n_rows ? table[r] : NO_UNIT;
            q.target = h == NO_UNIT ? KETO_NO_TARGET : h;
            q.flags = 1u;
        } else {
            q.target = p.subject;
        }
    }
    return q;
}

// the streamed requests tier 0 handed up (list[0 .. *count)), translated in place of the batch
__global__ void __launch_bounds__(256) list_pairs_to_handles(const keto_check_pair* __restrict__ in,
                                                             const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                             keto_check_ids* __restrict__ out, int32_t depth,
                                                             const uint32_t* __restrict__ table, uint32_t n_rows) {
    const uint32_t m = *count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t qi = list[i];
        bool mis;
        out[qi] = pair_to_ids(in[qi], depth, table, n_rows, mis);
    }
}

// The check of one device-resident batch: the tier plan and the kernel launches.  The caller holds
// D.mu and has set the device; `dq` / `da` are device buffers (`ss`: a streamed batch, dq unused).
void check_core(Snapshot& S, DeviceState& D, const keto_check_ids* dq, uint32_t n, int32_t gmd, uint8_t* da,
                hipStream_t st, const DevOverlay& dov, uint64_t* work_out, bool accumulate, uint32_t* d_steps,
                PipeStash* stash, int wsi, const ItemWork* items, const StreamSrc* ss = nullptr) {
    WorkSet& W = D.ws[wsi];
    if (S.part_mode == PART_MIGRATE)
        throw Error{KETO_E_INVALID, "a migrating part answers checks through keto_mig_begin / keto_mig_round"};
    if (n == 0) {
        if (!accumulate) D.last = keto_batch_timing{};
        return;
    }
    if (gmd > 65535) gmd = 65535;
    DevFree tmp;
    // check recursion holds at most gmd - 1 frames.  Tier 0 keeps them in LDS when they fit
    // (LdsStack<4> covers the default max-depth 5), else in HBM (GlobalStack).
    Plan p = make_plan(D, n, std::max(1, gmd - 1));
    const int fr = std::max(1, gmd - 1);
    const int kind = fr <= 4 ? 0 : fr <= 8 ? 1 : 2;
    p.frames[0] = kind == 2 ? std::min(fr, 64) : 0;
    for (int l = 0; l < 3; ++l) p.frames[l] *= 2;   // check frames on GlobalStack carry their edge block
    {
        // tier 2 keeps one 16-bit epoch per possible visit id (DirectVisited): 2 B per arena unit
        // and collision class, as many lanes (<= 256, a power of two) as 16 GiB allows
        const uint64_t ids = (uint64_t)std::min<uint32_t>(D.n_units, EDGE_VAL) + D.n_coll + 1;
        if ((ids + 3) / 4 > 0xFFFFFFFFull) throw Error{KETO_E_RANGE, "tier-2 visited table exceeds 2^32 words"};
        p.cap[2] = (uint32_t)((ids + 3) / 4);
        const uint64_t per = (uint64_t)p.cap[2] * sizeof(uint64_t);
        const char* es = getenv("KETO_T2_SLOTS");
        const uint64_t want = std::min<uint64_t>(es ? (uint64_t)atoi(es) : 256u, std::max<uint64_t>(1, (16ull << 30) / per));
        uint32_t s2 = 1;
        while (s2 * 2 <= want) s2 *= 2;
        p.slots[2] = s2;
    }
    // (deep_wave_kernel keeps one segment bit: arenas of up to 2 segments)
    const bool dw = kind == 2 && deep_wave(gmd) && (uint64_t)D.n_units <= (1ull << 31) && D.root_g == 0;
    if (ss && kind != 0) throw Error{KETO_E_INVALID, "streamed batches need max-depth <= 5"};
    int var = ss ? T0_VARIANTS + 3 + (t0_stream_v0() ? 1 : 0)
                 : kind == 0 ? t0_variant() : kind == 1 ? T0_VARIANTS : dw ? T0_VARIANTS + 2 : T0_VARIANTS + 1;
    // batches of fewer than 16 requests per lane of the 8-wave build take check_wave_kernel_w8
    // (variant 0's geometry at 8 waves per SIMD); KETO_T0 (tuning) or KETO_T0_W8=0 keep the variant
    constexpr int VAR_W8 = T0_VARIANTS + 5;
    // a wide arena (past 64 GiB) takes check_wave_kernel_wide as tier 0, whatever the variant
    const bool wide = D.root_g != 0;
    if (kind == 0 && !ss && !work_out && !wide && !getenv("KETO_T0") && !(getenv("KETO_T0_W8") && atoi(getenv("KETO_T0_W8")) == 0)) {
        if (!D.v1_lanes[VAR_W8]) {
            int per_cu = 0, cus = 0;
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, check_wave_kernel_w8<4, 4, 16>, 256, 0));
            HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, D.device));
            D.v1_lanes[VAR_W8] = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus) * 256u;
        }
        if ((uint64_t)n < 16ull * D.v1_lanes[VAR_W8]) var = VAR_W8;
    }
    if (!D.v1_lanes[var]) {
        // persistent grid = what is resident at the kernel's register / LDS budget (KETO_SLOTS overrides)
        int per_cu = 0, cus = 0;
        if (ss && wide)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, check_wave_kernel_wide<4, true>, 256, 0));
        else if (ss)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, t0_stream_kernel(), 256, 0));
        else if (wide && kind < 2)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, kind == 0 ? check_wave_kernel_wide<4, false> : check_wave_kernel_wide<8, false>, 256, 0));
        else if (dw)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, deep_wave_kernel<8, 8, false>, 256, 0));
        else if (kind == 2)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, check_kernel<GlobalStack, false, 0>, 256, 0));
        else
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, t0_kernel(var, false), 256, 0));
        HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, D.device));
        D.v1_lanes[var] = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus) * 256u;
    }
    uint32_t lanes = getenv("KETO_SLOTS") ? (uint32_t)hw_slots() : D.v1_lanes[var];
    // a batch of at most ~2 requests per resident lane (config #2: 1M requests) takes one lane per
    // request: the grid is then more than the chip holds at once, and a wave that finishes makes room
    // for the next instead of a lane walking its second request behind its first (0.158 -> 0.144
    // ms, profiles/r05aa_config2_grid.log).  KETO_T0_ONE_PER_LANE = the requests-per-lane bound
    // (default 2; 0 = off); tier-0 tables: 2 KB per lane
    if (var == VAR_W8 && !getenv("KETO_SLOTS")) {
        const char* e1 = getenv("KETO_T0_ONE_PER_LANE");
        const uint64_t k = e1 ? (uint64_t)std::max(0, atoi(e1)) : 2u;
        if ((uint64_t)n <= k * lanes) lanes = (uint32_t)(((uint64_t)n + 255) / 256 * 256);
    }
    p.slots[0] = (uint32_t)std::min<uint64_t>(lanes, ((uint64_t)n + 255) / 256 * 256);
    if (ss) {
        // a streamed launch leaves wave slots free: the runtime's H2D copies behind it run as blit
        // kernels, which a launch holding every slot starves until its lanes give up waiting
        // (tools/dev/stream_probe.hip: 8/8 of the slots never saw a chunk land, 7/8 did).
        // KETO_STREAM_EIGHTHS overrides the share (default 7)
        const char* e8 = getenv("KETO_STREAM_EIGHTHS");
        const uint32_t eighths = (uint32_t)std::min(8, std::max(1, e8 ? atoi(e8) : 7));
        p.slots[0] = std::max<uint32_t>(256, p.slots[0] / 8 * eighths / 256 * 256);
    }
    if (stash && kind < 2) {
        // KETO_CHUNK_LANES (tuning): a pipeline chunk's tier 0 on at most that many lanes, so that the
        // chunks of two compute streams (KETO_PIPE_STREAMS=2) can run side by side
        if (const char* e = getenv("KETO_CHUNK_LANES"))
            p.slots[0] = std::max<uint32_t>(256, std::min<uint32_t>(p.slots[0], (uint32_t)atoi(e) / 256 * 256));
    }
    if (kind == 2) {
        // deep requests (nested groups) visit thousands of sets.  Tier 0 gets tables of 64K entries
        // (32K visit ids before a lane borrows a tier-1 table, after which every test probes two
        // tables) and as many lanes as three quarters of the budget hold; tier 1 16K lanes with
        // tables of up to 128K entries in the rest (the borrow pool and the overflow tier).  The
        // budget is half of device memory (tables are reused across batches).  On config #3 the
        // items' tier 0 took 113 ms with 229K lanes of 64K entries against 132 ms with 327K lanes of
        // 32K (profiles/r03s_config3_tables.log, r03r_config3_tables.log).
        size_t free_b = 0, total_b = 0;
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        uint64_t held = 0;
        for (int l = 0; l < 2; ++l) held += (uint64_t)W.tiers[l].n_slots * W.tiers[l].cap * sizeof(uint64_t);
        uint64_t budget = std::min<uint64_t>(total_b / 2, (free_b + held) * 6 / 10);
        if (const char* eb = getenv("KETO_DEEP_BUDGET_GB"))
            budget = std::min<uint64_t>((uint64_t)atoi(eb) << 30, (free_b + held) * 3 / 4);
        const uint64_t b0 = budget / 4 * 3, b1 = budget - b0;
        const uint32_t full = pow2_at_least(2ull * D.vid_bound + 2);
        auto fit = [&](uint32_t slots, uint32_t lo, uint32_t hi, uint64_t b) {
            uint32_t c = lo;
            while (c < hi && (uint64_t)slots * (2ull * c) * sizeof(uint64_t) <= b) c *= 2;
            return std::min(c, full);
        };
        const char* e0 = getenv("KETO_T0_CAP");
        const char* e1 = getenv("KETO_T1_SLOTS");
        const char* e2 = getenv("KETO_T1_CAP");
        const uint32_t want0 = std::min(full, pow2_at_least(e0 ? (uint32_t)std::max(256, atoi(e0)) : 65536u));
        if (!getenv("KETO_SLOTS")) {
            const uint64_t fit_lanes = std::max<uint64_t>(256, b0 / ((uint64_t)want0 * sizeof(uint64_t)) / 256 * 256);
            p.slots[0] = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(lanes, fit_lanes), ((uint64_t)n + 255) / 256 * 256);
        }
        p.cap[0] = fit(p.slots[0], 256, want0, b0);
        p.slots[1] = (uint32_t)std::min<uint64_t>(e1 ? (uint32_t)atoi(e1) : 16384u, ((uint64_t)n + 255) / 256 * 256);
        p.cap[1] = std::max(p.cap[0], fit(p.slots[1], 1024, e2 ? (uint32_t)atoi(e2) : 131072u, b1));
        p.pool = getenv("KETO_NO_POOL") == nullptr;
    }
    if (const char* e = getenv("KETO_TEST_T2_FRAMES")) p.frames[2] = 2 * std::max(1, atoi(e));   // test hook
    DevSnap sv = D.view();
    unsigned long long* dwork = nullptr;
    if (work_out) {
        uint64_t acc = 0;
        dwork = dmalloc<unsigned long long>(2 * KETO_WORK_SLOTS, acc);   // + the SIMT profile
        tmp.p.push_back(dwork);
        HIP_OK(hipMemsetAsync(dwork, 0, 2 * KETO_WORK_SLOTS * sizeof(unsigned long long), st));
        if (d_steps) HIP_OK(hipMemsetAsync(d_steps, 0, (uint64_t)n * sizeof(uint32_t), st));
    }
    run_tiers(D, W, n, p, st,
              [&](int level, Tier& t, const uint32_t* il, const uint32_t* ic, uint32_t* ol, uint32_t* oc,
                  uint32_t slots) {
                  TierArgs a = tier_args(t, il, ic, ol, oc);
                  a.steps = dwork ? d_steps : nullptr;
                  if (items) {
                      a.items = 1u;
                      a.item_owner = items->owner;
                      a.item_acc = items->acc;
                  }
                  if (level == 0 && kind == 2 && !dw) {
                      // deep tier 0: one request per grab after each lane's first (KETO_T0_NEXT=0: runs)
                      const char* en = getenv("KETO_T0_NEXT");
                      if (!(en && atoi(en) == 0)) {
                          if (!W.heads) {
                              uint64_t acc = 0;
                              W.heads = dmalloc<uint32_t>(KETO_HEAD_WORDS, acc);
                          }
                          HIP_OK(hipMemsetAsync(W.heads, 0, sizeof(uint32_t), st));
                          a.next = W.heads;
                      }
                  }
                  if (level < 2 && p.pool) {
                      const Tier& tn = W.tiers[level + 1];
                      a.pool = tn.vtab;
                      a.pool_mask = tn.cap - 1;
                      a.pool_n = level == 1 ? std::min<uint32_t>(tn.n_slots, 256) : tn.n_slots;
                      a.pool_epoch = tn.slot_epoch;
                      a.pool_busy = W.pool_busy + (level == 1 ? 0 : 8);
                  }
                  const uint32_t bs = std::min<uint32_t>(256, slots);
                  const dim3 grid(slots / bs), block(bs);
                  const keto_check_ids* q = dq;
                  if (ss && level == 1) {
                      // the streamed requests tier 0 handed up, in the handle form the next tiers read
                      hipLaunchKernelGGL(list_pairs_to_handles, dim3(1024), dim3(256), 0, st, ss->pairs, il, ic, ss->xlate,
                                         ss->depth, D.row_handle, S.n_rows());
                      HIP_OK(hipGetLastError());
                  }
                  if (ss && level >= 1) q = ss->xlate;
                  auto go = [&](auto kern) {
                      hipLaunchKernelGGL(kern, grid, block, 0, st, sv, dov, q, n, gmd, da, a, dwork);
                  };
                  const bool local = p.frames[level] == 0;
                  if (level == 0 && ss) {
                      a.pairs = ss->pairs;
                      a.ready = ss->ready;
                      a.chunk_log2 = ss->chunk_log2;
                      a.row_handle = D.row_handle;
                      a.n_rows = S.n_rows();
                      a.pair_depth = ss->depth;
                      a.misrouted = W.counters + 4;
                      a.stalled = ss->stalled;
                      a.wait_ticks = ss->wait_ticks;
                      a.dyn = t0_stream_dyn();
                      if (!W.heads) {
                          uint64_t acc = 0;
                          W.heads = dmalloc<uint32_t>(KETO_HEAD_WORDS, acc);
                      }
                      HIP_OK(hipMemsetAsync(W.heads, 0, KETO_HEAD_WORDS * sizeof(uint32_t), st));
                      a.heads = W.heads;
                      if (wide) go(check_wave_kernel_wide<4, true>);
                      else go(t0_stream_kernel());
                  }
                  else if (level == 0 && kind < 2) {
                      a.dyn = t0_dyn(n, slots);
                      if (const char* wc = getenv("KETO_T0_WALK"))
                          if (atoi(wc) > 0) a.walk_cap = (uint32_t)atoi(wc);
                      if (a.dyn) {
                          if (!W.heads) {
                              uint64_t acc = 0;
                              W.heads = dmalloc<uint32_t>(KETO_HEAD_WORDS, acc);
                          }
                          HIP_OK(hipMemsetAsync(W.heads, 0, KETO_HEAD_WORDS * sizeof(uint32_t), st));
                          a.heads = W.heads;
                      }
                      if (var == VAR_W8) go(check_wave_kernel_w8<4, 4, 16>);
                      else if (wide) kind == 0 ? go(check_wave_kernel_wide<4, false>) : go(check_wave_kernel_wide<8, false>);
                      else go(t0_kernel(var, dwork != nullptr));
                  }
                  else if (level == 0 && dw) {
                      // frames: the tier's GlobalStack area as [frame][lane] 8-B words (DF per lane)
                      // (a search holds at most gmd - 1 saved frames)
                      if ((uint64_t)t.gstack_n * 2 < (uint64_t)std::max(1, gmd - 1))
                          throw Error{KETO_E_RANGE, "deep frame area too small"};
                      // items (one long search can take 30K+ iterations): every work request dealt one at a
                      // time by the XCD heads, so no lane holds two long searches back to back
                      a.dyn = items ? 1u : getenv("KETO_T0_DYN_FORCE") ? t0_dyn(n, slots) : 0u;
                      if (a.dyn) {
                          if (!W.heads) {
                              uint64_t acc = 0;
                              W.heads = dmalloc<uint32_t>(KETO_HEAD_WORDS, acc);
                          }
                          HIP_OK(hipMemsetAsync(W.heads, 0, KETO_HEAD_WORDS * sizeof(uint32_t), st));
                          a.heads = W.heads;
                      }
                      dwork ? go(deep_wave_kernel<8, 8, true>) : go(deep_wave_kernel<8, 8, false>);
                  }
                  else if (level == 0)
                      dwork ? go(check_kernel<GlobalStack, true, 0>) : go(check_kernel<GlobalStack, false, 0>);
                  else if (level == 2)         // direct-indexed visited tables (DirectVisited)
                      dwork ? go(check_kernel<GlobalStack, true, 2>) : go(check_kernel<GlobalStack, false, 2>);
                  else if (local)
                      dwork ? go(check_kernel<LocalStack<16>, true, 1>) : go(check_kernel<LocalStack<16>, false, 1>);
                  else
                      dwork ? go(check_kernel<GlobalStack, true, 1>) : go(check_kernel<GlobalStack, false, 1>);
                  HIP_OK(hipGetLastError());
              },
              Undecided{da, nullptr, (uint8_t)KETO_UNDECIDED}, accumulate, stash);
    if (work_out) {
        unsigned long long h[2 * KETO_WORK_SLOTS];
        HIP_OK(hipMemcpyAsync(h, dwork, sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        for (int i = 0; i < KETO_WORK_SLOTS; ++i) work_out[i] = h[i];
        if (getenv("KETO_SIMT_PROF"))       // tier-0 SIMT profile (tooling): wave / lane counts
            fprintf(stderr, "simt: iter %llu/%llu work %llu/%llu walk %llu/%llu enter %llu/%llu\n", h[16], h[17],
                    h[18], h[19], h[20], h[21], h[22], h[23]);
    }
}

// The check of one device-resident batch.  Deep batches (max-depth > 9, the check_kernel tiers)
// first go through reach.hip: requests split into top-level items, items a hop-bounded reachability
// pretest proves false dropped, the rest checked as work requests and folded back per request.  A
// pipeline chunk (stash) of a deep batch is decided whole here, without the deferred stash.
void check_locked(Snapshot& S, DeviceState& D, const keto_check_ids* dq, uint32_t n, int32_t gmd, uint8_t* da,
                  hipStream_t st, const DevOverlay& dov, uint64_t* work_out, bool accumulate,
                  uint32_t* d_steps = nullptr, PipeStash* stash = nullptr, int wsi = 0) {
    const int32_t g = std::min<int32_t>(gmd, 65535);
    // (the reachability pretest's indexes hold target handles only, below 2^31 in every layout; the
    // split reads a request's row by hword, so split and wide arenas take it too)
    const bool deep = n > 0 && g - 1 > 8 && S.part_mode != PART_MIGRATE;
    ItemWork iw;
    if (!deep || !reach_split(S, dq, n, gmd, da, dov.base, st, d_steps != nullptr, iw)) {
        check_core(S, D, dq, n, gmd, da, st, dov, work_out, accumulate, d_steps, stash, wsi, nullptr);
        return;
    }
    if (stash) {
        // the chunk's tier timing events still bracket it (the caller reads them)
        hipEvent_t* e = stash->ev.data() + 3 * stash->chunk;
        HIP_OK(hipEventRecord(e[0], st));
        HIP_OK(hipEventRecord(e[1], st));
    }
    const keto_batch_timing before = D.last;
    check_core(S, D, iw.work, iw.n_work, gmd, iw.dec, st, dov, work_out, false, iw.wsteps, nullptr, wsi, &iw);
    keto_batch_timing T = D.last;
    uint32_t und = 0;
    if (d_steps) HIP_OK(hipMemsetAsync(d_steps, 0, (uint64_t)n * sizeof(uint32_t), st));
    reach_merge(S, iw, n, da, d_steps, st, &und);
    if (stash) HIP_OK(hipEventRecord(stash->ev[3 * stash->chunk + 2], st));
    T.undecided = und;
    T.items_ms = iw.split_ms;
    T.items = iw.n_entries;
    T.items_kept = iw.n_work;
    T.index_ms = iw.index_ms;
    if (accumulate) {
        // a pipeline chunk: the caller times the chunk's tiers from the stash events
        keto_batch_timing& L = D.last;
        L = before;
        if (!stash) {
            for (int i = 0; i < 3; ++i) {
                L.tier_ms[i] += T.tier_ms[i];
                L.requests[i] += T.requests[i];
            }
        } else {
            // the chunk's tiers 0 and 1 are timed by the stash events around this call; its work
            // requests that went up the tiers are counted here
            L.requests[1] += T.requests[1];
            L.requests[2] += T.requests[2];
            L.tier_ms[2] += T.tier_ms[2];
        }
        L.undecided += T.undecided;
        L.items_ms += T.items_ms;
        L.items += T.items;
        L.items_kept += T.items_kept;
        L.index_ms += T.index_ms;
    } else {
        D.last = T;
    }
}

// Requests naming rows by row id (as they travel between parts) -> row handles of this device.
// A top-level row another part owns becomes KETO_NO_ROW and is counted in *misrouted; a subject-set
// target that is another part's root row becomes KETO_NO_TARGET (no tuple has it as subject, so
// the reference answers false for it too).
__global__ void __launch_bounds__(256) rows_to_handles(const keto_check_ids* __restrict__ in, keto_check_ids* __restrict__ out,
                                                       uint32_t n, const uint32_t* __restrict__ table, uint32_t n_rows,
                                                       uint32_t* misrouted) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keto_check_ids q = in[i];
    if (q.row != KETO_NO_ROW) {
        const uint32_t h = q.row < n_rows ? table[q.row] : NO_UNIT;
        if (h == NO_UNIT) atomicAdd(misrouted, 1u);
        q.row = h == NO_UNIT ? KETO_NO_ROW : h;
    }
    if ((q.flags & 1u) && q.target != KETO_NO_TARGET) {
        const uint32_t h = q.target < n_rows ? table[q.target] : NO_UNIT;
        q.target = h == NO_UNIT ? KETO_NO_TARGET : h;
    }
    out[i] = q;
}

void translate_rows_locked(Snapshot& S, DeviceState& D, const keto_check_ids* d_reqs, keto_check_ids* d_out, uint32_t n,
                           hipStream_t st, uint32_t* d_bad) {
    uint64_t acc = 0;
    if (!D.row_handle) {
        // room for the rows writes add (device_apply patches the map while they fit)
        D.row_handle_cap = (uint64_t)S.n_rows() + S.n_rows() / 64 + 4096;
        D.row_handle_rows = S.n_rows();
        D.row_handle = dmalloc<uint32_t>(D.row_handle_cap, acc);
        HIP_OK(hipMemcpy(D.row_handle, S.unit_of_row.data(), (uint64_t)S.n_rows() * sizeof(uint32_t),
                         hipMemcpyHostToDevice));
        // the slack rows writes add stays NO_UNIT until device_apply patches it
        HIP_OK(hipMemset(D.row_handle + S.n_rows(), 0xFF, (D.row_handle_cap - S.n_rows()) * sizeof(uint32_t)));
    }
    if (n) {
        hipLaunchKernelGGL(rows_to_handles, dim3((n + 255) / 256), dim3(256), 0, st, d_reqs, d_out, n, D.row_handle,
                           S.n_rows(), d_bad);
        HIP_OK(hipGetLastError());
    }
}

// 8-B requests (row id, subject: bit31 = subject-set row id, else subject-id string id) -> the
// 16-B handle form, with the batch's request depth.  Misrouted rows are counted like above.
__global__ void __launch_bounds__(256) pairs_to_handles(const keto_check_pair* __restrict__ in, keto_check_ids* __restrict__ out,
                                                        uint32_t n, int32_t depth, const uint32_t* __restrict__ table,
                                                        uint32_t n_rows, uint32_t* misrouted) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const keto_check_pair p = in[i];
    keto_check_ids q{KETO_NO_ROW, KETO_NO_TARGET, 0u, depth};
    if (p.row != KETO_NO_ROW) {
        const uint32_t h = p.row < n_rows ? table[p.row] : NO_UNIT;
        if (h == NO_UNIT) atomicAdd(misrouted, 1u);
        q.row = h == NO_UNIT ? KETO_NO_ROW : h;
    }
    if (p.subject != KETO_NO_TARGET) {
        if (p.subject & EDGE_SET) {
            const uint32_t r = p.subject & EDGE_VAL;
            const uint32_t h = r < n_rows ? table[r] : NO_UNIT;
            q.target = h == NO_UNIT ? KETO_NO_TARGET : h;
            q.flags = 1u;
        } else {
            q.target = p.subject;
        }
    }
    out[i] = q;
}

void translate_pairs_locked(Snapshot& S, DeviceState& D, const keto_check_pair* d_reqs, keto_check_ids* d_out, uint32_t n,
                            int32_t depth, hipStream_t st, uint32_t* d_bad) {
    translate_rows_locked(S, D, nullptr, nullptr, 0, st, d_bad);          // the row -> handle table
    if (n) {
        hipLaunchKernelGGL(pairs_to_handles, dim3((n + 255) / 256), dim3(256), 0, st, d_reqs, d_out, n, depth,
                           D.row_handle, S.n_rows(), d_bad);
        HIP_OK(hipGetLastError());
    }
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

uint64_t chunk_requests() {
    const char* e = getenv("KETO_CHUNK");               // tuning / tests
    const long long v = e ? atoll(e) : (4ll << 20);
    return (uint64_t)std::max<long long>(256, v);
}
// the first chunk of a host batch: shorter, so the check starts after a shorter copy
uint64_t first_chunk_requests(uint64_t C) {
    const char* e = getenv("KETO_CHUNK_FIRST");         // tuning / tests
    const long long v = e ? atoll(e) : (long long)C;
    return (uint64_t)std::min<long long>((long long)C, std::max<long long>(256, v));
}

}  // namespace

void device_check(Snapshot& S, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed, void* stream,
                  uint64_t* work_out, uint32_t* d_steps) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    // NULL = the default stream, as the header says: ordered after the caller's default-stream work
    // that produced the inputs (the snapshot's own stream is non-blocking and would not be)
    hipStream_t st = (hipStream_t)stream;
    check_locked(S, D, d_reqs, n, gmd, d_allowed, st, DevOverlay{nullptr, 0xFFFFFFFFu}, work_out, false, d_steps);
}

namespace {

// Streamed host batches: FORM_PAIRS from pinned memory, no overlay, max-depth <= 5, at least
// KETO_STREAM_MIN requests (default 1M); KETO_STREAM=0 turns it off
bool stream_ok(const Snapshot& S, uint32_t n, int32_t gmd, const Overlay* ovh) {
    const char* e = getenv("KETO_STREAM");
    if (e && atoi(e) == 0) return false;
    const char* m = getenv("KETO_STREAM_MIN");
    const uint64_t lo = m ? strtoull(m, nullptr, 10) : (1ull << 20);
    return n >= std::max<uint64_t>(lo, 1) && !(ovh && !ovh->empty()) && std::max(1, std::min(gmd, 65535) - 1) <= 4 &&
           S.part_mode != PART_MIGRATE;
}

// One tier-0 launch over the whole host batch, started before the requests have landed: the copy
// stream moves chunks of 2^KETO_STREAM_CHUNK_LOG2 pairs (default 2^20 = 8 MB) in and marks each
// landed with hipStreamWriteValue32; the kernel deals runs in batch order, waits for a run's chunk
// and turns row ids into handles itself (P_XLT).  The chunked pipeline below pays a launch tail
// and a translation pass per chunk (4 launches summed to 3.5 ms against 2.6 ms for one,
// DESIGN.md "Measurement").  Returns false, with nothing decided, if a lane waited longer than
// KETO_STREAM_WAIT_MS (default 1000) for a chunk: the caller then runs the chunked pipeline.
bool check_streamed(Snapshot& S, DeviceState& D, const keto_check_pair* reqs, uint32_t n, int32_t gmd, uint8_t* allowed,
                    int32_t depth) {
    uint64_t acc = 0;
    const char* ec = getenv("KETO_STREAM_CHUNK_LOG2");
    const uint32_t cl = (uint32_t)std::min(26, std::max(16, ec ? atoi(ec) : 20));
    const uint64_t chunks = ((uint64_t)n + (1ull << cl) - 1) >> cl;
    if (D.st_cap < n) {
        for (void* p : {(void*)D.st_pairs, (void*)D.st_dec, (void*)D.st_x, (void*)D.st_ready})
            if (p) (void)hipFree(p);
        D.st_pairs = nullptr;
        D.st_dec = nullptr;
        D.st_x = nullptr;
        D.st_ready = nullptr;
        D.st_cap = 0;
        D.st_pairs = dmalloc<keto_check_pair>((uint64_t)n + 4, acc);       // + the pair a 16-B load reads past an odd end
        D.st_dec = dmalloc<uint8_t>(((uint64_t)n + 3) & ~3ull, acc);
        D.st_x = dmalloc<keto_check_ids>(n, acc);
        D.st_ready = dmalloc<uint32_t>(((uint64_t)n >> 16) + 2, acc);
        D.st_cap = n;
    }
    WorkSet& W = D.ws[0];
    ensure_lists(W, n);
    uint32_t* d_bad = W.counters + 4;                                         // [4] misrouted, [5] stalled
    translate_rows_locked(S, D, nullptr, nullptr, 0, D.stream, d_bad);      // the row -> handle table
    HIP_OK(hipMemsetAsync(W.counters + 4, 0, 2 * sizeof(uint32_t), D.stream));
    HIP_OK(hipMemsetAsync(D.st_ready, 0, chunks * sizeof(uint32_t), D.stream));
    HIP_OK(hipEventRecord(D.pev[6], D.stream));
    HIP_OK(hipStreamWaitEvent(D.copy_in, D.pev[6], 0));
    const bool drop = getenv("KETO_STREAM_TEST_DROP") != nullptr;           // test hook: the last chunk is never marked
    for (uint64_t c = 0; c < chunks; ++c) {
        const uint64_t lo = c << cl, len = std::min<uint64_t>(n, lo + (1ull << cl)) - lo;
        HIP_OK(hipMemcpyAsync(D.st_pairs + lo, reqs + lo, len * sizeof(keto_check_pair), hipMemcpyHostToDevice, D.copy_in));
        if (!(drop && c + 1 == chunks)) HIP_OK(hipStreamWriteValue32(D.copy_in, D.st_ready + c, 1u, 0));
    }
    const char* ew = getenv("KETO_STREAM_WAIT_MS");
    StreamSrc ss;
    ss.pairs = D.st_pairs;
    ss.ready = D.st_ready;
    ss.chunk_log2 = cl;
    ss.depth = depth;
    ss.stalled = W.counters + 5;
    ss.wait_ticks = (uint64_t)std::max(1, ew ? atoi(ew) : 1000) * 100000ull;   // wall clock: 100 MHz
    ss.xlate = D.st_x;
    check_core(S, D, nullptr, n, gmd, D.st_dec, D.stream, DevOverlay{nullptr, 0xFFFFFFFFu}, nullptr, false, nullptr,
               nullptr, 0, nullptr, &ss);
    // the decisions and the two flags come back behind the check in one round trip; a stalled or
    // misrouted batch discards what was copied
    uint32_t flags[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(flags, W.counters + 4, sizeof(flags), hipMemcpyDeviceToHost, D.stream));
    HIP_OK(hipMemcpyAsync(allowed, D.st_dec, n, hipMemcpyDeviceToHost, D.stream));
    HIP_OK(hipStreamSynchronize(D.stream));
    HIP_OK(hipStreamSynchronize(D.copy_in));
    D.last.stream_stalls = flags[1];
    if (flags[1]) return false;
    if (flags[0]) throw Error{KETO_E_INVALID, std::to_string(flags[0]) + " requests name root rows another part owns"};
    D.last.chunks = (uint32_t)chunks;
    return true;
}

}  // namespace

// Host-buffer batches: the requests go to the device in chunks of KETO_CHUNK (default 4M), so the
// H2D copy of chunk c + 1 (copy_in stream) and the D2H copy of chunk c - 1 (copy_out) overlap the
// check of chunk c (the check stream).  Two device slots alternate.  Pinned caller buffers
// (keto_host_alloc / hipHostRegister) are copied directly; pageable ones through pinned staging.
// form: FORM_HANDLES (keto_check_ids with handles), FORM_ROWS (keto_check_ids naming rows by row
// id, translated on the device) or FORM_PAIRS (8-B keto_check_pair by row id, one request depth for
// the batch, expanded and translated on the device).
void device_check_host(Snapshot& S, const void* reqs_v, uint32_t n, int32_t gmd, uint8_t* allowed, int form,
                       int32_t pair_depth, const Overlay* ovh) {
    const uint64_t esz = form == FORM_PAIRS ? sizeof(keto_check_pair) : sizeof(keto_check_ids);
    const uint8_t* reqs = static_cast<const uint8_t*>(reqs_v);
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    const auto t_start = std::chrono::steady_clock::now();
    D.last = keto_batch_timing{};
    if (n == 0) return;
    if (form == FORM_PAIRS && stream_ok(S, n, gmd, ovh) && host_pinned(reqs) && host_pinned(allowed)) {
        if (check_streamed(S, D, reinterpret_cast<const keto_check_pair*>(reqs), n, gmd, allowed, pair_depth)) {
            D.last.wall_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count();
            D.last.streamed = 1;
            return;
        }
        const uint32_t stalls = D.last.stream_stalls;
        D.last = keto_batch_timing{};                    // a chunk did not land in time: the pipeline below
        D.last.stream_stalls = stalls;
        D.last.stream_fallbacks = 1;
    }
    OverlayBuf ov(S, ovh);
    const uint64_t C = std::min<uint64_t>(n, chunk_requests());
    const uint64_t C0 = first_chunk_requests(C);        // chunk 0; then chunks of C
    const uint32_t chunks = 1u + (uint32_t)((n - std::min<uint64_t>(n, C0) + C - 1) / C);
    uint64_t acc = 0;
    if (D.slot_cap < C) {
        for (int i = 0; i < 2; ++i) {
            if (D.slot_q[i]) (void)hipFree(D.slot_q[i]);
            if (D.slot_x[i]) (void)hipFree(D.slot_x[i]);
            if (D.slot_a[i]) (void)hipFree(D.slot_a[i]);
            D.slot_q[i] = D.slot_x[i] = nullptr;
            D.slot_a[i] = nullptr;
        }
        D.slot_cap = 0;
        for (int i = 0; i < 2; ++i) {
            D.slot_q[i] = dmalloc<keto_check_ids>(C, acc);
            D.slot_x[i] = dmalloc<keto_check_ids>(C, acc);
            D.slot_a[i] = dmalloc<uint8_t>((C + 3) & ~3ull, acc);
        }
        D.slot_cap = C;
    }
    const bool pinned = host_pinned(reqs) && host_pinned(allowed);
    if (!pinned && D.pin_cap < C) {
        for (int i = 0; i < 2; ++i) {
            if (D.pin_q[i]) (void)hipHostFree(D.pin_q[i]);
            if (D.pin_a[i]) (void)hipHostFree(D.pin_a[i]);
            D.pin_q[i] = nullptr;
            D.pin_a[i] = nullptr;
        }
        D.pin_cap = 0;
        for (int i = 0; i < 2; ++i) {
            HIP_OK(hipHostMalloc((void**)&D.pin_q[i], C * sizeof(keto_check_ids), hipHostMallocDefault));
            HIP_OK(hipHostMalloc((void**)&D.pin_a[i], C, hipHostMallocDefault));
        }
        D.pin_cap = C;
    }
    ensure_lists(D.ws[0], C);
    hipEvent_t* in_done = D.pev;
    hipEvent_t* kern_done = D.pev + 2;
    hipEvent_t* out_done = D.pev + 4;
    ensure_lists(D.ws[1], C);
    uint32_t* d_bad = D.ws[0].counters + 4;
    HIP_OK(hipMemsetAsync(d_bad, 0, sizeof(uint32_t), D.copy_in));     // the translations run on copy_in
    // requests that overflow tier 1 are stashed and decided after the last chunk (PipeStash)
    if (D.ps_cap < n) {
        if (D.ps_q) (void)hipFree(D.ps_q);
        if (D.ps_idx) (void)hipFree(D.ps_idx);
        D.ps_q = nullptr;
        D.ps_idx = nullptr;
        D.ps_cap = 0;
        D.ps_q = dmalloc<keto_check_ids>(n, acc);
        D.ps_idx = dmalloc<uint32_t>(n, acc);
        D.ps_cap = n;
    }
    if (!D.ps_count) D.ps_count = dmalloc<uint32_t>(2, acc);
    while (D.ps_ev.size() < 3ull * chunks) {
        hipEvent_t e;
        HIP_OK(hipEventCreate(&e));
        D.ps_ev.push_back(e);
    }
    HIP_OK(hipMemsetAsync(D.ps_count, 0, 2 * sizeof(uint32_t), D.stream));
    // KETO_PIPE_STREAMS=2: consecutive chunks check on two compute streams with their own workspaces
    // (ws[0], ws[1]), so that a chunk's check could start while the previous one drains its tail.
    // Measured no faster (4.64-4.77 vs 4.59 ms per 16.7M batch, profiles/r02aq_pipe_streams.log):
    // one stream stays the default
    const char* eps = getenv("KETO_PIPE_STREAMS");
    const bool two = eps && atoi(eps) == 2;
    if (two && !D.stream2) HIP_OK(hipStreamCreateWithFlags(&D.stream2, hipStreamNonBlocking));
    hipEvent_t setup_done = D.pev[6];
    HIP_OK(hipEventRecord(setup_done, D.stream));
    if (two) HIP_OK(hipStreamWaitEvent(D.stream2, setup_done, 0));
    PipeStash ps;
    ps.q = D.ps_q;
    ps.idx = D.ps_idx;
    ps.count = D.ps_count;
    ps.cap = D.ps_cap;
    ps.ev = D.ps_ev;
    auto lo = [&](uint32_t c) { return c == 0 ? 0 : std::min<uint64_t>(n, C0 + (uint64_t)(c - 1) * C); };
    auto len = [&](uint32_t c) { return (uint32_t)(std::min<uint64_t>(n, c == 0 ? C0 : lo(c) + C) - lo(c)); };
    // stage chunk c's requests and enqueue its H2D into slot c % 2 (slot reuse waits for chunk
    // c - 2's check, which read it, through kern_done)
    auto put = [&](uint32_t c) {
        const int k = c & 1;
        if (c >= 2) HIP_OK(hipStreamWaitEvent(D.copy_in, kern_done[k], 0));
        const uint8_t* src = reqs + lo(c) * esz;
        if (!pinned) {
            if (c >= 2) HIP_OK(hipEventSynchronize(in_done[k]));   // staging k free again
            uint8_t* dst = reinterpret_cast<uint8_t*>(D.pin_q[k]);
            const uint64_t bytes = (uint64_t)len(c) * esz, part = 1 << 20;
            host_parallel_for((bytes + part - 1) / part, [&](uint64_t i) {
                std::memcpy(dst + i * part, src + i * part, std::min(part, bytes - i * part));
            });
            src = dst;
        }
        HIP_OK(hipMemcpyAsync(D.slot_q[k], src, (uint64_t)len(c) * esz, hipMemcpyHostToDevice, D.copy_in));
        // row ids -> handles right behind the copy, on the copy stream: it runs beside the check of
        // the chunk before (in its tail) instead of between the two checks
        if (form == FORM_ROWS)
            translate_rows_locked(S, D, D.slot_q[k], D.slot_x[k], len(c), D.copy_in, d_bad);
        else if (form == FORM_PAIRS)
            translate_pairs_locked(S, D, reinterpret_cast<const keto_check_pair*>(D.slot_q[k]), D.slot_x[k], len(c),
                                   pair_depth, D.copy_in, d_bad);
        HIP_OK(hipEventRecord(in_done[k], D.copy_in));
    };
    // bring chunk c's decisions home (pageable: via staging, copied out once the D2H is done)
    auto drain = [&](uint32_t c) {
        const int k = c & 1;
        if (!pinned) {
            HIP_OK(hipEventSynchronize(out_done[k]));
            std::memcpy(allowed + lo(c), D.pin_a[k], len(c));
        }
    };
    put(0);
    for (uint32_t c = 0; c < chunks; ++c) {
        const int k = c & 1;
        const int wsi = two ? k : 0;
        hipStream_t cs = wsi ? D.stream2 : D.stream;
        if (c + 1 < chunks) put(c + 1);
        HIP_OK(hipStreamWaitEvent(cs, in_done[k], 0));
        if (c >= 2) HIP_OK(hipStreamWaitEvent(cs, out_done[k], 0));   // slot_a[k] drained
        const keto_check_ids* dq = form == FORM_HANDLES ? D.slot_q[k] : D.slot_x[k];   // translated on copy_in
        ps.base = (uint32_t)lo(c);
        ps.dq = dq;
        ps.chunk = c;
        check_locked(S, D, dq, len(c), gmd, D.slot_a[k], cs, ov.v, nullptr, true, nullptr, &ps, wsi);
        HIP_OK(hipEventRecord(kern_done[k], cs));
        HIP_OK(hipStreamWaitEvent(D.copy_out, kern_done[k], 0));
        if (!pinned && c >= 2) drain(c - 2);
        // decisions come home by a copy: the checks storing them straight into a pinned caller buffer
        // (scattered 4-B writes over PCIe) took 10-11 ms per batch instead of 3.5
        // (profiles/r03f_e2e_zerocopy_rejected.log)
        HIP_OK(hipMemcpyAsync(pinned ? allowed + lo(c) : D.pin_a[k], D.slot_a[k], len(c), hipMemcpyDeviceToHost,
                              D.copy_out));
        HIP_OK(hipEventRecord(out_done[k], D.copy_out));
    }
    for (uint32_t c = chunks >= 2 ? chunks - 2 : 0; c < chunks; ++c)
        if (!pinned) drain(c);
    HIP_OK(hipStreamSynchronize(D.copy_out));
    uint32_t bad = 0;
    if (form != FORM_HANDLES) {
        HIP_OK(hipMemcpyAsync(&bad, d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost, D.stream));
        HIP_OK(hipStreamSynchronize(D.stream));
    }
    // timing of the chunks' tiers 0 and 1, and the stash
    uint32_t pc[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(pc, D.ps_count, sizeof(pc), hipMemcpyDeviceToHost, D.stream));
    HIP_OK(hipStreamSynchronize(D.stream));
    D.last.requests[0] = n;
    D.last.requests[1] += pc[1];
    for (uint32_t c = 0; c < chunks; ++c) {
        float a = 0, b = 0;
        HIP_OK(hipEventElapsedTime(&a, D.ps_ev[3 * c], D.ps_ev[3 * c + 1]));
        HIP_OK(hipEventElapsedTime(&b, D.ps_ev[3 * c + 1], D.ps_ev[3 * c + 2]));
        D.last.tier_ms[0] += a;
        D.last.tier_ms[1] += b;
    }
    if (pc[0] && !bad) {
        // the stashed tier-1 overflows: one full check of them (tier 2, then per-request UNDECIDED),
        // and their decisions written over the ones the chunks left
        const uint32_t m = (uint32_t)std::min<uint64_t>(pc[0], D.ps_cap);
        const keto_batch_timing before = D.last;
        uint8_t* d_dec = nullptr;
        HIP_OK(hipMalloc(&d_dec, m));
        check_locked(S, D, D.ps_q, m, gmd, d_dec, D.stream, ov.v, nullptr, false);
        const keto_batch_timing stash_t = D.last;
        std::vector<uint8_t> dec(m);
        std::vector<uint32_t> idx(m);
        HIP_OK(hipMemcpyAsync(dec.data(), d_dec, m, hipMemcpyDeviceToHost, D.stream));
        HIP_OK(hipMemcpyAsync(idx.data(), D.ps_idx, m * sizeof(uint32_t), hipMemcpyDeviceToHost, D.stream));
        HIP_OK(hipStreamSynchronize(D.stream));
        (void)hipFree(d_dec);
        for (uint32_t i = 0; i < m; ++i) allowed[idx[i]] = dec[i];
        D.last = before;
        D.last.requests[2] += stash_t.requests[2];
        D.last.tier_ms[2] += stash_t.tier_ms[0] + stash_t.tier_ms[1] + stash_t.tier_ms[2];
        D.last.undecided += stash_t.undecided;
    }
    D.last.chunks = chunks;
    D.last.wall_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (bad) throw Error{KETO_E_INVALID, std::to_string(bad) + " requests name root rows another part owns"};
}

void* host_alloc(uint64_t bytes) {
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, std::max<uint64_t>(bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e)};
    return p;
}

void host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

void device_check_rows(Snapshot& S, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed,
                       void* stream, bool rows_valid) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    // NULL = the default stream, as the header says: ordered after the caller's default-stream work
    // that produced the inputs (the snapshot's own stream is non-blocking and would not be)
    hipStream_t st = (hipStream_t)stream;
    // the lock is held from the translation through the check: D.xlate is shared by all callers
    lock_trace("rows: waiting for D.mu");
    std::lock_guard<std::mutex> lk(D.mu);
    lock_trace("rows: D.mu");
    HIP_OK(hipSetDevice(D.device));
    uint64_t acc = 0;
    if (D.xlate_cap < n) {
        if (D.xlate) (void)hipFree(D.xlate);
        D.xlate = nullptr;
        D.xlate_cap = 0;
        D.xlate = dmalloc<keto_check_ids>(std::max<uint64_t>(n, 1024), acc);
        D.xlate_cap = std::max<uint64_t>(n, 1024);
    }
    ensure_lists(D.ws[0], n);
    HIP_OK(hipMemsetAsync(D.ws[0].counters + 4, 0, sizeof(uint32_t), st));
    translate_rows_locked(S, D, d_reqs, D.xlate, n, st, D.ws[0].counters + 4);
    if (!rows_valid) {
        uint32_t bad = 0;
        HIP_OK(hipMemcpyAsync(&bad, D.ws[0].counters + 4, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (bad) throw Error{KETO_E_INVALID, std::to_string(bad) + " requests name root rows another part owns"};
    }
    lock_trace("rows: translated");
    check_locked(S, D, D.xlate, n, gmd, d_allowed, st, DevOverlay{nullptr, 0xFFFFFFFFu}, nullptr, false);
    lock_trace("rows: check launched");
}

// A batch of requests in the handle form checked without a host round trip (the packed path's
// batches in flight, resolve_dev.hip): under the device lock, only enqueued -- on one of the
// ASYNC_STREAMS check streams in turn, after `ready`: tier 0 on that stream's workspace (ws[2 + k]),
// then t0_tail writes tier 0's overflow count to d_counts[0] and `done` is recorded.  Other batches'
// uploads, resolutions and checks run meanwhile on their own streams, and this call returns before
// the check ends.  A batch with d_counts[0] > 0 needs the next tiers and is checked again by the
// caller through device_check_rows.  Deep batches (max-depth > 9) and partitioned snapshots are not
// taken: false.
bool device_check_rows_async(Snapshot& S, const keto_check_ids* d_handles, uint32_t n, int32_t gmd,
                             uint8_t* d_allowed, uint32_t* d_counts, void* ready_event, void* done_event) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    hipEvent_t ready = (hipEvent_t)ready_event, done = (hipEvent_t)done_event;
    if (std::max(1, std::min<int32_t>(gmd, 65535) - 1) > 8 || S.n_parts != 1) return false;
    DeviceState& D = *S.dev;
    lock_trace("rows async: waiting for D.mu");
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    const uint32_t k = D.anext++ % ASYNC_STREAMS;
    WorkSet& W = D.ws[2 + k];
    if (!D.astream[k]) {
        HIP_OK(hipStreamCreateWithFlags(&D.astream[k], hipStreamNonBlocking));
        ensure_lists(W, n);
        HIP_OK(hipMemset(W.counters, 0, 8 * sizeof(uint32_t)));      // t0_tail keeps them zero after each batch
    }
    hipStream_t st = D.astream[k];
    if (n > D.amax[k]) {
        // a larger batch grows the workspace (its lists and tier tables are freed and allocated
        // again): the stream's earlier checks must be done with them
        HIP_OK(hipStreamSynchronize(st));
        D.amax[k] = n;
    }
    HIP_OK(hipStreamWaitEvent(st, ready, 0));
    PipeStash ps;
    ps.t0_only = true;
    ps.count = d_counts;
    ps.dq = d_handles;
    const keto_batch_timing before = D.last;
    check_locked(S, D, d_handles, n, gmd, d_allowed, st, DevOverlay{nullptr, 0xFFFFFFFFu}, nullptr, true, nullptr, &ps,
                 2 + (int)k);
    D.last = before;
    D.last.requests[0] = n;
    HIP_OK(hipEventRecord(done, st));
    lock_trace("rows async: enqueued");
    return true;
}

// The row id -> handle map on the device (built on first use; a write patches it under the
// exclusive lock): the packed path's resolution writes handles with it.  Call with the snapshot lock
// held shared; the map stays valid until it is released.
const uint32_t* device_row_handle_map(Snapshot& S) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    translate_rows_locked(S, D, nullptr, nullptr, 0, nullptr, nullptr);
    return D.row_handle;
}

// Expand output: set nodes carry row handles; map them to row ids on the device (binary search in
// the arena-order handle list; overlay handles >= ov_units_base are left for the host).
// the direct handle -> row map: every row header's unit gets its row (other units are never looked up)
__global__ void __launch_bounds__(256) scatter_unit_rows(uint32_t* __restrict__ unit_row, const uint32_t* __restrict__ units,
                                                         const uint32_t* __restrict__ rows, uint32_t n, uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && units[i] < cap) unit_row[units[i]] = rows[i];
}
__global__ void __launch_bounds__(256) handles_to_rows_direct(keto_tree_node* __restrict__ nodes, uint64_t n,
                                                              const uint32_t* __restrict__ unit_row, uint32_t ov_units_base) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = nodes[i].subject;
    if (!(x & EDGE_SET)) return;
    const uint32_t h = x & EDGE_VAL;
    if (h >= ov_units_base) return;
    nodes[i].subject = EDGE_SET | unit_row[h];
}
// the same over the trees a fill pass wrote at their offsets (ranges[2r], ranges[2r + 1] = first node,
// end): a wave per range
__global__ void __launch_bounds__(256) handles_to_rows_ranges(keto_tree_node* __restrict__ nodes,
                                                              const uint64_t* __restrict__ ranges, uint32_t n_ranges,
                                                              const uint32_t* __restrict__ unit_row, uint32_t ov_units_base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_ranges; r += waves) {
        const uint64_t b = ranges[2 * r], e = ranges[2 * r + 1];
        for (uint64_t i = b + lane; i < e; i += 64) {
            const uint32_t x = nodes[i].subject;
            if ((x & EDGE_SET) && (x & EDGE_VAL) < ov_units_base) nodes[i].subject = EDGE_SET | unit_row[x & EDGE_VAL];
        }
    }
}
__global__ void __launch_bounds__(256) handles_to_rows(keto_tree_node* __restrict__ nodes, uint64_t n,
                                                       const uint32_t* __restrict__ units, const uint32_t* __restrict__ rows,
                                                       uint32_t n_rows, uint32_t ov_units_base) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = nodes[i].subject;
    if (!(x & EDGE_SET)) return;
    const uint32_t h = x & EDGE_VAL;
    if (h >= ov_units_base) return;
    uint32_t lo = 0, hi = n_rows;                  // first unit >= h
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (units[m] < h) lo = m + 1;
        else hi = m;
    }
    nodes[i].subject = EDGE_SET | rows[lo];
}

// ---- the pinned block pool behind PinnedAlloc (snapshot.hpp); never destroyed, so an arena freed
// late in process exit still finds it
namespace {
struct PinPool {
    std::mutex mu;
    std::multimap<size_t, void*> idle;                              // idle blocks by size
    std::unordered_map<void*, std::pair<size_t, bool>> live;        // block -> (size, page-locked)
    size_t idle_bytes = 0;
};
PinPool& pin_pool() {
    static PinPool* p = new PinPool;
    return *p;
}
constexpr size_t PIN_IDLE_MAX = 1ull << 30;                         // idle pinned bytes kept for reuse
}  // namespace

void* pinned_take(size_t bytes) {
    PinPool& P = pin_pool();
    if (bytes == 0) bytes = 1;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.idle.lower_bound(bytes);
        if (it != P.idle.end() && it->first <= 2 * bytes + (1u << 20)) {   // not much bigger than asked
            void* p = it->second;
            P.idle_bytes -= it->first;
            P.idle.erase(it);
            return p;
        }
    }
    const size_t sz = (bytes + 4095) & ~(size_t)4095;
    void* p = nullptr;
    const bool pinned = hipHostMalloc(&p, sz, hipHostMallocDefault) == hipSuccess && p;
    if (!pinned) {
        (void)hipGetLastError();
        p = malloc(sz);
        if (!p) throw std::bad_alloc();
    }
    std::lock_guard<std::mutex> lk(P.mu);
    P.live[p] = {sz, pinned};
    return p;
}

void pinned_give(void* p) noexcept {
    if (!p) return;
    PinPool& P = pin_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.live.find(p);
    if (it == P.live.end()) return;
    const size_t sz = it->second.first;
    if (!it->second.second) {
        P.live.erase(it);
        free(p);
        return;
    }
    if (P.idle_bytes + sz <= PIN_IDLE_MAX) {      // keep it (still in `live`) for the next arena
        P.idle.emplace(sz, p);
        P.idle_bytes += sz;
        return;
    }
    P.live.erase(it);
    (void)hipHostFree(p);
}

void device_expand(Snapshot& S, const std::vector<uint32_t>& root_in, const std::vector<uint32_t>& root_flags,
                   const std::vector<uint32_t>& root_vid_in, const std::vector<int32_t>& depth, int32_t gmd,
                   const Overlay* ovh, ExpandResult& out,
                   const std::vector<std::pair<uint32_t, uint32_t>>* remote_roots,
                   const std::vector<uint32_t>* root_rows) {
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    if (S.n_units > (uint64_t)EDGE_VAL && (!root_rows || root_rows->size() != root_in.size()))
        throw Error{KETO_E_INVALID, "expand over an arena whose roots lie past 2^31 units needs the roots' row ids"};
    // a migrating part holds its own rows and stubs for the others' rows it points at: the rows a
    // tree needs from other parts are copied into the call's overlay (PullSet) from the host tables,
    // which every part holds whole
    const bool pulls = S.part_mode == PART_MIGRATE && S.n_parts > 1;
    std::unique_ptr<PullSet> ps;
    std::vector<uint32_t> root_m, vid_m;
    if (pulls) {
        ps = std::make_unique<PullSet>(S, ovh);
        root_m = root_in;
        vid_m = root_vid_in;
        if (remote_roots)
            for (const auto& rr : *remote_roots) {
                root_m[rr.first] = ps->identity(rr.second);
                vid_m[rr.first] = ps->vid(rr.second);
                ps->add(rr.second);
            }
    } else if (remote_roots && !remote_roots->empty()) {
        throw Error{KETO_E_INVALID, "expand root is owned by another part"};
    }
    const std::vector<uint32_t>& root = pulls ? root_m : root_in;
    const std::vector<uint32_t>& root_vid = pulls ? vid_m : root_vid_in;
    DeviceState& D = *S.dev;
    std::lock_guard<std::mutex> lk(D.mu);
    HIP_OK(hipSetDevice(D.device));
    const uint32_t n = (uint32_t)root.size();
    out.status.assign(n, EXP_NIL);
    out.offset.assign(n + 1, 0);
    out.nodes.clear();
    if (n == 0) return;
    if (gmd > 65535) gmd = 65535;
    hipStream_t st = D.stream;
    // KETO_EXPAND_TRACE=1: phase times on stderr (tooling)
    const bool trace = getenv("KETO_EXPAND_TRACE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace) return;
        (void)hipStreamSynchronize(st);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[expand] %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    OverlayBuf ov(S, pulls ? nullptr : ovh);          // (a migrating part: the PullSet's overlay)
    uint64_t acc = 0;
    // workspace, reused across calls: requests | counts (n + 1) | offsets (n + 1) | stage positions
    // (n) | statuses
    const uint64_t need = (uint64_t)n * sizeof(ExpandReq) + 3ull * (n + 1) * sizeof(uint64_t) + n + 64;
    if (D.ex_cap < need) {
        if (D.ex_buf) (void)hipFree(D.ex_buf);
        D.ex_cap = std::max<uint64_t>(need, 1 << 20);
        D.ex_buf = dmalloc<uint8_t>(D.ex_cap, acc);
    }
    uint8_t* base = (uint8_t*)D.ex_buf;
    uint64_t* dcount = reinterpret_cast<uint64_t*>(base);
    uint64_t* doff = dcount + (n + 1);
    uint64_t* dstage = doff + (n + 1);
    ExpandReq* dq = reinterpret_cast<ExpandReq*>(dstage + (n + 1));
    uint8_t* dstatus = reinterpret_cast<uint8_t*>(dq + n);
    {
        std::vector<ExpandReq> hq(n);
        for (uint32_t i = 0; i < n; ++i) hq[i] = ExpandReq{root[i], root_flags[i], root_vid[i], depth[i]};
        HIP_OK(hipMemcpyAsync(dq, hq.data(), n * sizeof(ExpandReq), hipMemcpyHostToDevice, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    lap("h2d");
    Plan p = make_plan(D, n, gmd);            // expand holds at most gmd frames
    DevSnap sv = D.view();
    DevOverlay dov = ov.v;
    // One pass (default): tier 0 writes every tree into its lane's staging region while it counts it;
    // the host scans the counts; a wave per root copies the staged trees to their offsets.  Trees that
    // did not fit (or that a later tier decided, counting only) are filled by a second pass over just
    // them.  KETO_EXPAND_STAGE=0: count pass + fill pass over every root (the two-pass form); =N > 1:
    // N nodes of staging per lane.
    const char* se = getenv("KETO_EXPAND_STAGE");
    const bool staged = !se || atoi(se) != 0;
    uint64_t stage_cap = 0, ovf_chunk = 0, ovf_cap = 0, ovf_base = 0;
    if (staged) {
        // staging nodes: KETO_EXPAND_STAGE_MB (default 1024 MB).  Bigger regions let fewer trees
        // spill to the second pass, but the lanes' regions then lie far apart and the copies into and
        // out of them miss the TLB page by page: the gather of config #5's 100k staged trees took
        // 34 us from 4 GiB of regions, 143 us from 8 GiB and 298 us from 16 GiB
        const char* sg = getenv("KETO_EXPAND_STAGE_MB");
        const uint64_t budget = (sg ? (uint64_t)std::max(16, atoi(sg)) : 1024ull) << 17;
        stage_cap = std::min<uint64_t>(16384, std::max<uint64_t>(64, budget / p.slots[0]));
        if (se && atoi(se) > 1) stage_cap = (uint64_t)atoi(se);            // tests: small regions spill
        // a tree past its region goes on in an overflow chunk of KETO_EXPAND_OVF_CHUNK nodes (default
        // 256K) from a pool of KETO_EXPAND_OVF_NODES (default a quarter of the regions' nodes, at
        // least 4 chunks, at most 32M nodes = 256 MB; 0: none, such trees are filled by the second pass)
        const char* oc = getenv("KETO_EXPAND_OVF_CHUNK");
        const char* on = getenv("KETO_EXPAND_OVF_NODES");
        ovf_chunk = oc ? (uint64_t)std::max(1, atoi(oc)) : 262144ull;
        ovf_cap = on ? (uint64_t)std::max(0ll, atoll(on))
                     : std::min<uint64_t>(32ull << 20, std::max<uint64_t>(4 * ovf_chunk, stage_cap * p.slots[0] / 4));
        ovf_cap -= ovf_cap % ovf_chunk;
        ovf_base = stage_cap * p.slots[0];
        const uint64_t nodes = ovf_base + ovf_cap;
        if (D.ex_stage_nodes < nodes) {
            if (D.ex_stage) (void)hipFree(D.ex_stage);
            D.ex_stage = nullptr;
            D.ex_stage_nodes = 0;
            D.ex_stage = dmalloc<keto_tree_node>(nodes, acc);
            D.ex_stage_nodes = nodes;
        }
        const uint32_t seg_cap = (uint32_t)(ovf_cap / ovf_chunk) + 1;
        if (D.ex_seg_cap < seg_cap) {
            if (D.ex_seg) (void)hipFree(D.ex_seg);
            D.ex_seg = nullptr;
            D.ex_seg_cap = 0;
            D.ex_seg = dmalloc<uint8_t>(16 + (uint64_t)seg_cap * sizeof(StageSeg), acc);
            D.ex_seg_cap = seg_cap;
        }
        HIP_OK(hipMemsetAsync(D.ex_seg, 0, 16, st));
    }
    // the id-run queues of tier 0's lanes (RUNS_PER_LANE entries each) | runs queued per lane
    const char* ri = getenv("KETO_EXPAND_RUN_INLINE");
    const uint32_t run_inline = ri ? (uint32_t)atoi(ri) : RUN_INLINE_DEFAULT;
    if (D.ex_runs_cap < p.slots[0]) {
        if (D.ex_runs) (void)hipFree(D.ex_runs);
        D.ex_runs = nullptr;
        D.ex_runs_cap = 0;
        D.ex_runs = reinterpret_cast<CopyRun*>(
            dmalloc<uint8_t>((uint64_t)p.slots[0] * (RUNS_PER_LANE * sizeof(CopyRun) + sizeof(uint32_t)), acc));
        D.ex_runs_cap = p.slots[0];
    }
    uint32_t* d_lane_runs = reinterpret_cast<uint32_t*>(D.ex_runs + (uint64_t)D.ex_runs_cap * RUNS_PER_LANE);
    // the big-run pieces: a run of L > BIG_RUN ids takes ceil(L / BIG_RUN) < 2 L / BIG_RUN pieces, so
    // 2 nodes / BIG_RUN bounds a pass, plus slack for roots that overflowed tier 0 part way (their
    // pieces are queued again); a queue that is full anyway copies the run in place
    auto ensure_big = [&](uint64_t nodes) {
        uint32_t cap = (uint32_t)std::min<uint64_t>(2 * nodes / BIG_RUN + 4096, 1u << 26);
        if (const char* bc = getenv("KETO_EXPAND_BIG_CAP")) {          // tests: a queue that fills
            cap = std::max(1, atoi(bc));
            if (D.ex_big_cap != cap && D.ex_big) {
                (void)hipFree(D.ex_big);
                D.ex_big = nullptr;
                D.ex_big_cap = 0;
            }
        }
        if (D.ex_big_cap >= cap) return;
        if (D.ex_big) (void)hipFree(D.ex_big);
        D.ex_big = nullptr;
        D.ex_big_cap = 0;
        D.ex_big = reinterpret_cast<CopyRun*>(dmalloc<uint8_t>((uint64_t)cap * sizeof(CopyRun) + 8, acc));
        D.ex_big_cap = cap;
    };
    for (int e = 0; e < 4; ++e)
        if (!D.ex_ev[e]) HIP_OK(hipEventCreate(&D.ex_ev[e]));
    // tier 0 walks with expand_sm (one access per iteration, frames in LDS) when the saved frames
    // fit its LDS stack; KETO_EXPAND_SM=0: expand_one (tooling)
    const char* sme = getenv("KETO_EXPAND_SM");
    const bool sm = gmd <= SM_FRAMES && !(sme && atoi(sme) == 0);
    // KETO_EXPAND_SPREAD=2|4 (A/B): tier 0's trees on 64 / spread lanes per wave
    const char* spe = getenv("KETO_EXPAND_SPREAD");
    const uint32_t spread = spe && (atoi(spe) == 2 || atoi(spe) == 4) ? (uint32_t)atoi(spe) : 1u;
    // (the batch timing sums the passes' tiers: keto_last_batch_timing after an expand)
    auto launch_pass = [&](bool fill, const ExpandOut& eo) {
        run_tiers(D, D.ews, n, p, st,
                  [&](int level, Tier& t, const uint32_t* il, const uint32_t* ic, uint32_t* ol, uint32_t* oc,
                      uint32_t slots) {
                      TierArgs a = tier_args(t, il, ic, ol, oc);
                      const uint32_t bs = std::min<uint32_t>(256, slots);
                      dim3 grid(slots / bs), block(bs);
                      const bool local = p.frames[level] == 0;
                      const int mode = fill ? EXP_FILL : (eo.stage && level == 0) ? EXP_STAGE : EXP_COUNT;
                      ExpandOut e = eo;
                      if (level > 0) {
                          e.runs = nullptr;                    // later tiers copy their runs in place
                          e.ovf_used = nullptr;                // and stage no tree
                      }
                      if (level == 0 && local && sm && spread > 1 && bs == 256) {
                          // (the same logical lanes, spread over spread x the waves)
                          const dim3 g2(grid.x * spread);
#define KETO_EXP_SPREAD(S)                                                                                          \
    if (mode == EXP_COUNT)                                                                                        \
        hipLaunchKernelGGL((expand_kernel<EXP_COUNT, SmFrames, S>), g2, block, 0, st, sv, dov, dq, n, gmd, e, a);  \
    else if (mode == EXP_STAGE)                                                                                   \
        hipLaunchKernelGGL((expand_kernel<EXP_STAGE, SmFrames, S>), g2, block, 0, st, sv, dov, dq, n, gmd, e, a);  \
    else                                                                                                          \
        hipLaunchKernelGGL((expand_kernel<EXP_FILL, SmFrames, S>), g2, block, 0, st, sv, dov, dq, n, gmd, e, a);
                          if (spread == 2) {
                              KETO_EXP_SPREAD(2)
                          } else {
                              KETO_EXP_SPREAD(4)
                          }
#undef KETO_EXP_SPREAD
                      } else if (level == 0 && local && sm) {
                          if (mode == EXP_COUNT)
                              hipLaunchKernelGGL((expand_kernel<EXP_COUNT, SmFrames>), grid, block, 0, st, sv, dov, dq, n, gmd, e, a);
                          else if (mode == EXP_STAGE)
                              hipLaunchKernelGGL((expand_kernel<EXP_STAGE, SmFrames>), grid, block, 0, st, sv, dov, dq, n, gmd, e, a);
                          else
                              hipLaunchKernelGGL((expand_kernel<EXP_FILL, SmFrames>), grid, block, 0, st, sv, dov, dq, n, gmd, e, a);
                      }
                      else if (mode == EXP_COUNT && local)
                          hipLaunchKernelGGL((expand_kernel<EXP_COUNT, LocalStack<16>>), grid, block, 0, st, sv, dov,
                                             dq, n, gmd, e, a);
                      else if (mode == EXP_COUNT)
                          hipLaunchKernelGGL((expand_kernel<EXP_COUNT, GlobalStack>), grid, block, 0, st, sv, dov, dq,
                                             n, gmd, e, a);
                      else if (mode == EXP_STAGE && local)
                          hipLaunchKernelGGL((expand_kernel<EXP_STAGE, LocalStack<16>>), grid, block, 0, st, sv, dov,
                                             dq, n, gmd, e, a);
                      else if (mode == EXP_STAGE)
                          hipLaunchKernelGGL((expand_kernel<EXP_STAGE, GlobalStack>), grid, block, 0, st, sv, dov, dq,
                                             n, gmd, e, a);
                      else if (local)
                          hipLaunchKernelGGL((expand_kernel<EXP_FILL, LocalStack<16>>), grid, block, 0, st, sv, dov,
                                             dq, n, gmd, e, a);
                      else
                          hipLaunchKernelGGL((expand_kernel<EXP_FILL, GlobalStack>), grid, block, 0, st, sv, dov, dq,
                                             n, gmd, e, a);
                      HIP_OK(hipGetLastError());
                  },
                  Undecided{dstatus, fill ? nullptr : dcount, (uint8_t)EXP_OVERFLOW}, fill);
    };
    // grids of the grid-stride copy kernels (a wave per lane / per root): capped, so that a launch is
    // not mostly the dispatch of waves with nothing to copy; KETO_EXPAND_COPY_BLOCKS overrides (tuning)
    const char* cbe = getenv("KETO_EXPAND_COPY_BLOCKS");
    const uint32_t cb_cap = cbe ? (uint32_t)std::max(1, atoi(cbe)) : 16384u;
    auto copy_blocks = [&](uint64_t want) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, cb_cap)); };
    uint32_t* d_nbig = nullptr;
    auto copy_queued = [&]() {
        hipLaunchKernelGGL(copy_lane_runs, dim3(copy_blocks((p.slots[0] + 7) / 8)), dim3(256), 0, st,
                           D.ex_runs, d_lane_runs, p.slots[0]);
        // (usually empty: a small grid-stride grid, not a wave per possible piece)
        hipLaunchKernelGGL(copy_big_runs, dim3(std::min<uint32_t>((D.ex_big_cap + 3) / 4, 512)), dim3(256), 0, st,
                           D.ex_big, d_nbig, D.ex_big_cap);
        HIP_OK(hipGetLastError());
    };
    auto big_queue = [&](uint64_t nodes) {
        ensure_big(nodes);
        d_nbig = reinterpret_cast<uint32_t*>(D.ex_big + D.ex_big_cap);
        HIP_OK(hipMemsetAsync(d_nbig, 0, sizeof(uint32_t), st));
    };
    if (pulls) {
        // rounds of the count pass over every root: each records the other parts' rows its walks met
        // without a copy; they are copied into the overlay and the pass runs again until no tree
        // needs one (a round finds every missing row a walk reaches through rows it has)
        constexpr uint32_t MISS_CAP = 1u << 16;
        DevBuf<uint32_t> miss(MISS_CAP + 1);
        const DevSnap base = sv;
        std::vector<uint8_t> stv(n);
        std::vector<uint32_t> ml;
        for (;;) {
            ps->build(dov, sv, base);
            HIP_OK(hipMemsetAsync(miss.p + MISS_CAP, 0, sizeof(uint32_t), st));
            ExpandOut eo{nullptr, nullptr, dcount, dstatus, nullptr, d_lane_runs, run_inline, nullptr, nullptr, 0, nullptr,
                         0, nullptr, nullptr, 0, 0, 0, nullptr, nullptr, 0, S.n_poisoned_rows == 0 ? 1u : 0u, 0u, 1u, nullptr};
            eo.miss = miss.p;
            eo.n_miss = miss.p + MISS_CAP;
            eo.miss_cap = MISS_CAP;
            launch_pass(false, eo);
            uint32_t nm = 0;
            HIP_OK(hipMemcpyAsync(stv.data(), dstatus, n, hipMemcpyDeviceToHost, st));
            HIP_OK(hipMemcpyAsync(&nm, miss.p + MISS_CAP, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            if (std::find(stv.begin(), stv.end(), (uint8_t)EXP_RETRY) == stv.end()) break;
            ml.resize(std::min(nm, MISS_CAP));
            if (!ml.empty()) HIP_OK(hipMemcpy(ml.data(), miss.p, ml.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
            bool added = false;
            for (uint32_t h : ml) {
                const int64_t r = ps->row_of(h);
                if (r >= 0) added |= ps->add((uint32_t)r);
            }
            if (!added) throw Error{KETO_E_HIP, "expand on a migrating part: a walk needs a row no part holds"};
        }
        if (trace) fprintf(stderr, "[expand] %zu rows of other parts copied\n", ps->pulled.size());
        lap("pulls");
    }
    // pass 1: count (and stage), then the staged trees' queued id runs
    HIP_OK(hipMemsetAsync(dstage, 0xFF, (uint64_t)n * sizeof(uint64_t), st));
    if (staged) big_queue(stage_cap * p.slots[0]);
    const uint32_t blind = S.n_poisoned_rows == 0 && getenv("KETO_EXPAND_LOAD_LEAVES") == nullptr;
    const char* pfe = getenv("KETO_EXPAND_PREFETCH");
    const uint32_t pf = pfe ? (uint32_t)(atoi(pfe) != 0) : 1u;
    const char* ebe = getenv("KETO_EXPAND_EDGE_BLOCKS");
    const uint32_t eb = ebe ? (uint32_t)(atoi(ebe) != 0) : 1u;
    // KETO_EXPAND_CLOCKS=1 (tooling): the first pass's per-root walk times, summarized on stderr
    uint32_t* d_clocks = nullptr;
    if (getenv("KETO_EXPAND_CLOCKS")) {
        d_clocks = dmalloc<uint32_t>(2ull * n, acc);
        HIP_OK(hipMemsetAsync(d_clocks, 0, 2ull * n * sizeof(uint32_t), st));
    }
    unsigned long long* d_ovf_used = staged && ovf_cap ? reinterpret_cast<unsigned long long*>(D.ex_seg) : nullptr;
    uint32_t* d_seg_n = staged ? reinterpret_cast<uint32_t*>(D.ex_seg + 8) : nullptr;
    StageSeg* d_segs = staged ? reinterpret_cast<StageSeg*>(D.ex_seg + 16) : nullptr;
    launch_pass(false, ExpandOut{nullptr, nullptr, dcount, dstatus, staged ? D.ex_runs : nullptr, d_lane_runs,
                                 run_inline, D.ex_big, d_nbig, D.ex_big_cap, D.ex_stage, stage_cap, dstage, d_ovf_used,
                                 ovf_base, ovf_cap, ovf_chunk, d_segs, d_seg_n, staged ? D.ex_seg_cap : 0u, blind, pf,
                                 eb, d_clocks});
    float extra_ms = 0;
    if (staged) {
        HIP_OK(hipEventRecord(D.ex_ev[0], st));
        copy_queued();
        HIP_OK(hipEventRecord(D.ex_ev[1], st));
    }
    lap("count");
    std::vector<uint64_t> cnt(n), spos;
    HIP_OK(hipMemcpyAsync(cnt.data(), dcount, n * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(out.status.data(), dstatus, n, hipMemcpyDeviceToHost, st));
    std::vector<uint8_t> segbuf;
    if (staged) {
        spos.resize(n);
        HIP_OK(hipMemcpyAsync(spos.data(), dstage, n * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        segbuf.resize(16 + (uint64_t)D.ex_seg_cap * sizeof(StageSeg));
        HIP_OK(hipMemcpyAsync(segbuf.data(), D.ex_seg, segbuf.size(), hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    if (pulls && std::find(out.status.begin(), out.status.end(), (uint8_t)EXP_RETRY) != out.status.end())
        throw Error{KETO_E_HIP, "expand on a migrating part: a tree still needs a row of another part"};
    if (staged) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, D.ex_ev[0], D.ex_ev[1]) == hipSuccess) extra_ms += ms;
    }
    if (d_clocks) {
        std::vector<uint32_t> ck(2ull * n);
        HIP_OK(hipMemcpy(ck.data(), d_clocks, 2ull * n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        {
            // per wave (64 consecutive roots of a lane block): the most accesses of one lane
            std::vector<uint32_t> it(ck.begin() + n, ck.end()), wmax;
            for (uint32_t b = 0; b < n; b += 64) wmax.push_back(*std::max_element(it.begin() + b, it.begin() + std::min(n, b + 64)));
            std::sort(it.begin(), it.end());
            std::sort(wmax.begin(), wmax.end());
            fprintf(stderr, "[expand clocks] accesses per root: p50 %u p90 %u p99 %u max %u; per wave (max lane): p50 %u p90 %u max %u\n",
                    it[n / 2], it[n * 9 / 10], it[n * 99 / 100], it[n - 1], wmax[wmax.size() / 2], wmax[wmax.size() * 9 / 10],
                    wmax.back());
        }
        (void)hipFree(d_clocks);
        std::vector<uint32_t> idx(n);
        std::iota(idx.begin(), idx.end(), 0u);
        std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return ck[x] > ck[y]; });
        auto q = [&](double f) { return ck[idx[std::min<size_t>(n - 1, (size_t)(f * n))]] / 100.0; };
        fprintf(stderr, "[expand clocks] walk us per root: max %.1f p0.1%% %.1f p1%% %.1f p10%% %.1f p50 %.1f\n",
                ck[idx[0]] / 100.0, q(0.001), q(0.01), q(0.1), q(0.5));
        for (uint32_t k = 0; k < std::min<uint32_t>(n, 12); ++k)
            fprintf(stderr, "[expand clocks]   root %u (handle %u): %.1f us, %llu nodes, %u accesses\n", idx[k], root[idx[k]],
                    ck[idx[k]] / 100.0, (unsigned long long)cnt[idx[k]], ck[n + idx[k]]);
    }
    uint32_t unstaged = 0;
    for (uint32_t i = 0; i < n; ++i) {
        out.offset[i + 1] = out.offset[i] + cnt[i];
        unstaged += (!staged || spos[i] == NOT_STAGED) && out.status[i] == EXP_TREE && cnt[i];
    }
    const uint64_t total = out.offset[n];
    out.nodes.resize(total);
    lap("scan");
    if (total == 0) {
        D.last.tier_ms[0] += extra_ms;
        return;
    }
    if (D.ex_nodes_cap < total) {
        if (D.ex_nodes) (void)hipFree(D.ex_nodes);
        D.ex_nodes_cap = std::max<uint64_t>(total, 1 << 16);
        D.ex_nodes = dmalloc<keto_tree_node>(D.ex_nodes_cap, acc);
    }
    if (!D.layout_units && !D.unit_row) {             // (a write patches the direct map in place)
        const uint64_t m = std::max<uint64_t>(1, S.layout_units.size());
        D.layout_units = dmalloc<uint32_t>(m, acc);
        D.rows_by_unit = dmalloc<uint32_t>(m, acc);
        HIP_OK(hipMemcpy(D.layout_units, S.layout_units.data(), S.layout_units.size() * sizeof(uint32_t),
                         hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(D.rows_by_unit, S.rows_by_unit.data(), S.rows_by_unit.size() * sizeof(uint32_t),
                         hipMemcpyHostToDevice));
        // the direct map (one word per arena unit) when it is small next to the arena; else the
        // handle -> row translation binary-searches the handle list
        // (only handles below 2^31 are translated -- a set node keeps 31 bits, and a tree's root past
        // them takes its row from the request -- so the map stops there: <= 8 GiB)
        if (S.n_units) {
            D.unit_row_cap = std::min<uint64_t>(1ull << 31, S.n_units + S.n_units / 64 + 4096);
            D.unit_row = dmalloc<uint32_t>(D.unit_row_cap, acc);
            // units that start no row (and the slack) read NO_UNIT, never a stale row id
            HIP_OK(hipMemsetAsync(D.unit_row, 0xFF, D.unit_row_cap * sizeof(uint32_t), st));
            const uint32_t m32 = (uint32_t)S.layout_units.size();
            if (m32)
                hipLaunchKernelGGL(scatter_unit_rows, dim3((m32 + 255) / 256), dim3(256), 0, st, D.unit_row,
                                   D.layout_units, D.rows_by_unit, m32, (uint32_t)D.unit_row_cap);
            HIP_OK(hipGetLastError());
        }
    }
    HIP_OK(hipMemcpyAsync(doff, out.offset.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // pass 2: the trees not staged, filled at their offsets (every root when not staging)
    if (unstaged) {
        big_queue(total);
        launch_pass(true, ExpandOut{D.ex_nodes, doff, dcount, dstatus, D.ex_runs, d_lane_runs, run_inline, D.ex_big,
                                    d_nbig, D.ex_big_cap, nullptr, 0, staged ? dstage : nullptr, nullptr, 0, 0, 0,
                                    nullptr, nullptr, 0, blind, pf, eb, nullptr});
    }
    HIP_OK(hipEventRecord(D.ex_ev[2], st));
    if (unstaged) copy_queued();
    // staged trees: copied to their offsets with their set handles turned into row ids on the way (16
    // lanes per root, their map loads independent); the trees a fill pass wrote at their offsets get
    // the translation over just their ranges.  (Round 3's fused version, a wave per tree, waited its
    // lanes' map loads one after another: 2.5x slower than a pass of its own.)
    const bool fuse = staged && D.unit_row;
    // a staged tree of more than `gbig` nodes goes to copy_stage_pieces in pieces of at most GPIECE
    // (a wave each) instead of one 16-lane group, whose copy of the biggest trees set the gather's
    // time (KETO_EXPAND_GATHER_BIG: the threshold, 0 = every single-piece tree in the gather)
    constexpr uint64_t GPIECE = 512;
    const char* gbe = getenv("KETO_EXPAND_GATHER_BIG");
    const uint64_t gbig = gbe ? (atoll(gbe) > 0 ? (uint64_t)atoll(gbe) : ~0ull) : 256u;
    if (staged)
        hipLaunchKernelGGL(gather_staged, dim3(copy_blocks((n + 15) / 16)), dim3(256), 0, st,
                           D.ex_nodes, D.ex_stage, dstage, doff, n, fuse ? D.unit_row : nullptr, (uint32_t)S.n_units,
                           gbig);
    HIP_OK(hipGetLastError());
    // staged trees in two pieces (a region, then an overflow chunk): copied piece by piece
    std::vector<uint64_t> pc;                          // (alive until the stream is synchronized below)
    uint32_t n_split = 0;
    if (staged) {
        uint32_t ns_ = 0;
        std::memcpy(&ns_, segbuf.data() + 8, 4);
        n_split = std::min<uint32_t>(ns_, D.ex_seg_cap);
        const StageSeg* sgs = reinterpret_cast<const StageSeg*>(segbuf.data() + 16);
        auto piece = [&](uint64_t src, uint64_t dst, uint64_t len) {
            for (uint64_t b = 0; b < len; b += GPIECE) {
                pc.push_back(src + b);
                pc.push_back(dst + b);
                pc.push_back(std::min<uint64_t>(GPIECE, len - b));
            }
        };
        if (gbig != ~0ull)
            for (uint32_t i = 0; i < n; ++i) {
                const uint64_t b = out.offset[i], len = out.offset[i + 1] - b;
                if (spos[i] < SPLIT_POS && len > gbig) piece(spos[i], b, len);
            }
        for (uint32_t k = 0; k < n_split; ++k) {
            const StageSeg& g = sgs[k];
            if (g.root >= n || spos[g.root] != (SPLIT_POS | k)) continue;   // (a record of another call)
            const uint64_t b = out.offset[g.root], len = out.offset[g.root + 1] - b;
            piece(g.region, b, std::min(g.split_at, len));
            if (len > g.split_at) piece(g.chunk, b + g.split_at, len - g.split_at);
        }
        if (!pc.empty()) {
            const uint64_t m = pc.size() / 3;
            if (D.ex_pieces_cap < m) {
                if (D.ex_pieces) (void)hipFree(D.ex_pieces);
                D.ex_pieces = nullptr;
                D.ex_pieces_cap = 0;
                D.ex_pieces = dmalloc<uint64_t>(3 * std::max<uint64_t>(m, 4096), acc);
                D.ex_pieces_cap = std::max<uint64_t>(m, 4096);
            }
            HIP_OK(hipMemcpyAsync(D.ex_pieces, pc.data(), pc.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(copy_stage_pieces, dim3(copy_blocks((m + 3) / 4)), dim3(256), 0, st, D.ex_nodes,
                               D.ex_stage, D.ex_pieces, (uint32_t)m, fuse ? D.unit_row : nullptr, (uint32_t)S.n_units);
            HIP_OK(hipGetLastError());
        }
    }
    std::vector<uint64_t> rg;                          // (alive until the stream is synchronized below)
    if (fuse && unstaged) {
        for (uint32_t i = 0; i < n; ++i)
            if (spos[i] == NOT_STAGED)   // in pieces of at most 2048 nodes: a big tree is not one wave's
                for (uint64_t b = out.offset[i]; b < out.offset[i + 1]; b += 2048) {
                    rg.push_back(b);
                    rg.push_back(std::min<uint64_t>(b + 2048, out.offset[i + 1]));
                }
        // (the big-run queue is free once the copies above ran: the ranges go through it, in pieces
        // that fit it; the copy of a piece waits for the kernel that read the last one)
        uint64_t* d_rg = reinterpret_cast<uint64_t*>(D.ex_big);
        const uint64_t per = std::max<uint64_t>(1, (uint64_t)D.ex_big_cap * sizeof(CopyRun) / 16);
        for (uint64_t r0 = 0; r0 < rg.size() / 2; r0 += per) {
            const uint32_t nr = (uint32_t)std::min<uint64_t>(per, rg.size() / 2 - r0);
            HIP_OK(hipMemcpyAsync(d_rg, rg.data() + 2 * r0, (uint64_t)nr * 16, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(handles_to_rows_ranges, dim3(std::min<uint32_t>((nr + 3) / 4, 4096)), dim3(256), 0, st,
                               D.ex_nodes, d_rg, nr, D.unit_row, (uint32_t)S.n_units);
        }
        HIP_OK(hipGetLastError());
    }
    HIP_OK(hipEventRecord(D.ex_ev[3], st));
    lap("fill");
    if (fuse) {
    } else if (D.unit_row)
        hipLaunchKernelGGL(handles_to_rows_direct, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, D.ex_nodes,
                           total, D.unit_row, (uint32_t)S.n_units);
    else
        hipLaunchKernelGGL(handles_to_rows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, D.ex_nodes, total,
                           D.layout_units, D.rows_by_unit, (uint32_t)S.layout_units.size(), (uint32_t)S.n_units);
    HIP_OK(hipGetLastError());
    const bool high_roots = S.n_units > (uint64_t)EDGE_VAL;
    lap("h2rows");
    HIP_OK(hipMemcpyAsync(out.nodes.data(), D.ex_nodes, total * sizeof(keto_tree_node), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    lap("d2h");
    // arenas with root rows past 2^31 units: a tree's root node lost its handle's bit 31 to EDGE_SET,
    // so it takes its row from the request (overlay roots: below)
    if (high_roots)
        for (uint32_t i = 0; i < n; ++i)
            if (root_flags[i] && out.offset[i + 1] > out.offset[i] && root[i] >= EDGE_VAL && root[i] < S.n_units)
                out.nodes[out.offset[i]].subject = EDGE_SET | (*root_rows)[i];
    {
        float ms = 0;
        if (hipEventElapsedTime(&ms, D.ex_ev[2], D.ex_ev[3]) == hipSuccess) extra_ms += ms;
        D.last.tier_ms[0] += extra_ms;
    }
    if (trace) {
        uint64_t big = 0, sum = 0;
        for (uint32_t i = 0; i < n; ++i)
            if ((!staged || spos[i] == NOT_STAGED) && out.status[i] == EXP_TREE) {
                big = std::max<uint64_t>(big, out.offset[i + 1] - out.offset[i]);
                sum += out.offset[i + 1] - out.offset[i];
            }
        fprintf(stderr, "[expand] %u of %u trees filled by the second pass (%llu nodes, the largest %llu); %u staged in two pieces\n",
                unstaged, n, (unsigned long long)sum, (unsigned long long)big, n_split);
    }
    // overlay handles -> ovh->base + overlay index (batch-local wildcard roots only); a migrating
    // part's identity slots -> the rows they name
    if (pulls) {
        const uint64_t wu = ps->wild_units;
        host_parallel_for(total, [&](uint64_t i) {
            keto_tree_node& x = out.nodes[i];
            if (!(x.subject & EDGE_SET)) return;
            const uint32_t h = x.subject & EDGE_VAL;
            if (h < S.n_units) return;
            const uint64_t u = (uint64_t)h - S.n_units;
            if (u < wu) {
                auto it = std::lower_bound(ovh->unit.begin(), ovh->unit.end(), (uint32_t)u);
                x.subject = EDGE_SET | (ovh->base + (uint32_t)(it - ovh->unit.begin()));
            } else {
                x.subject = EDGE_SET | ps->id_row[u - wu];
            }
        });
    } else if (ovh && !ovh->empty() && high_roots) {
        for (uint32_t i = 0; i < n; ++i) {
            if (!root_flags[i] || out.offset[i + 1] == out.offset[i] || root[i] < S.n_units) continue;
            auto it = std::lower_bound(ovh->unit.begin(), ovh->unit.end(), (uint32_t)(root[i] - S.n_units));
            out.nodes[out.offset[i]].subject = EDGE_SET | (ovh->base + (uint32_t)(it - ovh->unit.begin()));
        }
    } else if (ovh && !ovh->empty())
        host_parallel_for(total, [&](uint64_t i) {
            keto_tree_node& x = out.nodes[i];
            if (!(x.subject & EDGE_SET)) return;
            const uint32_t h = x.subject & EDGE_VAL;
            if (h < S.n_units) return;
            const uint32_t u = (uint32_t)(h - S.n_units);
            auto it = std::lower_bound(ovh->unit.begin(), ovh->unit.end(), u);
            x.subject = EDGE_SET | (ovh->base + (uint32_t)(it - ovh->unit.begin()));
        });
}

}  // namespace keto
