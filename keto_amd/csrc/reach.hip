// Deep check batches: top-level items and a hop-bounded reachability pretest (MI355X, gfx950).
//
// The reference answers a check with a DFS whose visited map is fresh for every top-level tuple of
// the request's row (the shadowed ctx at internal/check/engine.go:47-48) and shared below it.  Two
// exact consequences make deep searches (nested groups, max-depth 10..64) cheaper:
//
//   1. Top-level tuples are independent: each starts its own map, so the decision is the OR over
//      them (engine.go:47-77 returns on the first allowed one).  A request becomes one ITEM per
//      top-level subject set -- the set entered at max-depth - 1 with a map holding only itself --
//      and items run on separate lanes.  A request whose later item finds the subject no longer
//      waits for an earlier item's long search, and an item's search is the reference's search
//      below that tuple, event for event.
//   2. A match needs a row holding the requested subject id T that the search enters
//      (`requested.Subject.Equals(sr.Subject)`, engine.go:54), and the search enters only rows
//      within max-depth - 1 subject-set hops of the request's row (checkOneIndirectionFurther stops
//      at restDepth <= 0, engine.go:88-91).  So an item whose set has no row holding T within
//      max-depth - 2 hops is false, whatever order its search would take.  The pretest decides that
//      with a bidirectional BFS: forward from the item's set over subject-set edges, backward from
//      the rows holding T (a postings list) over reversed subject-set edges, expanding the smaller
//      frontier, until the frontiers meet (keep the item) or the hop budget is spent (drop it).
//      A search too big for its lane's bounds keeps the item: the pretest only ever drops items it
//      has proven false, so decisions equal the reference's.
//
// On the config #3 graph (100M tuples, nested groups with cycles, depths 5/16/32) half the requests
// are dropped by the pretest -- they are the long exhaustive searches (tools/dev/bidir_study.py:
// 3.53G reference DFS steps for 1M requests, 0.92G after the split and the pretest, and the longest
// chain 101K -> 58.5K steps).
//
// Index (per snapshot version, built on host threads, uploaded once): for every row some subject
// set points at, the handles of the rows pointing at it; for every subject id, the handles of the
// rows holding it.  Both are built from every stored edge, a superset of the effective (check)
// edges, which can only add paths: the pretest stays sound.  A write bumps the snapshot version;
// the next deep batch rebuilds the index first.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

namespace {

constexpr uint32_t RNONE = 0xFFFFFFFFu;

template <class T>
T* ralloc(uint64_t n, uint64_t& acc) {
    void* p = nullptr;
    if (n == 0) n = 1;
    const hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    acc += n * sizeof(T);
    return (T*)p;
}

struct RBuf {                     // a grow-only device buffer, freed with its owner
    void* p = nullptr;
    uint64_t cap = 0;
    RBuf() = default;
    RBuf(const RBuf&) = delete;
    RBuf& operator=(const RBuf&) = delete;
    template <class T>
    T* get(uint64_t n) {
        const uint64_t want = std::max<uint64_t>(16, n * sizeof(T));
        if (want > cap) {
            release();
            uint64_t acc = 0;
            p = ralloc<uint8_t>(want + want / 8, acc);
            cap = want + want / 8;
        }
        return (T*)p;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    ~RBuf() { release(); }
};

__host__ __device__ inline uint32_t rmix(uint32_t k) {
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}

// direct-indexed: dir[key] = the offset of the key's list [count, entries...], INLINE | the one
// entry of a single-entry list (one access fewer), or RNONE
constexpr uint32_t INLINE = 0x80000000u;
__device__ inline uint32_t dir_at(const uint32_t* __restrict__ dir, uint32_t n, uint32_t key) {
    return key < n ? dir[key] : RNONE;
}
// the list behind a table value: n entries, entry k = single (n == 1, inlined) or lists[off + k]
struct IdxList {
    uint32_t n, off, single;
    __device__ inline uint32_t at(const uint32_t* lists, uint32_t k) const { return off == RNONE ? single : lists[off + k]; }
};
__device__ inline IdxList list_of(uint32_t v, const uint32_t* lists) {
    if (v == RNONE) return IdxList{0, RNONE, 0};
    if (v & INLINE) return IdxList{1, RNONE, v & ~INLINE};
    return IdxList{lists[v], v + 1, 0};
}

// reverse lists: rdir[handle] = RD_NONE (nothing points at the row), tag << 62 | parents for one or
// two parents inlined (31 bits each), or 3 << 62 | offset of [count, parents...] in rev
constexpr uint64_t RD_NONE = ~0ull;
struct RevList {
    uint64_t e;
    uint32_t cnt;                                  // tag 3: the list's count (loaded separately)
    __device__ inline uint32_t tag() const { return e == RD_NONE ? 0u : (uint32_t)(e >> 62); }
    __device__ inline uint32_t n() const { const uint32_t t = tag(); return t == 3u ? cnt : t; }
    __device__ inline uint32_t at(const uint32_t* rev, uint32_t q) const {
        if (tag() == 3u) return rev[(uint32_t)e + 1 + q];
        return q == 0 ? (uint32_t)(e & EDGE_VAL) : (uint32_t)((e >> 31) & EDGE_VAL);
    }
};
__device__ inline uint64_t rdir_at(const uint64_t* __restrict__ d, uint32_t n, uint32_t key) {
    return key < n ? d[key] : RD_NONE;
}

struct ReachDev {
    const uint32_t* arena;
    const uint64_t* rdir;     // set-target handle -> the rows pointing at it (RevList)
    const uint32_t* rev;
    uint32_t rn;              // rdir entries
    const uint32_t* pdir;     // subject id -> list value over post: the rows holding it
    const uint32_t* post;
    uint32_t pn;              // pdir entries
    uint32_t ov_base;         // handles >= ov_base are batch-local overlay rows (never items)
    uint32_t root_g;          // wide arenas: root handles past 2^31 (snapshot.hpp hword)
};

__device__ inline uint32_t win(const uint4& w, uint32_t i) {
    const uint32_t lo = (i & 1u) ? w.y : w.x;
    const uint32_t hi = (i & 1u) ? w.w : w.z;
    return (i & 2u) ? hi : lo;
}

// a row's header (forwards followed) and window; beg = word index of its first edge (g: the arena's
// root unit, hword; only a request's own row can be a root)
__device__ inline void row_at(const uint32_t* a, uint32_t h, uint32_t g, uint4& h0, uint4& h1, uint64_t& beg) {
    uint64_t w = hword(h, g);
    h0 = *reinterpret_cast<const uint4*>(a + w);
    while (h0.z & HDR_FWD) {
        w = hword(h0.x, g);
        h0 = *reinterpret_cast<const uint4*>(a + w);
    }
    h1 = *reinterpret_cast<const uint4*>(a + w + HDR_WORDS);
    beg = w + HDR_WORDS;
}

// does a normal (not ROW_SEQ) row hold the subject id T?  Its ids follow its subject sets; a row
// with an id table answers from the header bloom filter and the table (snapshot.hpp layout).
__device__ inline bool holds_id(const uint32_t* a, const uint4& h0, const uint4& h1, uint64_t beg, uint32_t T) {
    const uint32_t n_sets = h0.x, n_ids = h0.y;
    if (n_ids == 0) return false;
    const uint32_t hl = (h0.z >> 8) & 31u;
    if (hl == 0) {
        bool hit = false;
        for (uint32_t i = 0; i < WINDOW_WORDS; ++i) hit |= (i >= n_sets) & (i < n_sets + n_ids) & (win(h1, i) == T);
        return hit;
    }
    uint32_t b1, b2;
    bloom_bits(T, b1, b2);
    if (!bloom_has(h0.z, h0.w, b1) || !bloom_has(h0.z, h0.w, b2)) return false;
    const uint32_t nb = (1u << hl) / BUCKET_WORDS;
    const uint64_t tb = beg - HDR_WORDS - ((h0.z & HDR_CLOSURE) ? CB_WORDS : 0u) - (1ull << hl);
    for (uint32_t b = rmix(T) & (nb - 1), k = 0; k < nb; b = (b + 1) & (nb - 1), ++k) {
        const uint4 v = *reinterpret_cast<const uint4*>(a + tb + (uint64_t)b * BUCKET_WORDS);
        if (v.x == T || v.y == T || v.z == T || v.w == T) return true;
        if (v.x == RNONE || v.y == RNONE || v.z == RNONE || v.w == RNONE) return false;
    }
    return false;
}

// per request: acc bit 4 = decided here (da written); count = work entries it needs (items, or
// 1 | PASS for a request checked whole)
constexpr uint32_t ACC_TRUE = 1u, ACC_UND = 2u, ACC_DONE = 4u;
constexpr uint32_t PASS = 0x80000000u;

__global__ void __launch_bounds__(256) split_count(ReachDev r, const keto_check_ids* __restrict__ q, uint32_t n,
                                                   int gmd, uint8_t* __restrict__ da, uint32_t* __restrict__ acc,
                                                   uint32_t* __restrict__ cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const keto_check_ids qq = q[i];
    int d = qq.max_depth;
    if (d <= 0 || gmd < d) d = gmd;                                    // engine.go:118-120
    uint32_t a = 0, c = 0;
    if (qq.row == KETO_NO_ROW || d <= 0 || qq.target == KETO_NO_TARGET) {
        da[i] = 0;
        a = ACC_DONE;
    } else if ((qq.flags & 1u) || qq.row >= r.ov_base) {
        c = 1u | PASS;                                                 // subject-set requests, overlay rows
    } else {
        uint4 h0, h1;
        uint64_t beg;
        row_at(r.arena, qq.row, r.root_g, h0, h1, beg);
        if (h0.z & HDR_SEQ) {
            c = 1u | PASS;                                             // ordered walk of colliding keys
        } else if (holds_id(r.arena, h0, h1, beg, qq.target)) {
            da[i] = 1;                                                 // a top-level id tuple (fresh map)
            a = ACC_DONE;
        } else if (d < 2 || h0.x == 0) {
            da[i] = 0;                                                 // no subject set can be entered
            a = ACC_DONE;
        } else {
            c = h0.x;                                                  // one item per top-level subject set
        }
    }
    acc[i] = a;
    cnt[i] = c;
}

__global__ void __launch_bounds__(256) split_fill(ReachDev r, const keto_check_ids* __restrict__ q, uint32_t n, int gmd,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                                  keto_check_ids* __restrict__ work, uint32_t* __restrict__ owner) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = cnt[i];
    if (!c) return;
    const keto_check_ids qq = q[i];
    const uint32_t o = off[i];
    if (c & PASS) {
        work[o] = qq;
        owner[o] = i;
        return;
    }
    int d = qq.max_depth;
    if (d <= 0 || gmd < d) d = gmd;
    uint4 h0, h1;
    uint64_t beg;
    row_at(r.arena, qq.row, r.root_g, h0, h1, beg);
    for (uint32_t j = 0; j < c; ++j) {
        const uint32_t e = j < WINDOW_WORDS ? win(h1, j) : r.arena[beg + j];
        work[o + j] = keto_check_ids{e & EDGE_VAL, qq.target, KETO_ITEM_FLAG, d - 1};
        owner[o + j] = i;
    }
}

// The pretest, one lane per item (a persistent grid handing items out dynamically).  Per lane: a
// mark table of 2 cap slots (epoch << 32 | side << 31 | handle) and two discovery lists of cap
// handles (forward, backward; a BFS level is a contiguous range).  keep[w] = 0 only when the search
// finished without the frontiers meeting.
struct Pretest {
    uint64_t* marks;
    uint32_t* lists;
    uint32_t* epochs;
    uint32_t cap;             // marks and list entries per lane (power of two)
    uint32_t work_cap;        // edges examined per item before giving up (keep)
    uint32_t* next;
};

__device__ inline int mark(uint64_t* M, uint32_t mmask, uint32_t ep, uint32_t& nm, uint32_t cap, uint32_t h, uint32_t side) {
    // 0 new (marked), 1 marked by this side, 2 marked by the other side (the frontiers meet), 3 full
    for (uint32_t i = rmix(h) & mmask;; i = (i + 1) & mmask) {
        const uint64_t e = M[i];
        if ((uint32_t)(e >> 32) != ep) {
            if (++nm > cap) return 3;
            M[i] = ((uint64_t)ep << 32) | (side << 31) | h;
            return 0;
        }
        if (((uint32_t)e & EDGE_VAL) == h) return (((uint32_t)e >> 31) == side) ? 1 : 2;
    }
}

__device__ bool within(const ReachDev& r, const Pretest& P, uint64_t* M, uint32_t* F, uint32_t* B, uint32_t ep,
                       uint32_t c, uint32_t T, int L) {
    const uint32_t mmask = 2 * P.cap - 1;
    uint32_t nm = 0, nf = 0, nb = 0;
    const IdxList pl = list_of(dir_at(r.pdir, r.pn, T), r.post);
    if (pl.n == 0) return false;                         // no row holds T
    const uint32_t pn = pl.n;
    if (pn >= P.cap) return true;                        // too many rows to start from: keep
    (void)mark(M, mmask, ep, nm, P.cap, c, 0);
    F[nf++] = c;
    for (uint32_t k = 0; k < pn; ++k) {
        const uint32_t h = pl.at(r.post, k);
        const int t = mark(M, mmask, ep, nm, P.cap, h, 1);
        if (t == 2 || t == 3) return true;               // c itself holds T, or full
        if (t == 0) B[nb++] = h;
    }
    uint32_t f0 = 0, f1 = nf, b0 = 0, b1 = nb, work = pn;
    int da = 0, db = 0;
    while (da + db < L && f1 > f0 && b1 > b0) {
        if (f1 - f0 <= b1 - b0) {
            for (uint32_t x = f0; x < f1; ++x) {
                uint4 h0, h1;
                uint64_t beg;
                row_at(r.arena, F[x], r.root_g, h0, h1, beg);
                const uint32_t ns = h0.x;                // ROW_SEQ: every edge, sets and ids mixed
                work += ns;
                if (work > P.work_cap) return true;
                for (uint32_t j = 0; j < ns; ++j) {
                    const uint32_t e = j < WINDOW_WORDS ? win(h1, j) : r.arena[beg + j];
                    if (!(e & EDGE_SET)) continue;
                    const uint32_t ch = e & EDGE_VAL;
                    const int t = mark(M, mmask, ep, nm, P.cap, ch, 0);
                    if (t == 2 || t == 3) return true;
                    if (t == 0) {
                        if (nf >= P.cap) return true;
                        F[nf++] = ch;
                    }
                }
            }
            f0 = f1;
            f1 = nf;
            ++da;
        } else {
            for (uint32_t x = b0; x < b1; ++x) {
                RevList rl{rdir_at(r.rdir, r.rn, B[x]), 0};
                if (rl.tag() == 3u) rl.cnt = r.rev[(uint32_t)rl.e];
                const uint32_t rn = rl.n();              // 0: a root row, nothing points at it
                work += rn;
                if (work > P.work_cap) return true;
                for (uint32_t k = 0; k < rn; ++k) {
                    const uint32_t u = rl.at(r.rev, k);
                    const int t = mark(M, mmask, ep, nm, P.cap, u, 1);
                    if (t == 2 || t == 3) return true;
                    if (t == 0) {
                        if (nb >= P.cap) return true;
                        B[nb++] = u;
                    }
                }
            }
            b0 = b1;
            b1 = nb;
            ++db;
        }
    }
    return false;
}

__global__ void __launch_bounds__(256) pretest_kernel(ReachDev r, Pretest P, const keto_check_ids* __restrict__ work,
                                                      uint32_t n, uint8_t* __restrict__ keep) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint64_t* M = P.marks + (uint64_t)lane * 2 * P.cap;
    uint32_t* F = P.lists + (uint64_t)lane * 2 * P.cap;
    uint32_t* B = F + P.cap;
    uint32_t ep = P.epochs[lane];
    for (uint32_t w = lane; w < n; w = stride + atomicAdd(P.next, 1u)) {
        const keto_check_ids it = work[w];
        if (!(it.flags & KETO_ITEM_FLAG)) {
            keep[w] = 1;
            continue;
        }
        if (++ep >= 0xFFFFFFF0u) {                       // epoch wrap: clear this lane's marks once
            for (uint32_t i = 0; i < 2 * P.cap; ++i) M[i] = 0;
            ep = 1;
        }
        // the item's set is entered at depth it.max_depth: rows it can enter are within
        // max_depth - 1 hops of it
        keep[w] = within(r, P, M, F, B, ep, it.row, it.target, it.max_depth - 1) ? 1 : 0;
    }
    P.epochs[lane] = ep;
}

// The pretest with one wave per item: a BFS level's nodes are expanded by the wave's lanes together
// (one round of header loads forward; one of table probes, then one of reverse lists, backward), and
// the marks live in LDS, claimed by compare-and-swap.  An item costs about two memory round trips per
// level instead of one per edge.  WP_CAP marks (4096 LDS slots) and WP_CAP handles per side bound a
// search; past them, or past work_cap edges, the item is kept.
constexpr uint32_t LEMPTY = 0xFFFFFFFFu;

template <uint32_t WP_SLOTS>
__device__ inline int lmark(uint32_t* tab, uint32_t* nm, uint32_t h, uint32_t side) {
    constexpr uint32_t WP_CAP = WP_SLOTS / 2;
    // 0 new (marked), 1 marked by this side, 2 marked by the other side (the frontiers meet), 3 full
    const uint32_t key = (side << 31) | h;
    for (uint32_t i = rmix(h) & (WP_SLOTS - 1);; i = (i + 1) & (WP_SLOTS - 1)) {
        uint32_t cur = tab[i];
        if (cur == LEMPTY) {
            if (atomicAdd(nm, 1u) >= WP_CAP) return 3;    // claimed slots stay below WP_SLOTS
            cur = atomicCAS(tab + i, LEMPTY, key);
            if (cur == LEMPTY) return 0;
            atomicSub(nm, 1u);                             // another lane took the slot: look at it
        }
        if ((cur & EDGE_VAL) == h) return (cur >> 31) == side ? 1 : 2;
    }
}

template <uint32_t WP_SLOTS>
__global__ void __launch_bounds__(64) pretest_wave_kernel(ReachDev r, const keto_check_ids* __restrict__ work, uint32_t n,
                                                         uint8_t* __restrict__ keep, uint32_t* __restrict__ next,
                                                         uint32_t work_cap, int min_depth) {
    constexpr uint32_t WP_CAP = WP_SLOTS / 2;
    __shared__ uint32_t tab[WP_SLOTS];
    // discovered handles: forward from the front, backward from the back (each is a distinct mark,
    // so together they never exceed WP_CAP)
    __shared__ uint32_t FB[WP_CAP];
    uint32_t* const F = FB;
    auto Bat = [&](uint32_t i) -> uint32_t& { return FB[WP_CAP - 1 - i]; };
    __shared__ uint32_t s_nf, s_nb, s_nm, s_hit, s_work, s_item;
    const uint32_t t = threadIdx.x;
    // work requests are taken 64 at a time (one atomic per chunk: one per request serialized the
    // grid on the counter, 13.8 ms for 1.2M requests); the chunk's requests that need a pretest are
    // found by a ballot and searched one after the other (keep[] starts all ones)
    for (;;) {
        if (t == 0) s_item = atomicAdd(next, 64u);
        __syncthreads();
        const uint32_t base = s_item;
        __syncthreads();
        if (base >= n) break;
        bool need = false;
        if (base + t < n) {
            const keto_check_ids c = work[base + t];
            need = (c.flags & KETO_ITEM_FLAG) && c.max_depth >= min_depth;
        }
        for (uint64_t mask = __ballot(need); mask; mask &= mask - 1) {
        const uint32_t w = base + (uint32_t)(__ffsll((unsigned long long)mask) - 1);
        const keto_check_ids it = work[w];
        for (uint32_t i = t; i < WP_SLOTS / 4; i += 64) reinterpret_cast<uint4*>(tab)[i] = make_uint4(LEMPTY, LEMPTY, LEMPTY, LEMPTY);
        if (t == 0) {
            s_nf = s_nb = s_nm = s_hit = s_work = 0;
        }
        __syncthreads();
        const int L = it.max_depth - 1;                    // hops from the item's set to a row it enters
        const IdxList pl = list_of(dir_at(r.pdir, r.pn, it.target), r.post);
        bool kept;
        if (pl.n == 0) {
            kept = false;                                  // no row holds T
        } else if (pl.n >= WP_CAP) {
            kept = true;
        } else {
            if (t == 0) {
                (void)lmark<WP_SLOTS>(tab, &s_nm, it.row, 0);
                F[0] = it.row;
                s_nf = 1;
            }
            __syncthreads();
            for (uint32_t k = t; k < pl.n; k += 64) {
                const uint32_t h = pl.at(r.post, k);
                const int m = lmark<WP_SLOTS>(tab, &s_nm, h, 1);
                if (m >= 2) s_hit = 1;                     // the item's set holds T, or full
                else if (m == 0) Bat(atomicAdd(&s_nb, 1u)) = h;
            }
            __syncthreads();
            uint32_t f0 = 0, f1 = 1, b0 = 0, b1 = s_nb;
            int da = 0, db = 0;
            while (!s_hit && da + db < L && f1 > f0 && b1 > b0) {
                // expand the smaller frontier; both in one round while they are of similar size and
                // the hop budget allows two more hops (a meet is then a path of <= da + db + 2 hops)
                const uint32_t fs = f1 - f0, bs = b1 - b0;
                const bool both = da + db + 2 <= L && max(fs, bs) <= 4 * min(fs, bs);
                const uint32_t nfw = (both || fs <= bs) ? fs : 0u, nbw = (both || fs > bs) ? bs : 0u;
                // each lane takes up to 4 nodes of the round at once: their header / reverse-list
                // loads are all issued before any is used, so a round costs ~one memory latency
                struct Pf {
                    uint4 h0, h1;
                    uint64_t beg;
                    RevList rl;
                };
                auto gather = [&](Pf& p, uint32_t x) {
                    p.rl = RevList{RD_NONE, 0};
                    if (x < nfw) row_at(r.arena, F[f0 + x], r.root_g, p.h0, p.h1, p.beg);
                    else if (x < nfw + nbw) p.rl.e = rdir_at(r.rdir, r.rn, Bat(b0 + x - nfw));
                };
                auto count = [&](Pf& p) {               // counts of reverse lists of 3+ parents
                    if (p.rl.tag() == 3u) p.rl.cnt = r.rev[(uint32_t)p.rl.e];
                };
                auto process = [&](const Pf& p, uint32_t x) {
                    if (x >= nfw + nbw || s_hit) return;
                    if (x < nfw) {
                        const uint32_t ns = p.h0.x;     // ROW_SEQ: every edge, sets and ids mixed
                        if (atomicAdd(&s_work, ns) + ns > work_cap) {
                            s_hit = 1;
                            return;
                        }
                        for (uint32_t j = 0; j < ns; ++j) {
                            const uint32_t e = j < WINDOW_WORDS ? win(p.h1, j) : r.arena[p.beg + j];
                            if (!(e & EDGE_SET)) continue;
                            const uint32_t ch = e & EDGE_VAL;
                            const int m = lmark<WP_SLOTS>(tab, &s_nm, ch, 0);
                            if (m >= 2) {
                                s_hit = 1;
                                return;
                            }
                            if (m == 0) {
                                const uint32_t at = atomicAdd(&s_nf, 1u);
                                if (at >= WP_CAP) {
                                    s_hit = 1;
                                    return;
                                }
                                F[at] = ch;
                            }
                        }
                    } else {
                        const uint32_t n_par = p.rl.n();
                        if (atomicAdd(&s_work, n_par) + n_par > work_cap) {
                            s_hit = 1;
                            return;
                        }
                        for (uint32_t q = 0; q < n_par; ++q) {   // 0: a root row, nothing points at it
                            const uint32_t u = p.rl.at(r.rev, q);
                            const int m = lmark<WP_SLOTS>(tab, &s_nm, u, 1);
                            if (m >= 2) {
                                s_hit = 1;
                                return;
                            }
                            if (m == 0) {
                                const uint32_t at = atomicAdd(&s_nb, 1u);
                                if (at >= WP_CAP) {
                                    s_hit = 1;
                                    return;
                                }
                                Bat(at) = u;
                            }
                        }
                    }
                };
                for (uint32_t base = 0; base < nfw + nbw && !s_hit; base += 256) {
                    Pf p0, p1, p2, p3;
                    gather(p0, base + t);
                    gather(p1, base + t + 64);
                    gather(p2, base + t + 128);
                    gather(p3, base + t + 192);
                    count(p0);
                    count(p1);
                    count(p2);
                    count(p3);
                    process(p0, base + t);
                    process(p1, base + t + 64);
                    process(p2, base + t + 128);
                    process(p3, base + t + 192);
                }
                __syncthreads();
                if (nfw) {
                    f0 = f1;
                    f1 = min(s_nf, WP_CAP);
                    ++da;
                }
                if (nbw) {
                    b0 = b1;
                    b1 = min(s_nb, WP_CAP);
                    ++db;
                }
            }
            kept = s_hit != 0;
        }
        if (t == 0) keep[w] = kept ? 1 : 0;
        __syncthreads();                                   // s_* and tab reused by the next item
        }
    }
}

// kept work requests in two classes: deep items (fa) and the rest (fb)
__global__ void __launch_bounds__(256) classify_kept(const keto_check_ids* __restrict__ work, const uint8_t* __restrict__ keep,
                                                     uint32_t m, int first_depth, uint8_t* __restrict__ fa,
                                                     uint8_t* __restrict__ fb) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= m) return;
    const bool k = keep[w] != 0;
    const bool deep = (work[w].flags & KETO_ITEM_FLAG) && work[w].max_depth >= first_depth;
    fa[w] = k && deep;
    fb[w] = k && !deep;
}

__global__ void __launch_bounds__(256) merge_kernel(const uint8_t* __restrict__ dec, const uint32_t* __restrict__ owner,
                                                    uint32_t m, uint32_t* __restrict__ acc,
                                                    const uint32_t* __restrict__ wsteps, uint32_t* __restrict__ steps) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= m) return;
    const uint8_t d = dec[w];
    const uint32_t o = owner[w];
    if (d == 1) atomicOr(acc + o, ACC_TRUE);
    else if (d != 0) atomicOr(acc + o, ACC_UND);
    if (steps) atomicMax(steps + o, wsteps[w]);          // a request's chain: its longest item
}

__global__ void __launch_bounds__(256) final_kernel(const uint32_t* __restrict__ acc, uint32_t n, uint8_t* __restrict__ da,
                                                    uint32_t* __restrict__ undecided) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = acc[i];
    if (a & ACC_DONE) return;
    // an allowed item decides the request (engine.go:73-75); else one the engine could not decide
    // leaves it undecided
    if (a & ACC_TRUE) da[i] = 1;
    else if (a & ACC_UND) {
        da[i] = (uint8_t)KETO_UNDECIDED;
        atomicAdd(undecided, 1u);
    } else da[i] = 0;
}

}  // namespace

struct ReachState {
    int device = 0;
    uint64_t version = ~0ull;
    bool built = false;
    uint64_t* rdir = nullptr;
    uint32_t* rev = nullptr;
    uint32_t rn = 0;
    uint32_t* pdir = nullptr;
    uint32_t* post = nullptr;
    uint32_t pn = 0;
    uint64_t bytes = 0;
    float build_ms = 0;
    // pretest lanes
    uint64_t* marks = nullptr;
    uint32_t* lists = nullptr;
    uint32_t* epochs = nullptr;
    uint32_t lanes = 0, cap = 0;
    uint32_t wave_blocks[2] = {0, 0};   // resident blocks of pretest_wave_kernel<4096>, <2048>
    // per batch (grow-only)
    RBuf acc, cnt, off, work, owner, keep, work2, owner2, dec, wsteps, nsel, tmp, ctr, flags;
    void free_index() {
        for (void* p : {(void*)rdir, (void*)rev, (void*)pdir, (void*)post})
            if (p) (void)hipFree(p);
        rdir = nullptr;
        rev = nullptr;
        pdir = nullptr;
        post = nullptr;
        bytes = 0;
        built = false;
    }
    ~ReachState() {
        (void)hipSetDevice(device);
        free_index();
        for (void* p : {(void*)marks, (void*)lists, (void*)epochs})
            if (p) (void)hipFree(p);
    }
};

void ReachStateDeleter::operator()(ReachState* r) const { delete r; }

namespace {

uint32_t pow2_ge(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    if (p > (1ull << 31)) throw Error{KETO_E_RANGE, "reach index table exceeds 2^31 slots"};
    return (uint32_t)p;
}

// keys -> list values, direct-indexed (RNONE where no list)
std::vector<uint32_t> make_dir(const std::vector<uint32_t>& keys, const std::vector<uint32_t>& vals, unsigned th) {
    uint32_t n = 0;
    for (uint32_t k : keys) n = std::max(n, k + 1);
    std::vector<uint32_t> dir(std::max<uint32_t>(n, 1), RNONE);
    par_chunks(keys.size(), th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t k = b; k < e; ++k) dir[keys[k]] = vals[k];
    });
    return dir;
}

// The reverse and postings index of the snapshot's current version (host threads, then one upload).
void build_index(const Snapshot& S, ReachState& R) {
    const auto t0 = std::chrono::steady_clock::now();
    R.free_index();
    const unsigned th = build_threads();
    const uint32_t NR = S.n_rows();
    // every stored edge of every row on this device (a superset of the effective edges)
    auto edges_of = [&](uint32_t r) { return S.row_edges(r); };
    // Only rows some subject set points at (row_cb: a target identity, kept while the row is one) go
    // into the index, as parents and as rows holding an id.  An item's forward search reaches only
    // targets (its own set is one), and a root row has no parent, so a backward path through a root
    // ends there without meeting the forward side: leaving roots out drops no meeting, i.e. changes no
    // kept item (and a T held by roots only now drops every item at once, as it should: no entered
    // row can hold it).  It keeps every handle in the index below 2^31 (targets), so arenas whose
    // roots lie past 2^31 units (split and wide layouts) take the pretest too, and it leaves out the
    // postings of the documents, most of the index on the power-law graphs.
    // (KETO_REACH_ROOTS=1, A/B tooling: roots too, as before round 6 -- arenas below 2^31 units only)
    const char* er = getenv("KETO_REACH_ROOTS");
    const bool roots_too = er && atoi(er) == 1 && S.n_units <= (uint64_t)EDGE_VAL;
    auto kept = [&](uint32_t r) { return S.present(r) && (roots_too || (r < S.row_cb.size() && S.row_cb[r])); };
    uint32_t max_id = 0;
    {
        std::vector<uint32_t> mx(th, 0);
        par_chunks(NR, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned t) {
            uint32_t m = mx[t];
            for (uint64_t r = b; r < e; ++r) {
                if (!kept((uint32_t)r)) continue;
                const auto ed = edges_of((uint32_t)r);
                for (uint64_t k = 0; k < ed.second; ++k) {
                    const uint32_t v = ed.first[k];
                    if (!(v & EDGE_SET) && v != EDGE_POISON) m = std::max(m, v);
                }
            }
            mx[t] = m;
        });
        for (uint32_t m : mx) max_id = std::max(max_id, m);
    }
    std::vector<uint32_t> indeg(NR, 0), idc((uint64_t)max_id + 1, 0);
    par_chunks(NR, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t r = b; r < e; ++r) {
            if (!kept((uint32_t)r)) continue;
            const auto ed = edges_of((uint32_t)r);
            for (uint64_t k = 0; k < ed.second; ++k) {
                const uint32_t v = ed.first[k];
                if (v & EDGE_SET) {
                    if ((v & EDGE_VAL) != EDGE_POISON) __atomic_fetch_add(&indeg[v & EDGE_VAL], 1u, __ATOMIC_RELAXED);
                } else if (v != EDGE_POISON) {
                    __atomic_fetch_add(&idc[v], 1u, __ATOMIC_RELAXED);
                }
            }
        }
    });
    // offsets: [count, entries...] per key
    std::vector<uint32_t> rkeys, roffs, pkeys, poffs;
    std::vector<uint64_t> rcur(NR), pcur(idc.size());
    uint64_t rw = 0, pw = 0;
    for (uint32_t r = 0; r < NR; ++r)
        if (indeg[r]) {
            if (!S.mapped(r)) throw Error{KETO_E_INVALID, "reach index: a subject set's row is not on this device"};
            rkeys.push_back(S.unit_of_row[r]);
            roffs.push_back((uint32_t)rw);
            rcur[r] = rw + 1;
            rw += 1ull + indeg[r];
            if (rw >= INLINE) throw Error{KETO_E_RANGE, "reach index exceeds 2^31 words"};
        }
    for (uint64_t v = 0; v < idc.size(); ++v)
        if (idc[v]) {
            pkeys.push_back((uint32_t)v);
            poffs.push_back((uint32_t)pw);
            pcur[v] = pw + 1;
            pw += 1ull + idc[v];
            if (pw >= INLINE) throw Error{KETO_E_RANGE, "reach index exceeds 2^31 words"};
        }
    std::vector<uint32_t> rev(std::max<uint64_t>(rw, 1)), post(std::max<uint64_t>(pw, 1));
    par_chunks(NR, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t r = b; r < e; ++r) {
            if (!kept((uint32_t)r)) continue;
            const uint32_t h = S.unit_of_row[r];
            const auto ed = edges_of((uint32_t)r);
            for (uint64_t k = 0; k < ed.second; ++k) {
                const uint32_t v = ed.first[k];
                if (v & EDGE_SET) {
                    if ((v & EDGE_VAL) == EDGE_POISON) continue;
                    const uint64_t at = __atomic_fetch_add(&rcur[v & EDGE_VAL], 1ull, __ATOMIC_RELAXED);
                    rev[at] = h;
                } else if (v != EDGE_POISON) {
                    const uint64_t at = __atomic_fetch_add(&pcur[v], 1ull, __ATOMIC_RELAXED);
                    post[at] = h;
                }
            }
        }
    });
    // counts: filled positions minus the start
    par_chunks(NR, th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t r = b; r < e; ++r)
            if (indeg[r]) rev[rcur[r] - indeg[r] - 1] = indeg[r];
    });
    par_chunks(idc.size(), th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t v = b; v < e; ++v)
            if (idc[v]) post[pcur[v] - idc[v] - 1] = idc[v];
    });
    // reverse lists of one or two parents go into the index word itself
    uint32_t rmax = 0;
    for (uint32_t k : rkeys) rmax = std::max(rmax, k + 1);
    std::vector<uint64_t> rd(std::max<uint32_t>(rmax, 1), ~0ull);
    par_chunks(rkeys.size(), th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t k = b; k < e; ++k) {
            const uint32_t o = roffs[k], c = rev[o];
            uint64_t v;
            if (c == 1) v = (1ull << 62) | rev[o + 1];
            else if (c == 2) v = (2ull << 62) | ((uint64_t)rev[o + 2] << 31) | rev[o + 1];
            else v = (3ull << 62) | o;
            rd[rkeys[k]] = v;
        }
    });
    par_chunks(pkeys.size(), th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t k = b; k < e; ++k)
            if (post[poffs[k]] == 1) poffs[k] = INLINE | post[poffs[k] + 1];
    });
    const std::vector<uint32_t> pd = make_dir(pkeys, poffs, th);
    uint64_t acc = 0;
    R.rdir = ralloc<uint64_t>(rd.size(), acc);
    R.rev = ralloc<uint32_t>(rev.size(), acc);
    R.pdir = ralloc<uint32_t>(pd.size(), acc);
    R.post = ralloc<uint32_t>(post.size(), acc);
    HIP_OK(hipMemcpy(R.rdir, rd.data(), rd.size() * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(R.rev, rev.data(), rev.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(R.pdir, pd.data(), pd.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(R.post, post.data(), post.size() * 4, hipMemcpyHostToDevice));
    R.rn = (uint32_t)rd.size();
    R.pn = (uint32_t)pd.size();
    R.bytes = acc;
    R.version = S.version;
    R.built = true;
    R.build_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e ? (uint32_t)std::max(0, atoi(e)) : dflt;
}

}  // namespace

bool reach_enabled(const Snapshot& S) {
    if (S.n_parts > 1 || S.part_mode == PART_MIGRATE) return false;
    const char* e = getenv("KETO_ITEMS");
    return !(e && atoi(e) == 0);
}

float reach_build_ms(const Snapshot& S) { return S.reach ? S.reach->build_ms : 0.f; }

bool reach_split(Snapshot& S, const keto_check_ids* dq, uint32_t n, int32_t gmd, uint8_t* da, uint32_t ov_base,
                 void* stream, bool steps, ItemWork& out) {
    if (!reach_enabled(S) || n == 0) return false;
    const DevView V = device_view(S);
    if (!S.reach) {
        S.reach.reset(new ReachState);
        S.reach->device = V.device;
    }
    ReachState& R = *S.reach;
    hipStream_t st = (hipStream_t)stream;
    out.index_ms = 0;
    if (!R.built || R.version != S.version) {
        build_index(S, R);
        out.index_ms = R.build_ms;
    }
    hipEvent_t e0, e1, ea, eb;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventCreate(&ea));
    HIP_OK(hipEventCreate(&eb));
    HIP_OK(hipEventRecord(e0, st));
    const ReachDev rd{V.arena, R.rdir, R.rev, R.rn, R.pdir, R.post, R.pn, ov_base, S.root_g};
    uint32_t* acc = R.acc.get<uint32_t>(n);
    uint32_t* cnt = R.cnt.get<uint32_t>((uint64_t)n + 1);
    uint32_t* off = R.off.get<uint32_t>((uint64_t)n + 1);
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(split_count, g, b, 0, st, rd, dq, n, gmd, da, acc, cnt);
    HIP_OK(hipGetLastError());
    // work entries: items and whole requests (PASS bit masked out of the counts)
    HIP_OK(hipMemsetAsync(cnt + n, 0, sizeof(uint32_t), st));
    struct Unpass {
        __host__ __device__ uint32_t operator()(uint32_t c) const { return c & ~PASS; }
    };
    hipcub::TransformInputIterator<uint32_t, Unpass, const uint32_t*> cit(cnt, Unpass{});
    size_t tb = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cit, off, (uint64_t)n + 1, st));
    void* tmp = R.tmp.get<uint8_t>(tb);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cit, off, (uint64_t)n + 1, st));
    uint32_t m = 0;
    HIP_OK(hipMemcpyAsync(&m, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    keto_check_ids* work = R.work.get<keto_check_ids>(m);
    uint32_t* owner = R.owner.get<uint32_t>(m);
    hipLaunchKernelGGL(split_fill, g, b, 0, st, rd, dq, n, gmd, cnt, off, work, owner);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ea, st));
    // pretest lanes: marks / lists kept across batches
    const uint32_t cap = pow2_ge(std::max<uint32_t>(64, env_u32("KETO_REACH_CAP", 2048)));
    const uint32_t want_lanes = std::min<uint32_t>(std::max<uint32_t>(256, env_u32("KETO_REACH_LANES", 65536)) / 256 * 256,
                                                   std::max<uint32_t>(256, (m + 255) / 256 * 256));
    if (R.lanes < want_lanes || R.cap != cap) {
        for (void* p : {(void*)R.marks, (void*)R.lists, (void*)R.epochs})
            if (p) (void)hipFree(p);
        R.marks = nullptr;
        R.lists = nullptr;
        R.epochs = nullptr;
        R.lanes = 0;
        uint64_t a = 0;
        R.marks = ralloc<uint64_t>((uint64_t)want_lanes * 2 * cap, a);
        R.lists = ralloc<uint32_t>((uint64_t)want_lanes * 2 * cap, a);
        R.epochs = ralloc<uint32_t>(want_lanes, a);
        HIP_OK(hipMemsetAsync(R.marks, 0, (uint64_t)want_lanes * 2 * cap * 8, st));
        HIP_OK(hipMemsetAsync(R.epochs, 0, (uint64_t)want_lanes * 4, st));
        R.lanes = want_lanes;
        R.cap = cap;
    }
    uint32_t* ctr = R.ctr.get<uint32_t>(4);
    HIP_OK(hipMemsetAsync(ctr, 0, 4 * sizeof(uint32_t), st));
    const Pretest P{R.marks, R.lists, R.epochs, cap, std::max<uint32_t>(1, env_u32("KETO_REACH_WORK", 4096)), ctr};
    uint8_t* keep = R.keep.get<uint8_t>(m);
    const uint32_t lanes = std::min<uint32_t>(R.lanes, std::max<uint32_t>(256, (m + 255) / 256 * 256));
    if (m) {
        const uint32_t mode = env_u32("KETO_REACH_PRETEST", 2);   // 2 = wave per item, 1 = lane per item
        if (mode == 2) {
            // LDS per wave: 4096 mark slots + 2048 handles (24 KB, 6 waves per CU), or half that
            const bool small = env_u32("KETO_REACH_WAVE_SLOTS", 4096) <= 2048;
            auto kern = small ? pretest_wave_kernel<2048> : pretest_wave_kernel<4096>;
            uint32_t& wb = R.wave_blocks[small ? 1 : 0];
            if (!wb) {
                int per_cu = 0, cus = 0;
                HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
                HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, V.device));
                wb = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus);
            }
            HIP_OK(hipMemsetAsync(keep, 1, m, st));
            const uint32_t blocks = std::min<uint32_t>(wb, std::max<uint32_t>(1, (m + 63) / 64));
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, st, rd, work, m, keep, ctr + 2, P.work_cap,
                               (int)env_u32("KETO_REACH_MIN_DEPTH", 16));
        } else if (mode == 1) {
            hipLaunchKernelGGL(pretest_kernel, dim3(lanes / 256), dim3(256), 0, st, rd, P, work, m, keep);
        } else {
            HIP_OK(hipMemsetAsync(keep, 1, m, st));
        }
        HIP_OK(hipGetLastError());
    }
    HIP_OK(hipEventRecord(eb, st));
    // the kept entries: deep items first (max-depth >= KETO_REACH_FIRST_DEPTH, default 16), so that the
    // searches that can run long hold lanes from the start of the check instead of waiting for one;
    // the rest after them, each class in request order
    keto_check_ids* work2 = R.work2.get<keto_check_ids>(m);
    uint32_t* owner2 = R.owner2.get<uint32_t>(m);
    uint32_t* nsel = R.nsel.get<uint32_t>(4);
    uint8_t* fl = R.flags.get<uint8_t>(2ull * std::max<uint32_t>(m, 1));
    uint32_t kept[2] = {0, 0};
    if (m) {
        hipLaunchKernelGGL(classify_kept, dim3((m + 255) / 256), dim3(256), 0, st, work, keep, m,
                           (int)env_u32("KETO_REACH_FIRST_DEPTH", 16), fl, fl + m);
        HIP_OK(hipGetLastError());
        size_t t1 = 0, t2 = 0;
        HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, t1, work, fl, work2, nsel, m, st));
        HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, t2, owner, fl, owner2, nsel + 1, m, st));
        tmp = R.tmp.get<uint8_t>(std::max(t1, t2));
        uint32_t first[2] = {0, 0};
        HIP_OK(hipcub::DeviceSelect::Flagged(tmp, t1, work, fl, work2, nsel, m, st));
        HIP_OK(hipcub::DeviceSelect::Flagged(tmp, t2, owner, fl, owner2, nsel + 1, m, st));
        HIP_OK(hipMemcpyAsync(first, nsel, sizeof(first), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipcub::DeviceSelect::Flagged(tmp, t1, work, fl + m, work2 + first[0], nsel + 2, m, st));
        HIP_OK(hipcub::DeviceSelect::Flagged(tmp, t2, owner, fl + m, owner2 + first[0], nsel + 3, m, st));
        uint32_t second[2] = {0, 0};
        HIP_OK(hipMemcpyAsync(second, nsel + 2, sizeof(second), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        kept[0] = first[0] + second[0];
        kept[1] = first[1] + second[1];
    }
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipStreamSynchronize(st));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    if (getenv("KETO_REACH_TRACE")) {          // phase timing (tooling)
        float a = 0, b2 = 0, c = 0;
        HIP_OK(hipEventElapsedTime(&a, e0, ea));
        HIP_OK(hipEventElapsedTime(&b2, ea, eb));
        HIP_OK(hipEventElapsedTime(&c, eb, e1));
        fprintf(stderr, "reach: split %.3f ms, pretest %.3f ms, select %.3f ms; %u requests, %u work, %u kept\n", a, b2, c, n,
                m, kept[0]);
    }
    (void)hipEventDestroy(ea);
    (void)hipEventDestroy(eb);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    out.work = work2;
    out.owner = owner2;
    out.n_work = kept[0];
    out.n_entries = m;
    out.acc = acc;
    out.dec = R.dec.get<uint8_t>(std::max<uint32_t>(kept[0], 1));
    out.wsteps = steps ? R.wsteps.get<uint32_t>(std::max<uint32_t>(kept[0], 1)) : nullptr;
    if (out.wsteps) HIP_OK(hipMemsetAsync(out.wsteps, 0, (uint64_t)std::max<uint32_t>(kept[0], 1) * 4, st));
    out.split_ms = ms;
    out.undecided = ctr + 1;
    return true;
}

void reach_merge(Snapshot& S, const ItemWork& w, uint32_t n, uint8_t* da, uint32_t* d_steps, void* stream,
                 uint32_t* undecided) {
    hipStream_t st = (hipStream_t)stream;
    (void)S;
    if (w.n_work) {
        hipLaunchKernelGGL(merge_kernel, dim3((w.n_work + 255) / 256), dim3(256), 0, st, w.dec, w.owner, w.n_work, w.acc,
                           w.wsteps, d_steps);
        HIP_OK(hipGetLastError());
    }
    hipLaunchKernelGGL(final_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.acc, n, da, w.undecided);
    HIP_OK(hipGetLastError());
    uint32_t u = 0;
    HIP_OK(hipMemcpyAsync(&u, w.undecided, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    *undecided = u;
}

}  // namespace keto
