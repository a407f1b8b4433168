// Migrating partition (PART_MIGRATE): check batches over a graph whose rows are ALL split across
// parts by hash(namespace id, object), for graphs whose shared rows (folders, groups) no longer fit
// on one GPU (SURVEY.md 8(e) "partitioned mode"; DESIGN.md "Multi-GPU").
//
// The reference answers a check with an ordered DFS whose visited map marks nodes on first
// encounter (internal/check/engine.go:36-114, internal/x/graph/graph_utils.go:13-35), so the
// search cannot be cut into level-synchronous frontier exchanges without changing answers.  It is
// cut at part crossings instead: a lane walks the DFS on its part; when the walk enters a subject
// set whose row another part owns (a stub: HDR_REMOTE), or pops back to a frame of a row another
// part owns, it writes the whole DFS state -- request, saved frames, visited map -- as a
// continuation record, and the owner resumes the DFS there in the next round.  The order of events
// inside every search stays the reference's, so answers stay exact.  Rounds exchange records with
// one all-to-all each (keto_amd/multi.py); a decided request sends its decision to the part that
// started it.
//
// Visit ids are global: (owner part, handle on the owner) for rows, (30, handle) for the hot rows
// every part holds at the same handle (the prefix [0, hot_units) of every part's arena), (31, class)
// for colliding Subject.String() keys (collision classes are computed on the host for the whole
// graph).
//
// Record (u32 words, 16-B units):
//   head 8 words: idx (request index on its origin part) | info (kind 0..1, tset 2, decision 3..4,
//   enter flags 5..7, origin part 8..15) | T (string id, or the set target's handle) | T's owner part
//   (set targets) | enter handle | enter remaining depth | saved frames ns | visit ids nv
//   ns frames of 16 B {pos lo, pos hi | part << 8, edges left, depth | flags << 16}
//   nv visit ids of 8 B
// ENTER: enter the row `enter` (a row of the receiving part) at the given depth, as the walk would
// after the hop; RESUME: pop the top saved frame (a frame of the receiving part); DECISION: the
// request's decision, for its origin part.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "snapshot.hpp"

namespace keto {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t MAX_ROUND_RECORDS = 1ull << 28;   // record counts are 28-bit fields of the grouping cursors
constexpr uint32_t HEAD_WORDS = 8;
constexpr uint32_t START_UNITS = 3;                 // a START record: the head and one visit id
constexpr uint32_t K_ENTER = 0, K_RESUME = 1, K_DECISION = 2;
constexpr uint32_t F_SEQ = 1, F_TOP = 2;            // frame flags
constexpr uint32_t MIG_FRAMES = 64;                 // saved frames of one search (max-depth <= 65)
constexpr uint64_t VID_CLASS_PART = 31;
constexpr uint32_t VID_HOT_PART = 30;                // rows every part holds (hot_units prefix)
constexpr uint32_t EPOCH_MAX = (1u << 28) - 1u;
constexpr int RES_FALSE = 0, RES_TRUE = 1, RES_UNDECIDED = 2, RES_BIG = 3;
// two lane tiers: many lanes with small visited tables, and a few with big ones for the searches
// whose maps outgrow the small ones (re-run from their input record, which is exact: a record's
// processing is deterministic and an overflowed lane has emitted nothing)
constexpr uint32_t VCAP_SMALL = 512, VCAP_BIG = 1u << 16;
constexpr uint32_t LANES_SMALL = 256 * 1024, LANES_BIG = 512;

__host__ __device__ inline uint32_t mixv(uint64_t v) {
    uint64_t k = v * 0x9E3779B97F4A7C15ull;
    k ^= k >> 29;
    k *= 0xBF58476D1CE4E5B9ull;
    return (uint32_t)(k >> 32);
}
__device__ inline uint64_t vid_row(uint32_t part, uint32_t handle) { return ((uint64_t)part << 31) | handle; }
__device__ inline uint64_t vid_class(uint32_t c) { return (VID_CLASS_PART << 31) | (c & 0x7FFFFFFFu); }

// the hash of engine.hip's id tables and collision table (same layouts)
__device__ inline uint32_t mix32d(uint32_t k) {
    k ^= k >> 16;
    k *= 0x7feb352dU;
    k ^= k >> 15;
    k *= 0x846ca68bU;
    k ^= k >> 16;
    return k;
}

__device__ inline uint32_t coll_find(const uint64_t* coll, uint32_t mask, uint32_t key) {
    if (mask == 0) return NONE;
    for (uint32_t i = mix32d(key) & mask;; i = (i + 1) & mask) {
        const uint64_t e = coll[i];
        if (e == ~0ull) return NONE;
        if ((uint32_t)(e >> 32) == key) return (uint32_t)e;
    }
}

// A visited map: its first MIG_LDS_VIDS ids in the lane's LDS column, behind a 64-bit filter in
// registers (a test the filter rules out, and an insert, touch no memory; a filter hit scans the
// column); past that, the lane's HBM table (epoch-tagged: entry = epoch << 36 | visit id) takes every
// id, as before round 6.  The insertion log (LDS column, then the HBM log) lets the whole map travel
// in a record.  (Every test had been a dependent HBM probe: profiles/r06y_migrate_lds_map.log.)
constexpr uint32_t MIG_LDS_VIDS = 16;
struct MigVisited {
    uint64_t* tab;
    uint64_t* log;
    uint32_t mask, cap;      // cap = ids a map may hold (half the table)
    uint32_t epoch, n;
    uint64_t* lv;            // the lane's LDS column: entry k at lv[k * 256]
    uint64_t filt;
    bool big;                // the map lives in the HBM table
    __device__ inline uint64_t at(uint32_t k) const { return big ? log[k] : lv[(uint64_t)k * 256]; }
    __device__ inline void fresh() {
        n = 0;
        filt = 0;
        big = false;
    }
    __device__ inline int tab_add(uint64_t vid) {
        uint32_t i = mixv(vid) & mask;
        const uint64_t want = ((uint64_t)epoch << 36) | vid;
        for (;;) {
            const uint64_t e = tab[i];
            if ((uint32_t)(e >> 36) != epoch) {
                if (n >= cap) return 2;
                tab[i] = want;
                log[n++] = vid;
                return 0;
            }
            if (e == want) return 1;
            i = (i + 1) & mask;
        }
    }
    // 0 = new, 1 = present, 2 = the map is full
    __device__ inline int test_add(uint64_t vid) {
        if (!big) {
            const uint64_t b = 1ull << (mixv(vid) & 63u);
            if (filt & b)
                for (uint32_t k = 0; k < n; ++k)
                    if (lv[(uint64_t)k * 256] == vid) return 1;
            if (n < MIG_LDS_VIDS && n < cap) {
                lv[(uint64_t)n * 256] = vid;
                ++n;
                filt |= b;
                return 0;
            }
            // the column is full: the map moves to the HBM table (a fresh epoch), then takes vid there
            if (++epoch > EPOCH_MAX) {
                for (uint32_t i = 0; i <= mask; ++i) tab[i] = 0;
                epoch = 1;
            }
            const uint32_t m = n;
            n = 0;
            big = true;
            for (uint32_t k = 0; k < m; ++k)
                if (tab_add(lv[(uint64_t)k * 256]) == 2) return 2;
        }
        return tab_add(vid);
    }
};

struct MigArgs {
    const uint32_t* arena;
    const uint64_t* coll;
    uint32_t coll_mask;
    uint32_t self;
    // input records: record j of source s (rec_base[s] <= j < rec_base[s + 1]) starts at unit
    // unit_base[s] + in_off[j]
    const uint32_t* in;
    const uint32_t* in_off;
    const uint32_t* rec_base;
    const uint64_t* unit_base;
    uint32_t n_src;
    uint32_t n_in;
    const uint32_t* list;        // NULL: every input record; else list[0 .. *n_list)
    const uint32_t* n_list;
    // output records (unordered pool) and their (destination, unit, length)
    uint32_t* pool;
    uint64_t pool_cap;
    unsigned long long* pool_used;
    uint32_t* out_dest;
    uint32_t* out_unit;
    uint32_t* out_len;
    uint32_t* out_count;
    uint32_t* spill;             // inputs whose record did not fit the pool
    uint32_t* n_spill;
    uint32_t* big;               // inputs whose map outgrew this tier's tables
    uint32_t* n_big;
    uint8_t* allowed;            // decisions of this part's own requests
    uint32_t* stats;             // [0] decided here, [1] undecided, [2] records handled
    // lane workspaces
    uint64_t* vtab;
    uint64_t* vlog;
    uint4* frames;
    uint32_t* lane_epoch;
    uint32_t vcap;
    // bounds of every index the kernel follows: a record or handle out of range is reported
    // (err: [0] count, [1] first code, [2] its input record, [3] its value) and the search is
    // dropped as KETO_UNDECIDED instead of reading out of bounds
    uint64_t arena_words;
    uint64_t in_units;
    uint32_t n_allowed;
    uint32_t n_parts;
    uint32_t* err;
    uint32_t hot_units;          // handles below it are rows every part holds at the same handle
};

constexpr uint32_t E_RECORD = 1, E_HANDLE = 2, E_POS = 3, E_IDX = 4, E_DEST = 5;
__device__ inline void report(const MigArgs& a, uint32_t code, uint32_t rj, uint64_t v) {
    if (atomicAdd(a.err, 1u) == 0) {
        a.err[1] = code;
        a.err[2] = rj;
        a.err[3] = (uint32_t)v;
    }
}

// What one input record turned into.
struct Outcome {
    int res;                     // RES_* decision, or -1: a continuation record (dest, kind, enter, k)
    uint32_t dest, kind, enter, k;
    uint32_t idx, origin;
    uint32_t t_lo, t_hi;
    bool tset;
    bool skip;                   // nothing to emit (a decision written here, a bad record, a re-run)
};

// The search of one input record on this part, until it is decided or crosses to another part.
// Uses the lane's visited table (V) and frame stack (fr); sp = saved frames on return.
__device__ inline Outcome run_record(const MigArgs& a, uint32_t rj, MigVisited& V, uint4* fr, uint32_t& sp) {
    Outcome o{-1, NONE, 0, 0, 0, 0, 0, 0, 0, false, true};
    sp = 0;
    uint32_t s = 0;
    while (s + 1 < a.n_src && a.rec_base[s + 1] <= rj) ++s;
    const uint64_t at_unit = a.unit_base[s] + a.in_off[rj];
    if (at_unit + 2 > a.in_units) {
        report(a, E_RECORD, rj, at_unit);
        return o;
    }
    const uint32_t* rec = a.in + at_unit * 4ull;
    const uint4 h0 = *reinterpret_cast<const uint4*>(rec);
    const uint4 h1 = *reinterpret_cast<const uint4*>(rec + 4);
    const uint32_t idx = h0.x, info = h0.y;
    const uint32_t kind = info & 3u, origin = (info >> 8) & 0xFFu;
    if (origin >= a.n_parts || kind > K_DECISION) {
        report(a, E_RECORD, rj, info);
        return o;
    }
    if (kind == K_DECISION) {
        if (origin != a.self || idx >= a.n_allowed) {
            report(a, E_IDX, rj, idx);
            return o;
        }
        a.allowed[idx] = (uint8_t)((info >> 3) & 3u);
        o.res = RES_FALSE;                                            // counted as decided here
        o.dest = NONE;
        o.skip = false;
        return o;
    }
    if (h1.z > MIG_FRAMES || at_unit + 2 + h1.z + (h1.w + 1ull) / 2 > a.in_units) {
        report(a, E_RECORD, rj, h1.z);
        return o;
    }
    o.idx = idx;
    o.origin = origin;
    o.t_lo = h0.z;
    o.t_hi = h0.w;
    const bool tset = (info >> 2) & 1u;
    o.tset = tset;
    const uint32_t T = h0.z;
    const uint64_t T64 = vid_row(h0.w, h0.z);
    uint32_t cw = 0, cb = 0;
    closure_bit(T, cw, cb);
    int res = -1;
    // restore the map and the saved frames
    V.fresh();
    const uint32_t ns = h1.z, nv = h1.w;
    if (nv > V.cap) res = RES_BIG;
    const uint64_t* rv = reinterpret_cast<const uint64_t*>(rec + HEAD_WORDS + 4ull * ns);
    for (uint32_t i = 0; i < nv && res < 0; ++i)
        if (V.test_add(rv[i]) == 2) res = RES_BIG;
    sp = ns;
    for (uint32_t i = 0; i < ns; ++i) fr[i] = *reinterpret_cast<const uint4*>(rec + HEAD_WORDS + 4ull * i);
    uint64_t pos = 0;
    uint32_t left = 0, k = 0, fl = 0;
    bool have = false;
    uint32_t enter = NONE, enter_k = 0, enter_fl = 0;
    if (kind == K_ENTER) {
        enter = h1.x;
        enter_k = h1.y;
        enter_fl = (info >> 5) & 7u;
    }
    while (res < 0) {
        if (enter != NONE) {
            uint64_t hw = (uint64_t)enter * HDR_WORDS;
            if (hw + 2 * HDR_WORDS > a.arena_words) {
                report(a, E_HANDLE, rj, enter);
                res = RES_UNDECIDED;
                break;
            }
            uint4 hd = *reinterpret_cast<const uint4*>(a.arena + hw);
            while ((hd.z & HDR_FWD) && (uint64_t)hd.x * HDR_WORDS + 2 * HDR_WORDS <= a.arena_words) {
                hw = (uint64_t)hd.x * HDR_WORDS;
                hd = *reinterpret_cast<const uint4*>(a.arena + hw);
            }
            const uint32_t n_sets = hd.x, n_ids = hd.y;
            const bool seq = (hd.z & HDR_SEQ) != 0;
            const uint32_t hl = (hd.z >> 8) & 31u;
            const uint64_t beg = hw + HDR_WORDS;
            const uint64_t tbl = (hl ? (1ull << hl) : 0ull) + ((hd.z & HDR_CLOSURE) ? CB_WORDS : 0u);
            if ((hd.z & (HDR_REMOTE | HDR_FWD)) || hl == 1 || beg + (uint64_t)n_sets + n_ids > a.arena_words ||
                hw < tbl) {
                report(a, E_POS, rj, enter);
                res = RES_UNDECIDED;
                break;
            }
            if (!seq && !tset && n_ids > 0) {                         // is the requested id in the row?
                bool hit = false;
                if (hl == 0) {
                    const uint4 w = *reinterpret_cast<const uint4*>(a.arena + beg);   // the window
                    for (uint32_t i = n_sets; i < n_sets + n_ids && i < WINDOW_WORDS; ++i)
                        hit |= (i == 0 ? w.x : i == 1 ? w.y : i == 2 ? w.z : w.w) == T;
                } else {
                    uint32_t b1, b2;
                    bloom_bits(T, b1, b2);
                    if (bloom_has(hd.z, hd.w, b1) && bloom_has(hd.z, hd.w, b2)) {
                        const uint32_t nb = (1u << hl) / BUCKET_WORDS;
                        const uint64_t tb = hw - tbl;
                        uint32_t b = mix32d(T) & (nb - 1);
                        for (uint32_t probe = 0; probe < nb; ++probe, b = (b + 1) & (nb - 1)) {   // load <= 1/2
                            const uint4 v = *reinterpret_cast<const uint4*>(a.arena + tb + (uint64_t)b * BUCKET_WORDS);
                            if (v.x == T || v.y == T || v.z == T || v.w == T) {
                                hit = true;
                                break;
                            }
                            if (v.x == NONE || v.y == NONE || v.z == NONE || v.w == NONE) break;
                        }
                    }
                }
                if (hit) {
                    res = RES_TRUE;
                    break;
                }
            }
            if (have && left > 0) {                                   // the parent keeps its place
                if (sp >= MIG_FRAMES) {
                    res = RES_UNDECIDED;
                    break;
                }
                fr[sp++] = make_uint4((uint32_t)pos, (uint32_t)(pos >> 32) | (a.self << 8), left, k | (fl << 16));
            }
            pos = beg;
            left = n_sets;
            k = enter_k;
            fl = enter_fl | (seq ? F_SEQ : 0u);
            have = true;
            enter = NONE;
            continue;
        }
        if (!have || left == 0) {                                     // row done: pop
            if (sp == 0) {
                res = RES_FALSE;
                break;
            }
            const uint4 f = fr[sp - 1];
            const uint32_t part = f.y >> 8;
            if (part >= a.n_parts ||
                (part == a.self && ((uint64_t)f.x | ((uint64_t)(f.y & 0xFFu) << 32)) + f.z > a.arena_words)) {
                report(a, E_POS, rj, f.x);
                res = RES_UNDECIDED;
                break;
            }
            if (part != a.self) {                                     // the parent lives elsewhere
                o.dest = part;
                o.kind = K_RESUME;
                break;
            }
            --sp;
            pos = (uint64_t)f.x | ((uint64_t)(f.y & 0xFFu) << 32);
            left = f.z;
            k = f.w & 0xFFFFu;
            fl = f.w >> 16;
            have = true;
            continue;
        }
        const uint32_t e = a.arena[pos];
        ++pos;
        --left;
        if (e & EDGE_SET) {
            const uint32_t child = e & EDGE_VAL;
            const uint64_t cw4 = (uint64_t)child * HDR_WORDS;
            if (cw4 < CB_WORDS || cw4 + 2 * HDR_WORDS > a.arena_words) {
                report(a, E_HANDLE, rj, child);
                res = RES_UNDECIDED;
                break;
            }
            const uint4 ch = *reinterpret_cast<const uint4*>(a.arena + cw4);
            const bool remote = (ch.z & HDR_REMOTE) != 0;
            if (remote && ch.x >= a.n_parts) {
                report(a, E_DEST, rj, ch.x);
                res = RES_UNDECIDED;
                break;
            }
            const uint64_t rvid = remote ? vid_row(ch.x, ch.y) : vid_row(child < a.hot_units ? VID_HOT_PART : a.self, child);
            uint64_t vid = rvid;
            if (fl & F_SEQ) {
                const uint32_t c = coll_find(a.coll, a.coll_mask, e);
                if (c != NONE) vid = vid_class(c);
            }
            if (fl & F_TOP) V.fresh();                                // a fresh map per top-level tuple
            const int t = V.test_add(vid);
            if (t == 2) {
                res = RES_BIG;
                break;
            }
            if (t == 1) continue;
            if (tset && rvid == T64) {                                // engine.go:54-57
                res = RES_TRUE;
                break;
            }
            if (k < 2) continue;                                      // remaining depth after the hop >= 1
            if (!tset && (ch.z & HDR_CLOSURE) && !((a.arena[cw4 - CB_WORDS + cw] >> cb) & 1u))
                continue;                                             // T is not below this set
            if (remote) {                                             // the walk goes on on the owner
                if (left > 0) {
                    if (sp >= MIG_FRAMES) {
                        res = RES_UNDECIDED;
                        break;
                    }
                    fr[sp++] = make_uint4((uint32_t)pos, (uint32_t)(pos >> 32) | (a.self << 8), left, k | (fl << 16));
                }
                o.dest = ch.x;
                o.kind = K_ENTER;
                o.enter = ch.y;
                o.k = k - 1;
                break;
            }
            enter = child;
            enter_k = k - 1;
            enter_fl = 0;
        } else {                                                      // a subject id of an ordered row
            int t = 0;
            if (!(fl & F_TOP)) {
                const uint32_t c = coll_find(a.coll, a.coll_mask, e);
                if (c != NONE) t = V.test_add(vid_class(c));
            }
            if (t == 2) {
                res = RES_BIG;
                break;
            }
            if (t == 0 && !tset && e == T) res = RES_TRUE;
        }
    }
    if (res == RES_BIG) {                                             // re-run on the big tier
        if (a.big) {
            a.big[atomicAdd(a.n_big, 1u)] = rj;
            return o;                                                 // skip
        }
        res = RES_UNDECIDED;
    }
    o.res = res;
    if (res >= 0) {
        if (origin == a.self) {
            if (idx >= a.n_allowed) {
                report(a, E_IDX, rj, idx);
                return o;
            }
            a.allowed[idx] = (uint8_t)res;
            o.dest = NONE;                                            // decided here: nothing to send
        } else {
            o.dest = origin;
            o.kind = K_DECISION;
        }
    }
    o.skip = false;
    return o;
}

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// inclusive prefix sum over the 64 lanes of a wave (every lane active)
__device__ inline uint32_t wave_scan(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(v, (unsigned)d);
        if (lane >= (uint32_t)d) v += x;
    }
    return v;
}

// One search state machine per lane over the round's input records (persistent grid).  The loop
// runs the same number of times on every lane of a wave, so a record's output is placed with
// wave-wide prefix sums and one atomic per wave instead of one per record.
__global__ void __launch_bounds__(256) mig_kernel(MigArgs a) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t stride = gridDim.x * blockDim.x;
    __shared__ uint64_t s_vids[MIG_LDS_VIDS * 256];
    MigVisited V{a.vtab + (uint64_t)slot * a.vcap, a.vlog + (uint64_t)slot * (a.vcap / 2), a.vcap - 1u, a.vcap / 2,
                 a.lane_epoch[slot], 0, s_vids + threadIdx.x, 0, false};
    uint4* const fr = a.frames + (uint64_t)slot * MIG_FRAMES;
    const uint32_t total = a.list ? *a.n_list : a.n_in;
    uint32_t n_dec = 0, n_und = 0, n_in = 0;
    for (uint32_t base = slot - lane; base < total; base += stride) {
        const uint32_t j = base + lane;
        uint32_t sp = 0;
        Outcome o{-1, NONE, 0, 0, 0, 0, 0, 0, 0, false, true};
        if (j < total) {
            ++n_in;
            o = run_record(a, a.list ? a.list[j] : j, V, fr, sp);
        }
        const bool out = !o.skip && o.dest != NONE;
        if (!o.skip && o.res >= 0 && o.dest == NONE) {
            ++n_dec;
            if (o.res == RES_UNDECIDED) ++n_und;
        }
        if (!o.skip && o.res == RES_UNDECIDED && o.dest != NONE) ++n_und;
        // place the record: units and record slots by wave prefix sums, one atomic each per wave
        const uint32_t units = out ? (o.res >= 0 ? 2u : 2u + sp + (V.n + 1) / 2) : 0u;
        const uint32_t incl = wave_scan(units);
        const uint32_t wave_units = __shfl(incl, 63);
        if (wave_units == 0) continue;
        unsigned long long ub = 0;
        if (lane == 0) ub = atomicAdd(a.pool_used, (unsigned long long)wave_units);
        ub = __shfl(ub, 0);
        const unsigned long long u = ub + incl - units;
        const bool fits = out && u + units <= a.pool_cap;
        const uint64_t m = __ballot(fits);
        uint32_t rb = 0;
        if (lane == 0 && m) rb = atomicAdd(a.out_count, (uint32_t)__popcll(m));
        rb = __shfl(rb, 0);
        if (out && !fits) a.spill[atomicAdd(a.n_spill, 1u)] = a.list ? a.list[j] : j;   // re-run once the pool has grown
        if (!fits) continue;
        const uint32_t at = rb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint32_t nso = o.res >= 0 ? 0u : sp, nvo = o.res >= 0 ? 0u : V.n;
        uint32_t* ow = a.pool + u * 4ull;
        // (an ENTER record's row is never a top-level row: enter flags 0)
        const uint32_t oinfo = o.kind | (o.tset ? 4u : 0u) | ((o.res >= 0 ? (uint32_t)o.res : 0u) << 3) | (o.origin << 8);
        *reinterpret_cast<uint4*>(ow) = make_uint4(o.idx, oinfo, o.t_lo, o.t_hi);
        *reinterpret_cast<uint4*>(ow + 4) = make_uint4(o.enter, o.k, nso, nvo);
        for (uint32_t i = 0; i < nso; ++i) *reinterpret_cast<uint4*>(ow + HEAD_WORDS + 4ull * i) = fr[i];
        uint64_t* ov = reinterpret_cast<uint64_t*>(ow + HEAD_WORDS + 4ull * nso);
        for (uint32_t i = 0; i < nvo; ++i) ov[i] = V.at(i);
        if (nvo & 1u) ov[nvo] = 0;
        a.out_dest[at] = o.dest;
        a.out_unit[at] = (uint32_t)u;
        a.out_len[at] = units;
    }
    a.lane_epoch[slot] = V.epoch;
    // statistics: one atomic per wave
    const uint32_t d = wave_scan(n_dec), un = wave_scan(n_und), ni = wave_scan(n_in);
    if (lane == 63) {
        if (d) atomicAdd(a.stats + 0, d);
        if (un) atomicAdd(a.stats + 1, un);
        if (ni) atomicAdd(a.stats + 2, ni);
    }
}

// START records of a routed batch (row-id requests of this part): the depth clamp
// (engine.go:118-120), the row's handle, a set target's global identity.  Trivial requests become
// DECISION records for this part.  Each record takes START_UNITS units: the head, and room for one
// visit id -- a request for one top-level tuple of a wildcard query (KETO_CHILD_FLAG, when
// `child_entries`) enters its row below the top, the map holding the tuple's visit key, as
// run_record does after the hop from a top-level frame.
__global__ void __launch_bounds__(256) mig_start(const keto_check_ids* __restrict__ q, uint32_t n, int32_t gmd,
                                                 const uint32_t* __restrict__ g_handle,
                                                 const uint8_t* __restrict__ owner, uint32_t n_rows, uint32_t self,
                                                 uint32_t hot_units, uint32_t child_entries,
                                                 uint32_t* __restrict__ out, uint32_t* __restrict__ off,
                                                 uint32_t* misrouted) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const keto_check_ids r = q[i];
    int d = r.max_depth;
    if (d <= 0 || gmd < d) d = gmd;
    const bool child = child_entries && (r.flags & KETO_CHILD_FLAG);
    uint32_t info = K_ENTER | ((child ? 0u : F_TOP) << 5) | (self << 8);
    uint32_t t_lo = r.target, t_hi = 0, enter = NONE;
    bool trivial = r.row == KETO_NO_ROW || d <= 0 || r.target == KETO_NO_TARGET;
    if (!trivial) {
        if (r.row >= n_rows || owner[r.row] != self) {
            atomicAdd(misrouted, 1u);
            trivial = true;
        } else {
            enter = g_handle[r.row];
        }
    }
    if (!trivial && (r.flags & 1u)) {
        info |= 4u;
        if (r.target >= n_rows) {
            trivial = true;                                      // no such row: no tuple names it
        } else {
            t_lo = g_handle[r.target];
            t_hi = t_lo < hot_units ? VID_HOT_PART : owner[r.target];
        }
    }
    if (trivial) info = K_DECISION | (self << 8);              // denied (decision 0)
    uint32_t nv = 0;
    uint64_t vid = 0;
    if (!trivial && child) {
        const uint32_t cls = r.flags >> 8;
        vid = cls ? vid_class(cls - 1u) : vid_row(enter < hot_units ? VID_HOT_PART : self, enter);
        nv = 1;
    }
    uint32_t* o = out + (uint64_t)i * 4 * START_UNITS;
    *reinterpret_cast<uint4*>(o) = make_uint4(i, info, t_lo, t_hi);
    *reinterpret_cast<uint4*>(o + 4) = make_uint4(enter, (uint32_t)d, 0u, nv);
    *reinterpret_cast<uint4*>(o + 8) = make_uint4((uint32_t)vid, (uint32_t)(vid >> 32), 0u, 0u);
    off[i] = START_UNITS * i;
}

// group the round's output records by destination part, without a global atomic: each block takes
// a chunk of GROUP_CHUNK records and counts them per destination in LDS (mig_group_count), one block
// per destination turns the per-block counts into exclusive prefixes and the destination's total
// (mig_group_scan), and each block then places its chunk's records in input order after its prefix
// (mig_group_scatter).  (One 64-bit atomic per wave and destination on P cursors had serialized at
// the L2: 0.3-0.7 ms per round at 200K records, profiles/r06p_migrate_local.log.)  Counts are
// records << 36 | units.
constexpr uint32_t GROUP_CHUNK = 2048;               // records per block: 256 threads x 8
__device__ inline uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}
__global__ void __launch_bounds__(256) mig_group_count(const uint32_t* __restrict__ dest, const uint32_t* __restrict__ len,
                                                       uint32_t n, uint32_t n_parts, uint32_t n_blocks,
                                                       unsigned long long* __restrict__ bcnt) {
    __shared__ unsigned long long c[MIG_MAX_PARTS];
    if (threadIdx.x < n_parts) c[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * GROUP_CHUNK;
    for (uint32_t k = 0; k < GROUP_CHUNK / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        const bool valid = i < n;
        const uint32_t d = valid ? dest[i] : NONE, l = valid ? len[i] : 0u;
        for (uint32_t p = 0; p < n_parts; ++p) {
            const uint64_t m = __ballot(d == p);
            if (!m) continue;
            const uint32_t units = wave_sum(d == p ? l : 0u);
            if (lane_id() == 0) atomicAdd(&c[p], ((unsigned long long)__popcll(m) << 36) | units);
        }
    }
    __syncthreads();
    if (threadIdx.x < n_parts) bcnt[(uint64_t)threadIdx.x * n_blocks + blockIdx.x] = c[threadIdx.x];
}
// one block per destination: its column of per-block counts -> exclusive prefixes; total[p]
__global__ void __launch_bounds__(256) mig_group_scan(unsigned long long* __restrict__ bcnt, uint32_t n_blocks,
                                                      unsigned long long* __restrict__ total) {
    __shared__ unsigned long long s[256];
    unsigned long long* col = bcnt + (uint64_t)blockIdx.x * n_blocks;
    unsigned long long carry = 0;
    for (uint32_t at = 0; at < n_blocks; at += 256) {
        const uint32_t i = at + threadIdx.x;
        const unsigned long long v = i < n_blocks ? col[i] : 0ull;
        s[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t d = 1; d < 256; d <<= 1) {
            const unsigned long long t = threadIdx.x >= d ? s[threadIdx.x - d] : 0ull;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n_blocks) col[i] = carry + s[threadIdx.x] - v;
        carry += s[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) total[blockIdx.x] = carry;
}
struct GroupBases {
    uint64_t unit[MIG_MAX_PARTS];     // first unit of each destination's segment of the send buffer
    uint32_t rec[MIG_MAX_PARTS];      // first record of each destination's segment
};
__global__ void __launch_bounds__(256) mig_group_scatter(const uint32_t* __restrict__ dest,
                                                         const uint32_t* __restrict__ unit,
                                                         const uint32_t* __restrict__ len, uint32_t n,
                                                         uint32_t n_parts, uint32_t n_blocks,
                                                         const unsigned long long* __restrict__ bcnt,
                                                         const uint32_t* __restrict__ pool, GroupBases gb,
                                                         uint32_t* __restrict__ send, uint32_t* __restrict__ send_off) {
    __shared__ unsigned long long run[MIG_MAX_PARTS];
    __shared__ unsigned long long wt[4][MIG_MAX_PARTS];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x < n_parts) run[threadIdx.x] = bcnt[(uint64_t)threadIdx.x * n_blocks + blockIdx.x];
    __syncthreads();
    const uint32_t base = blockIdx.x * GROUP_CHUNK;
    for (uint32_t k = 0; k < GROUP_CHUNK / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        const bool valid = i < n;
        const uint32_t d = valid ? dest[i] : NONE, l = valid ? len[i] : 0u;
        uint32_t my_u = 0, my_r = 0;
        for (uint32_t p = 0; p < n_parts; ++p) {
            const uint64_t m = __ballot(d == p);
            if (!m) {
                if (lane == 0) wt[w][p] = 0;
                continue;
            }
            const uint32_t incl = wave_scan(d == p ? l : 0u);
            if (lane == 63) wt[w][p] = ((unsigned long long)__popcll(m) << 36) | incl;
            if (d == p) {
                my_u = incl - l;
                my_r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            }
        }
        __syncthreads();
        if (d < n_parts) {
            unsigned long long off = run[d];
            for (uint32_t v = 0; v < w; ++v) off += wt[v][d];
            const uint64_t u_in = (off & ((1ull << 36) - 1)) + my_u;
            const uint64_t r_in = (off >> 36) + my_r;
            const uint4* src = reinterpret_cast<const uint4*>(pool) + unit[i];
            uint4* dst = reinterpret_cast<uint4*>(send) + gb.unit[d] + u_in;
            for (uint32_t x = 0; x < l; ++x) dst[x] = src[x];
            send_off[gb.rec[d] + r_in] = (uint32_t)u_in;
        }
        __syncthreads();
        if (threadIdx.x < n_parts) run[threadIdx.x] += wt[0][threadIdx.x] + wt[1][threadIdx.x] + wt[2][threadIdx.x] + wt[3][threadIdx.x];
        __syncthreads();
    }
}

inline uint32_t pow2_floor(uint32_t v) {
    uint32_t p = 1;
    while (p * 2 <= v) p *= 2;
    return p;
}
template <class T>
T* dalloc(uint64_t n) {
    void* p = nullptr;
    if (n == 0) n = 1;
    const hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    return (T*)p;
}
template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

struct Lanes {
    uint64_t* vtab = nullptr;
    uint64_t* vlog = nullptr;
    uint4* frames = nullptr;
    uint32_t* epoch = nullptr;
    uint32_t n = 0, vcap = 0;
    void alloc(uint32_t lanes, uint32_t cap) {
        n = lanes;
        vcap = cap;
        vtab = dalloc<uint64_t>((uint64_t)lanes * cap);
        HIP_OK(hipMemset(vtab, 0, (uint64_t)lanes * cap * 8));
        vlog = dalloc<uint64_t>((uint64_t)lanes * (cap / 2));
        frames = dalloc<uint4>((uint64_t)lanes * MIG_FRAMES);
        epoch = dalloc<uint32_t>(lanes);
        HIP_OK(hipMemset(epoch, 0, (uint64_t)lanes * 4));
        // the memsets run on the null stream, which does not order the caller's non-blocking
        // streams: finish them before any batch uses the lanes (a late epoch reset would bring
        // back the epochs of marks still in the tables)
        HIP_OK(hipDeviceSynchronize());
    }
    void release() {
        dfree(vtab);
        dfree(vlog);
        dfree(frames);
        dfree(epoch);
    }
};

}  // namespace

struct MigState {
    int device = 0;
    uint32_t n_rows = 0;
    uint32_t* g_handle = nullptr;
    uint8_t* owner = nullptr;
    Lanes small, bigl;
    // the batch
    uint8_t* allowed = nullptr;
    uint32_t n = 0;
    int32_t gmd = 5;
    bool active = false;
    // START records
    uint32_t* start = nullptr;
    uint32_t* start_off = nullptr;
    uint64_t start_cap = 0;
    // outputs of a round
    uint32_t* pool = nullptr;
    uint64_t pool_cap = 0;             // units
    uint32_t *out_dest = nullptr, *out_unit = nullptr, *out_len = nullptr;
    uint32_t *spill = nullptr, *spill2 = nullptr, *bigq = nullptr;
    uint64_t out_cap = 0;
    uint32_t* ctr = nullptr;           // [0] out_count [1] n_spill [2] n_big [3] scratch [4..7] stats [8..11] err
    unsigned long long* pool_used = nullptr;
    unsigned long long* cursor = nullptr;   // [MIG_MAX_PARTS] records << 36 | units per destination
    unsigned long long* bcnt = nullptr;     // per block and destination (mig_group_*)
    uint64_t bcnt_cap = 0;
    uint64_t* unit_base = nullptr;          // [MIG_MAX_PARTS] source / destination unit bases
    uint32_t* rec_base = nullptr;           // [MIG_MAX_PARTS + 1]
    uint32_t* send = nullptr;
    uint64_t send_cap = 0;
    uint32_t* send_off = nullptr;
    uint64_t send_off_cap = 0;

    ~MigState() {
        (void)hipSetDevice(device);
        dfree(g_handle);
        dfree(owner);
        small.release();
        bigl.release();
        dfree(start);
        dfree(start_off);
        dfree(pool);
        dfree(out_dest);
        dfree(out_unit);
        dfree(out_len);
        dfree(spill);
        dfree(spill2);
        dfree(bigq);
        dfree(ctr);
        dfree(pool_used);
        dfree(cursor);
        dfree(bcnt);
        dfree(unit_base);
        dfree(rec_base);
        dfree(send);
        dfree(send_off);
    }
};

void MigStateDeleter::operator()(MigState* m) const { delete m; }

void mig_release(Snapshot& S) { S.mig.reset(); }

namespace {

MigState& mig_state(Snapshot& S) {
    if (S.part_mode != PART_MIGRATE) throw Error{KETO_E_INVALID, "not a migrating part (keto_snapshot_upload_part_mode)"};
    if (!S.dev) throw Error{KETO_E_HIP, "snapshot has no device copy"};
    if (!S.mig_ready) throw Error{KETO_E_INVALID, "closure filter exchange not finished (keto_part_closure_done)"};
    if (!S.mig) {
        const DevView dv = device_view(S);
        HIP_OK(hipSetDevice(dv.device));
        auto M = std::unique_ptr<MigState, MigStateDeleter>(new MigState);
        M->device = dv.device;
        M->n_rows = S.n_rows();
        M->g_handle = dalloc<uint32_t>(S.n_rows());
        HIP_OK(hipMemcpy(M->g_handle, S.g_handle.data(), (uint64_t)S.n_rows() * 4, hipMemcpyHostToDevice));
        std::vector<uint8_t> own(S.n_rows());
        for (uint32_t r = 0; r < S.n_rows(); ++r) own[r] = (uint8_t)S.root_owner(r, S.n_parts);
        M->owner = dalloc<uint8_t>(S.n_rows());
        HIP_OK(hipMemcpy(M->owner, own.data(), own.size(), hipMemcpyHostToDevice));
        M->ctr = dalloc<uint32_t>(16);
        M->pool_used = dalloc<unsigned long long>(1);
        M->cursor = dalloc<unsigned long long>(MIG_MAX_PARTS);
        M->unit_base = dalloc<uint64_t>(MIG_MAX_PARTS);
        M->rec_base = dalloc<uint32_t>(MIG_MAX_PARTS + 1);
        S.mig.reset(M.release());
    }
    return *S.mig;
}

void ensure_out(MigState& M, uint64_t n_in) {
    if (M.out_cap >= n_in && M.out_dest) return;
    dfree(M.out_dest);
    dfree(M.out_unit);
    dfree(M.out_len);
    dfree(M.spill);
    dfree(M.spill2);
    dfree(M.bigq);
    M.out_cap = std::max<uint64_t>(n_in, 4096);
    M.out_dest = dalloc<uint32_t>(M.out_cap);
    M.out_unit = dalloc<uint32_t>(M.out_cap);
    M.out_len = dalloc<uint32_t>(M.out_cap);
    M.spill = dalloc<uint32_t>(M.out_cap);
    M.spill2 = dalloc<uint32_t>(M.out_cap);
    M.bigq = dalloc<uint32_t>(M.out_cap);
}

// grow the output pool, keeping the records already written (all below the old capacity)
void grow_pool(MigState& M, uint64_t want, hipStream_t st) {
    uint64_t cap = want;
    if (cap <= M.pool_cap) return;
    uint32_t* p = dalloc<uint32_t>(cap * 4);
    if (M.pool) HIP_OK(hipMemcpyAsync(p, M.pool, M.pool_cap * 16, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    dfree(M.pool);
    M.pool = p;
    M.pool_cap = cap;
}

// Process one round's input (n_in records in n_src source segments) and group the outputs.
void run_round(Snapshot& S, MigState& M, const uint32_t* d_in, const uint32_t* d_in_off, uint32_t n_in,
               const uint32_t* in_records, const uint64_t* in_units, uint32_t n_src, hipStream_t st, MigOut& out) {
    const DevView dv = device_view(S);
    const uint32_t P = S.n_parts;
    ensure_out(M, n_in);
    if (!M.pool) {
        // records are ~10 units at max-depth 5; a short pool only costs reruns (tests force them)
        uint64_t want = std::max<uint64_t>((uint64_t)n_in * 16, 1ull << 20);
        if (const char* e = getenv("KETO_MIG_POOL_UNITS")) want = std::max<uint64_t>(64, strtoull(e, nullptr, 0));
        grow_pool(M, want, st);
    }
    if (!M.small.vtab) {
        // KETO_MIG_LANES / KETO_MIG_VCAP: the small tier's lanes and table entries (measurement knobs)
        uint32_t lanes = LANES_SMALL, vcap = VCAP_SMALL;
        if (const char* e = getenv("KETO_MIG_LANES")) lanes = std::max<uint32_t>(256, (uint32_t)strtoul(e, nullptr, 0) / 256 * 256);
        if (const char* e = getenv("KETO_MIG_VCAP")) vcap = pow2_floor(std::max<uint32_t>(16, std::min<uint32_t>(VCAP_BIG, (uint32_t)strtoul(e, nullptr, 0))));
        M.small.alloc(lanes, vcap);
    }
    if (!M.bigl.vtab) M.bigl.alloc(LANES_BIG, VCAP_BIG);
    // source segments
    uint32_t rb[MIG_MAX_PARTS + 1];
    uint64_t ub[MIG_MAX_PARTS];
    rb[0] = 0;
    uint64_t acc = 0;
    for (uint32_t s = 0; s < n_src; ++s) {
        ub[s] = acc;
        acc += in_units[s];
        rb[s + 1] = rb[s] + in_records[s];
    }
    if (rb[n_src] != n_in) throw Error{KETO_E_INVALID, "record counts do not add up"};
    HIP_OK(hipMemcpyAsync(M.rec_base, rb, (n_src + 1) * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(M.unit_base, ub, n_src * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(M.ctr, 0, 16 * 4, st));
    HIP_OK(hipMemsetAsync(M.pool_used, 0, 8, st));
    MigArgs a{};
    a.arena = dv.arena;
    a.coll = dv.coll;
    a.coll_mask = dv.coll_mask;
    a.self = S.part;
    a.in = d_in;
    a.in_off = d_in_off;
    a.rec_base = M.rec_base;
    a.unit_base = M.unit_base;
    a.n_src = n_src;
    a.n_in = n_in;
    a.pool_used = M.pool_used;
    a.out_dest = M.out_dest;
    a.out_unit = M.out_unit;
    a.out_len = M.out_len;
    a.out_count = M.ctr + 0;
    a.n_spill = M.ctr + 1;
    a.n_big = M.ctr + 2;
    a.allowed = M.allowed;
    a.stats = M.ctr + 4;
    a.err = M.ctr + 8;
    a.arena_words = dv.arena_words;
    a.in_units = acc;
    a.n_allowed = M.n;
    a.n_parts = P;
    a.hot_units = S.hot_units;
    auto launch = [&](Lanes& L, const uint32_t* list, const uint32_t* n_list, uint32_t n_max, uint32_t* big,
                      uint32_t* spill) {
        a.list = list;
        a.n_list = n_list;
        a.big = big;
        a.spill = spill;
        a.pool = M.pool;
        a.pool_cap = M.pool_cap;
        a.vtab = L.vtab;
        a.vlog = L.vlog;
        a.frames = L.frames;
        a.lane_epoch = L.epoch;
        a.vcap = L.vcap;
        const uint32_t lanes = (uint32_t)std::min<uint64_t>(L.n, ((uint64_t)n_max + 255) / 256 * 256);
        if (lanes == 0) return;
        hipLaunchKernelGGL(mig_kernel, dim3(lanes / 256), dim3(256), 0, st, a);
        HIP_OK(hipGetLastError());
    };
    // small tier over every input, then the big tier over the inputs whose maps outgrew it, then the
    // inputs whose output did not fit the pool (with a bigger pool), until none is left
    uint32_t cnt[16];
    if (n_in) launch(M.small, nullptr, nullptr, n_in, M.bigq, M.spill);
    HIP_OK(hipMemcpyAsync(cnt, M.ctr, 16 * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    uint32_t n_big = cnt[2];
    uint32_t spilled = 0;
    for (int pass = 0; pass < 2; ++pass) {       // pass 0: the small tier's spills, pass 1: the big tier
        uint32_t n_sp = cnt[1];
        bool small_tier = pass == 0;
        while (n_sp) {
            spilled += n_sp;
            // rerun the spilled inputs with a pool twice the size (list copied: the rerun spills into spill)
            unsigned long long used = 0;
            HIP_OK(hipMemcpyAsync(&used, M.pool_used, 8, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            const unsigned long long cap_used = std::min<unsigned long long>(used, M.pool_cap);
            grow_pool(M, std::max<uint64_t>(M.pool_cap * 2, used * 2), st);
            HIP_OK(hipMemcpyAsync(M.spill2, M.spill, (uint64_t)n_sp * 4, hipMemcpyDeviceToDevice, st));
            HIP_OK(hipMemcpyAsync(M.ctr + 3, M.ctr + 1, 4, hipMemcpyDeviceToDevice, st));
            HIP_OK(hipMemsetAsync(M.ctr + 1, 0, 4, st));
            HIP_OK(hipMemcpyAsync(M.pool_used, &cap_used, 8, hipMemcpyHostToDevice, st));
            if (small_tier) launch(M.small, M.spill2, M.ctr + 3, n_sp, M.bigq, M.spill);
            else launch(M.bigl, M.spill2, M.ctr + 3, n_sp, nullptr, M.spill);
            HIP_OK(hipMemcpyAsync(cnt, M.ctr, 16 * 4, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            n_sp = cnt[1];
        }
        if (pass == 0) {
            n_big = cnt[2];
            if (n_big == 0) break;
            HIP_OK(hipMemsetAsync(M.ctr + 1, 0, 4, st));
            launch(M.bigl, M.bigq, M.ctr + 2, n_big, nullptr, M.spill);
            HIP_OK(hipMemcpyAsync(cnt, M.ctr, 16 * 4, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
        }
    }
    const uint32_t n_out = cnt[0];
    if (getenv("KETO_MIG_DEBUG"))
        fprintf(stderr, "mig part %u: in %u big %u out %u decided %u undecided %u pool %llu spilled %u\n", S.part, n_in,
                n_big, n_out, cnt[4], cnt[5], (unsigned long long)M.pool_cap, spilled);
    if (cnt[8])
        throw Error{KETO_E_INVALID, std::to_string(cnt[8]) + " malformed continuation records or handles (first: code " +
                                        std::to_string(cnt[9]) + ", input record " + std::to_string(cnt[10]) +
                                        ", value " + std::to_string(cnt[11]) + ")"};
    // group by destination (mig_group_*): per-block counts, their prefixes, then the records in place
    const uint32_t nb = (uint32_t)(((uint64_t)n_out + GROUP_CHUNK - 1) / GROUP_CHUNK);
    if (M.bcnt_cap < (uint64_t)nb * P || !M.bcnt) {
        dfree(M.bcnt);
        M.bcnt_cap = std::max<uint64_t>((uint64_t)nb * P * 2, 1024);
        M.bcnt = dalloc<unsigned long long>(M.bcnt_cap);
    }
    unsigned long long c[MIG_MAX_PARTS] = {};
    if (n_out) {
        hipLaunchKernelGGL(mig_group_count, dim3(nb), dim3(256), 0, st, M.out_dest, M.out_len, n_out, P, nb, M.bcnt);
        HIP_OK(hipGetLastError());
        hipLaunchKernelGGL(mig_group_scan, dim3(P), dim3(256), 0, st, M.bcnt, nb, M.cursor);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(c, M.cursor, P * 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    GroupBases gb{};
    uint64_t total_units = 0;
    uint32_t total_recs = 0;
    for (uint32_t p = 0; p < P; ++p) {
        out.units[p] = c[p] & ((1ull << 36) - 1);
        out.records[p] = (uint32_t)(c[p] >> 36);
        gb.unit[p] = total_units;
        gb.rec[p] = total_recs;
        total_units += out.units[p];
        total_recs += out.records[p];
    }
    for (uint32_t p = P; p < MIG_MAX_PARTS; ++p) {
        out.units[p] = 0;
        out.records[p] = 0;
    }
    if (total_recs != n_out) throw Error{KETO_E_INVALID, "continuation records with a bad destination part"};
    if (M.send_cap < total_units || !M.send) {
        dfree(M.send);
        M.send_cap = std::max<uint64_t>(total_units * 2, 1ull << 16);
        M.send = dalloc<uint32_t>(M.send_cap * 4);
    }
    if (M.send_off_cap < n_out || !M.send_off) {
        dfree(M.send_off);
        M.send_off_cap = std::max<uint64_t>((uint64_t)n_out * 2, 4096);
        M.send_off = dalloc<uint32_t>(M.send_off_cap);
    }
    if (n_out) {
        hipLaunchKernelGGL(mig_group_scatter, dim3(nb), dim3(256), 0, st, M.out_dest, M.out_unit, M.out_len, n_out, P,
                           nb, M.bcnt, M.pool, gb, M.send, M.send_off);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(st));
    }
    out.d_buf = M.send;
    out.d_off = M.send_off;
    out.decided = cnt[4];
    out.undecided = cnt[5];
    out.processed = cnt[6];
    out.reruns = spilled + n_big;
}

}  // namespace

void mig_begin(Snapshot& S, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed, void* stream,
               MigOut& out, bool child_entries) {
    std::lock_guard<std::mutex> lk(S.mu);
    MigState& M = mig_state(S);
    HIP_OK(hipSetDevice(M.device));
    // NULL = the default stream, as the header says: ordered after the caller's default-stream work
    // that produced the inputs (the snapshot's own stream is non-blocking and would not be)
    hipStream_t st = (hipStream_t)stream;
    if (gmd > 65535) gmd = 65535;
    if (n && (!d_reqs || !d_allowed)) throw Error{KETO_E_INVALID, "NULL argument"};
    // the grouping packs a destination's record count into 28 bits (records << 36 | units); a round
    // emits at most one record per input, so capping the inputs caps every count
    if (n >= MAX_ROUND_RECORDS) throw Error{KETO_E_RANGE, "a migrating batch holds fewer than 2^28 requests"};
    M.allowed = d_allowed;
    M.n = n;
    M.gmd = gmd;
    M.active = true;
    if (M.start_cap < n || !M.start) {
        dfree(M.start);
        dfree(M.start_off);
        M.start_cap = std::max<uint64_t>(n, 4096);
        M.start = dalloc<uint32_t>(M.start_cap * 4 * START_UNITS);
        M.start_off = dalloc<uint32_t>(M.start_cap);
    }
    HIP_OK(hipMemsetAsync(M.ctr, 0, 4, st));
    if (n) {
        hipLaunchKernelGGL(mig_start, dim3((n + 255) / 256), dim3(256), 0, st, d_reqs, n, gmd, M.g_handle, M.owner,
                           M.n_rows, S.part, S.hot_units, child_entries ? 1u : 0u, M.start, M.start_off, M.ctr);
        HIP_OK(hipGetLastError());
    }
    uint32_t bad = 0;
    HIP_OK(hipMemcpyAsync(&bad, M.ctr, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (bad) throw Error{KETO_E_INVALID, std::to_string(bad) + " requests name rows another part owns"};
    const uint32_t recs = n;
    const uint64_t units = (uint64_t)START_UNITS * n;
    run_round(S, M, M.start, M.start_off, n, &recs, &units, 1, st, out);
}

void mig_round(Snapshot& S, const void* d_in, const uint32_t* d_in_off, const uint32_t* in_records,
               const uint64_t* in_units, void* stream, MigOut& out) {
    std::lock_guard<std::mutex> lk(S.mu);
    MigState& M = mig_state(S);
    HIP_OK(hipSetDevice(M.device));
    if (!M.active) throw Error{KETO_E_INVALID, "no migrating batch (keto_mig_begin)"};
    // NULL = the default stream, as the header says: ordered after the caller's default-stream work
    // that produced the inputs (the snapshot's own stream is non-blocking and would not be)
    hipStream_t st = (hipStream_t)stream;
    uint64_t n_in = 0;
    for (uint32_t s = 0; s < S.n_parts; ++s) n_in += in_records[s];
    if (n_in >= MAX_ROUND_RECORDS) throw Error{KETO_E_RANGE, "a round takes fewer than 2^28 records"};
    if (n_in && (!d_in || !d_in_off)) throw Error{KETO_E_INVALID, "NULL argument"};
    run_round(S, M, static_cast<const uint32_t*>(d_in), d_in_off, (uint32_t)n_in, in_records, in_units, S.n_parts, st,
              out);
}

void device_memory(int device, uint64_t& free_bytes, uint64_t& total_bytes) {
    int cur = 0;
    HIP_OK(hipGetDevice(&cur));
    HIP_OK(hipSetDevice(device));
    size_t f = 0, t = 0;
    const hipError_t e = hipMemGetInfo(&f, &t);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) throw Error{KETO_E_HIP, std::string("hipMemGetInfo: ") + hipGetErrorString(e)};
    free_bytes = f;
    total_bytes = t;
}

void device_copy(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (bytes == 0) return;
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
}

}  // namespace keto
