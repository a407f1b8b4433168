// Host-side snapshot builder: interning, reference ORDER BY, CSR, wildcard materialization,
// poisoned-page detection and visit-key collision classes.
//
// What it reproduces (paths relative to the reference tree):
//   * row order and edge order = ORDER BY nid, namespace_id, object, relation, subject_id,
//     subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time
//     (internal/persistence/sql/relationtuples.go:250) under SQLite semantics: NULL first, so
//     subject sets precede subject ids; TEXT compared byte-wise (BINARY collation).
//   * whereQuery (relationtuples.go:178-198): an empty namespace/object/relation is no filter.
//     Stored subject sets with empty fields become materialized "wildcard rows" whose edges
//     are the concatenation of all matching rows in ORDER BY order.
//   * toInternal (relationtuples.go:43-80): a row whose namespace id, or whose subject-set
//     namespace id, is not configured fails its whole page with ErrNotFound.  check turns that
//     into `false` for the node (internal/check/engine.go:98-100) -> the row is truncated at the
//     first poisoned page; expand returns the error (internal/expand/engine.go:63-66).
//   * visited identity is Subject.String() (internal/x/graph/graph_utils.go:13-35;
//     internal/relationtuple/definitions.go:163-169): keys shared by two different subjects get
//     a shared visit id ("collision class") and their rows take the ordered ROW_SEQ path.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_set>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

namespace {

// KETO_BUILD_TRACE=1: builder phase times on stderr (tooling)
struct PhaseClock {
    bool on = getenv("KETO_BUILD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto build] %-28s %8.3f s\n", what, std::chrono::duration<double>(n - t).count());
        t = n;
    }
};

std::atomic<uint64_t> g_snapshot_uid{0};

inline std::string_view sv(const keto_str& s) { return std::string_view(s.p ? s.p : "", s.n); }

void load_namespaces(Snapshot& S, const keto_namespace* ns, uint32_t n_ns) {
    if (n_ns && !ns) throw Error{KETO_E_INVALID, "namespaces == NULL"};
    for (uint32_t i = 0; i < n_ns; ++i) {
        std::string name(sv(ns[i].name));
        if (S.ns_by_id.count(ns[i].id) || S.ns_by_name.count(name))
            throw Error{KETO_E_CONFIG, "duplicate namespace id or name in config: " + name};
        S.ns_by_id[ns[i].id] = (int)i;
        S.ns_by_name[name] = (int)i;
        S.ns_ids.push_back(ns[i].id);
        S.ns_names.push_back(std::move(name));
    }
    for (uint32_t i = 0; i < (uint32_t)S.ns_names.size(); ++i) S.ns_view.emplace(S.ns_names[i], (int)i);
}

// Sharded parallel interning of the tuple table's strings (objects, relations, subject ids, subject-set
// objects and relations) plus extra strings: every occurrence is hashed in parallel, thread t owns
// the shards h % S == t (mod threads) and dedups its occurrences with an open-addressing table, the
// unique strings are sorted byte-wise with the parallel sample sort, and each occurrence gets its
// string's rank (= its id: numeric id order is byte order).
struct ParInterner {
    static constexpr int FIELDS = 4;    // per tuple: object, relation, subject id | set object, set relation
    std::vector<uint32_t> occ;          // per occurrence: global unique id, then rank
    std::vector<std::string_view> uniq; // unique strings by global id
    std::vector<uint32_t> rank;         // global id -> rank

    static std::string_view field(const keto_tuple& t, int f) {
        switch (f) {
            case 0: return std::string_view(t.object.p ? t.object.p : "", t.object.n);
            case 1: return std::string_view(t.relation.p ? t.relation.p : "", t.relation.n);
            case 2:
                return t.subject_kind ? std::string_view(t.set_object.p ? t.set_object.p : "", t.set_object.n)
                                      : std::string_view(t.subject_id.p ? t.subject_id.p : "", t.subject_id.n);
            default:
                return t.subject_kind ? std::string_view(t.set_relation.p ? t.set_relation.p : "", t.set_relation.n)
                                      : std::string_view();
        }
    }

    // occurrences: FIELDS per tuple, then the extras; slot 3 of a subject-id tuple is unused
    void run(const keto_tuple* tup, uint64_t n, const std::vector<std::string_view>& extra, unsigned threads) {
        const uint64_t m = n * FIELDS + extra.size();
        auto view = [&](uint64_t i) -> std::string_view {
            return i < n * FIELDS ? field(tup[i / FIELDS], (int)(i % FIELDS)) : extra[i - n * FIELDS];
        };
        auto used = [&](uint64_t i) { return i >= n * FIELDS || i % FIELDS != 3 || tup[i / FIELDS].subject_kind; };
        PhaseClock clk;
        std::vector<uint64_t> hv(m);                // hash | 1; 0 = unused slot
        // hash pass over static slices; each slice bins its occurrences by owner thread, so an owner
        // reads only its own occurrences
        std::vector<std::vector<std::vector<uint64_t>>> bins(threads, std::vector<std::vector<uint64_t>>(threads));
        par_threads(threads, [&](unsigned t) {
            const uint64_t lo = (uint64_t)((unsigned __int128)t * m / threads);
            const uint64_t hi = (uint64_t)((unsigned __int128)(t + 1) * m / threads);
            for (auto& b : bins[t]) b.reserve((hi - lo) / threads + 16);
            for (uint64_t i = lo; i < hi; ++i) {
                if (!used(i)) {
                    hv[i] = 0;
                    continue;
                }
                const uint64_t h = hash_bytes(view(i)) | 1;
                hv[i] = h;
                bins[t][(h >> 40) % threads].push_back(i);
            }
        });
        clk.lap("  intern: hash");
        occ.assign(m, 0xFFFFFFFFu);
        // thread t: occurrences whose hash picks it; local ids, then global = base[t] + local
        std::vector<std::vector<std::string_view>> loc(threads);
        std::vector<std::vector<uint32_t>> local_id(threads);
        par_threads(threads, [&](unsigned t) {
            std::vector<std::string_view>& L = loc[t];
            uint64_t cap = 1024;
            std::vector<uint64_t> th(cap, 0);          // hash | 1 (0 = empty)
            std::vector<uint32_t> tid(cap, 0);
            uint64_t cnt = 0;
            auto grow = [&]() {
                std::vector<uint64_t> nh(cap * 2, 0);
                std::vector<uint32_t> ni(cap * 2, 0);
                for (uint64_t i = 0; i < cap; ++i)
                    if (th[i]) {
                        uint64_t j = (th[i] >> 1) & (cap * 2 - 1);
                        while (nh[j]) j = (j + 1) & (cap * 2 - 1);
                        nh[j] = th[i];
                        ni[j] = tid[i];
                    }
                th.swap(nh);
                tid.swap(ni);
                cap *= 2;
            };
            for (unsigned src = 0; src < threads; ++src)
              for (const uint64_t i : bins[src][t]) {
                const uint64_t h = hv[i];
                const std::string_view v = view(i);
                const uint64_t key = h;
                uint64_t j = (h >> 1) & (cap - 1);
                for (;;) {
                    if (!th[j]) {
                        th[j] = key;
                        tid[j] = (uint32_t)L.size();
                        L.push_back(v);
                        occ[i] = tid[j];
                        if (++cnt * 2 > cap) grow();
                        break;
                    }
                    if (th[j] == key && L[tid[j]] == v) {
                        occ[i] = tid[j];
                        break;
                    }
                    j = (j + 1) & (cap - 1);
                }
            }
        });
        clk.lap("  intern: shard tables");
        bins.clear();
        std::vector<uint32_t> base(threads + 1, 0);
        for (unsigned t = 0; t < threads; ++t) base[t + 1] = base[t] + (uint32_t)loc[t].size();
        uniq.resize(base[threads]);
        for (unsigned t = 0; t < threads; ++t) std::copy(loc[t].begin(), loc[t].end(), uniq.begin() + base[t]);
        par_chunks(m, threads, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i)
                if (hv[i]) occ[i] += base[(hv[i] >> 40) % threads];
        });
        std::vector<uint64_t>().swap(hv);
        clk.lap("  intern: global ids");
        std::vector<uint32_t> order(uniq.size());
        std::iota(order.begin(), order.end(), 0u);
        parallel_sort(order, [&](uint32_t a, uint32_t b) { return uniq[a] < uniq[b]; }, threads);
        clk.lap("  intern: sort uniques");
        rank.assign(uniq.size(), 0);
        for (uint32_t r = 0; r < order.size(); ++r) rank[order[r]] = r;
        par_chunks(m, threads, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i)
                if (occ[i] != 0xFFFFFFFFu) occ[i] = rank[occ[i]];
        });
        std::vector<std::string_view> sorted(uniq.size());
        for (uint32_t r = 0; r < order.size(); ++r) sorted[r] = uniq[order[r]];
        uniq.swap(sorted);                      // now by rank
        clk.lap("  intern: ranks");
    }
};

struct T {                    // one interned tuple
    int32_t ns;
    uint32_t obj, rel;
    uint8_t kind;
    uint32_t a;               // kind 0: sid ; kind 1: sobj
    int32_t sns;
    uint32_t srel;
    uint64_t seq;             // commit order
};

bool tuple_less(const T& x, const T& y) {
    if (x.ns != y.ns) return x.ns < y.ns;
    if (x.obj != y.obj) return x.obj < y.obj;
    if (x.rel != y.rel) return x.rel < y.rel;
    // subject_id: NULL (sets) first
    if (x.kind != y.kind) return x.kind == 1;
    if (x.kind == 0) {
        if (x.a != y.a) return x.a < y.a;
    } else {
        if (x.sns != y.sns) return x.sns < y.sns;
        if (x.a != y.a) return x.a < y.a;
        if (x.srel != y.srel) return x.srel < y.srel;
    }
    return x.seq < y.seq;
}

int64_t key_cmp(const RowKey& a, const RowKey& b) {
    if (a.ns != b.ns) return a.ns < b.ns ? -1 : 1;
    if (a.obj != b.obj) return a.obj < b.obj ? -1 : 1;
    if (a.rel != b.rel) return a.rel < b.rel ? -1 : 1;
    return 0;
}

// row flags + effective counts, once edges, poison pages and collision classes are known
void finalize_rows(Snapshot& S, const std::vector<uint64_t>& row_ptr, const std::vector<uint8_t>& is_wild) {
    uint32_t R = (uint32_t)row_ptr.size() - 1;
    S.rows.resize(R);
    S.n_seq_rows = 0;
    S.n_poisoned_rows = 0;
    for (uint32_t r = 0; r < R; ++r) {
        uint64_t b = row_ptr[r], e = row_ptr[r + 1], n = e - b;
        if (b >= (1ull << 40)) throw Error{KETO_E_RANGE, "more than 2^40 edges"};
        uint32_t pp = S.row_pp[r];
        uint64_t L = pp == NO_PAGE ? n : std::min<uint64_t>(n, (uint64_t)pp * S.page_size);
        if (pp != NO_PAGE) S.n_poisoned_rows++;
        bool seq = is_wild[r] != 0;
        if (!seq && !S.coll.empty()) {
            for (uint64_t k = b; k < b + L; ++k)
                if (S.coll.count(S.edges[k])) { seq = true; break; }
        }
        RowRec rec;
        rec.edge_lo = (uint32_t)b;
        rec.hi_flags = (uint32_t)(b >> 32) | ((seq ? ROW_SEQ : 0u) << 8);
        if (L > 0xFFFFFFFFull) throw Error{KETO_E_RANGE, "row with more than 2^32 edges"};
        if (seq) {
            rec.n_sets = (uint32_t)L;
            rec.n_ids = 0;
            S.n_seq_rows++;
        } else {
            uint64_t ns = 0;
            while (ns < L && (S.edges[b + ns] & EDGE_SET)) ++ns;
            rec.n_sets = (uint32_t)ns;
            rec.n_ids = (uint32_t)(L - ns);
        }
        S.rows[r] = rec;
    }
}

}  // namespace

uint64_t next_snapshot_uid() { return ++g_snapshot_uid; }

int Snapshot::key_cmp_bytes(const RowKey& a, const RowKey& b) const {
    if (a.ns != b.ns) return a.ns < b.ns ? -1 : 1;
    if (a.obj != b.obj) return str_cmp(a.obj, b.obj);
    if (a.rel != b.rel) return str_cmp(a.rel, b.rel);
    return 0;
}

std::vector<uint32_t> Snapshot::rows_in_key_order(const RowKey& k) const {
    auto match = [&](const RowKey& rk) {
        return (k.ns == ANY_NS || rk.ns == k.ns) && (k.obj == ANY || rk.obj == k.obj) && (k.rel == ANY || rk.rel == k.rel);
    };
    std::vector<uint32_t> out, extra;
    for (uint32_t q = 0; q < n_real_rows; ++q)
        if (match(row_key[q])) out.push_back(q);
    // rows outside the build's sorted range that hold tuples now (written by keto_snapshot_apply)
    for (uint32_t q = n_real_rows; q < n_rows(); ++q) {
        const RowKey& rk = row_key[q];
        if (rk.ns == ANY_NS || rk.obj == ANY || rk.rel == ANY || !row_over.count(q)) continue;
        if (row_over.at(q).empty() || !match(rk)) continue;
        extra.push_back(q);
    }
    if (extra.empty()) return out;
    auto less = [&](uint32_t a, uint32_t b) { return key_cmp_bytes(row_key[a], row_key[b]) < 0; };
    std::sort(extra.begin(), extra.end(), less);
    std::vector<uint32_t> all(out.size() + extra.size());
    std::merge(out.begin(), out.end(), extra.begin(), extra.end(), all.begin(), less);
    return all;
}

int Snapshot::str_cmp(uint32_t a, uint32_t b) const {
    if (a == b) return 0;
    if (a < n_sorted_strs && b < n_sorted_strs) return a < b ? -1 : 1;
    const int c = strs[a].compare(strs[b]);
    return c < 0 ? -1 : c > 0 ? 1 : 0;
}

uint32_t overlay_row(const Snapshot& S, Overlay& ov, const RowKey& k) {
    auto f = ov.map.find(k);
    if (f != ov.map.end()) return f->second;
    uint32_t id = ov.base + (uint32_t)ov.rows.size();
    uint64_t b = ov.edges.size(), pos = 0;
    uint32_t pp = NO_PAGE;
    for (uint32_t q : S.rows_in_key_order(k)) {              // matching real rows in ORDER BY order
        const auto e = S.row_edges(q);
        for (uint64_t i = 0; i < e.second; ++i, ++pos) {
            if (e.first[i] == EDGE_POISON && pp == NO_PAGE) pp = (uint32_t)(pos / S.page_size);
            ov.edges.push_back(e.first[i]);
        }
    }
    uint64_t n = ov.edges.size() - b;
    uint64_t L = pp == NO_PAGE ? n : std::min<uint64_t>(n, (uint64_t)pp * S.page_size);
    RowRec rec;
    rec.edge_lo = (uint32_t)b;
    rec.hi_flags = (uint32_t)(b >> 32) | (ROW_SEQ << 8);
    rec.n_sets = (uint32_t)L;
    rec.n_ids = 0;
    ov.rows.push_back(rec);
    ov.pp.push_back(pp);
    ov.keys.push_back(k);
    ov.map.emplace(k, id);
    ov.unit.push_back((uint32_t)ov.n_units);                  // overlay rows: header + edges, no table
    ov.n_units += 1 + (n + 3) / 4;
    if (S.n_units + ov.n_units >= (uint64_t)HANDLE_MAX) throw Error{KETO_E_RANGE, "overlay exceeds the handle space"};
    return id;
}

namespace {
uint64_t row_size(const Snapshot& S, uint32_t r) { return S.row_edges(r).second; }
uint32_t ceil_log2(uint64_t x) {
    uint32_t k = 0;
    while ((1ull << k) < x) ++k;
    return k;
}
}  // namespace

uint32_t Snapshot::row_hlog2(uint32_t r) const {
    if (row_flags(r) & ROW_SEQ) return 0;
    const RowRec& x = rows[r];
    if (x.n_ids == 0 || (uint64_t)x.n_sets + x.n_ids <= WINDOW_WORDS) return 0;   // ids sit in the window
    return std::max<uint32_t>(2, ceil_log2(2ull * x.n_ids));                      // load <= 1/2, >= 1 bucket
}

uint64_t arena_fit(uint64_t w, uint64_t table, uint64_t cb, uint64_t n_edges, uint64_t& total) {
    // line placement: a row that fits in a 128-B line never straddles one (closure filter, header,
    // window and id table come in with one miss); a bigger row keeps closure filter + header +
    // window in one line
    const uint64_t slot = cb + HDR_WORDS + WINDOW_WORDS;         // read together on a visit
    total = table + cb + HDR_WORDS + ((n_edges + 3) & ~3ull);
    const uint64_t fit = std::max(total, table + slot);          // a short row's window included
    auto align = [&](uint64_t x) {
        if (fit <= LINE_WORDS) {
            if (x % LINE_WORDS + fit > LINE_WORDS) x = (x + LINE_WORDS - 1) / LINE_WORDS * LINE_WORDS;
        } else {
            const uint64_t o = (x + table) % LINE_WORDS;         // closure filter + header + window
            if (o + slot > LINE_WORDS) x += LINE_WORDS - o;
        }
        return x;
    };
    w = align(w);
    if ((w >> 32) != ((w + fit - 1) >> 32)) w = align(((w >> 32) + 1) << 32);   // rows stay in a segment
    return w;
}

uint64_t arena_fit_g(uint64_t w, uint64_t table, uint64_t cb, uint64_t n_edges, uint64_t& total, uint32_t g) {
    // wide layouts: a header past word 2^33 sits on a multiple of 4 << g words from there (its handle
    // counts such units, hword).  That alignment (>= 8 words, and 2^33 is line-aligned) already keeps
    // header + window inside one line; the rest of the line rule gives way to it, the segment rule
    // does not
    const uint64_t x = arena_fit(w, table, cb, n_edges, total);
    if (g == 0 || x + table + cb < TARGET_MAX_WORDS) return x;
    const uint64_t a = 4ull << g, pre = table + cb;
    const uint64_t fit = std::max(total, pre + HDR_WORDS + WINDOW_WORDS);
    auto up = [&](uint64_t h) { return TARGET_MAX_WORDS + (std::max(h, TARGET_MAX_WORDS) - TARGET_MAX_WORDS + a - 1) / a * a; };
    uint64_t h = up(w + pre);
    if (((h - pre) >> 32) != ((h - pre + fit - 1) >> 32)) h = up(((((h - pre) >> 32) + 1) << 32) + pre);   // stay in a segment
    return h - pre;
}

namespace {
// The arena layout of one part: which rows it holds, where, and (PART_MIGRATE) its stubs.
struct PartLayout {
    std::vector<uint32_t> unit_of_row, rows_by_unit, layout_units;
    std::vector<uint8_t> stub;
    uint64_t n_units = 0, n_words = 0, shared_words = 0, n_stubs = 0, hot_words = 0, hot_rows = 0;
    uint64_t tgt_tail = 0, tgt_end = 0, roots_at = 0;
    uint32_t root_g = 0;
};

// hot_band (PART_MIGRATE): rows of in-degree band >= hot_band are kept on every part; sorted
// hottest first, they come first in every part's layout, identically
void layout_part(const Snapshot& S, const std::vector<uint8_t>& band, uint32_t part, uint32_t n_parts, int mode,
                 uint32_t hot_band, PartLayout& L) {
    const uint32_t R = S.n_rows();
    L.unit_of_row.assign(R, NO_UNIT);
    // edge partitioning: PART_SHARED leaves other parts' root rows out of this device's arena;
    // PART_MIGRATE keeps only this part's rows, plus a stub for every other part's row that one of
    // them points at
    std::vector<uint8_t> keep(R, 1);
    L.stub.clear();
    L.n_stubs = 0;
    if (n_parts > 1) {
        if (mode == PART_MIGRATE) {
            L.stub.assign(R, 0);
            for (uint32_t r = 0; r < R; ++r) keep[r] = S.root_owner(r, n_parts) == part || band[r] >= hot_band;
            for (uint32_t r = 0; r < R; ++r) {
                if (!keep[r]) continue;
                const auto ed = S.row_edges(r);
                for (uint64_t i = 0; i < ed.second; ++i) {
                    const uint32_t e = ed.first[i];
                    if (!(e & EDGE_SET) || e == EDGE_POISON) continue;
                    const uint32_t t = e & EDGE_VAL;
                    if (t < R && !keep[t] && !L.stub[t]) {
                        L.stub[t] = 1;
                        ++L.n_stubs;
                    }
                }
            }
        } else {
            for (uint32_t r = 0; r < R; ++r)
                if (S.is_root[r] && S.root_owner(r, n_parts) != part) keep[r] = 0;
        }
    }
    auto held = [&](uint32_t r) { return keep[r] || (!L.stub.empty() && L.stub[r]); };
    uint64_t kept = 0;
    std::vector<uint64_t> start(35, 0);                  // key = 33 - band: hottest first
    for (uint32_t r = 0; r < R; ++r)
        if (held(r)) {
            ++start[33 - band[r] + 1];
            ++kept;
        }
    for (int b = 1; b < 35; ++b) start[b] += start[b - 1];
    L.rows_by_unit.assign(kept, 0);
    for (uint32_t r = 0; r < R; ++r)
        if (held(r)) L.rows_by_unit[start[33 - band[r]]++] = r;
    L.layout_units.assign(kept, 0);
    L.shared_words = 0;
    L.hot_words = 0;
    L.hot_rows = 0;
    // test hook: start the layout this many words into the arena, so a small graph straddles the
    // segment boundary at 2^32 words (tests/test_gpu_synth.py)
    uint64_t w = 0;
    if (const char* base = getenv("KETO_TEST_ARENA_BASE")) w = strtoull(base, nullptr, 0) & ~(uint64_t)(LINE_WORDS - 1);
    // test hook: a split layout whose root rows start at this word (tests/test_gpu_arena_split.py)
    const char* root_base = getenv("KETO_TEST_ROOT_BASE");
    // what the placement needs of each row, gathered in arena order on the builder's threads (the
    // rows come in band order, so these are random reads): edge count (bits 0..39), id-table log2
    // (40..45), closure filter (46), stub (47), root row (48)
    constexpr uint64_t P_CB = 1ull << 46, P_STUB = 1ull << 47, P_ROOT = 1ull << 48;
    std::vector<uint64_t> pk(kept);
    std::vector<uint64_t> root_part(std::max(1u, build_threads()), 0);
    const unsigned th = kept >= par_min() ? build_threads() : 1u;
    par_chunks(kept, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned t) {
        uint64_t rw = 0;
        for (uint64_t x = b; x < e; ++x) {
            const uint32_t r = L.rows_by_unit[x];
            const bool stub = !keep[r], root = S.is_root[r] != 0;
            const uint64_t h = stub ? 0 : S.row_hlog2(r), n = stub ? 0 : row_size(S, r);
            pk[x] = n | (h << 40) | (root ? P_ROOT : P_CB) | (stub ? P_STUB : 0);
            // the root rows' words, to see whether the layout must split (roots come last)
            if (root && !stub) rw += (h ? (1ull << h) : 0) + HDR_WORDS + ((n + 3) & ~3ull) + LINE_WORDS;   // + alignment
        }
        root_part[t] += rw;
    });
    uint64_t root_words = 0;
    for (uint64_t v : root_part) root_words += v;
    L.tgt_tail = L.tgt_end = L.roots_at = 0;
    L.root_g = 0;
    // test hook: the target reserve's size in words (a small one fills after a few writes)
    const char* reserve_words = getenv("KETO_TEST_TGT_RESERVE");
    bool in_roots = false;
    for (uint64_t x = 0; x < kept; ++x) {
        const uint64_t p = pk[x];
        const bool stub = (p & P_STUB) != 0;                         // header + closure block only
        const bool root = (p & P_ROOT) != 0;
        if (root && !stub && !in_roots) {
            in_roots = true;
            if (root_base || w + root_words > TARGET_MAX_WORDS) {
                // split: targets end here; a reserve for targets writes add, then the roots
                if (mode == PART_MIGRATE) throw Error{KETO_E_RANGE, "a migrating part's arena exceeds 2^31 16-byte units"};
                L.tgt_tail = w;
                const uint64_t reserve = reserve_words ? strtoull(reserve_words, nullptr, 0) : std::max<uint64_t>(1ull << 20, w / 8);
                L.tgt_end = std::min<uint64_t>(TARGET_MAX_WORDS, w + reserve);
                L.roots_at = std::max<uint64_t>(L.tgt_end, root_base ? strtoull(root_base, nullptr, 0) & ~(uint64_t)(LINE_WORDS - 1) : 0);
                w = L.roots_at;
                // wide: the roots run past 64 GiB, so those past word 2^33 take handles in units of
                // 16 << g bytes, the smallest g leaving an eighth of the handles for writes and
                // overlays (root_words allows a line of alignment per root, >= 4 << g words)
                // (test hook KETO_TEST_ROOT_G: at least this g, whatever the size)
                const char* force_g = getenv("KETO_TEST_ROOT_G");
                const uint64_t end = w + root_words;
                if (end > NARROW_MAX_WORDS || force_g) {
                    L.root_g = force_g ? std::max<uint32_t>(1, std::min<uint32_t>(ROOT_G_MAX, (uint32_t)atoi(force_g))) : 1;
                    auto fits = [&](uint32_t g) {
                        const uint64_t hu = end <= TARGET_MAX_WORDS ? 0 : (end - TARGET_MAX_WORDS + (4ull << g) - 1) >> (2 + g);
                        return 0x80000000ull + hu + hu / 8 < HANDLE_MAX;
                    };
                    while (L.root_g < ROOT_G_MAX && !fits(L.root_g)) ++L.root_g;
                }
            }
        }
        const uint32_t h = (uint32_t)(p >> 40) & 63u;
        const uint64_t table = h ? (1ull << h) : 0;
        const uint64_t cb = (p & P_CB) ? CB_WORDS : 0;              // closure filter
        uint64_t total = 0;
        w = arena_fit_g(w, table, cb, p & ((1ull << 40) - 1), total, L.root_g);
        const uint64_t unit = handle_at_word(w + table + cb, L.root_g);
        if (!root || stub ? unit >= (uint64_t)EDGE_VAL : unit >= HANDLE_MAX)
            throw Error{KETO_E_RANGE, root && !stub ? "device arena exceeds the 2^32 handles (288 GiB)"
                                                    : "subject-set targets exceed 2^31 16-byte units"};
        L.layout_units[x] = (uint32_t)unit;
        if (!root && !stub) L.shared_words += total;
        w += total;
        if (mode == PART_MIGRATE && band[L.rows_by_unit[x]] >= hot_band) {   // the replicated prefix so far
            L.hot_words = w;
            ++L.hot_rows;
        }
    }
    par_chunks(kept, th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t x = b; x < e; ++x) L.unit_of_row[L.rows_by_unit[x]] = L.layout_units[x];
    });
    if (w > (L.root_g ? ARENA_MAX_WORDS : NARROW_MAX_WORDS))
        throw Error{KETO_E_RANGE, "device arena exceeds 2^34 words (64 GiB) in 16-byte handles"};
    if (mode == PART_MIGRATE && w > TARGET_MAX_WORDS)
        throw Error{KETO_E_RANGE, "a migrating part's arena exceeds 2^31 16-byte units"};
    L.n_words = w;
    L.n_units = handle_end(w, L.root_g);
}
}  // namespace

void compute_layout(Snapshot& S) {
    const uint32_t R = S.n_rows();
    // Hot rows first: rows that many subject sets point at (popular folders, groups) are laid out
    // densely at the front of the arena, most-referenced first, so the lines most traversals touch
    // stay in L2 and the Infinity Cache.  A stable counting sort by floor(log2(in-degree)).
    std::vector<uint8_t> band(R, 0);
    {
        std::vector<uint32_t> indeg(R, 0);
        const unsigned th = R >= par_min() ? build_threads() : 1u;
        par_chunks(R, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t r = b; r < e; ++r) {
                const auto ed = S.row_edges((uint32_t)r);
                for (uint64_t i = 0; i < ed.second; ++i) {
                    const uint32_t x = ed.first[i];
                    if ((x & EDGE_SET) && x != EDGE_POISON && (x & EDGE_VAL) < R)
                        __atomic_fetch_add(&indeg[x & EDGE_VAL], 1u, __ATOMIC_RELAXED);
                }
            }
        });
        S.is_root.assign(R, 0);
        par_chunks(R, th, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t r = b; r < e; ++r) {
                band[r] = indeg[r] ? (uint8_t)(32 - __builtin_clz(indeg[r])) : 0;
                S.is_root[r] = indeg[r] == 0;
            }
        });
    }
    if (S.part_mode == PART_MIGRATE && S.n_parts > MIG_MAX_PARTS)
        throw Error{KETO_E_INVALID, "a migrating partition has at most 30 parts"};
    // PART_MIGRATE: the hottest in-degree bands whose rows fit S.hot_bytes are replicated
    uint32_t hot_band = 64;                              // none
    if (S.part_mode == PART_MIGRATE && S.hot_bytes > 0 && S.n_parts > 1) {
        std::vector<uint64_t> bw(34, 0);
        for (uint32_t r = 0; r < R; ++r) {
            if (!band[r]) continue;
            const uint32_t h = S.row_hlog2(r);
            bw[band[r]] += (h ? (1ull << h) : 0) + CB_WORDS + HDR_WORDS + ((row_size(S, r) + 3) & ~3ull);
        }
        uint64_t acc = 0;
        for (uint32_t b = 33; b >= 1; --b) {
            if ((acc + bw[b]) * 4 > S.hot_bytes) break;
            acc += bw[b];
            hot_band = b;
        }
    }
    PartLayout L;
    layout_part(S, band, S.part, S.n_parts, S.part_mode, hot_band, L);
    S.unit_of_row = std::move(L.unit_of_row);
    S.rows_by_unit = std::move(L.rows_by_unit);
    S.layout_units = std::move(L.layout_units);
    S.stub = std::move(L.stub);
    S.n_stubs = L.n_stubs;
    S.n_units = L.n_units;
    S.n_words = L.n_words;
    S.root_g = L.root_g;
    S.tgt_tail = L.tgt_tail;
    S.tgt_end = L.tgt_end;
    S.roots_at = L.roots_at;
    S.shared_words = L.shared_words;
    S.hot_units = (uint32_t)(L.hot_words / HDR_WORDS);
    S.hot_rows = L.hot_rows;
    S.g_handle.clear();
    if (S.part_mode == PART_MIGRATE) {
        // every row's handle on its owner part: the layouts of the other parts are computed here too
        // (each is a deterministic function of the snapshot and the part)
        S.g_handle.assign(R, NO_UNIT);
        for (uint32_t q = 0; q < S.n_parts; ++q) {
            const std::vector<uint32_t>* u = &S.unit_of_row;
            PartLayout Q;
            if (q != S.part) {
                layout_part(S, band, q, S.n_parts, S.part_mode, hot_band, Q);
                u = &Q.unit_of_row;
            }
            for (uint32_t r = 0; r < R; ++r)
                if (S.root_owner(r, S.n_parts) == q) S.g_handle[r] = (*u)[r];
        }
    }
    S.row_cb.assign(R, 0);
    for (uint32_t r = 0; r < R; ++r) S.row_cb[r] = !S.is_root[r];
    S.row_place.clear();
}

uint32_t Snapshot::root_owner(uint32_t r, uint32_t parts) const {
    // hash(namespace id, object): every relation of one object lives on one part
    uint64_t h = (uint64_t)(uint32_t)row_key[r].ns * 0x9E3779B97F4A7C15ull ^ (uint64_t)row_key[r].obj * 0xC2B2AE3D27D4EB4Full;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return parts ? (uint32_t)(h % parts) : 0;
}

int64_t Snapshot::row_of_handle(uint32_t unit) const {
    auto it = std::lower_bound(layout_units.begin(), layout_units.end(), unit);   // increasing
    if (it == layout_units.end() || *it != unit) return -1;
    return rows_by_unit[it - layout_units.begin()];
}

uint32_t handle_of(const Snapshot& S, const Overlay* ov, uint32_t row) {
    if (ov && row >= ov->base) return (uint32_t)(S.n_units + ov->unit[row - ov->base]);
    return S.unit_of_row[row];
}

uint32_t Snapshot::vid_of_row(uint32_t row) const {
    if (!coll.empty()) {
        auto it = coll.find(EDGE_SET | row);
        if (it != coll.end()) return it->second;
    }
    // a root row past 2^31 units (split layout): no subject set points at it, so nothing in its own
    // tree can be it; its handle could read as a collision class's visit id (VID_CLASS | c)
    const uint32_t u = unit_of_row[row];
    return u != NO_UNIT && u >= EDGE_VAL ? 0xFFFFFFF0u : u;
}

std::string Snapshot::row_field_ns(uint32_t row) const {
    const RowKey& k = row_key[row];
    if (k.ns == ANY_NS) return "";
    auto it = ns_by_id.find((int32_t)k.ns);
    return it == ns_by_id.end() ? std::string() : ns_names[it->second];
}

std::string Snapshot::row_field(uint32_t row, int which) const {
    uint32_t v = which == 1 ? row_key[row].obj : row_key[row].rel;
    if (v == ANY || v >= strs.size()) return "";
    return strs[v];
}

std::string Snapshot::subject_string(uint32_t ref) const {
    if (ref & EDGE_SET) {
        uint32_t r = ref & EDGE_VAL;
        return row_field_ns(r) + ":" + row_field(r, 1) + "#" + row_field(r, 2);
    }
    return ref < strs.size() ? strs[ref] : std::string();
}

std::unique_ptr<Snapshot> build_snapshot(const keto_namespace* ns, uint32_t n_ns, const keto_tuple* tup, uint64_t n,
                                         uint32_t page_size) {
    auto Sp = std::make_unique<Snapshot>();
    Snapshot& S = *Sp;
    S.page_size = page_size ? page_size : 100;
    S.n_tuples = n;
    load_namespaces(S, ns, n_ns);
    if (n && !tup) throw Error{KETO_E_INVALID, "tuples == NULL"};

    // ---- intern strings (ids = ranks in byte order), in parallel
    PhaseClock clk;
    const unsigned threads = n >= par_min() ? build_threads() : 1u;
    std::vector<T> ts(n);
    {
        std::vector<std::string_view> extra{std::string_view("")};
        for (const auto& nm : S.ns_names) extra.push_back(nm);
        ParInterner in;
        in.run(tup, n, extra, threads);
        S.strs.resize(in.uniq.size());
        S.n_sorted_strs = (uint32_t)in.uniq.size();
        par_chunks(in.uniq.size(), threads, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i) S.strs[i] = std::string(in.uniq[i]);
        });
        S.empty_str = in.occ[n * ParInterner::FIELDS];
        const uint32_t* o = in.occ.data();
        par_chunks(n, threads, 1 << 16, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i) {
                const keto_tuple& t = tup[i];
                T& x = ts[i];
                const uint32_t* q = o + i * ParInterner::FIELDS;
                x.ns = t.namespace_id;
                x.obj = q[0];
                x.rel = q[1];
                x.kind = t.subject_kind ? 1 : 0;
                x.seq = i;
                x.a = q[2];
                x.sns = x.kind ? t.set_namespace_id : 0;
                x.srel = x.kind ? q[3] : 0;
            }
        });
    }

    clk.lap("intern");
    // ---- reference ORDER BY (parallel sample sort; tuple_less is a total order: commit seq last)
    parallel_sort(ts, tuple_less, threads);
    clk.lap("order by");

    // ---- real rows
    std::vector<uint64_t> real_ptr;   // per real row begin (in tuple index space)
    for (uint64_t i = 0; i < n; ++i) {
        if (i == 0 || ts[i].ns != ts[i - 1].ns || ts[i].obj != ts[i - 1].obj || ts[i].rel != ts[i - 1].rel) {
            real_ptr.push_back(i);
            S.row_key.push_back(RowKey{ts[i].ns, ts[i].obj, ts[i].rel});
        }
    }
    real_ptr.push_back(n);
    if (real_ptr.size() - 1 >= (uint64_t)EDGE_VAL) throw Error{KETO_E_RANGE, "more than 2^31-1 rows"};
    S.n_real_rows = (uint32_t)(real_ptr.size() - 1);

    // ---- subject sets -> target rows (real, empty or wildcard)
    std::vector<RowKey> wild_keys;          // wildcard rows, in creation order
    std::vector<uint8_t> extra_is_wild;     // for rows >= n_real_rows
    auto target_row = [&](int32_t sns, uint32_t sobj, uint32_t srel, bool& poison) -> uint32_t {
        auto it = S.ns_by_id.find(sns);
        if (it == S.ns_by_id.end()) { poison = true; return EDGE_POISON; }
        poison = false;
        const std::string& name = S.ns_names[it->second];
        RowKey k{name.empty() ? ANY_NS : (int64_t)sns, sobj == S.empty_str ? ANY : sobj,
                 srel == S.empty_str ? ANY : srel};
        bool wild = k.ns == ANY_NS || k.obj == ANY || k.rel == ANY;
        if (!wild) {
            uint32_t lo = 0, hi = S.n_real_rows;
            while (lo < hi) {
                uint32_t m = lo + (hi - lo) / 2;
                int64_t c = key_cmp(S.row_key[m], k);
                if (c == 0) return m;
                if (c < 0) lo = m + 1; else hi = m;
            }
        }
        auto f = S.row_of.find(k);
        if (f != S.row_of.end()) return f->second;
        uint32_t id = (uint32_t)S.row_key.size();
        if (id >= EDGE_VAL) throw Error{KETO_E_RANGE, "more than 2^31-1 rows"};
        S.row_key.push_back(k);
        S.row_of.emplace(k, id);
        extra_is_wild.push_back(wild ? 1 : 0);
        if (wild) wild_keys.push_back(k);
        return id;
    };

    // ---- real-row edges: subject sets whose target is a real row are resolved in parallel (binary
    // search over the sorted real rows); the rest (unknown namespaces, empty and wildcard targets)
    // go through target_row in tuple order, which creates their rows in the sequential order
    std::vector<uint32_t> real_edges(n);
    std::vector<uint8_t> poison(n, 0);
    constexpr uint32_t LATER = 0xFFFFFFFEu;
    par_chunks(n, threads, 1 << 15, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t i = b; i < e; ++i) {
            const T& x = ts[i];
            const bool own_unknown = !S.ns_by_id.count(x.ns);
            real_edges[i] = x.a;
            poison[i] = own_unknown;
            if (x.kind == 1) {
                real_edges[i] = LATER;
                auto it = S.ns_by_id.find(x.sns);
                if (it == S.ns_by_id.end() || S.ns_names[it->second].empty() || x.a == S.empty_str ||
                    x.srel == S.empty_str)
                    continue;
                const RowKey k{(int64_t)x.sns, x.a, x.srel};
                uint32_t lo = 0, hi = S.n_real_rows;
                while (lo < hi) {
                    const uint32_t m = lo + (hi - lo) / 2;
                    const int64_t c = key_cmp(S.row_key[m], k);
                    if (c == 0) {
                        real_edges[i] = EDGE_SET | m;
                        break;
                    }
                    if (c < 0) lo = m + 1; else hi = m;
                }
            }
            if (poison[i] && real_edges[i] != LATER) real_edges[i] = EDGE_POISON;
        }
    });
    for (uint64_t i = 0; i < n; ++i) {
        if (real_edges[i] != LATER) continue;
        const T& x = ts[i];
        bool p;
        const uint32_t r = target_row(x.sns, x.a, x.srel, p);
        real_edges[i] = p ? EDGE_POISON : (EDGE_SET | r);
        poison[i] = p || poison[i];
        if (poison[i]) real_edges[i] = EDGE_POISON;
    }
    uint32_t R = (uint32_t)S.row_key.size();
    S.n_wild_rows = (uint32_t)wild_keys.size();

    // ---- assemble edges: real rows, then empty rows (no edges), then wildcard rows
    std::vector<uint64_t> row_ptr(R + 1, 0);
    S.row_pp.assign(R, NO_PAGE);
    S.edges.reserve(n);
    for (uint32_t r = 0; r < S.n_real_rows; ++r) {
        row_ptr[r] = S.edges.size();
        for (uint64_t i = real_ptr[r]; i < real_ptr[r + 1]; ++i) {
            if (poison[i] && S.row_pp[r] == NO_PAGE) S.row_pp[r] = (uint32_t)((i - real_ptr[r]) / S.page_size);
            S.edges.push_back(real_edges[i]);
        }
    }
    std::vector<uint8_t> is_wild(R, 0);
    for (uint32_t r = S.n_real_rows; r < R; ++r) {
        row_ptr[r] = S.edges.size();
        if (!extra_is_wild[r - S.n_real_rows]) continue;
        is_wild[r] = 1;
        S.wild_rows.push_back(r);
        const RowKey& k = S.row_key[r];
        uint64_t pos = 0;
        for (uint32_t q = 0; q < S.n_real_rows; ++q) {          // matching real rows in ORDER BY order
            const RowKey& rk = S.row_key[q];
            if ((k.ns != ANY_NS && rk.ns != k.ns) || (k.obj != ANY && rk.obj != k.obj) ||
                (k.rel != ANY && rk.rel != k.rel))
                continue;
            for (uint64_t i = real_ptr[q]; i < real_ptr[q + 1]; ++i, ++pos) {
                if (poison[i] && S.row_pp[r] == NO_PAGE) S.row_pp[r] = (uint32_t)(pos / S.page_size);
                S.edges.push_back(real_edges[i]);
            }
        }
    }
    row_ptr[R] = S.edges.size();

    clk.lap("rows + edges");
    // ---- visit-key collision classes over every typed subject: rows (sets) and subject ids.  A
    // 64-bit hash of every key (rows' String() and used ids, in parallel) is sorted; only keys whose
    // hash occurs twice are materialized and grouped exactly.
    {
        std::vector<uint8_t> id_used(S.strs.size(), 0);
        for (uint32_t e : S.edges)
            if (!(e & EDGE_SET) && e != EDGE_POISON) id_used[e] = 1;
        auto row_subject = [&](uint32_t r) {          // unknown-ns rows are never subjects
            const RowKey& k = S.row_key[r];
            return k.ns == ANY_NS || S.ns_by_id.count((int32_t)k.ns) != 0;
        };
        constexpr uint32_t ROW_TAG = 0x80000000u;
        std::vector<std::pair<uint64_t, uint32_t>> hk(R + S.strs.size());
        std::vector<uint8_t> keep(R + S.strs.size(), 0);
        par_chunks(R + S.strs.size(), threads, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i) {
                if (i < R) {
                    if (!row_subject((uint32_t)i)) continue;
                    hk[i] = {hash_bytes(S.subject_string(EDGE_SET | (uint32_t)i)), ROW_TAG | (uint32_t)i};
                } else {
                    const uint32_t sid = (uint32_t)(i - R);
                    if (!id_used[sid]) continue;
                    hk[i] = {hash_bytes(S.strs[sid]), sid};
                }
                keep[i] = 1;
            }
        });
        {
            uint64_t w = 0;
            for (uint64_t i = 0; i < hk.size(); ++i)
                if (keep[i]) hk[w++] = hk[i];
            hk.resize(w);
        }
        parallel_sort(hk, [](const std::pair<uint64_t, uint32_t>& x, const std::pair<uint64_t, uint32_t>& y) {
            return x.first != y.first ? x.first < y.first : x.second < y.second;
        }, threads);
        std::unordered_map<std::string, std::vector<uint32_t>> owners;   // candidate key -> typed subjects
        for (uint64_t i = 0; i < hk.size();) {
            uint64_t j = i + 1;
            while (j < hk.size() && hk[j].first == hk[i].first) ++j;
            if (j - i >= 2)
                for (uint64_t k = i; k < j; ++k) {
                    const uint32_t tag = hk[k].second;
                    owners[(tag & ROW_TAG) ? S.subject_string(EDGE_SET | (tag & ~ROW_TAG)) : S.strs[tag]].push_back(tag);
                }
            i = j;
        }
        S.n_coll_keys = 0;
        for (auto& kv : owners) {
            if (kv.second.size() < 2) continue;             // a hash collision, not a key collision
            const uint32_t c = VID_CLASS | S.n_coll_keys++;
            for (uint32_t tag : kv.second) S.coll[(tag & ROW_TAG) ? (EDGE_SET | (tag & ~ROW_TAG)) : tag] = c;
        }
    }

    clk.lap("collision classes");
    S.n_base_rows = R;
    finalize_rows(S, row_ptr, is_wild);
    compute_layout(S);
    clk.lap("rows + layout");
    return Sp;
}

std::unique_ptr<Snapshot> build_snapshot_csr(const keto_namespace* ns, uint32_t n_ns, uint32_t n_rows,
                                             const int32_t* row_ns, const uint32_t* row_obj,
                                             const uint32_t* row_rel, const uint64_t* row_ptr,
                                             const uint32_t* edges, const keto_str* strings, uint32_t n_strings,
                                             uint32_t page_size) {
    auto Sp = std::make_unique<Snapshot>();
    Snapshot& S = *Sp;
    S.page_size = page_size ? page_size : 100;
    load_namespaces(S, ns, n_ns);
    if (!row_ns || !row_obj || !row_rel || !row_ptr || (row_ptr[n_rows] && !edges))
        throw Error{KETO_E_INVALID, "NULL array"};
    if (n_rows >= EDGE_VAL) throw Error{KETO_E_RANGE, "more than 2^31-1 rows"};
    if (strings) {
        S.strs.resize(n_strings);
        par_chunks(n_strings, n_strings >= par_min() ? build_threads() : 1u, 1 << 14,
                   [&](uint64_t b, uint64_t e, unsigned) {
                       for (uint64_t i = b; i < e; ++i) S.strs[i] = std::string(sv(strings[i]));
                   });
        S.n_sorted_strs = n_strings;
        S.empty_str = n_strings && S.strs[0].empty() ? 0u : ANY;      // "" sorts first
    }
    S.row_key.resize(n_rows);
    for (uint32_t r = 0; r < n_rows; ++r) {
        S.row_key[r] = RowKey{row_ns[r], row_obj[r], row_rel[r]};
        if (r && key_cmp(S.row_key[r - 1], S.row_key[r]) >= 0)
            throw Error{KETO_E_INVALID, "rows not in (namespace_id, object, relation) order"};
    }
    S.n_real_rows = n_rows;
    uint64_t E = row_ptr[n_rows];
    S.n_tuples = E;
    S.edges.assign(edges, edges + E);
    S.row_pp.assign(n_rows, NO_PAGE);
    std::vector<uint64_t> rp(row_ptr, row_ptr + n_rows + 1);
    std::vector<uint8_t> is_wild(n_rows, 0);
    S.n_base_rows = n_rows;
    finalize_rows(S, rp, is_wild);
    compute_layout(S);
    return Sp;
}

// A host copy of a snapshot for another device (keto_snapshot_clone): every host table the engine
// reads, at the snapshot's current version, laid out afresh (as a host-only snapshot is after writes,
// delta.cpp).  The resolution indexes are rebuilt on the copy's first lookup.
std::unique_ptr<Snapshot> clone_host(const Snapshot& S) {
    if (S.n_parts > 1) throw Error{KETO_E_INVALID, "a part of a partitioned snapshot cannot be cloned"};
    auto Cp = std::make_unique<Snapshot>();
    Snapshot& C = *Cp;
    C.ns_ids = S.ns_ids;
    C.ns_names = S.ns_names;
    C.ns_by_name = S.ns_by_name;
    C.ns_by_id = S.ns_by_id;
    for (uint32_t i = 0; i < (uint32_t)C.ns_names.size(); ++i) C.ns_view.emplace(C.ns_names[i], (int)i);
    C.page_size = S.page_size;
    C.strs = S.strs;
    C.empty_str = S.empty_str;
    C.n_real_rows = S.n_real_rows;
    C.n_wild_rows = S.n_wild_rows;
    C.wild_rows = S.wild_rows;
    C.row_key = S.row_key;
    C.row_of = S.row_of;
    C.rows = S.rows;
    C.row_pp = S.row_pp;
    C.edges = S.edges;
    C.row_has_coll = S.row_has_coll;
    C.coll = S.coll;
    C.n_coll_keys = S.n_coll_keys;
    C.coll_dirty = false;
    C.n_tuples = S.n_tuples;
    C.n_poisoned_rows = S.n_poisoned_rows;
    C.n_seq_rows = S.n_seq_rows;
    C.version = S.version.load();
    C.n_sorted_strs = S.n_sorted_strs;
    C.added_str = S.added_str;
    C.n_base_rows = S.n_base_rows;
    C.row_over = S.row_over;
    compute_layout(C);
    return Cp;
}

}  // namespace keto
