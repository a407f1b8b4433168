// Snapshot lifecycle: writes applied to a live snapshot as a delta, with a version.
//
// The reference reads the live table on every check (internal/persistence/sql/relationtuples.go:
// 238-277), so a snapshot must follow the writes.  keto_snapshot_apply takes one transaction the way
// TransactRelationTuples runs it (relationtuples.go:289-297): the inserts first (InsertRelationTuple,
// :128-149: a new row with commit_time = now, i.e. after every equal tuple), then the deletes
// (DeleteRelationTuples, :200-223: every tuple equal to the given one -- namespace, object,
// relation and the exact subject).  A namespace name that is not configured fails the whole
// transaction, as GetNamespaceByName does there.
//
// Every row the transaction touches gets its new edge list in ORDER BY order (sets before ids,
// sets by namespace id then object / relation bytes, ids by bytes, ties in commit order) in
// Snapshot::row_over; device_apply (engine.hip) rewrites those rows in the device arena.  New strings
// are appended after the build's byte-ordered ones and compared by bytes wherever order matters.
//
// A write that creates a Subject.String() collision gives the colliding subjects a collision class and
// re-flags the rows that hold them ROW_SEQ, as the build would have.  A stored subject set with an
// empty field (a wildcard set: its query leaves that field out, relationtuples.go:178-198) points at
// a materialized wildcard row, the concatenation of every row its query matches in ORDER BY order
// (snapshot.cpp); a write that inserts a new wildcard set creates that row, and a write that changes
// a row some wildcard row matches re-materializes the wildcard row from the staged edges.  Writes
// outside this delta path throw KETO_E_REBUILD and leave the snapshot unchanged; the caller rebuilds
// it (keto_snapshot_build from the table): a write that touches a poisoned row (one whose pages hold
// a tuple of an unknown namespace), or a wildcard row that matches one.  A part of an
// edge-partitioned snapshot (KETO_PART_SHARED) takes every transaction: its host tables are the whole
// graph's, and device_apply writes the rows the part holds (every subject-set target and its own root
// rows); a migrating part takes none.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

namespace {

inline std::string_view sv(const keto_str& s) { return std::string_view(s.p ? s.p : "", s.n); }
inline bool wild_key(const RowKey& k) { return k.ns == ANY_NS || k.obj == ANY || k.rel == ANY; }
inline bool key_matches(const RowKey& w, const RowKey& k) {     // does wildcard query w return row k
    return (w.ns == ANY_NS || w.ns == k.ns) && (w.obj == ANY || w.obj == k.obj) && (w.rel == ANY || w.rel == k.rel);
}

struct Txn {
    Snapshot& S;
    std::unordered_map<uint32_t, std::vector<uint32_t>> rows;    // staged edges per touched row
    std::vector<uint32_t> order;                                  // touched rows, first-touch order
    std::vector<std::string> new_strs;                            // strings this transaction adds
    std::unordered_map<std::string, uint32_t> new_str_id;
    std::vector<RowKey> new_keys;                                 // rows this transaction adds
    std::unordered_map<RowKey, uint32_t, RowKeyHash> new_row_id;
    std::vector<uint32_t> new_targets;                            // rows some inserted subject set points at

    explicit Txn(Snapshot& s) : S(s) {}

    int32_t ns_id(std::string_view name) const {
        auto it = S.ns_by_name.find(std::string(name));
        if (it == S.ns_by_name.end())
            throw Error{KETO_E_INVALID, "Unknown namespace with name " + std::string(name) + "."};
        return S.ns_ids[it->second];
    }
    int32_t ns_id_checked(int32_t id) const {
        if (!S.ns_by_id.count(id)) throw Error{KETO_E_INVALID, "Unknown namespace with id " + std::to_string(id) + "."};
        return id;
    }
    // string id, existing or staged (-1: absent and !add)
    int64_t str(std::string_view s, bool add) {
        const int64_t id = S.lookup_str(s);
        if (id >= 0) return id;
        auto it = new_str_id.find(std::string(s));
        if (it != new_str_id.end()) return it->second;
        if (!add) return -1;
        const uint32_t nid = (uint32_t)(S.strs.size() + new_strs.size());
        if (nid >= EDGE_VAL) throw Error{KETO_E_RANGE, "more than 2^31-1 strings"};
        new_strs.emplace_back(s);
        new_str_id.emplace(std::string(s), nid);
        return nid;
    }
    const std::string& str_of(uint32_t id) const {
        return id < S.strs.size() ? S.strs[id] : new_strs[id - S.strs.size()];
    }
    int cmp(uint32_t a, uint32_t b) const {
        if (a == b) return 0;
        if (a < S.n_sorted_strs && b < S.n_sorted_strs) return a < b ? -1 : 1;
        const int c = str_of(a).compare(str_of(b));
        return c < 0 ? -1 : c > 0 ? 1 : 0;
    }
    const RowKey& key(uint32_t r) const { return r < S.row_key.size() ? S.row_key[r] : new_keys[r - S.row_key.size()]; }
    // a key field of a subject set's target row: ANY stands for the empty string the tuple stored
    int field_cmp(uint32_t a, uint32_t b) const {
        if (a == b) return 0;
        static const std::string empty;
        const std::string& x = a == ANY ? empty : str_of(a);
        const std::string& y = b == ANY ? empty : str_of(b);
        if (a != ANY && b != ANY) return cmp(a, b);
        const int c = x.compare(y);
        return c < 0 ? -1 : c > 0 ? 1 : 0;
    }
    int64_t ns_field(int64_t ns) const {              // ANY_NS: the namespace named "" (its config id)
        if (ns != ANY_NS) return ns;
        auto it = S.ns_by_name.find("");
        return it == S.ns_by_name.end() ? ANY_NS : (int64_t)S.ns_ids[it->second];
    }
    // ORDER BY position of a subject set: (namespace id, object bytes, relation bytes)
    int set_cmp(uint32_t ra, uint32_t rb) const {
        const RowKey &a = key(ra), &b = key(rb);
        const int64_t na = ns_field(a.ns), nb = ns_field(b.ns);
        if (na != nb) return na < nb ? -1 : 1;
        if (a.obj != b.obj) return field_cmp(a.obj, b.obj);
        if (a.rel != b.rel) return field_cmp(a.rel, b.rel);
        return 0;
    }
    // row of a complete key (-1: none yet)
    int64_t row(const RowKey& k) const {
        uint32_t lo = 0, hi = S.n_real_rows;
        while (lo < hi) {
            const uint32_t m = lo + (hi - lo) / 2;
            const RowKey& x = S.row_key[m];
            const int c = x.ns != k.ns ? (x.ns < k.ns ? -1 : 1) : x.obj != k.obj ? (x.obj < k.obj ? -1 : 1)
                                                                    : x.rel != k.rel ? (x.rel < k.rel ? -1 : 1) : 0;
            if (c == 0) return m;
            if (c < 0) lo = m + 1; else hi = m;
        }
        auto it = S.row_of.find(k);
        if (it != S.row_of.end()) return it->second;
        auto jt = new_row_id.find(k);
        return jt == new_row_id.end() ? -1 : (int64_t)jt->second;
    }
    uint32_t row_or_new(const RowKey& k) {
        const int64_t r = row(k);
        if (r >= 0) return (uint32_t)r;
        const uint32_t id = (uint32_t)(S.row_key.size() + new_keys.size());
        if (id >= EDGE_VAL) throw Error{KETO_E_RANGE, "more than 2^31-1 rows"};
        new_keys.push_back(k);
        new_row_id.emplace(k, id);
        return id;
    }
    std::vector<uint32_t>& edges(uint32_t r) {
        auto it = rows.find(r);
        if (it != rows.end()) return it->second;
        if (r < S.rows.size() && S.row_pp[r] != NO_PAGE)           // holds EDGE_POISON entries
            throw Error{KETO_E_REBUILD, "a write touches a poisoned row"};
        const auto e = r < S.rows.size() ? S.row_edges(r) : std::pair<const uint32_t*, uint64_t>{nullptr, 0};
        order.push_back(r);
        return rows.emplace(r, std::vector<uint32_t>(e.first, e.first + e.second)).first->second;
    }
    // 0 < position of edge value v among e (sets before ids), after every equal edge
    uint64_t upper(const std::vector<uint32_t>& e, uint32_t v) const {
        uint64_t lo = 0, hi = e.size();
        while (lo < hi) {
            const uint64_t m = (lo + hi) / 2;
            if (less(v, e[m])) hi = m; else lo = m + 1;
        }
        return lo;
    }
    bool less(uint32_t a, uint32_t b) const {           // strict ORDER BY of two edge values
        const bool sa = a & EDGE_SET, sb = b & EDGE_SET;
        if (sa != sb) return sa;                        // subject_id NULL (sets) first
        if (sa) return set_cmp(a & EDGE_VAL, b & EDGE_VAL) < 0;
        return cmp(a, b) < 0;
    }

    RowKey tuple_key(const keto_tuple& t, bool add) {
        RowKey k;
        k.ns = ns_id_checked(t.namespace_id);
        const int64_t o = str(sv(t.object), add), r = str(sv(t.relation), add);
        k.obj = o < 0 ? ANY : (uint32_t)o;                                // ANY: absent (delete only)
        k.rel = r < 0 ? ANY : (uint32_t)r;
        return k;
    }
    // edge value of the tuple's subject; ~0 when it cannot exist (delete of unknown strings)
    uint32_t subject_value(const keto_tuple& t, bool add) {
        if (!t.subject_kind) {
            const int64_t id = str(sv(t.subject_id), add);
            return id < 0 ? NONE : (uint32_t)id;
        }
        const int32_t sns = ns_id_checked(t.set_namespace_id);
        // an empty field is left out of the set's query (the build's target_row): ANY
        RowKey k{S.ns_names[S.ns_by_id.at(sns)].empty() ? ANY_NS : (int64_t)sns, ANY, ANY};
        if (t.set_object.n) {
            const int64_t o = str(sv(t.set_object), add);
            if (o < 0) return NONE;
            k.obj = (uint32_t)o;
        }
        if (t.set_relation.n) {
            const int64_t r = str(sv(t.set_relation), add);
            if (r < 0) return NONE;
            k.rel = (uint32_t)r;
        }
        if (!add) {
            const int64_t x = row(k);
            return x < 0 ? NONE : (EDGE_SET | (uint32_t)x);
        }
        const uint32_t x = row_or_new(k);
        new_targets.push_back(x);
        return EDGE_SET | x;
    }
    static constexpr uint32_t NONE = 0xFFFFFFFFu;

    // ORDER BY position of two complete row keys: (namespace id, object bytes, relation bytes)
    bool key_less(uint32_t ra, uint32_t rb) const {
        const RowKey &a = key(ra), &b = key(rb);
        if (a.ns != b.ns) return a.ns < b.ns;
        if (a.obj != b.obj) return cmp(a.obj, b.obj) < 0;
        return cmp(a.rel, b.rel) < 0;
    }
    // the edges of wildcard row w as the staged table holds them: the rows its query returns
    // (relationtuples.go:250 ORDER BY), concatenated -- the build's materialization (snapshot.cpp)
    std::vector<uint32_t> materialize(const RowKey& w) const {
        std::vector<uint32_t> sorted, extra;
        uint32_t lo = 0, hi = S.n_real_rows;           // real rows sort by namespace first
        if (w.ns != ANY_NS) {
            lo = (uint32_t)(std::lower_bound(S.row_key.begin(), S.row_key.begin() + hi, w.ns,
                                             [](const RowKey& x, int64_t n) { return x.ns < n; }) - S.row_key.begin());
            hi = (uint32_t)(std::upper_bound(S.row_key.begin() + lo, S.row_key.begin() + hi, w.ns,
                                             [](int64_t n, const RowKey& x) { return n < x.ns; }) - S.row_key.begin());
        }
        for (uint32_t q = lo; q < hi; ++q)
            if (key_matches(w, S.row_key[q])) sorted.push_back(q);
        // rows outside the build's sorted range that hold tuples: changed by earlier writes or staged now
        auto extra_row = [&](uint32_t q) {
            if (q < S.n_real_rows || wild_key(key(q)) || !key_matches(w, key(q))) return;
            extra.push_back(q);
        };
        for (const auto& kv : S.row_over) extra_row(kv.first);
        for (const auto& kv : rows)
            if (!S.row_over.count(kv.first)) extra_row(kv.first);
        std::sort(extra.begin(), extra.end(), [&](uint32_t a, uint32_t b) { return key_less(a, b); });
        std::vector<uint32_t> order(sorted.size() + extra.size());
        std::merge(sorted.begin(), sorted.end(), extra.begin(), extra.end(), order.begin(),
                   [&](uint32_t a, uint32_t b) { return key_less(a, b); });
        std::vector<uint32_t> out;
        for (uint32_t q : order) {
            if (q < S.rows.size() && S.row_pp[q] != NO_PAGE)
                throw Error{KETO_E_REBUILD, "a wildcard row that changes matches a poisoned row"};
            auto st = rows.find(q);
            if (st != rows.end()) {
                out.insert(out.end(), st->second.begin(), st->second.end());
            } else {
                const auto e = S.row_edges(q);
                out.insert(out.end(), e.first, e.first + e.second);
            }
        }
        return out;
    }
};

std::string key_string(const Snapshot& S, const Txn& T, const RowKey& k) {     // Subject.String()
    auto it = k.ns == ANY_NS ? S.ns_by_id.end() : S.ns_by_id.find((int32_t)k.ns);
    const std::string ns = it == S.ns_by_id.end() ? "" : S.ns_names[it->second];
    return ns + ":" + (k.obj == ANY ? std::string() : T.str_of(k.obj)) + "#" +
           (k.rel == ANY ? std::string() : T.str_of(k.rel));
}

// Room for a transaction's new rows in every per-row table, made before the exclusive lock: a table
// at capacity is copied into a larger buffer here (reads only -- batches keep running) and swapped in
// at commit, so the commit never reallocates a table of every row (50 B a row: 11 GB at the 1B-tuple
// graph's rows, seconds of blocked batches).  The old buffers go to Snapshot::retired, freed after
// the exclusive lock is released.
struct Grown {
    std::vector<RowKey> row_key;
    std::vector<RowRec> rows;
    std::vector<uint32_t> row_pp, unit_of_row, layout_units, rows_by_unit;
    std::vector<uint8_t> is_root, row_cb;
    template <class V>
    static void make(const V& v, size_t extra, V& next) {
        if (!extra || v.size() + extra <= v.capacity()) return;
        next.reserve(v.size() + std::max<size_t>(extra, v.size() / 4 + 1024));
        next.assign(v.begin(), v.end());
    }
    template <class V>
    static void put(V& v, V& next, std::vector<std::shared_ptr<void>>& retired) {
        if (!next.capacity()) return;
        v.swap(next);
        retired.push_back(std::make_shared<V>(std::move(next)));
    }
    // k new rows; `placed` rows that may get an arena place (device_apply appends them to the layout)
    Grown(const Snapshot& S, size_t k, size_t placed) {
        make(S.row_key, k, row_key);
        make(S.rows, k, rows);
        make(S.row_pp, k, row_pp);
        make(S.unit_of_row, k, unit_of_row);
        make(S.is_root, k, is_root);
        make(S.row_cb, k, row_cb);
        if (S.dev) {
            make(S.layout_units, placed, layout_units);
            make(S.rows_by_unit, placed, rows_by_unit);
        }
    }
    void swap_in(Snapshot& S) {
        put(S.row_key, row_key, S.retired);
        put(S.rows, rows, S.retired);
        put(S.row_pp, row_pp, S.retired);
        put(S.unit_of_row, unit_of_row, S.retired);
        put(S.is_root, is_root, S.retired);
        put(S.row_cb, row_cb, S.retired);
        put(S.layout_units, layout_units, S.retired);
        put(S.rows_by_unit, rows_by_unit, S.retired);
    }
};

}  // namespace

void apply_writes(Snapshot& S, const keto_tuple* ins, uint64_t n_ins, const keto_tuple* del, uint64_t n_del,
                  const std::function<void()>& commit) {
    // a part of an edge-partitioned snapshot holds the whole graph's host tables: every part applies
    // every transaction.  A shared-rows part writes the rows it holds in place (device_apply); a
    // migrating part's stubs carry their owners' handles and filters, which a write on the owner can
    // move, so device_apply lays the part out afresh from the host tables (every part computes every
    // part's layout the same way) and the next routed batch exchanges the closure filters again
    if ((n_ins && !ins) || (n_del && !del)) throw Error{KETO_E_INVALID, "NULL tuples"};
    Txn T(S);
    // ---- inserts (commit order: after every equal tuple), then deletes (every equal tuple)
    for (uint64_t i = 0; i < n_ins; ++i) {
        const keto_tuple& t = ins[i];
        const RowKey k = T.tuple_key(t, true);
        const uint32_t v = T.subject_value(t, true);
        const uint32_t r = T.row_or_new(k);
        std::vector<uint32_t>& e = T.edges(r);
        e.insert(e.begin() + T.upper(e, v), v);
    }
    for (uint64_t i = 0; i < n_del; ++i) {
        const keto_tuple& t = del[i];
        const RowKey k = T.tuple_key(t, false);
        const uint32_t v = T.subject_value(t, false);
        if (k.obj == ANY || k.rel == ANY || v == Txn::NONE) continue;     // nothing can match
        const int64_t r = T.row(k);
        if (r < 0) continue;
        std::vector<uint32_t>& e = T.edges((uint32_t)r);
        e.erase(std::remove(e.begin(), e.end(), v), e.end());
    }
    // ---- Subject.String() collisions (graph_utils.go:13-35 keys) this transaction creates: a new row
    // whose String() is another subject's (a subject id -- conservatively, any existing string -- or
    // another row's), or a new subject id equal to some row's String().  The typed subjects sharing
    // a key get one collision class as their visit id (an existing class is joined), and every row
    // holding one of them as an edge is walked edge by edge from now on (ROW_SEQ), as the build does
    // (snapshot.cpp, collision classes); its closure filter becomes all ones, and the re-closing in
    // device_apply carries that up to every row above it, so pruning stays exact.
    std::unordered_map<uint32_t, uint32_t> new_coll;     // edge value -> class (values not classed before)
    uint32_t classes = 0;
    {
        std::unordered_map<std::string, std::vector<uint32_t>> groups;
        auto group_of = [&](const std::string& ks) -> std::vector<uint32_t>& {
            auto it = groups.find(ks);
            if (it != groups.end()) return it->second;
            std::vector<uint32_t>& g = groups[ks];
            for (uint32_t r : S.rows_of_string(ks)) g.push_back(EDGE_SET | r);
            const int64_t sid = T.str(ks, false);       // existing or staged string
            if (sid >= 0) g.push_back((uint32_t)sid);
            return g;
        };
        for (uint32_t i = 0; i < T.new_keys.size(); ++i) {
            const uint32_t r = (uint32_t)S.row_key.size() + i;
            group_of(key_string(S, T, T.key(r))).push_back(EDGE_SET | r);
        }
        for (uint64_t i = 0; i < n_ins; ++i) {
            const keto_tuple& t = ins[i];
            if (t.subject_kind) continue;
            const std::string_view sid = sv(t.subject_id);
            if (sid.find(':') == std::string_view::npos || sid.find('#') == std::string_view::npos) continue;
            group_of(std::string(sid));                  // holds the id itself (staged string)
        }
        for (auto& kv : groups) {
            std::vector<uint32_t>& g = kv.second;
            std::sort(g.begin(), g.end());
            g.erase(std::unique(g.begin(), g.end()), g.end());
            if (g.size() < 2) continue;
            uint32_t c = NO_UNIT;
            for (uint32_t v : g) {
                auto it = S.coll.find(v);
                if (it != S.coll.end()) c = it->second;
            }
            if (c == NO_UNIT) c = VID_CLASS | (S.n_coll_keys + classes++);
            for (uint32_t v : g)
                if (!S.coll.count(v)) new_coll[v] = c;
        }
    }
    if (!new_coll.empty()) {
        // the rows holding a newly classed subject as an edge (rows already ROW_SEQ look classes up as
        // they walk): a parallel scan of every row's current edges
        const uint32_t R = S.n_rows();
        std::vector<uint8_t> hit(R, 0);
        // a transaction classes a handful of values: a branch-free compare against each of them per
        // edge (many values: a 64-bit prefilter before the hash lookup).  The whole scan is one pass
        // over the edge array: 15-24 ms of the write at 15.6M tuples on 8 threads
        // (profiles/r04_apply_latency_cpu.log), linear in the tuples
        std::vector<uint32_t> vals;
        for (auto& kv : new_coll) vals.push_back(kv.first);
        uint64_t mask = 0;
        for (uint32_t v : vals) mask |= 1ull << ((v * 0x9E3779B1u) >> 26);
        auto holds = [&](const uint32_t* e, uint64_t n) {
            if (vals.size() <= 8) {
                uint32_t v8[8];
                for (int k = 0; k < 8; ++k) v8[k] = vals[(size_t)k < vals.size() ? k : 0];
                for (uint64_t i = 0; i < n; ++i) {
                    bool any = false;
                    for (int k = 0; k < 8; ++k) any |= e[i] == v8[k];
                    if (any) return true;
                }
                return false;
            }
            for (uint64_t i = 0; i < n; ++i)
                if (((mask >> ((e[i] * 0x9E3779B1u) >> 26)) & 1u) && new_coll.count(e[i])) return true;
            return false;
        };
        // one streaming pass over the base edge array (no per-row lookups); a match is mapped to its
        // row by binary search, and rows a write overrode are checked on their current edges
        const unsigned th = S.edges.size() >= par_min() ? build_threads() : 1u;
        std::vector<std::vector<uint64_t>> found(std::max(1u, th));
        par_chunks(S.edges.size(), th, 1 << 20, [&](uint64_t b, uint64_t e, unsigned t) {
            for (uint64_t i = b; i < e;) {
                const uint64_t n = std::min<uint64_t>(e - i, 256);
                if (holds(S.edges.data() + i, n))
                    for (uint64_t x = i; x < i + n; ++x)
                        if (holds(S.edges.data() + x, 1)) found[t].push_back(x);
                i += n;
            }
        });
        const uint32_t NB = S.n_base_rows;
        for (auto& f : found)
            for (uint64_t x : f) {
                uint32_t lo = 0, hi = NB;                    // the last base row starting at or before x
                while (hi - lo > 1) {
                    const uint32_t m = lo + (hi - lo) / 2;
                    if (S.row_begin(m) <= x) lo = m;
                    else hi = m;
                }
                if (lo < R && !S.row_over.count(lo) && !(S.row_flags(lo) & ROW_SEQ)) hit[lo] = 1;
            }
        for (auto& kv : S.row_over)
            if (kv.first < R && !(S.row_flags(kv.first) & ROW_SEQ) && holds(kv.second.data(), kv.second.size()))
                hit[kv.first] = 1;
        for (auto& kv : T.rows)
            if (kv.first < R) hit[kv.first] = 0;         // staged rows: checked below
        for (uint32_t r = 0; r < R; ++r)
            if (hit[r]) T.edges(r);                      // re-imaged with the new flag (poisoned: rebuild)
    }
    // ---- wildcard rows: every new one, and every one whose query returns a row this transaction
    // staged, is materialized again from the staged edges
    std::vector<uint32_t> new_wild;
    for (uint32_t i = 0; i < T.new_keys.size(); ++i)
        if (wild_key(T.new_keys[i])) new_wild.push_back((uint32_t)S.row_key.size() + i);
    if (!S.wild_rows.empty() || !new_wild.empty()) {
        std::vector<uint32_t> changed;
        for (uint32_t r : T.order)
            if (!wild_key(T.key(r))) changed.push_back(r);
        auto redo = [&](uint32_t w, bool always) {
            const RowKey& wk = T.key(w);
            bool hit = always;
            for (uint32_t r = 0; !hit && r < changed.size(); ++r) hit = key_matches(wk, T.key(changed[r]));
            if (!hit) return;
            if (w < S.rows.size() && S.row_pp[w] != NO_PAGE)
                throw Error{KETO_E_REBUILD, "a write changes a wildcard row that matches a poisoned row"};
            std::vector<uint32_t> e = T.materialize(wk);
            auto it = T.rows.find(w);
            if (it == T.rows.end()) {
                T.order.push_back(w);
                T.rows.emplace(w, std::move(e));
            } else {
                it->second = std::move(e);
            }
        };
        for (uint32_t w : S.wild_rows) redo(w, false);
        for (uint32_t w : new_wild) redo(w, true);
    }
    // ---- what the delta path cannot express: the caller rebuilds
    for (uint32_t r : T.order)
        if (r < S.rows.size() && S.row_pp[r] != NO_PAGE) throw Error{KETO_E_REBUILD, "a write touches a poisoned row"};
    // ---- commit
    Grown grown(S, T.new_keys.size(), T.new_keys.size() + T.order.size() + T.new_targets.size());
    if (commit) commit();
    grown.swap_in(S);
    const uint32_t R0 = S.n_rows();
    if (!new_coll.empty()) {
        for (auto& kv : new_coll) S.coll[kv.first] = kv.second;
        S.n_coll_keys += classes;
        S.coll_dirty = true;
    }
    for (auto& x : T.new_strs) {
        S.added_str.emplace(x, (uint32_t)S.strs.size());
        S.strs.push_back(std::move(x));
    }
    for (auto& k : T.new_keys) {
        S.row_of.emplace(k, (uint32_t)S.row_key.size());
        S.row_key.push_back(k);
        S.rows.push_back(RowRec{0, 0, 0, 0});
        S.row_pp.push_back(NO_PAGE);
        S.unit_of_row.push_back(NO_UNIT);
        S.is_root.push_back(1);
        S.row_cb.push_back(0);
    }
    S.dirty.clear();
    S.needs_cb.clear();
    for (uint32_t w : new_wild) S.wild_rows.push_back(w);
    S.n_wild_rows += (uint32_t)new_wild.size();
    for (uint32_t r : T.order) {
        std::vector<uint32_t>& e = T.rows[r];
        const bool wild = wild_key(S.row_key[r]);          // materialized: walked edge by edge
        bool seq = wild;
        for (uint32_t v : e)
            if (!seq && S.coll.count(v)) { seq = true; break; }
        // base rows keep their build edge range (row_edges of the row before reads it as its end)
        RowRec rec{r < R0 ? S.rows[r].edge_lo : 0u,
                   (r < R0 ? (S.rows[r].hi_flags & 0xFFu) : 0u) | ((seq ? ROW_SEQ : 0u) << 8), 0, 0};
        if (seq) {
            rec.n_sets = (uint32_t)e.size();
        } else {
            uint32_t ns = 0;
            while (ns < e.size() && (e[ns] & EDGE_SET)) ++ns;
            rec.n_sets = ns;
            rec.n_ids = (uint32_t)(e.size() - ns);
        }
        if (S.row_flags(r) & ROW_SEQ) S.n_seq_rows -= 1;
        if (seq) S.n_seq_rows += 1;
        // the place its content had before this write (base rows: their build layout)
        if (S.dev && !S.row_place.count(r) && r < R0 && S.unit_of_row[r] != NO_UNIT) {
            const auto old = S.row_edges(r);
            S.row_place[r] = Snapshot::RowPlace{S.unit_of_row[r], S.row_hlog2(r), (old.second + 3) & ~3ull,
                                                S.row_cb[r] != 0};
        }
        S.rows[r] = rec;
        if (!wild) {                                        // a wildcard row's edges are other rows' tuples
            S.n_tuples += e.size();
            S.n_tuples -= r < R0 ? S.row_edges(r).second : 0;
        }
        S.row_over[r] = std::move(e);
        S.dirty.push_back(r);
    }
    for (uint32_t i = 0; i < T.new_keys.size(); ++i) {            // new rows only subject sets point at
        const uint32_t r = R0 + i;
        if (S.row_over.count(r)) continue;
        S.row_over[r] = {};
        S.dirty.push_back(r);
    }
    for (uint32_t x : T.new_targets)
        if (S.is_root[x]) {
            S.is_root[x] = 0;
            if (!S.row_cb[x]) S.needs_cb.push_back(x);
        }
    std::sort(S.needs_cb.begin(), S.needs_cb.end());
    S.needs_cb.erase(std::unique(S.needs_cb.begin(), S.needs_cb.end()), S.needs_cb.end());
    S.version += 1;
    if (!S.dev) {                             // host-only: a later upload lays everything out afresh
        const auto t0 = std::chrono::steady_clock::now();
        compute_layout(S);
        if (getenv("KETO_APPLY_TRACE"))
            fprintf(stderr, "[apply] host-only layout %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
}

}  // namespace keto
