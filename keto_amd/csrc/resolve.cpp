// Request resolution: names -> snapshot ids, the role whereQuery plays for every SQL page query of
// the reference engines (internal/persistence/sql/relationtuples.go:178-198).  A check request
// (namespace, object, relation, subject) becomes {top-level row handle, target, flags, depth}.
//
// The snapshot's strings have byte-order ids and its real rows are sorted, so both could be found
// by binary search; at 10^8 strings that is ~27 dependent cache misses per lookup, three lookups
// and a row search per request.  Instead two flat open-addressing tables (linear probing, load
// <= 3/4, huge pages) index the build's strings and real rows.  Their 16-B slots hold what verifies a
// hit -- a string's length and first 11 bytes, a row's whole (namespace, object, relation) key -- so
// the common short identifier and every row are matched inside the slot; only a longer string reads
// its bytes from strs.  The bulk resolver is a software pipeline over groups of requests: each step
// runs five stages on five different groups, and every stage prefetches what the next stage of its
// group reads, one step (a whole group's work) ahead:
//   stage 0  the request's strings (prefetched the step before) -> hashes; prefetch the string slots
//   stage 1  string slots -> ids (long strings: prefetch their bytes)
//   stage 2  verify long strings; the row key's hash; prefetch the row slot
//   stage 3  row slot -> row; prefetch its handle
//   stage 4  the device-form request
// so a request costs ~6 independent misses (two request strings, two string slots, the row slot,
// the handle) that overlap across the groups in flight.
#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

namespace {

using StrSlot = Snapshot::StrSlot;
using RowSlot = Snapshot::RowSlot;
constexpr uint32_t INLINE = sizeof(StrSlot::b);   // leading bytes kept in a string slot

inline std::string_view sv(const keto_str& s) { return std::string_view(s.p ? s.p : "", s.n); }

inline uint64_t row_hash(int64_t ns, uint32_t obj, uint32_t rel) {
    return mix64((uint64_t)ns * 0x9E3779B97F4A7C15ull ^ mix64(((uint64_t)obj << 32) | rel));
}

inline uint64_t table_cap(uint64_t n) {
    uint64_t cap = 16;
    while (cap < n + n / 3 + 1) cap <<= 1;                 // load <= 3/4
    return cap;
}

// does slot x hold string s?  exact for strings of up to INLINE bytes; longer ones compare the
// leading bytes here and the rest in strs
inline bool str_slot_eq(const Snapshot& S, const StrSlot& x, std::string_view s) {
    const uint32_t n = (uint32_t)std::min<size_t>(s.size(), 255);
    if (x.n != n || std::memcmp(x.b, s.data(), std::min<size_t>(s.size(), INLINE)) != 0) return false;
    return s.size() <= INLINE || std::string_view(S.strs[x.id1 - 1]) == s;
}

int64_t find_str(const Snapshot& S, uint64_t h, std::string_view s) {
    const StrSlot* t = static_cast<const StrSlot*>(S.str_idx.p);
    if (!t) return -1;
    for (uint64_t j = h & S.str_mask;; j = (j + 1) & S.str_mask) {
        if (!t[j].id1) return -1;
        if (str_slot_eq(S, t[j], s)) return t[j].id1 - 1;
    }
}

int64_t find_row(const Snapshot& S, uint64_t h, int32_t ns, uint32_t obj, uint32_t rel) {
    const RowSlot* t = static_cast<const RowSlot*>(S.row_idx.p);
    if (!t) return -1;
    for (uint64_t j = h & S.row_mask;; j = (j + 1) & S.row_mask) {
        const RowSlot& x = t[j];
        if (!x.row1) return -1;
        if (x.ns == ns && x.obj == obj && x.rel == rel) return x.row1 - 1;
    }
}

inline void prefetch(const void* p) { __builtin_prefetch(p, 0, 3); }

}  // namespace

Snapshot::HugeBuf::~HugeBuf() {
    if (p) munmap(p, bytes);
}

void Snapshot::HugeBuf::alloc(uint64_t n) {
    if (p) munmap(p, bytes);
    p = nullptr;
    bytes = 0;
    void* m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    madvise(m, n, MADV_HUGEPAGE);                          // advisory: 4 KB pages still work
    p = m;
    bytes = n;
}

void Snapshot::ensure_index() const {
    std::call_once(idx_once, [this] {
        const unsigned th = std::max<uint64_t>(n_sorted_strs, n_real_rows) >= par_min() ? build_threads() : 1u;
        {
            const uint64_t cap = table_cap(n_sorted_strs);
            str_idx.alloc(cap * sizeof(StrSlot));
            str_mask = cap - 1;
            StrSlot* t = static_cast<StrSlot*>(str_idx.p);
            par_chunks(n_sorted_strs, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
                for (uint64_t id = b; id < e; ++id) {
                    const std::string_view s = strs[id];
                    for (uint64_t j = hash_bytes(s) & str_mask;; j = (j + 1) & str_mask) {
                        uint32_t zero = 0;   // claim the slot by its id word; nothing reads the table yet
                        if (__atomic_compare_exchange_n(&t[j].id1, &zero, (uint32_t)id + 1, false, __ATOMIC_RELAXED,
                                                        __ATOMIC_RELAXED)) {
                            t[j].n = (uint8_t)std::min<size_t>(s.size(), 255);
                            std::memcpy(t[j].b, s.data(), std::min<size_t>(s.size(), INLINE));
                            break;
                        }
                    }
                }
            });
        }
        {
            const uint64_t cap = table_cap(n_real_rows);
            row_idx.alloc(cap * sizeof(RowSlot));
            row_mask = cap - 1;
            RowSlot* t = static_cast<RowSlot*>(row_idx.p);
            par_chunks(n_real_rows, th, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
                for (uint64_t r = b; r < e; ++r) {
                    const RowKey& k = row_key[r];
                    for (uint64_t j = row_hash(k.ns, k.obj, k.rel) & row_mask;; j = (j + 1) & row_mask) {
                        uint32_t zero = 0;
                        if (__atomic_compare_exchange_n(&t[j].row1, &zero, (uint32_t)r + 1, false, __ATOMIC_RELAXED,
                                                        __ATOMIC_RELAXED)) {
                            t[j].ns = (int32_t)k.ns;
                            t[j].obj = k.obj;
                            t[j].rel = k.rel;
                            break;
                        }
                    }
                }
            });
        }
    });
}

int Snapshot::ns_index(std::string_view name) const {
    if (ns_names.size() <= 8) {                          // the usual handful: compare in place
        for (uint32_t i = 0; i < ns_names.size(); ++i)
            if (ns_names[i].size() == name.size() && std::memcmp(ns_names[i].data(), name.data(), name.size()) == 0)
                return (int)i;
        return -1;
    }
    auto it = ns_view.find(name);
    return it == ns_view.end() ? -1 : it->second;
}

int64_t Snapshot::lookup_str(std::string_view s) const {
    ensure_index();
    const int64_t id = find_str(*this, hash_bytes(s), s);
    if (id >= 0 || added_str.empty()) return id;
    auto f = added_str.find(std::string(s));
    return f == added_str.end() ? -1 : (int64_t)f->second;
}

int64_t Snapshot::real_row(const RowKey& k) const {
    ensure_index();
    if (k.ns < INT32_MIN || k.ns > INT32_MAX) return -1;
    return find_row(*this, row_hash(k.ns, k.obj, k.rel), (int32_t)k.ns, k.obj, k.rel);
}

int64_t Snapshot::resolve_query(std::string_view ns, std::string_view obj, std::string_view rel,
                                RowKey* key_out) const {
    RowKey k;
    if (ns.empty()) {
        k.ns = ANY_NS;
    } else {
        const int c = ns_index(ns);
        if (c < 0) return -2;                                                    // ErrNotFound
        k.ns = ns_ids[c];
    }
    if (obj.empty()) k.obj = ANY;
    else {
        const int64_t o = lookup_str(obj);
        if (o < 0) return -1;          // no row can match an unknown string
        k.obj = (uint32_t)o;
    }
    if (rel.empty()) k.rel = ANY;
    else {
        const int64_t r = lookup_str(rel);
        if (r < 0) return -1;
        k.rel = (uint32_t)r;
    }
    if (key_out) *key_out = k;
    if (k.ns != ANY_NS && k.obj != ANY && k.rel != ANY) {
        const int64_t r = real_row(k);
        if (r >= 0) return r;
    }
    auto it = row_of.find(k);
    if (it != row_of.end()) return it->second;
    if (k.ns == ANY_NS || k.obj == ANY || k.rel == ANY) return -3;
    return -1;
}

std::vector<uint32_t> Snapshot::rows_of_string(std::string_view key) const {
    std::vector<uint32_t> out;
    // the snapshot's subject sets: rows of configured namespaces, and wildcard rows (namespace ANY
    // prints as ""); a field that is "" is the empty string's id or, in a wildcard row, ANY
    auto field_ids = [&](std::string_view f, std::vector<uint32_t>& ids) {
        ids.clear();
        if (f.empty()) ids.push_back(ANY);
        const int64_t x = lookup_str(f);
        if (x >= 0) ids.push_back((uint32_t)x);
    };
    std::vector<uint32_t> objs, rels;
    for (size_t p = key.find(':'); p != std::string_view::npos; p = key.find(':', p + 1)) {
        const std::string_view ns = key.substr(0, p), rest = key.substr(p + 1);
        std::vector<int64_t> nss;
        const int c = ns_index(ns);
        if (c >= 0) nss.push_back(ns_ids[c]);
        if (ns.empty()) nss.push_back(ANY_NS);
        if (nss.empty()) continue;
        for (size_t q = rest.find('#'); q != std::string_view::npos; q = rest.find('#', q + 1)) {
            field_ids(rest.substr(0, q), objs);
            field_ids(rest.substr(q + 1), rels);
            for (int64_t n : nss)
                for (uint32_t o : objs)
                    for (uint32_t r : rels) {
                        const RowKey k{n, o, r};
                        int64_t row = n != ANY_NS && o != ANY && r != ANY ? real_row(k) : -1;
                        if (row < 0) {
                            auto it = row_of.find(k);
                            if (it != row_of.end()) row = it->second;
                        }
                        if (row >= 0) out.push_back((uint32_t)row);
                    }
        }
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

uint32_t Snapshot::vid_of_key(std::string_view key) const {
    const std::vector<uint32_t> rows = rows_of_string(key);
    return rows.empty() ? 0xFFFFFFF0u : vid_of_row(rows[0]);   // 0xFFFFFFF0: no snapshot subject
}

namespace {

[[noreturn]] void foreign_row(const Snapshot& S, uint32_t row) {
    throw Error{KETO_E_INVALID, "the request's row is a root row owned by part " +
                                    std::to_string(S.root_owner(row, S.n_parts)) + " (keto_row_owner)"};
}

// one request, any form (wildcards, subject sets, unknown namespaces)
keto_check_ids resolve_general(const Snapshot& S, const keto_check_req& q, uint64_t i, uint8_t& status,
                               std::vector<WildReq>& wild, bool by_row) {
    keto_check_ids r{KETO_NO_ROW, KETO_NO_TARGET, 0, q.max_depth};
    status = KETO_CHECK_OK;
    RowKey wkey;
    const int64_t row = S.resolve_query(sv(q.namespace_), sv(q.object), sv(q.relation), &wkey);
    if (row == -2) status = KETO_CHECK_UNKNOWN_NAMESPACE;
    else if (row == -3) wild.push_back(WildReq{(uint32_t)i, wkey});
    else if (row >= 0) {
        if (by_row) {
            r.row = (uint32_t)row;
        } else {
            if (!S.present((uint32_t)row)) foreign_row(S, (uint32_t)row);
            r.row = S.handle((uint32_t)row);
        }
    }
    if (q.subject.kind == 0) {
        const int64_t sid = S.lookup_str(sv(q.subject.id));
        if (sid >= 0) r.target = (uint32_t)sid;
    } else {
        const int64_t t = S.resolve_query(sv(q.subject.set_namespace), sv(q.subject.set_object), sv(q.subject.set_relation));
        if (t >= 0) {
            r.target = by_row ? (uint32_t)t : S.handle((uint32_t)t);
            r.flags = 1;
        }
    }
    return r;
}

constexpr int DEPTH = 5;         // groups in flight (one per stage)

struct Lane {
    uint64_t i;                  // request index
    int32_t ns;                  // config namespace id (if ns_ok)
    bool ns_ok;
    std::string_view f[3];       // object, relation, subject id
    uint64_t h[3];
    int64_t id[3];               // string ids (-1 absent)
    uint64_t hrow;
    int64_t row;                 // -1: none
    bool keyed;                  // namespace, object and relation all known: a row key exists
};
template <int G>                 // requests per group
struct Group {
    Lane l[G];
    int n = 0;
};

template <int G>
void resolve_group_pipeline(const Snapshot& S, const keto_check_req* q, uint64_t b, uint64_t e, keto_check_ids* out,
                            uint8_t* status, std::vector<WildReq>& wild, bool by_row) {
    const StrSlot* ST = static_cast<const StrSlot*>(S.str_idx.p);
    const RowSlot* RT = static_cast<const RowSlot*>(S.row_idx.p);
    const uint64_t n_groups = (e - b + G - 1) / G;
    Group<G> ring[DEPTH];
    auto prefetch_strings = [&](uint64_t g) {            // the caller's request strings of group g
        if (g >= n_groups) return;
        const uint64_t g0 = b + g * G, g1 = std::min(e, g0 + G);
        for (uint64_t i = g0; i < g1; ++i) {
            prefetch(q[i].object.p);
            prefetch(q[i].subject.id.p);
        }
    };
    // stage 0: classify (the common form ns:obj#rel@id with every field set is pipelined; the rest
    // goes through resolve_general at once), hash, prefetch the string slots
    auto stage0 = [&](uint64_t g) {
        Group<G>& G_ = ring[g % DEPTH];
        G_.n = 0;
        const uint64_t g0 = b + g * G, g1 = std::min(e, g0 + G);
        for (uint64_t i = g0; i < g1; ++i) {
            const keto_check_req& x = q[i];
            if (!x.namespace_.n || !x.object.n || !x.relation.n || x.subject.kind != 0) {
                out[i] = resolve_general(S, x, i, status[i], wild, by_row);
                continue;
            }
            Lane& l = G_.l[G_.n++];
            l.i = i;
            const int c = S.ns_index(sv(x.namespace_));
            l.ns_ok = c >= 0;
            l.ns = l.ns_ok ? S.ns_ids[c] : 0;
            l.f[0] = sv(x.object);
            l.f[1] = sv(x.relation);
            l.f[2] = sv(x.subject.id);
            for (int k = 0; k < 3; ++k) {
                l.h[k] = hash_bytes(l.f[k]);
                prefetch(ST + (l.h[k] & S.str_mask));
            }
        }
    };
    // stage 1: the string slots -> ids (a long string's bytes are prefetched for stage 2)
    auto stage1 = [&](uint64_t g) {
        Group<G>& G_ = ring[g % DEPTH];
        for (int a = 0; a < G_.n; ++a) {
            Lane& l = G_.l[a];
            for (int k = 0; k < 3; ++k) {
                const std::string_view s = l.f[k];
                const uint32_t n = (uint32_t)std::min<size_t>(s.size(), 255);
                int64_t id = -1;
                for (uint64_t j = l.h[k] & S.str_mask;; j = (j + 1) & S.str_mask) {
                    const StrSlot& x = ST[j];
                    if (!x.id1) break;
                    if (x.n == n && std::memcmp(x.b, s.data(), std::min<size_t>(s.size(), INLINE)) == 0) {
                        id = x.id1 - 1;                      // exact for short strings, verified in stage 2 else
                        if (s.size() > INLINE) prefetch(&S.strs[id]);
                        break;
                    }
                }
                l.id[k] = id;
            }
        }
    };
    // stage 2: verify long strings (a mismatch re-probes), strings added by writes, the row key
    auto stage2 = [&](uint64_t g) {
        Group<G>& G_ = ring[g % DEPTH];
        for (int a = 0; a < G_.n; ++a) {
            Lane& l = G_.l[a];
            for (int k = 0; k < 3; ++k) {
                const std::string_view s = l.f[k];
                if (l.id[k] >= 0 && s.size() > INLINE && std::string_view(S.strs[l.id[k]]) != s)
                    l.id[k] = find_str(S, l.h[k], s);
                if (l.id[k] < 0 && !S.added_str.empty()) l.id[k] = S.lookup_str(s);
            }
            l.keyed = l.ns_ok && l.id[0] >= 0 && l.id[1] >= 0;
            if (l.keyed) {
                l.hrow = row_hash(l.ns, (uint32_t)l.id[0], (uint32_t)l.id[1]);
                prefetch(RT + (l.hrow & S.row_mask));
            }
        }
    };
    // stage 3: the row slot -> row (empty rows and rows added by writes: row_of), prefetch its handle
    auto stage3 = [&](uint64_t g) {
        Group<G>& G_ = ring[g % DEPTH];
        for (int a = 0; a < G_.n; ++a) {
            Lane& l = G_.l[a];
            l.row = -1;
            if (!l.keyed) continue;
            l.row = find_row(S, l.hrow, l.ns, (uint32_t)l.id[0], (uint32_t)l.id[1]);
            if (l.row < 0 && !S.row_of.empty()) {
                auto it = S.row_of.find(RowKey{l.ns, (uint32_t)l.id[0], (uint32_t)l.id[1]});
                if (it != S.row_of.end()) l.row = it->second;
            }
            if (l.row >= 0) prefetch(&S.unit_of_row[l.row]);
        }
    };
    // stage 4: the device-form request
    auto stage4 = [&](uint64_t g) {
        Group<G>& G_ = ring[g % DEPTH];
        for (int a = 0; a < G_.n; ++a) {
            const Lane& l = G_.l[a];
            keto_check_ids r{KETO_NO_ROW, KETO_NO_TARGET, 0, q[l.i].max_depth};
            status[l.i] = l.ns_ok ? KETO_CHECK_OK : KETO_CHECK_UNKNOWN_NAMESPACE;
            if (l.row >= 0) {
                if (by_row) {
                    r.row = (uint32_t)l.row;
                } else {
                    if (!S.present((uint32_t)l.row)) foreign_row(S, (uint32_t)l.row);
                    r.row = S.handle((uint32_t)l.row);
                }
            }
            if (l.id[2] >= 0) r.target = (uint32_t)l.id[2];
            out[l.i] = r;
        }
    };
    prefetch_strings(0);
    for (uint64_t t = 0; t < n_groups + DEPTH - 1; ++t) {
        prefetch_strings(t + 1);
        if (t >= 4 && t - 4 < n_groups) stage4(t - 4);
        if (t >= 3 && t - 3 < n_groups) stage3(t - 3);
        if (t >= 2 && t - 2 < n_groups) stage2(t - 2);
        if (t >= 1 && t - 1 < n_groups) stage1(t - 1);
        if (t < n_groups) stage0(t);
    }
}

}  // namespace

void resolve_checks(const Snapshot& S, const keto_check_req* q, uint64_t b, uint64_t e, keto_check_ids* out,
                    uint8_t* status, std::vector<WildReq>& wild, bool by_row) {
    S.ensure_index();
    // KETO_RESOLVE_GROUP (tuning): requests per pipeline group, 8 / 16 / 32 (8: 96 M requests/s on 16
    // EPYC 9575F threads at 1B tuples, 16: 88 M, 32: 91 M; profiles/r03d_resolve.log)
    const char* v = getenv("KETO_RESOLVE_GROUP");
    const int group = v ? atoi(v) : 8;
    if (group == 8) resolve_group_pipeline<8>(S, q, b, e, out, status, wild, by_row);
    else if (group == 32) resolve_group_pipeline<32>(S, q, b, e, out, status, wild, by_row);
    else resolve_group_pipeline<16>(S, q, b, e, out, status, wild, by_row);
}

}  // namespace keto
