// Synthetic ACL graphs and request batches for bench.py and the large-size tests (tooling, not
// part of the engine).  Graphs come out already interned and in the reference ORDER BY, ready for
// keto_snapshot_from_csr; names are fixed-width lowercase hex ("d%08x", "f%08x", "g%08x",
// "u%08x"), so numeric id order equals byte order and no Subject.String() can collide.
//
// "power-law ACL" graph (BASELINE config #4):
//   namespaces docs(1) / folders(2) / groups(3); rows docs:d#view, folders:f#view, groups:g#member
//   docs:d#view    -> (folders:f#view) parent, f ~ power law over folders; 0-2 x (groups:g#member),
//                     g ~ power law; Pareto(1.8) direct user shares
//   folders:f#view -> (folders:p#view) parent (random recursive forest, p < f; 1/64 are roots);
//                     0-3 x (groups:g#member); Pareto(1.6) users
//   groups:g#member-> (groups:h#member) nested, h < g with p = 0.5, h > g (cycles) with p = 0.001;
//                     Pareto(1.3) users, capped at 2^21 (heavy-tailed group sizes)
//   users drawn with a power law (popular users are in many groups); total edges adjusted to
//   exactly `target_edges` by adding / removing direct user shares on documents.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

#include "../include/keto_mi355x.h"

namespace {

inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(splitmix(seed)) {}
    uint64_t next() { return s = splitmix(s); }
    double u01() { return ((next() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
};

// P(x < k) = (k/n)^(1/3): heavy preference for low indices
inline uint64_t skewed(Rng& r, uint64_t n, double power = 3.0) {
    uint64_t x = (uint64_t)(std::pow(r.u01(), power) * (double)n);
    return x >= n ? n - 1 : x;
}
inline uint64_t pareto(Rng& r, double xm, double a, uint64_t cap) {
    double v = xm / std::pow(r.u01(), 1.0 / a) - xm;   // starts at 0
    uint64_t k = (uint64_t)v;
    return k > cap ? cap : k;
}

template <class F>
void parallel_for(uint64_t n, int threads, F f) {
    if (threads < 1) threads = 1;
    std::atomic<uint64_t> next{0};
    const uint64_t chunk = 1 << 14;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&] {
            for (;;) {
                uint64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                uint64_t e = std::min(n, b + chunk);
                for (uint64_t i = b; i < e; ++i) f(i);
            }
        });
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

typedef struct {
    uint64_t n_docs, n_folders, n_groups, n_users, target_edges, seed;
} synth_params;

typedef struct {
    uint32_t n_rows;
    int32_t* row_ns;
    uint32_t* row_obj;
    uint32_t* row_rel;
    uint64_t* row_ptr;
    uint32_t* edges;
    uint64_t n_edges;
    uint64_t n_set_edges;
} synth_graph;

enum { REL_MEMBER = 0, REL_VIEW = 1 };

static void row_degrees(const synth_params* p, uint64_t r, uint32_t& ns, uint32_t& ni) {
    const uint64_t F0 = p->n_docs, G0 = p->n_docs + p->n_folders;
    Rng g(p->seed * 0x100000001B3ull ^ (r * 0x9E3779B97F4A7C15ull));
    if (r < F0) {
        uint64_t u = g.next() % 5;
        ns = 1 + (u < 2 ? 0 : u < 4 ? 1 : 2);
        ni = (uint32_t)pareto(g, 1.0, 1.8, 64);
    } else if (r < G0) {
        uint64_t f = r - F0;
        bool root = f < p->n_folders / 64;
        ns = (root ? 0 : 1) + (uint32_t)(g.next() % 4);
        ni = (uint32_t)pareto(g, 3.0, 1.6, 10000);
    } else {
        uint64_t x = g.next() % 1000;
        ns = x < 500 ? 1 : 0;
        if (x == 999) ns++;
        ni = (uint32_t)pareto(g, 16.0, 1.3, 1u << 21);
    }
}

int synth_generate(const synth_params* p, int threads, synth_graph* out) {
    const uint64_t R = p->n_docs + p->n_folders + p->n_groups;
    if (R >= 0x7FFFFFFFull || p->n_users >= 0x7FFFFFFFull) return -1;
    const uint64_t F0 = p->n_docs, G0 = p->n_docs + p->n_folders;
    std::vector<uint32_t> nset(R), nid(R);
    parallel_for(R, threads, [&](uint64_t r) { row_degrees(p, r, nset[r], nid[r]); });
    uint64_t tot = 0;
    for (uint64_t r = 0; r < R; ++r) tot += nset[r] + nid[r];
    // hit target_edges exactly by adjusting document shares
    if (p->target_edges) {
        int64_t diff = (int64_t)p->target_edges - (int64_t)tot;
        uint64_t r = 0, guard = 0;
        while (diff != 0 && p->n_docs && guard < 64 * p->n_docs) {
            if (diff > 0) { nid[r]++; diff--; }
            else if (nid[r] > 0) { nid[r]--; diff++; }
            r = (r + 7919) % p->n_docs;
            ++guard;
        }
    }
    out->n_rows = (uint32_t)R;
    out->row_ns = (int32_t*)malloc(R * sizeof(int32_t));
    out->row_obj = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_rel = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_ptr = (uint64_t*)malloc((R + 1) * sizeof(uint64_t));
    uint64_t acc = 0, sets = 0;
    for (uint64_t r = 0; r < R; ++r) {
        out->row_ptr[r] = acc;
        acc += nset[r] + nid[r];
        sets += nset[r];
    }
    out->row_ptr[R] = acc;
    out->n_edges = acc;
    out->n_set_edges = sets;
    out->edges = (uint32_t*)malloc(std::max<uint64_t>(acc, 1) * sizeof(uint32_t));
    if (!out->row_ns || !out->row_obj || !out->row_rel || !out->row_ptr || !out->edges) return -2;
    parallel_for(R, threads, [&](uint64_t r) {
        if (r < F0) { out->row_ns[r] = 1; out->row_obj[r] = (uint32_t)r; out->row_rel[r] = REL_VIEW; }
        else if (r < G0) { out->row_ns[r] = 2; out->row_obj[r] = (uint32_t)(r - F0); out->row_rel[r] = REL_VIEW; }
        else { out->row_ns[r] = 3; out->row_obj[r] = (uint32_t)(r - G0); out->row_rel[r] = REL_MEMBER; }
        Rng g(p->seed * 0xC2B2AE3D27D4EB4Full ^ (r * 0xD6E8FEB86659FD93ull) ^ 0x5555);
        uint32_t* e = out->edges + out->row_ptr[r];
        uint32_t k = 0;
        const uint32_t ns = nset[r], ni = nid[r];
        if (r < F0) {
            e[k++] = 0x80000000u | (uint32_t)(F0 + skewed(g, p->n_folders));
            while (k < ns) e[k++] = 0x80000000u | (uint32_t)(G0 + skewed(g, p->n_groups));
        } else if (r < G0) {
            uint64_t f = r - F0;
            bool root = f < p->n_folders / 64;
            if (!root) e[k++] = 0x80000000u | (uint32_t)(F0 + g.next() % f);
            while (k < ns) e[k++] = 0x80000000u | (uint32_t)(G0 + skewed(g, p->n_groups));
        } else {
            uint64_t gi = r - G0;
            while (k < ns) {
                uint64_t h;
                if (k == 0 && gi > 0) h = g.next() % gi;                       // nested, acyclic
                else h = gi + 1 + g.next() % std::max<uint64_t>(1, p->n_groups - gi - 1);   // back-edge
                if (h >= p->n_groups) h = g.next() % p->n_groups;
                e[k++] = 0x80000000u | (uint32_t)(G0 + h);
            }
        }
        std::sort(e, e + ns);                     // subject sets by (namespace id, object, relation)
        for (uint32_t j = 0; j < ni; ++j) e[ns + j] = (uint32_t)skewed(g, p->n_users, 1.5);
        std::sort(e + ns, e + ns + ni);           // subject ids by bytes
    });
    return 0;
}

// "nested groups" graph (BASELINE config #3): groups:g#member only.  Groups form chains of
// `chain` groups (g -> g+1 inside a chain, so membership nests up to `chain` levels), with a
// 0.3-probability cross edge to a random later group and a 0.01-probability back-edge to an earlier
// group (cycles).  Users per group ~ Pareto(1.5); users drawn with a power law.
int synth_generate_nested(const synth_params* p, uint32_t chain, int threads, synth_graph* out) {
    const uint64_t R = p->n_groups;
    if (R >= 0x7FFFFFFFull || chain == 0) return -1;
    std::vector<uint32_t> nset(R), nid(R);
    parallel_for(R, threads, [&](uint64_t r) {
        Rng g(p->seed * 0x2545F4914F6CDD1Dull ^ (r * 0x9E3779B97F4A7C15ull));
        uint32_t k = (r % chain != chain - 1 && r + 1 < R) ? 1 : 0;
        if (g.u01() < 0.3) ++k;
        if (g.u01() < 0.01) ++k;
        nset[r] = k;
        nid[r] = (uint32_t)pareto(g, 2.0, 1.5, 1u << 16);
    });
    // hit target_edges exactly (when set) by spreading extra / fewer direct members over groups
    if (p->target_edges) {
        int64_t diff = (int64_t)p->target_edges;
        for (uint64_t r = 0; r < R; ++r) diff -= (int64_t)nset[r] + nid[r];
        const uint64_t stride = 0x9E3779B1ull % R | 1;   // odd: a permutation of the rows when R is 2^k
        for (uint64_t i = 0; diff != 0 && i < 64 * R; ++i) {
            const uint64_t r = (i * stride) % R;
            if (diff > 0) {
                ++nid[r];
                --diff;
            } else if (nid[r] > 0) {
                --nid[r];
                ++diff;
            }
        }
        if (diff != 0) return -3;
    }
    out->n_rows = (uint32_t)R;
    out->row_ns = (int32_t*)malloc(R * sizeof(int32_t));
    out->row_obj = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_rel = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_ptr = (uint64_t*)malloc((R + 1) * sizeof(uint64_t));
    uint64_t acc = 0, sets = 0;
    for (uint64_t r = 0; r < R; ++r) {
        out->row_ptr[r] = acc;
        acc += nset[r] + nid[r];
        sets += nset[r];
    }
    out->row_ptr[R] = acc;
    out->n_edges = acc;
    out->n_set_edges = sets;
    out->edges = (uint32_t*)malloc(std::max<uint64_t>(acc, 1) * sizeof(uint32_t));
    if (!out->row_ns || !out->row_obj || !out->row_rel || !out->row_ptr || !out->edges) return -2;
    parallel_for(R, threads, [&](uint64_t r) {
        out->row_ns[r] = 3;
        out->row_obj[r] = (uint32_t)r;
        out->row_rel[r] = REL_MEMBER;
        Rng g(p->seed * 0x2545F4914F6CDD1Dull ^ (r * 0x9E3779B97F4A7C15ull));
        const bool in_chain = r % chain != chain - 1 && r + 1 < R;
        const bool cross = g.u01() < 0.3;
        const bool back = g.u01() < 0.01;
        uint32_t* e = out->edges + out->row_ptr[r];
        uint32_t k = 0;
        Rng h(p->seed ^ (r * 0xD1B54A32D192ED03ull));
        if (in_chain) e[k++] = 0x80000000u | (uint32_t)(r + 1);
        if (cross) e[k++] = 0x80000000u | (uint32_t)(r + 1 + h.next() % std::max<uint64_t>(1, R - r - 1)) % (uint32_t)R;
        if (back) e[k++] = 0x80000000u | (uint32_t)(r ? h.next() % r : 0);
        std::sort(e, e + nset[r]);
        for (uint32_t j = 0; j < nid[r]; ++j) e[nset[r] + j] = (uint32_t)skewed(h, p->n_users, 1.5);
        std::sort(e + nset[r], e + nset[r] + nid[r]);
    });
    return 0;
}

// Requests groups:g#member@u for the nested graph: half a user of a group reached by walking
// 0..depth-1 nesting edges, half random users; request depth cycles through `depths`.
int synth_queries_nested(const synth_graph* g, const synth_params* p, uint64_t n, uint64_t seed,
                         const int32_t* depths, uint32_t n_depths, keto_check_ids* out, int threads) {
    parallel_for(n, threads, [&](uint64_t i) {
        Rng r(seed * 0xA24BAED4963EE407ull ^ (i * 0x9FB21C651E98DF25ull));
        uint32_t row = (uint32_t)(r.next() % g->n_rows);
        int32_t d = depths[i % n_depths];
        keto_check_ids q{row, 0, 0, d};
        if (r.next() & 1) {
            uint32_t cur = row;
            int hops = (int)(r.next() % (uint64_t)std::max(1, d));
            for (int h = 0; h < hops; ++h) {
                uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1], ns = 0;
                while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
                if (!ns) break;
                cur = g->edges[b + r.next() % ns] & 0x7FFFFFFFu;
            }
            uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1], ns = 0;
            while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
            q.target = e - b > ns ? g->edges[b + ns + r.next() % (e - b - ns)] : (uint32_t)(r.next() % p->n_users);
        } else {
            q.target = (uint32_t)(r.next() % p->n_users);
        }
        out[i] = q;
    });
    return 0;
}

// "Drive-like" graph (BASELINE config #2, SURVEY.md 8(d) exactly): namespaces files(1) /
// folders(2) / groups(3); relations member(0) < owner(1) < view(2) (byte order).
//   rows (in (namespace, object, relation) order): files:d#owner = 2d, files:d#view = 2d + 1,
//        folders:f#view = 2 n_files + f, groups:g#member = 2 n_files + n_folders + g
//   files:d#view    -> (files:d#owner)  [same object, another relation; ns 1 sorts first]
//                      (folders:p#view) [the file's folder, uniform over folders]
//   files:d#owner   -> 1 + Pareto(2.0) users (<= 16)
//   folders:f#view  -> (folders:parent#view) unless f is a tree root; 0/1/2 x (groups:g#member)
//                      (p = .6/.3/.1, popular groups preferred); Pareto(1.5) users (<= 1000)
//   groups:g#member -> users; group sizes Zipf(1.1) (size of the k-th group ~ C / k^1.1),
//                      scaled so the graph has exactly `target_edges` tuples
// The folders form a forest of complete 8-ary trees in heap order (folder j of a tree has parent
// (j - 1) / 8), at most 37,449 folders per tree, i.e. depth <= 6 (levels 0..5).
constexpr uint64_t DRIVE_TREE = 1 + 8 + 64 + 512 + 4096 + 32768;

static void drive_degrees(const synth_params* p, uint64_t r, uint32_t& ns, uint32_t& ni) {
    const uint64_t NF = p->n_docs, NO = p->n_folders;
    Rng g(p->seed * 0x9FB21C651E98DF25ull ^ (r * 0x9E3779B97F4A7C15ull));
    if (r < 2 * NF) {
        if (r & 1) { ns = 2; ni = 0; }                                   // files:d#view
        else { ns = 0; ni = 1 + (uint32_t)pareto(g, 1.0, 2.0, 15); }      // files:d#owner
    } else if (r < 2 * NF + NO) {
        const uint64_t f = r - 2 * NF;
        const uint64_t u = g.next() % 10;
        ns = (f % DRIVE_TREE == 0 ? 0u : 1u) + (u < 6 ? 0u : u < 9 ? 1u : 2u);
        ni = (uint32_t)pareto(g, 1.0, 1.5, 1000);
    } else {
        ns = 0;
        ni = 0;                                                           // groups: sized below
    }
}

int synth_generate_drive(const synth_params* p, int threads, synth_graph* out) {
    const uint64_t NF = p->n_docs, NO = p->n_folders, NG = p->n_groups;
    const uint64_t R = 2 * NF + NO + NG;
    if (R >= 0x7FFFFFFFull || p->n_users >= 0x7FFFFFFFull || !NF || !NO || !NG || !p->n_users) return -1;
    std::vector<uint32_t> nset(R), nid(R);
    parallel_for(R, threads, [&](uint64_t r) { drive_degrees(p, r, nset[r], nid[r]); });
    uint64_t fixed = 0;
    for (uint64_t r = 0; r < 2 * NF + NO; ++r) fixed += nset[r] + nid[r];
    const uint64_t target = p->target_edges ? p->target_edges : fixed + 16 * NG;
    if (target < fixed + NG) return -4;                                   // every group gets >= 1 member
    // Zipf(1.1) sizes for the remaining tuples, then +/-1 from the largest groups down to hit it exactly
    const uint64_t rem = target - fixed;
    double H = 0;
    for (uint64_t k = 1; k <= NG; ++k) H += std::pow((double)k, -1.1);
    uint64_t got = 0;
    for (uint64_t k = 0; k < NG; ++k) {
        uint64_t s = (uint64_t)((double)rem / H * std::pow((double)(k + 1), -1.1));
        if (s < 1) s = 1;
        if (s > 0xFFFFFFF0ull) s = 0xFFFFFFF0ull;
        nid[2 * NF + NO + k] = (uint32_t)s;
        got += s;
    }
    for (uint64_t k = 0; got != rem; k = (k + 1) % NG) {
        uint32_t& s = nid[2 * NF + NO + k];
        if (got < rem) { ++s; ++got; }
        else if (s > 1) { --s; --got; }
    }
    out->n_rows = (uint32_t)R;
    out->row_ns = (int32_t*)malloc(R * sizeof(int32_t));
    out->row_obj = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_rel = (uint32_t*)malloc(R * sizeof(uint32_t));
    out->row_ptr = (uint64_t*)malloc((R + 1) * sizeof(uint64_t));
    uint64_t acc = 0, sets = 0;
    for (uint64_t r = 0; r < R; ++r) {
        out->row_ptr[r] = acc;
        acc += nset[r] + nid[r];
        sets += nset[r];
    }
    out->row_ptr[R] = acc;
    out->n_edges = acc;
    out->n_set_edges = sets;
    out->edges = (uint32_t*)malloc(std::max<uint64_t>(acc, 1) * sizeof(uint32_t));
    if (!out->row_ns || !out->row_obj || !out->row_rel || !out->row_ptr || !out->edges) return -2;
    enum { D_MEMBER = 0, D_OWNER = 1, D_VIEW = 2 };
    const uint32_t FO = (uint32_t)(2 * NF), GR = (uint32_t)(2 * NF + NO);
    parallel_for(R, threads, [&](uint64_t r) {
        Rng g(p->seed * 0xC2B2AE3D27D4EB4Full ^ (r * 0xD6E8FEB86659FD93ull) ^ 0xD21Eull);
        uint32_t* e = out->edges + out->row_ptr[r];
        uint32_t k = 0;
        const uint32_t ns = nset[r], ni = nid[r];
        if (r < 2 * NF) {
            out->row_ns[r] = 1;
            out->row_obj[r] = (uint32_t)(r >> 1);
            out->row_rel[r] = (r & 1) ? D_VIEW : D_OWNER;
            if (r & 1) {
                e[k++] = 0x80000000u | (uint32_t)(r - 1);                        // (files:d#owner)
                e[k++] = 0x80000000u | (FO + (uint32_t)(g.next() % NO));         // (folders:p#view)
            }
        } else if (r < GR) {
            const uint64_t f = r - FO;
            out->row_ns[r] = 2;
            out->row_obj[r] = (uint32_t)f;
            out->row_rel[r] = D_VIEW;
            const uint64_t j = f % DRIVE_TREE;
            if (j) e[k++] = 0x80000000u | (FO + (uint32_t)(f - j + (j - 1) / 8));   // parent folder
            while (k < ns) e[k++] = 0x80000000u | (GR + (uint32_t)skewed(g, NG, 2.0));
        } else {
            out->row_ns[r] = 3;
            out->row_obj[r] = (uint32_t)(r - GR);
            out->row_rel[r] = D_MEMBER;
        }
        std::sort(e, e + ns);                     // subject sets by (namespace id, object, relation)
        for (uint32_t j = 0; j < ni; ++j) e[ns + j] = (uint32_t)skewed(g, p->n_users, 1.5);
        std::sort(e + ns, e + ns + ni);           // subject ids by bytes
    });
    return 0;
}

// Requests files:d#view@u for the Drive-like graph: d uniform; half a user of a row reached by a
// random walk of 1..depth-1 subject-set hops from files:d#view (real paths), half random users.
int synth_queries_drive(const synth_graph* g, const synth_params* p, uint64_t n, uint64_t seed, int32_t depth,
                        keto_check_ids* out, int threads) {
    parallel_for(n, threads, [&](uint64_t i) {
        Rng r(seed * 0xA24BAED4963EE407ull ^ (i * 0x9FB21C651E98DF25ull) ^ 0xD21Eull);
        const uint32_t row = (uint32_t)(2 * (r.next() % p->n_docs) + 1);
        keto_check_ids q{row, 0, 0, depth};
        q.target = (uint32_t)(r.next() % p->n_users);
        if (r.next() & 1) {
            uint32_t cur = row;
            const int hops = 1 + (int)(r.next() % (uint64_t)std::max(1, depth - 1));
            for (int h = 0; h < hops; ++h) {
                uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1], ns = 0;
                while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
                if (!ns) break;
                cur = g->edges[b + r.next() % ns] & 0x7FFFFFFFu;
            }
            uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1], ns = 0;
            while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
            if (e - b > ns) q.target = g->edges[b + ns + r.next() % (e - b - ns)];
        }
        out[i] = q;
    });
    return 0;
}

void synth_free(synth_graph* g) {
    free(g->row_ns);
    free(g->row_obj);
    free(g->row_rel);
    free(g->row_ptr);
    free(g->edges);
    memset(g, 0, sizeof(*g));
}

// Requests docs:d#view@u: half sampled along a real path (a random walk of 0..depth-1 subject-set
// hops from d, then one of the reached row's users), half uniformly random users.
int synth_queries(const synth_graph* g, const synth_params* p, uint64_t n, uint64_t seed, int32_t depth,
                  keto_check_ids* out, int threads) {
    parallel_for(n, threads, [&](uint64_t i) {
        Rng r(seed * 0xA24BAED4963EE407ull ^ (i * 0x9FB21C651E98DF25ull));
        uint32_t doc = (uint32_t)(r.next() % p->n_docs);
        keto_check_ids q{doc, 0, 0, depth};
        if (r.next() & 1) {
            uint32_t cur = doc;
            int hops = (int)(r.next() % (uint64_t)std::max(1, depth));
            for (int h = 0; h < hops; ++h) {
                uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1];
                uint64_t ns = 0;
                while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
                if (!ns) break;
                cur = g->edges[b + r.next() % ns] & 0x7FFFFFFFu;
            }
            uint64_t b = g->row_ptr[cur], e = g->row_ptr[cur + 1];
            uint64_t ns = 0;
            while (b + ns < e && (g->edges[b + ns] & 0x80000000u)) ++ns;
            if (e - b > ns) q.target = g->edges[b + ns + r.next() % (e - b - ns)];
            else q.target = (uint32_t)(r.next() % p->n_users);
        } else {
            q.target = (uint32_t)(r.next() % p->n_users);
        }
        out[i] = q;
    });
    return 0;
}

// ---- oracle table extraction (cpu_baseline sample): every row a depth-bounded check from the
// sample's rows can query (subject-set hops 0..depth-1), as tuples in ORDER BY order.
typedef struct {
    uint64_t n;
    int32_t* ns;
    uint32_t *obj, *rel;
    uint8_t* kind;
    uint32_t* sid;
    int32_t* sns;
    uint32_t *sobj, *srel, *key;
} synth_table;

int synth_extract(const synth_graph* g, const synth_params* p, const keto_check_ids* q, uint64_t nq, int32_t depth,
                  synth_table* out) {
    std::vector<uint8_t> seen(g->n_rows, 0);
    std::vector<uint32_t> frontier, next, rows;
    for (uint64_t i = 0; i < nq; ++i)
        if (q[i].row < g->n_rows && !seen[q[i].row]) { seen[q[i].row] = 1; frontier.push_back(q[i].row); }
    rows = frontier;
    for (int h = 1; h < depth && !frontier.empty(); ++h) {
        next.clear();
        for (uint32_t r : frontier)
            for (uint64_t k = g->row_ptr[r]; k < g->row_ptr[r + 1]; ++k) {
                uint32_t e = g->edges[k];
                if (!(e & 0x80000000u)) break;
                uint32_t t = e & 0x7FFFFFFFu;
                if (!seen[t]) { seen[t] = 1; next.push_back(t); rows.push_back(t); }
            }
        frontier.swap(next);
    }
    std::sort(rows.begin(), rows.end());
    uint64_t n = 0;
    for (uint32_t r : rows) n += g->row_ptr[r + 1] - g->row_ptr[r];
    out->n = n;
    out->ns = (int32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->obj = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->rel = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->kind = (uint8_t*)malloc(std::max<uint64_t>(n, 1));
    out->sid = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->sns = (int32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->sobj = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->srel = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    out->key = (uint32_t*)malloc(std::max<uint64_t>(n, 1) * 4);
    uint64_t k = 0;
    for (uint32_t r : rows) {
        for (uint64_t i = g->row_ptr[r]; i < g->row_ptr[r + 1]; ++i, ++k) {
            uint32_t e = g->edges[i];
            out->ns[k] = g->row_ns[r];
            out->obj[k] = g->row_obj[r];
            out->rel[k] = g->row_rel[r];
            if (e & 0x80000000u) {
                uint32_t t = e & 0x7FFFFFFFu;
                out->kind[k] = 1;
                out->sid[k] = 0;
                out->sns[k] = g->row_ns[t];
                out->sobj[k] = g->row_obj[t];
                out->srel[k] = g->row_rel[t];
                out->key[k] = (uint32_t)(p->n_users + t);
            } else {
                out->kind[k] = 0;
                out->sid[k] = e;
                out->sns[k] = 0;
                out->sobj[k] = out->srel[k] = 0;
                out->key[k] = e;
            }
        }
    }
    return 0;
}

// ---- the same graph as keto_relation_tuples rows (strings, commit order) for keto_snapshot_build:
// objects are "%08x" of their per-namespace id, relations rel_names[id] (byte order = id order),
// users "u%08x"; tuples come in a seeded pseudo-random commit order (i -> (a i + b) mod E).  Strings
// are shared: every keto_str points into one name table.
typedef struct {
    uint64_t n;
    keto_tuple* tuples;
    char* names;
    uint64_t obj_base, user_base, rel_base;   // offsets of the three tables in `names`
    uint32_t rel_off[8], rel_len[8];
} synth_strings;

static inline keto_str kstr(const char* p, uint32_t n) {
    keto_str s;
    s.p = p;
    s.n = n;
    return s;
}

static int emit_strings(const synth_graph* g, const synth_params* p, const char* const* rel_names, uint32_t n_rel,
                        uint64_t seed, int threads, bool with_tuples, synth_strings* out);

int synth_emit_strings(const synth_graph* g, const synth_params* p, const char* const* rel_names, uint32_t n_rel,
                       uint64_t seed, int threads, synth_strings* out) {
    return emit_strings(g, p, rel_names, n_rel, seed, threads, true, out);
}

// the name table alone (no tuple rows): objects "%08x", users "u%08x", relation names
int synth_emit_names(const synth_graph* g, const synth_params* p, const char* const* rel_names, uint32_t n_rel,
                     int threads, synth_strings* out) {
    return emit_strings(g, p, rel_names, n_rel, 0, threads, false, out);
}

// The graph in one string id space for keto_snapshot_from_csr (ids = byte-order ranks): object o ->
// obj_base + o, user u -> user_base + u, relation r -> rel_id[r] (the caller orders the three blocks).
// Writes the string table (keto_str into st->names), the rows' object / relation ids and the edges
// (subject ids moved into the user block; subject sets unchanged).
int synth_unify(const synth_graph* g, const synth_strings* st, uint64_t n_objs, uint64_t n_users, uint32_t obj_base,
                uint32_t user_base, const uint32_t* rel_id, uint32_t n_rel, keto_str* strs, uint32_t* row_obj,
                uint32_t* row_rel, uint32_t* edges, int threads) {
    parallel_for(n_objs, threads, [&](uint64_t i) { strs[obj_base + i] = kstr(st->names + st->obj_base + i * 8, 8); });
    parallel_for(n_users, threads, [&](uint64_t i) { strs[user_base + i] = kstr(st->names + st->user_base + i * 9, 9); });
    for (uint32_t r = 0; r < n_rel; ++r) strs[rel_id[r]] = kstr(st->names + st->rel_base + st->rel_off[r], st->rel_len[r]);
    parallel_for(g->n_rows, threads, [&](uint64_t r) {
        row_obj[r] = obj_base + g->row_obj[r];
        row_rel[r] = rel_id[g->row_rel[r]];
    });
    parallel_for((g->n_edges + 65535) / 65536, threads, [&](uint64_t c) {
        const uint64_t b = c * 65536, e = std::min<uint64_t>(g->n_edges, b + 65536);
        for (uint64_t i = b; i < e; ++i) {
            const uint32_t x = g->edges[i];
            edges[i] = (x & 0x80000000u) ? x : user_base + x;
        }
    });
    return 0;
}

static int emit_strings(const synth_graph* g, const synth_params* p, const char* const* rel_names, uint32_t n_rel,
                        uint64_t seed, int threads, bool with_tuples, synth_strings* out) {
    if (n_rel > 8) return -1;
    uint32_t max_obj = 0;
    for (uint32_t r = 0; r < g->n_rows; ++r) max_obj = std::max(max_obj, g->row_obj[r]);
    const uint64_t objs = (uint64_t)max_obj + 1, users = p->n_users;
    uint64_t rel_bytes = 0;
    for (uint32_t i = 0; i < n_rel; ++i) rel_bytes += strlen(rel_names[i]);
    out->obj_base = 0;
    out->user_base = objs * 8;
    out->rel_base = out->user_base + users * 9;
    out->names = (char*)malloc(out->rel_base + rel_bytes + 1);
    out->n = with_tuples ? g->n_edges : 0;
    out->tuples = with_tuples ? (keto_tuple*)calloc(std::max<uint64_t>(1, g->n_edges), sizeof(keto_tuple)) : nullptr;
    if (!out->names || (with_tuples && !out->tuples)) return -2;
    static const char* hex = "0123456789abcdef";
    parallel_for(objs, threads, [&](uint64_t i) {
        char* d = out->names + out->obj_base + i * 8;
        for (int k = 7; k >= 0; --k) d[7 - k] = hex[(i >> (4 * k)) & 15];
    });
    parallel_for(users, threads, [&](uint64_t i) {
        char* d = out->names + out->user_base + i * 9;
        d[0] = 'u';
        for (int k = 7; k >= 0; --k) d[8 - k] = hex[(i >> (4 * k)) & 15];
    });
    uint64_t at = out->rel_base;
    for (uint32_t i = 0; i < n_rel; ++i) {
        out->rel_off[i] = (uint32_t)(at - out->rel_base);
        out->rel_len[i] = (uint32_t)strlen(rel_names[i]);
        memcpy(out->names + at, rel_names[i], out->rel_len[i]);
        at += out->rel_len[i];
    }
    if (!with_tuples) return 0;
    const uint64_t E = g->n_edges;
    uint64_t a = (splitmix(seed) | 1) % std::max<uint64_t>(E, 1);
    while (E > 1 && std::gcd(a, E) != 1) a = (a + 2) % E;
    const uint64_t b = splitmix(seed + 1) % std::max<uint64_t>(E, 1);
    auto obj = [&](uint32_t o) { return kstr(out->names + out->obj_base + (uint64_t)o * 8, 8); };
    auto rel = [&](uint32_t r) { return kstr(out->names + out->rel_base + out->rel_off[r], out->rel_len[r]); };
    parallel_for(g->n_rows, threads, [&](uint64_t r) {
        for (uint64_t i = g->row_ptr[r]; i < g->row_ptr[r + 1]; ++i) {
            const uint64_t pos = E > 1 ? (uint64_t)(((unsigned __int128)i * a + b) % E) : i;
            keto_tuple& t = out->tuples[pos];
            t.namespace_id = g->row_ns[r];
            t.object = obj(g->row_obj[r]);
            t.relation = rel(g->row_rel[r]);
            const uint32_t e = g->edges[i];
            if (e & 0x80000000u) {
                const uint32_t x = e & 0x7FFFFFFFu;
                t.subject_kind = 1;
                t.set_namespace_id = g->row_ns[x];
                t.set_object = obj(g->row_obj[x]);
                t.set_relation = rel(g->row_rel[x]);
            } else {
                t.subject_kind = 0;
                t.subject_id = kstr(out->names + out->user_base + (uint64_t)e * 9, 9);
            }
        }
    });
    return 0;
}

// keto_check_ids with CSR row ids and user targets -> keto_check_req by name (namespace names
// ns_names[namespace id])
int synth_check_reqs(const synth_graph* g, const synth_strings* st, const keto_check_ids* q, uint64_t n,
                     const char* const* ns_names, keto_check_req* out, int threads) {
    parallel_for(n, threads, [&](uint64_t i) {
        keto_check_req& r = out[i];
        memset(&r, 0, sizeof r);
        const uint32_t row = q[i].row;
        const char* nm = ns_names[g->row_ns[row]];
        r.namespace_ = kstr(nm, (uint32_t)strlen(nm));
        r.object = kstr(st->names + st->obj_base + (uint64_t)g->row_obj[row] * 8, 8);
        r.relation = kstr(st->names + st->rel_base + st->rel_off[g->row_rel[row]], st->rel_len[g->row_rel[row]]);
        r.subject.kind = 0;
        r.subject.id = kstr(st->names + st->user_base + (uint64_t)q[i].target * 9, 9);
        r.max_depth = q[i].max_depth;
    });
    return 0;
}

// keto_check_req -> keto_check_packed: every request's fields back to back in blob (which holds
// cap bytes); returns the bytes used, or -1 when blob is too small or a field exceeds 65535 bytes.
// Offsets are a prefix sum over the requests' field lengths (threads: per-chunk sums, then copies).
int64_t synth_pack_reqs(const keto_check_req* q, uint64_t n, uint8_t* blob, uint64_t cap, keto_check_packed* out,
                        int threads) {
    auto fields = [&](const keto_check_req& r, keto_str* f) {
        f[0] = r.namespace_;
        f[1] = r.object;
        f[2] = r.relation;
        if (r.subject.kind == 0) {
            f[3] = r.subject.id;
            f[4] = f[5] = keto_str{nullptr, 0};
            return 4;
        }
        f[3] = r.subject.set_namespace;
        f[4] = r.subject.set_object;
        f[5] = r.subject.set_relation;
        return 6;
    };
    const uint64_t T = (uint64_t)std::max(1, threads);
    const uint64_t chunk = (n + T - 1) / T;
    std::vector<uint64_t> sum(T + 1, 0);
    std::atomic<int> bad{0};
    parallel_for(T, threads, [&](uint64_t t) {
        uint64_t s = 0;
        for (uint64_t i = t * chunk; i < std::min(n, (t + 1) * chunk); ++i) {
            keto_str f[6];
            const int k = fields(q[i], f);
            for (int j = 0; j < k; ++j) {
                if (f[j].n > 65535) bad = 1;
                s += f[j].n;
            }
        }
        sum[t + 1] = s;
    });
    for (uint64_t t = 0; t < T; ++t) sum[t + 1] += sum[t];
    if (bad || sum[T] > cap || sum[T] >= (1ull << 32)) return -1;
    parallel_for(T, threads, [&](uint64_t t) {
        uint64_t at = sum[t];
        for (uint64_t i = t * chunk; i < std::min(n, (t + 1) * chunk); ++i) {
            keto_str f[6];
            const int k = fields(q[i], f);
            keto_check_packed& p = out[i];
            memset(&p, 0, sizeof p);
            p.off = (uint32_t)at;
            p.kind = q[i].subject.kind;
            p.max_depth = q[i].max_depth;
            for (int j = 0; j < k; ++j) {
                p.len[j] = (uint16_t)f[j].n;
                if (f[j].n) memcpy(blob + at, f[j].p, f[j].n);
                at += f[j].n;
            }
        }
    });
    return (int64_t)sum[T];
}

void synth_strings_free(synth_strings* s) {
    free(s->tuples);
    free(s->names);
    memset(s, 0, sizeof(*s));
}

void synth_table_free(synth_table* t) {
    free(t->ns); free(t->obj); free(t->rel); free(t->kind); free(t->sid);
    free(t->sns); free(t->sobj); free(t->srel); free(t->key);
    memset(t, 0, sizeof(*t));
}

}  // extern "C"
