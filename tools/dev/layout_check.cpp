// Host-only check (no GPU): every part of a migrating partition computes the layouts of all the
// other parts (to fill its stubs with the owners' handles); they must equal each part's own layout.
//   g++ -O2 -std=c++17 tools/dev/layout_check.cpp -Lketo_amd -lketo_mi355x -Ltools -lketo_synth -o /tmp/lc
#include <cstdio>
#include <cstdlib>

#include "../../keto_amd/csrc/snapshot.hpp"

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
int synth_generate(const synth_params* p, int threads, synth_graph* out);
}

int main(int argc, char** argv) {
    const double scale = argc > 1 ? atof(argv[1]) : 1.0 / 64;
    const uint32_t P = argc > 2 ? (uint32_t)atoi(argv[2]) : 2;
    const uint64_t hot = argc > 3 ? strtoull(argv[3], nullptr, 0) : 0;   // replicated hot rows (bytes)
    auto sc = [&](uint64_t x) { return std::max<uint64_t>(64, (uint64_t)(x * scale)); };
    synth_params p{sc(1ull << 27), sc(1ull << 24), sc(1ull << 22), sc(1ull << 26), (uint64_t)(1e9 * scale), 4};
    synth_graph g{};
    if (synth_generate(&p, 16, &g)) return 2;
    keto_namespace ns[3] = {{1, {"docs", 4}}, {2, {"folders", 7}}, {3, {"groups", 6}}};
    std::vector<std::unique_ptr<keto::Snapshot>> parts;
    for (uint32_t q = 0; q < P; ++q) {
        parts.push_back(keto::build_snapshot_csr(ns, 3, g.n_rows, g.row_ns, g.row_obj, g.row_rel, g.row_ptr, g.edges,
                                                 nullptr, 0, 100));
        keto::Snapshot& S = *parts.back();
        S.part = q;
        S.n_parts = P;
        S.part_mode = keto::PART_MIGRATE;
        S.hot_bytes = hot;
        keto::compute_layout(S);
    }
    uint64_t bad = 0, checked = 0;
    for (uint32_t q = 0; q < P; ++q)
        for (uint32_t r = 0; r < g.n_rows; ++r) {
            const uint32_t own = parts[q]->root_owner(r, P);
            if (own != q) continue;
            for (uint32_t v = 0; v < P; ++v) {
                ++checked;
                if (parts[v]->g_handle[r] != parts[q]->unit_of_row[r]) {
                    if (bad < 5)
                        fprintf(stderr, "row %u owner %u: part %u says %u, owner has %u\n", r, q, v, parts[v]->g_handle[r],
                                parts[q]->unit_of_row[r]);
                    ++bad;
                }
            }
        }
    // the replicated hot rows: the same prefix, at the same handle, on every part
    uint64_t hot_rows = 0;
    for (uint32_t q = 1; q < P; ++q)
        if (parts[q]->hot_units != parts[0]->hot_units) {
            fprintf(stderr, "hot_units differ: part %u %u, part 0 %u\n", q, parts[q]->hot_units, parts[0]->hot_units);
            ++bad;
        }
    for (uint32_t r = 0; r < g.n_rows; ++r) {
        const uint32_t u = parts[0]->unit_of_row[r];
        if (u == keto::NO_UNIT || u >= parts[0]->hot_units || (!parts[0]->stub.empty() && parts[0]->stub[r])) continue;
        ++hot_rows;
        for (uint32_t q = 1; q < P; ++q)
            if (parts[q]->unit_of_row[r] != u || (!parts[q]->stub.empty() && parts[q]->stub[r])) {
                if (bad < 10) fprintf(stderr, "hot row %u: part %u at %u, part 0 at %u\n", r, q, parts[q]->unit_of_row[r], u);
                ++bad;
            }
    }
    printf("rows %u parts %u hot rows %llu (units %u) stubs/part %llu checked %llu mismatches %llu\n", g.n_rows, P,
           (unsigned long long)hot_rows, parts[0]->hot_units, (unsigned long long)parts[0]->n_stubs,
           (unsigned long long)checked, (unsigned long long)bad);
    return bad != 0;
}
