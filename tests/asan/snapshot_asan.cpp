// Host-side sanitizer run of the C-ABI (tests/test_asan_host.py builds this with the library's
// host code under -fsanitize=address,undefined; no GPU is touched).  Random tuple tables with the
// reference's quirks -- empty fields (wildcards), '#' and ':' inside objects, subject ids whose text
// equals a set's String() (visit-key collisions), subject sets in unconfigured namespaces (poisoned
// pages), duplicates, tiny page sizes -- go through keto_snapshot_build (host-only snapshot),
// keto_snapshot_get_stats, keto_resolve_checks and keto_row_handles; random CSR graphs go through
// keto_snapshot_from_csr; compute calls must fail with KETO_E_HIP on a host-only snapshot.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../../include/keto_mi355x.h"

namespace {

uint64_t rng_state = 0x9E3779B97F4A7C15ull;
uint64_t next() {
    uint64_t x = (rng_state += 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
uint32_t pick(uint32_t n) { return (uint32_t)(next() % n); }
keto_str ks(const std::string& s) { return keto_str{s.data(), (uint32_t)s.size()}; }

int fail(const char* what) {
    std::fprintf(stderr, "FAIL %s: %s\n", what, keto_last_error());
    return 1;
}

int tuple_round(int it) {
    static const char* names[] = {"n", "m", "", "docs"};
    static const char* objs[] = {"a", "b", "", "a#b", "x:y", "B", "\xc3\xa9"};
    static const char* rels[] = {"r", "s", "", "b#c"};
    std::deque<std::string> pool;                           // keeps every string alive (stable addresses)
    auto keep = [&](std::string s) -> keto_str {
        pool.push_back(std::move(s));
        return ks(pool.back());
    };
    const uint32_t n_ns = 1 + pick(3);
    std::vector<keto_namespace> ns(n_ns);
    for (uint32_t i = 0; i < n_ns; ++i) ns[i] = keto_namespace{(int32_t)(i * 3 + pick(2)), keep(names[i])};
    const uint32_t n = pick(200);
    std::vector<keto_tuple> t(n);
    for (uint32_t i = 0; i < n; ++i) {
        keto_tuple& x = t[i];
        std::memset(&x, 0, sizeof x);
        x.namespace_id = ns[pick(n_ns)].id;
        x.object = keep(objs[pick(7)]);
        x.relation = keep(rels[pick(4)]);
        if (pick(2)) {
            x.subject_kind = 0;
            const uint32_t k = pick(4);
            x.subject_id = k == 3 ? keep(std::string(names[pick(n_ns)]) + ":" + objs[pick(7)] + "#" + rels[pick(4)])
                                  : keep("u" + std::to_string(k));
        } else {
            x.subject_kind = 1;
            x.set_namespace_id = pick(10) == 0 ? 99 : ns[pick(n_ns)].id;   // 99: unconfigured -> poisoned page
            x.set_object = keep(objs[pick(7)]);
            x.set_relation = keep(rels[pick(4)]);
        }
    }
    keto_snapshot_opts opts{1u + pick(3), -1, 0};
    keto_snapshot* s = nullptr;
    int rc = keto_snapshot_build(ns.data(), n_ns, n ? t.data() : nullptr, n, &opts, &s);
    if (rc == KETO_E_CONFIG) return 0;                      // duplicate namespace names / ids: rejected
    if (rc != KETO_OK) return fail("keto_snapshot_build");
    keto_snapshot_stats st;
    if (keto_snapshot_get_stats(s, &st) != KETO_OK) return fail("stats");
    std::vector<keto_check_req> q(64);
    for (auto& r : q) {
        std::memset(&r, 0, sizeof r);
        r.namespace_ = keep(pick(8) ? names[pick(n_ns)] : "unknown");
        r.object = keep(objs[pick(7)]);
        r.relation = keep(rels[pick(4)]);
        r.subject.kind = (uint8_t)pick(2);
        if (r.subject.kind == 0) r.subject.id = keep("u" + std::to_string(pick(5)));
        else {
            r.subject.set_namespace = keep(names[pick(n_ns)]);
            r.subject.set_object = keep(objs[pick(7)]);
            r.subject.set_relation = keep(rels[pick(4)]);
        }
        r.max_depth = (int32_t)pick(7) - 1;
    }
    std::vector<keto_check_ids> ids(q.size());
    std::vector<uint8_t> status(q.size());
    rc = keto_resolve_checks(s, q.data(), (uint32_t)q.size(), ids.data(), status.data());
    if (rc != KETO_OK && rc != KETO_E_INVALID) return fail("resolve");   // INVALID: an unmaterialized wildcard
    std::vector<uint32_t> rows(st.n_rows + 1), hs(st.n_rows + 1);
    for (uint32_t i = 0; i < st.n_rows; ++i) rows[i] = i;
    rows[st.n_rows] = KETO_NO_ROW;
    if (keto_row_handles(s, rows.data(), rows.size(), hs.data()) != KETO_OK) return fail("row_handles");
    // partition layouts (host side of keto_snapshot_upload_part_mode): both modes, 1..4 parts; a
    // migrating part's stubs are other parts' rows
    for (uint32_t mode = KETO_PART_SHARED; mode <= KETO_PART_MIGRATE; ++mode) {
        const uint32_t P = 1 + pick(4);
        uint64_t rows_total = 0;
        for (uint32_t p = 0; p < P; ++p) {
            keto_part_stats ps;
            if (keto_snapshot_part_stats_mode(s, p, P, mode, &ps) != KETO_OK) return fail("part_stats_mode");
            rows_total += ps.rows;
            if (mode == KETO_PART_SHARED && ps.stub_rows) return fail("stubs in a shared-rows part");
            if (mode == KETO_PART_MIGRATE && P == 1 && ps.stub_rows) return fail("stubs with one part");
        }
        if (mode == KETO_PART_MIGRATE && rows_total != st.n_rows) return fail("migrating parts do not split the rows");
    }
    if (keto_snapshot_part_stats_mode(s, 0, 32, KETO_PART_MIGRATE, nullptr) == KETO_OK) return fail("NULL stats");
    std::vector<uint8_t> allowed(q.size());
    if (keto_check_batch(s, q.data(), (uint32_t)q.size(), 5, allowed.data(), nullptr) != KETO_E_HIP) {
        std::fprintf(stderr, "FAIL round %d: compute on a host-only snapshot did not fail with KETO_E_HIP\n", it);
        return 1;
    }
    // writes (keto_snapshot_apply) on the host-only snapshot: inserts with new strings and new rows,
    // deletes of existing and absent tuples; refusals (KETO_E_REBUILD) and unknown namespaces
    // (KETO_E_INVALID) leave it as it was
    auto random_tuple = [&](keto_tuple& x) {
        std::memset(&x, 0, sizeof x);
        x.namespace_id = pick(20) ? ns[pick(n_ns)].id : 99;
        x.object = pick(3) ? keep(objs[pick(7)]) : keep("new" + std::to_string(pick(30)));
        x.relation = keep(rels[pick(4)]);
        if (pick(2)) {
            x.subject_kind = 0;
            x.subject_id = pick(4) ? keep("u" + std::to_string(pick(9))) : keep("w" + std::to_string(pick(50)));
        } else {
            x.subject_kind = 1;
            x.set_namespace_id = ns[pick(n_ns)].id;
            x.set_object = pick(3) ? keep(objs[pick(7)]) : keep("new" + std::to_string(pick(30)));
            x.set_relation = keep(rels[pick(4)]);
        }
    };
    for (int w = 0; w < 6; ++w) {
        std::vector<keto_tuple> ins(pick(7)), del(pick(4));
        for (auto& x : ins) random_tuple(x);
        for (auto& x : del) {
            if (n && pick(2)) x = t[pick(n)];
            else random_tuple(x);
        }
        uint64_t ver = 0;
        rc = keto_snapshot_apply(s, ins.empty() ? nullptr : ins.data(), ins.size(), del.empty() ? nullptr : del.data(),
                                 del.size(), &ver);
        if (rc != KETO_OK && rc != KETO_E_REBUILD && rc != KETO_E_INVALID) return fail("apply");
        if (keto_snapshot_get_stats(s, &st) != KETO_OK) return fail("stats after apply");
        rc = keto_resolve_checks(s, q.data(), (uint32_t)q.size(), ids.data(), status.data());
        if (rc != KETO_OK && rc != KETO_E_INVALID) return fail("resolve after apply");
    }
    keto_snapshot_release(s);
    return 0;
}

int csr_round() {
    const uint32_t R = 1 + pick(300);
    std::vector<int32_t> rns(R);
    std::vector<uint32_t> robj(R), rrel(R);
    std::vector<uint64_t> rp(R + 1, 0);
    std::vector<uint32_t> edges;
    for (uint32_t r = 0; r < R; ++r) {
        rns[r] = 1;
        robj[r] = r;
        rrel[r] = 0;
        rp[r] = edges.size();
        const uint32_t ns = pick(4), ni = pick(40);
        for (uint32_t k = 0; k < ns; ++k) edges.push_back(0x80000000u | pick(R));
        std::vector<uint32_t> idv;
        for (uint32_t k = 0; k < ni; ++k) idv.push_back(R + pick(1000));
        std::sort(idv.begin(), idv.end());
        edges.insert(edges.end(), idv.begin(), idv.end());
    }
    rp[R] = edges.size();
    std::vector<std::string> strs;
    for (uint32_t i = 0; i < R + 1000; ++i) {
        char b[16];
        std::snprintf(b, sizeof b, "%08x", i);
        strs.push_back(b);
    }
    std::vector<keto_str> ks_(strs.size());
    for (size_t i = 0; i < strs.size(); ++i) ks_[i] = ks(strs[i]);
    std::string nsn = "docs";
    keto_namespace ns{1, ks(nsn)};
    keto_snapshot_opts opts{100, -1, 0};
    keto_snapshot* s = nullptr;
    if (keto_snapshot_from_csr(&ns, 1, R, rns.data(), robj.data(), rrel.data(), rp.data(),
                               edges.empty() ? nullptr : edges.data(), ks_.data(), (uint32_t)ks_.size(), &opts,
                               &s) != KETO_OK)
        return fail("from_csr");
    keto_snapshot_stats st;
    if (keto_snapshot_get_stats(s, &st) != KETO_OK || st.n_rows != R) return fail("csr stats");
    keto_snapshot_release(s);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 300;
    for (int i = 0; i < rounds; ++i) {
        if (tuple_round(i)) return 1;
        if (i % 3 == 0 && csr_round()) return 1;
    }
    std::printf("asan host rounds ok: %d\n", rounds);
    return 0;
}
