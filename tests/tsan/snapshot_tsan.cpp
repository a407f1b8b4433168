// ThreadSanitizer run of the library's host concurrency (tests/test_tsan_host.py builds this with the
// library's host code under -fsanitize=thread; no GPU is touched).  The reference serves concurrent
// Check / Expand calls and writes from goroutines (internal/check/handler.go:168-184,
// internal/persistence/sql/relationtuples.go:279-297) and runs its suite under -race
// (.circleci/config.yml:63); the C-ABI makes the same promise (include/keto_mi355x.h: calls on one
// snapshot may come from any thread).  On one host-only snapshot, at once:
//   * a writer applies transactions (keto_snapshot_apply: staged under the shared lock, committed
//     under the exclusive one; new strings, new rows, subject sets, deletes, visit-key collisions);
//   * readers resolve named requests (keto_resolve_checks: the flat string / row indexes are built on
//     first use, by whichever reader gets there first), map rows to handles and owners, read stats,
//     versions and subject strings, and call a compute entry point that must fail (no device);
//   * a copier clones the snapshot host-only, saves it and loads it back;
//   * a planner asks for partition statistics (keto_snapshot_part_stats_mode lays the snapshot out
//     for a part and back).
// Each call must return KETO_OK or the documented error; TSan reports any data race.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/keto_mi355x.h"

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t x = (s += 0x9E3779B97F4A7C15ull);
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    }
    uint32_t pick(uint32_t n) { return (uint32_t)(next() % n); }
};

keto_str ks(const std::string& s) { return keto_str{s.data(), (uint32_t)s.size()}; }

std::atomic<int> failures{0};

void fail(const char* what, int rc) {
    std::fprintf(stderr, "FAIL %s: rc %d: %s\n", what, rc, keto_last_error());
    failures.fetch_add(1);
}

const char* NS[] = {"docs", "folders", "groups"};
const char* RELS[] = {"view", "owner", "member"};

// A tuple of a small ACL graph: docs / folders point at folders and groups, groups at groups; objects
// o0..o(n_obj-1), users u0..; a few subject ids spelled like a subject set's String() (collisions).
struct TupleMaker {
    std::deque<std::string> pool;      // stable string storage for the keto_str views
    keto_str keep(std::string s) {
        pool.push_back(std::move(s));
        return ks(pool.back());
    }
    keto_tuple make(Rng& r, uint32_t n_obj) {
        keto_tuple t;
        std::memset(&t, 0, sizeof t);
        const uint32_t ns = r.pick(3);
        t.namespace_id = (int32_t)ns + 1;
        t.object = keep("o" + std::to_string(r.pick(n_obj)));
        t.relation = keep(RELS[ns == 2 ? 2 : r.pick(2)]);
        const uint32_t k = r.pick(10);
        if (k < 5) {
            t.subject_kind = 0;
            t.subject_id = keep(k == 0 ? std::string("groups:o") + std::to_string(r.pick(n_obj)) + "#member"
                                       : "u" + std::to_string(r.pick(400)));
        } else {
            t.subject_kind = 1;
            const uint32_t sn = ns == 2 ? 2 : 1 + r.pick(2);
            t.set_namespace_id = (int32_t)sn + 1;
            t.set_object = keep("o" + std::to_string(r.pick(n_obj)));
            t.set_relation = keep(RELS[sn == 2 ? 2 : r.pick(2)]);
        }
        return t;
    }
};

}  // namespace

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 60;
    const char* dir = argc > 2 ? argv[2] : "/tmp";
    std::vector<keto_namespace> ns;
    std::deque<std::string> names;
    for (int i = 0; i < 3; ++i) {
        names.push_back(NS[i]);
        ns.push_back(keto_namespace{i + 1, ks(names.back())});
    }
    TupleMaker base_maker;
    Rng r0{1};
    std::vector<keto_tuple> base;
    for (int i = 0; i < 4000; ++i) base.push_back(base_maker.make(r0, 300));
    keto_snapshot_opts opts{};
    opts.page_size = 7;
    opts.device = -1;
    keto_snapshot* snap = nullptr;
    int rc = keto_snapshot_build(ns.data(), (uint32_t)ns.size(), base.data(), base.size(), &opts, &snap);
    if (rc != KETO_OK) {
        fail("build", rc);
        return 1;
    }
    std::atomic<bool> done{false};
    std::atomic<uint64_t> reads{0}, writes{0}, copies{0}, plans{0};

    std::thread writer([&] {
        TupleMaker m;
        Rng r{7};
        std::vector<keto_tuple> live(base);
        for (int it = 0; it < rounds; ++it) {
            std::vector<keto_tuple> ins, del;
            const uint32_t ni = 1 + r.pick(12);
            for (uint32_t k = 0; k < ni; ++k) ins.push_back(m.make(r, 300 + 4 * (uint32_t)it));   // new objects: rows, strings
            for (uint32_t k = r.pick(4); k > 0 && !live.empty(); --k) del.push_back(live[r.pick((uint32_t)live.size())]);
            uint64_t ver = 0;
            const int rc = keto_snapshot_apply(snap, ins.data(), ins.size(), del.data(), del.size(), &ver);
            if (rc != KETO_OK && rc != KETO_E_REBUILD) fail("apply", rc);
            if (rc == KETO_OK) live.insert(live.end(), ins.begin(), ins.end());
            writes.fetch_add(1);
        }
        done = true;
    });

    std::vector<std::thread> readers;
    for (int t = 0; t < 4; ++t)
        readers.emplace_back([&, t] {
            TupleMaker m;
            Rng r{100u + (uint64_t)t};
            while (!done.load()) {
                std::vector<keto_check_req> q(64);
                for (auto& x : q) {
                    std::memset(&x, 0, sizeof x);
                    const uint32_t n = r.pick(3);
                    x.namespace_ = ks(names[n]);
                    x.object = m.keep("o" + std::to_string(r.pick(500)));
                    x.relation = m.keep(RELS[n == 2 ? 2 : r.pick(2)]);
                    x.subject.kind = 0;
                    x.subject.id = m.keep("u" + std::to_string(r.pick(400)));
                    x.max_depth = (int32_t)r.pick(7);
                }
                std::vector<keto_check_ids> ids(q.size());
                std::vector<uint8_t> st(q.size());
                int rc = keto_resolve_checks(snap, q.data(), (uint32_t)q.size(), ids.data(), st.data());
                if (rc != KETO_OK) fail("resolve", rc);
                keto_snapshot_stats s{};
                rc = keto_snapshot_get_stats(snap, &s);
                if (rc != KETO_OK) fail("stats", rc);
                std::vector<uint32_t> rows(16), hs(16);
                for (auto& x : rows) x = r.pick(s.n_rows);
                rc = keto_row_handles(snap, rows.data(), rows.size(), hs.data());
                if (rc != KETO_OK) fail("row_handles", rc);
                std::vector<int32_t> own(rows.size());
                rc = keto_row_owner(snap, rows.data(), rows.size(), 4, own.data());
                if (rc != KETO_OK) fail("row_owner", rc);
                char buf[256];
                if (keto_subject_string(snap, r.pick(s.n_strings), buf, sizeof buf) < 0) fail("subject_string", -1);
                (void)keto_snapshot_version(snap);
                std::vector<uint8_t> allowed(q.size());
                rc = keto_check_batch(snap, q.data(), (uint32_t)q.size(), 5, allowed.data(), st.data());
                if (rc != KETO_E_HIP) fail("check_batch on a host-only snapshot must fail with KETO_E_HIP", rc);
                reads.fetch_add(1);
            }
        });

    std::thread copier([&] {
        int k = 0;
        while (!done.load()) {
            keto_snapshot* c = nullptr;
            int rc = keto_snapshot_clone(snap, -1, &c);
            if (rc != KETO_OK) fail("clone", rc);
            else keto_snapshot_release(c);
            const std::string path = std::string(dir) + "/tsan_snap_" + std::to_string(k++ % 2) + ".bin";
            rc = keto_snapshot_save(snap, path.c_str(), 42);
            if (rc != KETO_OK) fail("save", rc);
            keto_snapshot* l = nullptr;
            uint64_t tag = 0;
            rc = keto_snapshot_load(path.c_str(), -1, &l, &tag);
            if (rc != KETO_OK || tag != 42) fail("load", rc);
            if (l) keto_snapshot_release(l);
            std::remove(path.c_str());
            copies.fetch_add(1);
        }
    });

    std::thread planner([&] {
        uint32_t p = 0;
        while (!done.load()) {
            keto_part_stats st{};
            const int rc = keto_snapshot_part_stats_mode(snap, p % 3, 3, p % 2 ? KETO_PART_MIGRATE : KETO_PART_SHARED, &st);
            if (rc != KETO_OK) fail("part_stats", rc);
            ++p;
            plans.fetch_add(1);
        }
    });

    writer.join();
    for (auto& t : readers) t.join();
    copier.join();
    planner.join();
    keto_snapshot_release(snap);
    if (failures.load()) return 1;
    std::printf("tsan host rounds ok: %d writes, %llu reads, %llu copies, %llu plans\n", (int)writes.load(),
                (unsigned long long)reads.load(), (unsigned long long)copies.load(), (unsigned long long)plans.load());
    return 0;
}
