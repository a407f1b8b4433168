// Multi-GPU check batches behind the C-ABI: the exchanges keto_amd/multi.py runs over
// torch.distributed, here in the library so that a caller without Python -- the Go server
// (internal/driver/daemon.go:62-69) -- can use every multi-GPU mode:
//
//   keto_check_batch_sharded    replicated snapshot: rank r checks the r-th contiguous shard of the
//                               batch, one all-gather returns every decision to every rank
//   keto_check_batch_routed     edge-partitioned snapshot (keto_snapshot_upload_part_mode): every
//                               rank's own batch is routed to the parts owning the requests' rows
//                               (one all-to-all), decided there, and the decisions come back (a
//                               second all-to-all); on a migrating partition the owners run the
//                               continuation-record rounds (an all-gather and all-to-alls a round)
//   keto_expand_batch_routed    edge-partitioned snapshot (shared rows): every rank's expand roots
//                               whose root row another part owns go to that part (one all-to-all),
//                               are expanded there, and their trees come back (a second all-to-all)
//   keto_comm_close_filters     a migrating partition's closure-filter exchange after upload
//
// Two transports carry the collectives:
//   RCCL  (keto_comm_init)        one process per GPU over xGMI: grouped ncclSend / ncclRecv
//                                 all-to-alls and all-gathers on the communicator's stream
//   local (keto_comm_init_local)  the ranks are threads of one process, each with its own stream
//                                 (on one GPU or several): a rendezvous in host memory and device
//                                 copies (peer copies over xGMI between GPUs).  One server process
//                                 can serve a partitioned graph over the node's GPUs this way, and
//                                 the multi-rank logic runs on a one-GPU box.
//
// Errors never leave a peer waiting: a rank-local failure (a bad argument, a request that cannot be
// routed, an allocation, a kernel error) is caught, and before every data exchange the ranks agree
// on their status (an all-gather of error codes, folded into the count exchanges where there is
// one).  If any rank failed, every rank returns the code of the lowest failing rank.  Only a failure
// of the transport itself (RCCL, or a local peer that never arrives: KETO_COMM_TIMEOUT_MS, default
// 10 minutes) ends a call without agreement, and it marks the communicator broken.
//
// The reference serves each check on one goroutine against one database
// (internal/check/handler.go:108-184); batching across GPUs is this engine's.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <unordered_map>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "capi_internal.hpp"

using namespace keto;

namespace {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)
#define NCCL_OK(x)                                                                                  \
    do {                                                                                            \
        ncclResult_t r__ = (x);                                                                     \
        if (r__ != ncclSuccess) throw Error{KETO_E_HIP, std::string(#x) + ": " + ncclGetErrorString(r__)}; \
    } while (0)

struct DBuf {                     // grow-only device buffer
    void* p = nullptr;
    uint64_t cap = 0;
    template <class T>
    T* get(uint64_t n) {
        const uint64_t want = std::max<uint64_t>(64, n * sizeof(T));
        if (want > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            const hipError_t e = hipMalloc(&p, want + want / 8);
            if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
            cap = want + want / 8;
        }
        return static_cast<T*>(p);
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};

// ------------------------------------------------------------------ transports
// Collectives over the ranks of one communicator.  Device-buffer calls are enqueued on `st` and
// complete before they return (the callers read the results on the host or launch on `st`).
struct Transport {
    virtual ~Transport() = default;
    // bytes: send[sdisp(p), +scount[p]) to rank p; recv[rdisp(p), +rcount[p]) from rank p (device)
    virtual void alltoallv(const void* send, const std::vector<uint64_t>& scount, void* recv,
                           const std::vector<uint64_t>& rcount, hipStream_t st) = 0;
    // two all-to-alls of one step (a migrating round's records and their offsets)
    virtual void alltoallv2(const void* s1, const std::vector<uint64_t>& sc1, void* r1, const std::vector<uint64_t>& rc1,
                            const void* s2, const std::vector<uint64_t>& sc2, void* r2, const std::vector<uint64_t>& rc2,
                            hipStream_t st) {
        alltoallv(s1, sc1, r1, rc1, st);
        alltoallv(s2, sc2, r2, rc2, st);
    }
    // every rank's `bytes` at send -> recv + p * bytes (device)
    virtual void allgather(const void* send, void* recv, uint64_t bytes, hipStream_t st) = 0;
    // host words: in[p * k + j] goes to rank p, arriving as out[src * k + j]
    virtual std::vector<uint64_t> alltoall_u64(const std::vector<uint64_t>& in, int k, hipStream_t st) = 0;
    // host words: every rank's `in` (the same length on every rank), in rank order
    virtual std::vector<uint64_t> allgather_u64(const std::vector<uint64_t>& in, hipStream_t st) = 0;
};

struct RcclTransport final : Transport {
    ncclComm_t comm = nullptr;
    int n = 1;
    DBuf small;
    ~RcclTransport() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    void alltoallv(const void* send, const std::vector<uint64_t>& scount, void* recv, const std::vector<uint64_t>& rcount,
                   hipStream_t st) override {
        uint64_t so = 0, ro = 0;
        NCCL_OK(ncclGroupStart());
        for (int p = 0; p < n; ++p) {
            if (scount[p]) NCCL_OK(ncclSend(static_cast<const uint8_t*>(send) + so, scount[p], ncclUint8, p, comm, st));
            if (rcount[p]) NCCL_OK(ncclRecv(static_cast<uint8_t*>(recv) + ro, rcount[p], ncclUint8, p, comm, st));
            so += scount[p];
            ro += rcount[p];
        }
        NCCL_OK(ncclGroupEnd());
        HIP_OK(hipStreamSynchronize(st));
    }
    void allgather(const void* send, void* recv, uint64_t bytes, hipStream_t st) override {
        if (bytes) NCCL_OK(ncclAllGather(send, recv, bytes, ncclUint8, comm, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    std::vector<uint64_t> alltoall_u64(const std::vector<uint64_t>& in, int k, hipStream_t st) override {
        uint64_t* d_in = small.get<uint64_t>((uint64_t)n * k * 2);
        uint64_t* d_out = d_in + (uint64_t)n * k;
        HIP_OK(hipMemcpyAsync(d_in, in.data(), in.size() * 8, hipMemcpyHostToDevice, st));
        NCCL_OK(ncclGroupStart());
        for (int p = 0; p < n; ++p) {
            NCCL_OK(ncclSend(d_in + (uint64_t)p * k, k, ncclUint64, p, comm, st));
            NCCL_OK(ncclRecv(d_out + (uint64_t)p * k, k, ncclUint64, p, comm, st));
        }
        NCCL_OK(ncclGroupEnd());
        std::vector<uint64_t> out((uint64_t)n * k);
        HIP_OK(hipMemcpyAsync(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        return out;
    }
    std::vector<uint64_t> allgather_u64(const std::vector<uint64_t>& in, hipStream_t st) override {
        const uint64_t k = in.size();
        uint64_t* d_in = small.get<uint64_t>(k * (n + 1));
        uint64_t* d_out = d_in + k;
        HIP_OK(hipMemcpyAsync(d_in, in.data(), k * 8, hipMemcpyHostToDevice, st));
        NCCL_OK(ncclAllGather(d_in, d_out, k, ncclUint64, comm, st));
        std::vector<uint64_t> out(k * n);
        HIP_OK(hipMemcpyAsync(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        return out;
    }
};

// The rendezvous of a local communicator: what each rank posted for the current collective, and a
// generation barrier.  Ranks find it by the caller's 128-B id (a process-wide registry).
struct LocalHub {
    int n = 0;
    int refs = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    bool broken = false;
    std::string why;
    struct Post {
        const void* dsend[2] = {nullptr, nullptr};
        int device = 0;
        std::vector<uint64_t> sdisp[2], scount[2], host;
    };
    std::vector<Post> post;
};
std::mutex g_hubs_mu;
std::map<std::string, std::shared_ptr<LocalHub>> g_hubs;

int64_t timeout_ms() {
    const char* e = getenv("KETO_COMM_TIMEOUT_MS");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? v : 600000;
}

struct LocalTransport final : Transport {
    std::shared_ptr<LocalHub> hub;
    std::string key;
    int rank = 0, n = 1, device = 0;
    ~LocalTransport() override {
        std::lock_guard<std::mutex> g(g_hubs_mu);
        if (hub && --hub->refs == 0) g_hubs.erase(key);
    }
    [[noreturn]] void fail(const std::string& why) {
        {
            std::lock_guard<std::mutex> lk(hub->mu);
            if (!hub->broken) {
                hub->broken = true;
                hub->why = why;
            }
        }
        hub->cv.notify_all();
        throw Error{KETO_E_HIP, "local communicator broken: " + why};
    }
    // every rank arrives before any leaves; a peer that does not arrive within the timeout, or a
    // broken hub, fails the call on every rank still waiting
    void barrier() {
        std::unique_lock<std::mutex> lk(hub->mu);
        if (hub->broken) throw Error{KETO_E_HIP, "local communicator broken: " + hub->why};
        const uint64_t g = hub->gen;
        if (++hub->arrived == n) {
            hub->arrived = 0;
            ++hub->gen;
            lk.unlock();
            hub->cv.notify_all();
            return;
        }
        const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms());
        if (!hub->cv.wait_until(lk, until, [&] { return hub->gen != g || hub->broken; })) {
            lk.unlock();
            fail("rank " + std::to_string(rank) + " timed out waiting for its peers");
        }
        if (hub->gen == g) throw Error{KETO_E_HIP, "local communicator broken: " + hub->why};
    }
    void put(const void* d0, const std::vector<uint64_t>& c0, const void* d1, const std::vector<uint64_t>* c1,
             std::vector<uint64_t> host) {
        std::lock_guard<std::mutex> lk(hub->mu);
        LocalHub::Post& p = hub->post[rank];
        p.device = device;
        for (int a = 0; a < 2; ++a) {
            const std::vector<uint64_t>& c = a == 0 ? c0 : c1 ? *c1 : c0;
            p.dsend[a] = a == 0 ? d0 : d1;
            p.scount[a] = a == 0 || c1 ? c : std::vector<uint64_t>(c.size(), 0);
            p.sdisp[a].assign(c.size(), 0);
            for (size_t q = 1; q < c.size(); ++q) p.sdisp[a][q] = p.sdisp[a][q - 1] + p.scount[a][q - 1];
        }
        p.host = std::move(host);
    }
    // One exchange step of one or two arrays.  The peers' segments for this rank are copied by one
    // launch (copy_segments) when they lie on this device, instead of one runtime copy per peer and
    // array: a migrating round on 8 parts had spent most of its copy time in ~2.7K blit launches per
    // batch (profiles/r06p_migrate_local.log).
    void exchange(const void* s1, const std::vector<uint64_t>& sc1, void* r1, const std::vector<uint64_t>& rc1,
                  const void* s2, const std::vector<uint64_t>* sc2, void* r2, const std::vector<uint64_t>* rc2,
                  hipStream_t st) {
        HIP_OK(hipStreamSynchronize(st));            // this rank's send data is complete
        put(s1, sc1, s2, sc2, {});
        barrier();
        CopySegments cs{};
        for (int a = 0; a < (sc2 ? 2 : 1); ++a) {
            const std::vector<uint64_t>& rcount = a == 0 ? rc1 : *rc2;
            void* recv = a == 0 ? r1 : r2;
            uint64_t ro = 0;
            for (int p = 0; p < n; ++p) {
                const LocalHub::Post& src = hub->post[p];
                if (src.scount[a][rank] != rcount[p])
                    fail("rank " + std::to_string(rank) + " expected " + std::to_string(rcount[p]) + " bytes from rank " +
                         std::to_string(p) + ", which sends " + std::to_string(src.scount[a][rank]));
                if (rcount[p]) {
                    const void* from = static_cast<const uint8_t*>(src.dsend[a]) + src.sdisp[a][rank];
                    void* to = static_cast<uint8_t*>(recv) + ro;
                    if (src.device != device) {
                        HIP_OK(hipMemcpyPeerAsync(to, device, from, src.device, rcount[p], st));
                    } else {
                        if (cs.n == COPY_SEGMENTS) {
                            copy_segments(cs, st);
                            cs.n = 0;
                        }
                        cs.src[cs.n] = from;
                        cs.dst[cs.n] = to;
                        cs.bytes[cs.n++] = rcount[p];
                    }
                }
                ro += rcount[p];
            }
        }
        if (cs.n) copy_segments(cs, st);
        HIP_OK(hipStreamSynchronize(st));
        barrier();                                  // every copy out of the send buffers is done
    }
    void alltoallv(const void* send, const std::vector<uint64_t>& scount, void* recv, const std::vector<uint64_t>& rcount,
                   hipStream_t st) override {
        exchange(send, scount, recv, rcount, nullptr, nullptr, nullptr, nullptr, st);
    }
    void alltoallv2(const void* s1, const std::vector<uint64_t>& sc1, void* r1, const std::vector<uint64_t>& rc1,
                    const void* s2, const std::vector<uint64_t>& sc2, void* r2, const std::vector<uint64_t>& rc2,
                    hipStream_t st) override {
        exchange(s1, sc1, r1, rc1, s2, &sc2, r2, &rc2, st);
    }
    void allgather(const void* send, void* recv, uint64_t bytes, hipStream_t st) override {
        HIP_OK(hipStreamSynchronize(st));
        put(send, std::vector<uint64_t>(n, 0), nullptr, nullptr, {});
        barrier();
        for (int p = 0; p < n; ++p) {
            const LocalHub::Post& src = hub->post[p];
            void* to = static_cast<uint8_t*>(recv) + (uint64_t)p * bytes;
            if (!bytes) continue;
            if (src.device == device) HIP_OK(hipMemcpyAsync(to, src.dsend[0], bytes, hipMemcpyDeviceToDevice, st));
            else HIP_OK(hipMemcpyPeerAsync(to, device, src.dsend[0], src.device, bytes, st));
        }
        HIP_OK(hipStreamSynchronize(st));
        barrier();
    }
    std::vector<uint64_t> alltoall_u64(const std::vector<uint64_t>& in, int k, hipStream_t) override {
        put(nullptr, std::vector<uint64_t>(n, 0), nullptr, nullptr, in);
        barrier();
        std::vector<uint64_t> out((uint64_t)n * k);
        for (int p = 0; p < n; ++p) {
            const std::vector<uint64_t>& h = hub->post[p].host;
            if (h.size() != (uint64_t)n * k) fail("all-to-all of words with different sizes");
            std::copy(h.begin() + (uint64_t)rank * k, h.begin() + (uint64_t)(rank + 1) * k, out.begin() + (uint64_t)p * k);
        }
        barrier();
        return out;
    }
    std::vector<uint64_t> allgather_u64(const std::vector<uint64_t>& in, hipStream_t) override {
        put(nullptr, std::vector<uint64_t>(n, 0), nullptr, nullptr, in);
        barrier();
        std::vector<uint64_t> out;
        out.reserve(in.size() * n);
        for (int p = 0; p < n; ++p) {
            const std::vector<uint64_t>& h = hub->post[p].host;
            if (h.size() != in.size()) fail("all-gather of words with different sizes");
            out.insert(out.end(), h.begin(), h.end());
        }
        barrier();
        return out;
    }
};

}  // namespace

struct keto_comm {
    std::unique_ptr<Transport> t;
    int rank = 0, n = 1, device = 0;
    hipStream_t stream = nullptr;
    // device buffers, kept across calls: a requests, b their order, c routing workspace / output,
    // d routed requests out, g routed requests in, h their decisions, i decisions back, k / l the
    // migrating rounds' records and offsets
    DBuf a, b, c, d, e, g, h, i, k, l, p;   // e: a packed batch's host-resolved requests; p: its device-resolved ones
    // owner part per row id (int16, -1 = every part) of the last routed snapshot (its uid, version,
    // partitioning: a snapshot freed and another allocated at its address is not mistaken for it)
    uint64_t owner_uid = 0, owner_version = ~0ull, owner_layout = ~0ull;
    DBuf owner;
    ~keto_comm() {
        (void)hipSetDevice(device);
        t.reset();
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

void sync(keto_comm& c) { HIP_OK(hipStreamSynchronize(c.stream)); }

// A rank's status before an exchange: the first error of its local work.
struct Local {
    int code = KETO_OK;
    std::string msg;
    template <class F>
    void run(F&& f) {
        if (code != KETO_OK) return;
        try {
            f();
        } catch (const Error& e) {
            code = e.code;
            msg = e.msg;
        } catch (const std::bad_alloc&) {
            code = KETO_E_NOMEM;
            msg = "out of host memory";
        } catch (const std::exception& e) {
            code = KETO_E_INVALID;
            msg = e.what();
        }
    }
};

// KETO_COMM_INJECT="<rank>:<point>" fails that rank's local work at that point (tests of the
// agreement): resolve, check, mig_begin, mig_round, filters
void injected(const keto_comm& c, const char* point) {
    const char* e = getenv("KETO_COMM_INJECT");
    if (!e) return;
    const char* colon = strchr(e, ':');
    if (!colon || atoi(e) != c.rank || strcmp(colon + 1, point) != 0) return;
    throw Error{KETO_E_INVALID, std::string("injected failure at ") + point};
}

// the agreed outcome of every rank's codes (rank order): the lowest failing rank's code on every
// rank; this rank's own message when it failed, else the failing peer's rank
void settle(const keto_comm& c, const Local& mine, const std::vector<int64_t>& codes) {
    for (int p = 0; p < c.n; ++p) {
        if (codes[p] == KETO_OK) continue;
        if (p == c.rank) throw Error{mine.code, mine.msg};
        std::string msg = "rank " + std::to_string(p) + " failed with code " + std::to_string(codes[p]) +
                          "; every rank of the collective call returns it";
        if (mine.code != KETO_OK) msg += " (this rank failed too: " + mine.msg + ")";
        throw Error{(int)codes[p], msg};
    }
}

void agree(keto_comm& c, const Local& mine) {
    const std::vector<uint64_t> all = c.t->allgather_u64({(uint64_t)(int64_t)mine.code}, c.stream);
    std::vector<int64_t> codes(all.begin(), all.end());
    settle(c, mine, codes);
}

void shard(uint32_t n, int rank, int world, uint32_t& lo, uint32_t& hi) {
    const uint32_t base = n / world, extra = n % world;
    lo = rank * base + std::min<uint32_t>(rank, extra);
    hi = lo + base + ((uint32_t)rank < extra ? 1u : 0u);
}

const int16_t* owner_table(keto_comm& c, const Snapshot& S) {
    const uint64_t layout = ((uint64_t)S.part_mode << 40) | ((uint64_t)S.n_parts << 20) | S.part;
    if (c.owner_uid != S.uid || c.owner_version != S.version || c.owner_layout != layout) {
        const uint32_t R = S.n_rows();
        std::vector<int16_t> own(std::max<uint32_t>(R, 1), -1);
        for (uint32_t r = 0; r < R; ++r) own[r] = (int16_t)S.row_owner(r, S.n_parts);
        int16_t* d = c.owner.get<int16_t>(own.size());
        HIP_OK(hipMemcpy(d, own.data(), own.size() * 2, hipMemcpyHostToDevice));
        c.owner_uid = S.uid;
        c.owner_version = S.version;
        c.owner_layout = layout;
    }
    return static_cast<const int16_t*>(c.owner.p);
}

// the migrating partition's record rounds for the requests routed to this part (decisions into
// d_dec, in routed order); every rank calls it collectively, `mine` carrying its status so far
void mig_rounds(keto_comm& c, Snapshot& S, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_dec,
                Local& mine) {
    MigOut out{};
    const int P = c.n;
    mine.run([&] {
        injected(c, "mig_begin");
        mig_begin(S, d_reqs, n, gmd, d_dec, c.stream, out, true);
    });
    for (uint32_t rounds = 0;; ++rounds) {
        // one all-to-all of words per round: to every rank, this rank's status, the records it emitted
        // in all, and the units and records it sends that rank
        uint64_t emitted = 0;
        if (mine.code == KETO_OK)
            for (int q = 0; q < P; ++q) emitted += out.records[q];
        std::vector<uint64_t> cnt((uint64_t)P * 4);
        for (int q = 0; q < P; ++q) {
            const bool ok = mine.code == KETO_OK;
            cnt[4 * q] = (uint64_t)(int64_t)mine.code;
            cnt[4 * q + 1] = emitted;
            cnt[4 * q + 2] = ok ? out.units[q] : 0;
            cnt[4 * q + 3] = ok ? out.records[q] : 0;
        }
        const std::vector<uint64_t> in = c.t->alltoall_u64(cnt, 4, c.stream);
        std::vector<int64_t> codes(P);
        uint64_t total = 0;
        for (int p = 0; p < P; ++p) {
            codes[p] = (int64_t)in[4 * p];
            total += in[4 * p + 1];
        }
        settle(c, mine, codes);
        if (total == 0) return;
        if (rounds >= (1u << 20)) throw Error{KETO_E_RANGE, "migrating check did not finish in 2^20 rounds"};
        std::vector<uint64_t> su(P), sr(P), ru(P), rr(P);
        std::vector<uint32_t> in_recs(MIG_MAX_PARTS, 0);
        std::vector<uint64_t> in_units(MIG_MAX_PARTS, 0);
        uint64_t tu = 0, tr = 0;
        for (int q = 0; q < P; ++q) {
            su[q] = out.units[q] * 16;
            sr[q] = (uint64_t)out.records[q] * 4;
            ru[q] = in[4 * q + 2] * 16;
            rr[q] = in[4 * q + 3] * 4;
            in_units[q] = in[4 * q + 2];
            in_recs[q] = (uint32_t)in[4 * q + 3];
            tu += in[4 * q + 2];
            tr += in[4 * q + 3];
        }
        uint8_t* rbuf = nullptr;
        uint32_t* roff = nullptr;
        mine.run([&] {
            rbuf = c.k.get<uint8_t>(tu * 16);
            roff = c.l.get<uint32_t>(tr);
        });
        agree(c, mine);
        c.t->alltoallv2(out.d_buf, su, rbuf, ru, out.d_off, sr, roff, rr, c.stream);
        out = MigOut{};
        mine.run([&] {
            injected(c, "mig_round");
            mig_round(S, rbuf, roff, in_recs.data(), in_units.data(), c.stream, out);
        });
    }
}

std::unique_ptr<keto_comm> new_comm(int32_t n_ranks, int32_t rank, int32_t device) {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || n_ranks > (int32_t)MIG_MAX_PARTS)
        throw Error{KETO_E_INVALID, "bad rank / rank count"};
    HIP_OK(hipSetDevice(device));
    auto c = std::make_unique<keto_comm>();
    c->rank = rank;
    c->n = n_ranks;
    c->device = device;
    HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return c;
}

}  // namespace

extern "C" {

int keto_comm_id(uint8_t* id_out) {
    return guarded([&] {
        if (!id_out) throw Error{KETO_E_INVALID, "NULL argument"};
        ncclUniqueId id;
        NCCL_OK(ncclGetUniqueId(&id));
        std::memcpy(id_out, id.internal, KETO_COMM_ID_BYTES);
        return KETO_OK;
    });
}

int keto_comm_init(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, keto_comm** out) {
    return guarded([&] {
        if (!id || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        auto c = new_comm(n_ranks, rank, device);
        auto t = std::make_unique<RcclTransport>();
        t->n = n_ranks;
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, KETO_COMM_ID_BYTES);
        NCCL_OK(ncclCommInitRank(&t->comm, n_ranks, uid, rank));
        c->t = std::move(t);
        *out = c.release();
        return KETO_OK;
    });
}

int keto_comm_init_local(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, keto_comm** out) {
    return guarded([&] {
        if (!id || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        auto c = new_comm(n_ranks, rank, device);
        auto t = std::make_unique<LocalTransport>();
        t->key.assign(reinterpret_cast<const char*>(id), KETO_COMM_ID_BYTES);
        t->rank = rank;
        t->n = n_ranks;
        t->device = device;
        {
            std::lock_guard<std::mutex> g(g_hubs_mu);
            std::shared_ptr<LocalHub>& h = g_hubs[t->key];
            if (!h) {
                h = std::make_shared<LocalHub>();
                h->n = n_ranks;
                h->post.resize(n_ranks);
            }
            if (h->n != n_ranks) throw Error{KETO_E_INVALID, "local communicator id in use with another rank count"};
            ++h->refs;
            t->hub = h;
        }
        // peer copies between the ranks' GPUs over xGMI (already enabled, or one GPU: nothing to do)
        int nd = 0;
        if (hipGetDeviceCount(&nd) == hipSuccess)
            for (int d = 0; d < nd; ++d)
                if (d != device) {
                    int ok = 0;
                    if (hipDeviceCanAccessPeer(&ok, device, d) == hipSuccess && ok) (void)hipDeviceEnablePeerAccess(d, 0);
                }
        (void)hipGetLastError();
        c->t = std::move(t);
        *out = c.release();
        return KETO_OK;
    });
}

void keto_comm_free(keto_comm* c) { delete c; }

int keto_check_batch_sharded(keto_comm* c, keto_snapshot* h, const keto_check_req* reqs, uint32_t n,
                             int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!c) throw Error{KETO_E_INVALID, "NULL communicator"};
        HIP_OK(hipSetDevice(c->device));
        Local mine;
        uint32_t lo = 0, hi = 0, w0 = 0, w1 = 0;
        shard(n, c->rank, c->n, lo, hi);
        shard(n, 0, c->n, w0, w1);
        const uint32_t width = w1 - w0;          // the largest shard; every shard is padded to it
        std::vector<uint8_t> part(2ull * std::max<uint32_t>(width, 1), 0);
        uint8_t *d_send = nullptr, *d_recv = nullptr;
        mine.run([&] {
            if (!h || (n && (!reqs || !allowed_out || !status_out))) throw Error{KETO_E_INVALID, "NULL argument"};
            if (h->s->n_parts > 1) throw Error{KETO_E_INVALID, "a partitioned snapshot: keto_check_batch_routed"};
            injected(*c, "check");
            if (hi > lo) {
                const int rc = keto_check_batch(h, reqs + lo, hi - lo, global_max_depth, part.data(), part.data() + width);
                if (rc != KETO_OK) throw Error{rc, g_err};
            }
            d_send = c->a.get<uint8_t>(2ull * std::max<uint32_t>(width, 1));
            d_recv = c->b.get<uint8_t>(2ull * std::max<uint32_t>(width, 1) * c->n);
            HIP_OK(hipMemcpyAsync(d_send, part.data(), 2ull * width, hipMemcpyHostToDevice, c->stream));
        });
        agree(*c, mine);
        // decisions and statuses of every shard, all-gathered as [allowed (width) | status (width)]
        c->t->allgather(d_send, d_recv, 2ull * width, c->stream);
        std::vector<uint8_t> all(2ull * width * c->n);
        HIP_OK(hipMemcpyAsync(all.data(), d_recv, all.size(), hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        for (int r = 0; r < c->n; ++r) {
            uint32_t a, b;
            shard(n, r, c->n, a, b);
            const uint8_t* src = all.data() + 2ull * width * r;
            std::memcpy(allowed_out + a, src, b - a);
            std::memcpy(status_out + a, src + width, b - a);
        }
        return KETO_OK;
    });
}

void close_filters(keto_comm* c, keto_snapshot* h, uint32_t* rounds_out);

}  // extern "C"

namespace {

// A packed batch (keto_check_batch_routed_packed): the requests' strings back to back in one blob
// and 24-B records, resolved on the device.
struct PackedIn {
    const char* blob;
    uint64_t blob_len;
    const keto_check_packed* reqs;
};

// keto_check_batch_routed's body, for named requests (reqs: resolved on host threads) or a packed
// batch (pk: resolved on the device, the wildcard queries it leaves to the host resolved here).
int routed_check(keto_comm* c, keto_snapshot* h, const keto_check_req* reqs, const PackedIn* pk, uint32_t n,
                 int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!c) throw Error{KETO_E_INVALID, "NULL communicator"};
        HIP_OK(hipSetDevice(c->device));
        Local mine;
        Snapshot* Sp = nullptr;
        std::shared_lock<RwGate> lk;
        std::vector<uint64_t> cnt(c->n, 0);
        std::vector<WildReq> wild;     // wildcard queries no stored set uses: answered here (below)
        keto_check_ids* d_send = nullptr;
        uint32_t* d_order = nullptr;
        uint64_t wb = 0;
        // named requests: every request's row-id form; a packed batch: the requests the device left to
        // the host (wildcard queries), in hidx order, the others in d_pk on the device
        std::vector<keto_check_ids> ids;
        std::vector<uint32_t> hidx;
        std::unordered_map<uint32_t, uint32_t> hpos;     // packed: batch index -> position in ids / wr
        std::vector<keto_check_req> wr;                  // packed: those requests by name (into the blob)
        keto_check_ids* d_pk = nullptr;
        auto idref = [&](uint32_t i) -> keto_check_ids& { return pk ? ids[hpos.at(i)] : ids[i]; };
        // a migrating part's wildcard queries: one request per matching row after the batch's own
        // (parent = the query's index), their decisions OR-ed into the query's below
        std::vector<uint32_t> parent;
        std::vector<keto_check_ids> extra;               // those requests
        std::vector<uint32_t> decided;                   // queries a top-level tuple allows outright
        uint32_t N = n;                                  // requests routed: the batch's + those
        // row-id requests to the device, grouped by owner (d_send, d_order); counts per part
        auto route = [&] {
            keto_check_ids* d_reqs = c->a.get<keto_check_ids>(N);
            if (!pk) {
                HIP_OK(hipMemcpyAsync(d_reqs, ids.data(), (uint64_t)n * sizeof(keto_check_ids), hipMemcpyHostToDevice,
                                      c->stream));
            } else {
                if (n) HIP_OK(hipMemcpyAsync(d_reqs, d_pk, (uint64_t)n * sizeof(keto_check_ids), hipMemcpyDeviceToDevice,
                                             c->stream));
                if (!hidx.empty()) {                     // the host-resolved requests into their places
                    const uint64_t m = hidx.size();
                    uint8_t* tmp = c->e.get<uint8_t>(m * (sizeof(keto_check_ids) + 4));
                    HIP_OK(hipMemcpyAsync(tmp, ids.data(), m * sizeof(keto_check_ids), hipMemcpyHostToDevice, c->stream));
                    HIP_OK(hipMemcpyAsync(tmp + m * sizeof(keto_check_ids), hidx.data(), m * 4, hipMemcpyHostToDevice,
                                          c->stream));
                    scatter_ids(d_reqs, reinterpret_cast<const uint32_t*>(tmp + m * sizeof(keto_check_ids)),
                                reinterpret_cast<const keto_check_ids*>(tmp), (uint32_t)m, c->stream);
                }
            }
            if (!extra.empty())
                HIP_OK(hipMemcpyAsync(d_reqs + n, extra.data(), extra.size() * sizeof(keto_check_ids),
                                      hipMemcpyHostToDevice, c->stream));
            const int16_t* d_owner = owner_table(*c, *Sp);
            wb = route_work_bytes(N, c->n);
            uint8_t* work = c->c.get<uint8_t>(std::max<uint64_t>(wb, N));
            d_send = c->d.get<keto_check_ids>(N);
            d_order = c->b.get<uint32_t>(N);
            std::vector<uint32_t> cs(c->n);
            route_rows(d_reqs, N, d_owner, Sp->n_rows(), c->rank, c->n, work, wb, d_send, d_order, cs.data(), c->stream);
            cnt.assign(cs.begin(), cs.end());
        };
        mine.run([&] {
            if (!h || (n && ((!reqs && !pk) || (pk && (!pk->reqs || (pk->blob_len && !pk->blob))) || !allowed_out ||
                             !status_out)))
                throw Error{KETO_E_INVALID, "NULL argument"};
            Sp = h->s.get();
            lk = std::shared_lock<RwGate>(Sp->rw);
            if ((int)Sp->n_parts != c->n || (int)Sp->part != c->rank)
                throw Error{KETO_E_INVALID, "the snapshot is not this rank's part (keto_snapshot_upload_part_mode with "
                                            "part = rank and n_parts = ranks)"};
            injected(*c, "resolve");
            // names -> row ids (routing needs rows, not this part's handles)
            if (!pk) {
                ids.resize(std::max<uint32_t>(n, 1));
                wild = resolve_all(*Sp, reqs, n, ids.data(), status_out, true);
            } else {
                // on the device: whereQuery per request against this part's copy of the indexes (every
                // part's host tables are the whole graph's), then the wildcard queries it leaves to
                // the host, by name, exactly as the named form resolves them
                d_pk = c->p.get<keto_check_ids>(std::max<uint32_t>(n, 1));
                device_resolve_packed_rows(*Sp, reinterpret_cast<const uint8_t*>(pk->blob), pk->blob_len, pk->reqs, n,
                                           d_pk, status_out, hidx, c->stream);
                const uint32_t m = (uint32_t)hidx.size();
                wr.resize(m);
                for (uint32_t k = 0; k < m; ++k) {
                    const keto_check_packed& p = pk->reqs[hidx[k]];
                    const char* f = pk->blob + p.off;
                    keto_str fs[6];
                    for (int j = 0; j < 6; ++j) {
                        fs[j] = keto_str{f, (uint32_t)(p.kind || j < 4 ? p.len[j] : 0u)};
                        f += fs[j].n;
                    }
                    keto_check_req& q = wr[k];
                    std::memset(&q, 0, sizeof q);
                    q.namespace_ = fs[0];
                    q.object = fs[1];
                    q.relation = fs[2];
                    q.subject.kind = p.kind;
                    if (p.kind == 0) {
                        q.subject.id = fs[3];
                    } else {
                        q.subject.set_namespace = fs[3];
                        q.subject.set_object = fs[4];
                        q.subject.set_relation = fs[5];
                    }
                    q.max_depth = p.max_depth;
                    hpos[hidx[k]] = k;
                }
                ids.resize(std::max<uint32_t>(m, 1));
                std::vector<uint8_t> hst(std::max<uint32_t>(m, 1));
                for (const WildReq& w : resolve_all(*Sp, wr.data(), m, ids.data(), hst.data(), true))
                    wild.push_back(WildReq{hidx[w.i], w.key});
                for (uint32_t k = 0; k < m; ++k) status_out[hidx[k]] = hst[k];
            }
            if (!wild.empty() && Sp->part_mode == PART_MIGRATE) {
                // A wildcard query that no stored subject set uses has no row here, and its
                // batch-local row would hold other parts' subject sets.  Its tuples are every
                // matching row's, and each top-level tuple is searched with a fresh visited map
                // (the shadowed ctx, internal/check/engine.go:47-48), so the query is allowed iff
                // one of the matching rows is, checked as a request of its own at the same depth:
                // those requests travel like any other.
                //
                // The query's ORDER BY sequence is its rows' tuples one after another, read a page at a
                // time until a page fails toInternal (relationtuples.go:64-71, 250-277): the search sees
                // the first L tuples, L = the failing page's start (engine.go:98-100 then answers
                // false).  Rows wholly before L go as above (none holds a failing tuple, so each is
                // whole in its owner's arena).  The row L cuts is taken a tuple at a time, each with the
                // fresh map of a top-level tuple: a subject id or the requested set itself decides here;
                // any other set is a request that enters its row as the walk would after the hop
                // (remaining depth d - 1, the map holding the set's visit key; migrate.hip mig_start).
                const int32_t g = std::min<int32_t>(global_max_depth, 65535);
                for (const WildReq& w : wild) {
                    const keto_check_ids q = idref(w.i);
                    const std::vector<uint32_t> rows = Sp->rows_in_key_order(w.key);
                    uint64_t L = UINT64_MAX, at = 0;
                    for (uint32_t r : rows) {
                        const auto e = Sp->row_edges(r);
                        if (Sp->row_pp[r] != NO_PAGE) {
                            uint64_t i = 0;
                            while (i < e.second && e.first[i] != EDGE_POISON) ++i;
                            L = (at + i) / Sp->page_size * Sp->page_size;
                            break;
                        }
                        at += e.second;
                    }
                    int32_t d = q.max_depth;
                    if (d <= 0 || g < d) d = g;
                    if (d <= 0) L = 0;                           // engine.go:88-91: nothing is read
                    bool yes = false;
                    at = 0;
                    for (uint32_t r : rows) {
                        if (at >= L || yes) break;
                        const auto e = Sp->row_edges(r);
                        if (at + e.second <= L) {
                            keto_check_ids x = q;
                            x.row = r;
                            extra.push_back(x);
                            parent.push_back(w.i);
                        } else {
                            for (uint64_t i = 0; i < L - at && !yes; ++i) {
                                const uint32_t v = e.first[i];
                                const bool set = (v & EDGE_SET) != 0;
                                if (set != ((q.flags & 1u) != 0) || (v & EDGE_VAL) != q.target) {
                                    if (!set || d < 2 || q.target == KETO_NO_TARGET) continue;
                                    uint32_t cls = 0;                // the set's visit key: its class if it collides
                                    if (auto it = Sp->coll.find(v); it != Sp->coll.end()) cls = (it->second & ~VID_CLASS) + 1u;
                                    if (cls >= (1u << 24)) throw Error{KETO_E_RANGE, "collision class past 2^24"};
                                    keto_check_ids x = q;
                                    x.row = v & EDGE_VAL;
                                    x.flags = (q.flags & 1u) | KETO_CHILD_FLAG | (cls << 8);
                                    x.max_depth = d - 1;
                                    extra.push_back(x);
                                    parent.push_back(w.i);
                                } else {
                                    yes = true;                      // engine.go:54-57 on a top-level tuple
                                }
                            }
                        }
                        at += e.second;
                    }
                    if (yes) decided.push_back(w.i);
                    idref(w.i).row = KETO_NO_ROW;                // decided by its rows' requests
                }
                if ((uint64_t)n + parent.size() >= 0xFFFFFFFFull) throw Error{KETO_E_RANGE, "too many wildcard rows"};
                N = n + (uint32_t)parent.size();
                wild.clear();
            }
            route();
        });
        // the counts to their owners, each with this rank's status, whether writes left this
        // (migrating) part's closure filters stale, and the snapshot version it is at: the exchange is
        // the agreement
        const uint64_t stale = mine.code == KETO_OK && Sp->part_mode == PART_MIGRATE && !Sp->mig_ready ? 1u : 0u;
        const uint64_t version = mine.code == KETO_OK ? Sp->version.load() : 0;
        std::vector<uint64_t> cw(4ull * c->n);
        for (int p = 0; p < c->n; ++p) {
            cw[4 * p] = mine.code == KETO_OK ? cnt[p] : 0;
            cw[4 * p + 1] = (uint64_t)(int64_t)mine.code;
            cw[4 * p + 2] = stale;
            cw[4 * p + 3] = version;
        }
        const std::vector<uint64_t> inw = c->t->alltoall_u64(cw, 4, c->stream);
        std::vector<int64_t> codes(c->n);
        std::vector<uint64_t> in(c->n), versions(c->n);
        bool any_stale = false;
        for (int p = 0; p < c->n; ++p) {
            in[p] = inw[4 * p];
            codes[p] = (int64_t)inw[4 * p + 1];
            any_stale |= inw[4 * p + 2] != 0;
            versions[p] = inw[4 * p + 3];
        }
        settle(*c, mine, codes);
        // Every part must be at the same snapshot version: a migrating part's records name rows by
        // their owners' handles, which each write lays out afresh, and a shared-rows part routes rows
        // that a write may have added on one part only.  Every rank saw the same versions, so every
        // rank refuses the batch here, before anything travels.
        for (int p = 0; p < c->n; ++p)
            if (versions[p] != versions[0])
                throw Error{KETO_E_INVALID, "parts at different snapshot versions (rank 0 at " +
                                                std::to_string(versions[0]) + ", rank " + std::to_string(p) + " at " +
                                                std::to_string(versions[p]) +
                                                "): apply every write to every part before a routed batch"};
        // a write lays a migrating part out afresh (its stubs' filters start empty): every rank saw the
        // same flags, so all of them run the exchange again before the batch's records travel.  The
        // exchange rewrites filters in the arena, so it runs under the exclusive lock (no other batch
        // on this part sees half-closed filters); a write that slips in between is caught below.
        if (any_stale) {
            lk.unlock();
            {
                std::unique_lock<RwGate> xl(Sp->rw);
                close_filters(c, h, nullptr);
            }
            lk.lock();
            mine.run([&] {
                if (Sp->version != version)
                    throw Error{KETO_E_INVALID, "a write was applied to this part during the routed batch"};
                // the exchange used the communicator's scratch buffers: route again (same owners, same counts)
                route();
            });
            agree(*c, mine);
        }
        Snapshot& S = *Sp;
        const uint64_t m = std::accumulate(in.begin(), in.end(), 0ull);
        keto_check_ids* d_recv = nullptr;
        uint8_t *d_dec = nullptr, *d_back = nullptr;
        mine.run([&] {
            if (m >= 0xFFFFFFFFull) throw Error{KETO_E_RANGE, "more than 2^32 - 1 requests routed to one part"};
            d_recv = c->g.get<keto_check_ids>(std::max<uint64_t>(m, 1));
            d_dec = c->h.get<uint8_t>(std::max<uint64_t>(m, 1));
            d_back = c->i.get<uint8_t>(std::max<uint32_t>(N, 1));
        });
        agree(*c, mine);
        std::vector<uint64_t> sb(c->n), rb(c->n);
        for (int p = 0; p < c->n; ++p) {
            sb[p] = cnt[p] * sizeof(keto_check_ids);
            rb[p] = in[p] * sizeof(keto_check_ids);
        }
        c->t->alltoallv(d_send, sb, d_recv, rb, c->stream);
        if (S.part_mode == PART_MIGRATE) {
            mig_rounds(*c, S, d_recv, (uint32_t)m, global_max_depth, d_dec, mine);   // agreed inside
        } else {
            mine.run([&] {
                injected(*c, "check");
                device_check_rows(S, d_recv, (uint32_t)m, global_max_depth, d_dec, c->stream);
            });
            agree(*c, mine);
        }
        // decisions back to their origins, in the origin's order
        c->t->alltoallv(d_dec, in, d_back, cnt, c->stream);
        uint8_t* d_out = c->c.get<uint8_t>(std::max<uint64_t>(wb, N));
        unroute_rows(d_back, d_order, N, d_out, c->stream);
        std::vector<uint8_t> sub(N - n);
        if (n) HIP_OK(hipMemcpyAsync(allowed_out, d_out, n, hipMemcpyDeviceToHost, c->stream));
        if (N > n) HIP_OK(hipMemcpyAsync(sub.data(), d_out + n, N - n, hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        for (uint32_t i : decided) allowed_out[i] = 1;
        for (size_t k = 0; k < parent.size(); ++k) {     // allowed if a row is; undecided if one is, none allowed
            uint8_t& a = allowed_out[parent[k]];
            if (sub[k] == 1) a = 1;
            else if (sub[k] > 1 && a != 1) a = sub[k];
        }
        for (uint32_t i = 0; i < n; ++i)
            if (allowed_out[i] > 1) {            // KETO_UNDECIDED (and the migrating kernel's unset 255)
                allowed_out[i] = 0;
                if (status_out[i] == KETO_CHECK_OK) status_out[i] = KETO_CHECK_UNDECIDED;
            }
        // A wildcard query that no stored subject set uses (whereQuery with an empty field,
        // relationtuples.go:178-198) has no row to route by; it went to this part as a request without
        // a row.  Every part holds the whole graph's host tables, so this part builds its batch-local
        // row (every matching row's tuples in ORDER BY order, as keto_check_batch does) and answers
        // it: below its top level a search only enters subject-set targets, which every part holds.
        if (!wild.empty()) {
            std::vector<keto_check_req> wq(wild.size());
            for (size_t k = 0; k < wild.size(); ++k) wq[k] = pk ? wr[hpos.at(wild[k].i)] : reqs[wild[k].i];
            std::vector<uint8_t> wa(wild.size()), ws(wild.size());
            check_named(S, wq.data(), (uint32_t)wq.size(), global_max_depth, wa.data(), ws.data());
            for (size_t k = 0; k < wild.size(); ++k) {
                allowed_out[wild[k].i] = wa[k];
                status_out[wild[k].i] = ws[k];
            }
        }
        return KETO_OK;
    });
}

}  // namespace

extern "C" {

int keto_check_batch_routed(keto_comm* c, keto_snapshot* h, const keto_check_req* reqs, uint32_t n,
                            int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return routed_check(c, h, reqs, nullptr, n, global_max_depth, allowed_out, status_out);
}

int keto_check_batch_routed_packed(keto_comm* c, keto_snapshot* h, const char* blob, uint64_t blob_len,
                                   const keto_check_packed* reqs, uint32_t n, int32_t global_max_depth,
                                   uint8_t* allowed_out, uint8_t* status_out) {
    const PackedIn pk{blob, blob_len, reqs};
    return routed_check(c, h, nullptr, &pk, n, global_max_depth, allowed_out, status_out);
}

// BuildTree (internal/expand/engine.go:33-102) for every rank's own roots over an edge-partitioned
// snapshot.  A migrating part expands all of them itself (device_expand copies the other parts' rows
// a tree reaches into the call's overlay); on shared-rows parts:  A root whose row this part holds (a subject-set target, which
// every part keeps, or one of this part's own root rows), a subject id, an unknown namespace, a
// missing row or a wildcard query is expanded here, exactly as keto_expand_batch does it.  A root
// row another part owns goes there as one word (row id, max depth); the owner expands it -- every
// row below a root is a subject-set target, which the owner holds -- and returns the tree as
// {status, node count, nodes}.  Node subjects are row and string ids of the whole graph, which every
// part's host tables share, so a returned tree reads like a local one.  Both exchanges carry each
// rank's status, so a failure anywhere ends the call with the same code on every rank.
int keto_expand_batch_routed(keto_comm* c, keto_snapshot* h, const keto_expand_req* reqs, uint32_t n,
                             int32_t global_max_depth, keto_tree_arena** out) {
    return guarded([&] {
        if (!c) throw Error{KETO_E_INVALID, "NULL communicator"};
        HIP_OK(hipSetDevice(c->device));
        const int P = c->n;
        Local mine;
        Snapshot* Sp = nullptr;
        std::shared_lock<RwGate> lk;
        std::vector<uint8_t> routed(std::max<uint32_t>(n, 1), 0);
        std::vector<std::vector<uint32_t>> to(P);        // request indices per owner part, in request order
        std::vector<uint64_t> words;                     // (row id | max depth << 32), grouped by owner
        auto local = std::make_unique<keto_tree_arena>();
        if (out) *out = nullptr;
        mine.run([&] {
            if (!h || !out || (n && !reqs)) throw Error{KETO_E_INVALID, "NULL argument"};
            Sp = h->s.get();
            lk = std::shared_lock<RwGate>(Sp->rw);
            if ((int)Sp->n_parts != P || (int)Sp->part != c->rank)
                throw Error{KETO_E_INVALID, "the snapshot is not this rank's part (keto_snapshot_upload_part_mode with "
                                            "part = rank and n_parts = ranks)"};
            injected(*c, "resolve");
            const Snapshot& S = *Sp;
            // a migrating part expands every root itself (device_expand copies the other parts' rows
            // a tree needs from the host tables, which every part holds whole): nothing is routed,
            // and the exchanges below carry only the agreement
            const bool migrating = Sp->part_mode == PART_MIGRATE;
            for (uint32_t i = 0; i < n && !migrating; ++i) {
                const keto_subject& sj = reqs[i].subject;
                if (sj.kind != 1) continue;
                const int64_t r = S.resolve_query(std::string_view(sj.set_namespace.p ? sj.set_namespace.p : "", sj.set_namespace.n),
                                                  std::string_view(sj.set_object.p ? sj.set_object.p : "", sj.set_object.n),
                                                  std::string_view(sj.set_relation.p ? sj.set_relation.p : "", sj.set_relation.n));
                if (r < 0 || S.present((uint32_t)r)) continue;
                const int32_t o = S.row_owner((uint32_t)r, (uint32_t)P);
                if (o < 0 || o >= P || o == c->rank) throw Error{KETO_E_INVALID, "expand root " + std::to_string(i) + " has no owner part"};
                routed[i] = 1;
                to[o].push_back(i);
            }
            for (int p = 0; p < P; ++p)
                for (uint32_t i : to[p]) {
                    const keto_subject& sj = reqs[i].subject;
                    const int64_t r = S.resolve_query(std::string_view(sj.set_namespace.p ? sj.set_namespace.p : "", sj.set_namespace.n),
                                                      std::string_view(sj.set_object.p ? sj.set_object.p : "", sj.set_object.n),
                                                      std::string_view(sj.set_relation.p ? sj.set_relation.p : "", sj.set_relation.n));
                    words.push_back((uint64_t)(uint32_t)r | ((uint64_t)(uint32_t)reqs[i].max_depth << 32));
                }
            injected(*c, "expand");
            if (n) expand_named(*Sp, reqs, n, global_max_depth, *local, routed.data());
        });
        // the roots to their owners, each count with this rank's status and snapshot version (the
        // exchange is the agreement)
        const uint64_t version = mine.code == KETO_OK ? Sp->version.load() : 0;
        std::vector<uint64_t> cw(3ull * P);
        for (int p = 0; p < P; ++p) {
            cw[3 * p] = mine.code == KETO_OK ? to[p].size() : 0;
            cw[3 * p + 1] = (uint64_t)(int64_t)mine.code;
            cw[3 * p + 2] = version;
        }
        const std::vector<uint64_t> inw = c->t->alltoall_u64(cw, 3, c->stream);
        std::vector<int64_t> codes(P);
        std::vector<uint64_t> in(P), sb(P), rb(P);
        for (int p = 0; p < P; ++p) {
            in[p] = inw[3 * p];
            codes[p] = (int64_t)inw[3 * p + 1];
            sb[p] = to[p].size() * 8;
            rb[p] = in[p] * 8;
        }
        settle(*c, mine, codes);
        for (int p = 0; p < P; ++p)           // every rank refuses alike (see keto_check_batch_routed)
            if (inw[3 * p + 2] != inw[2])
                throw Error{KETO_E_INVALID, "parts at different snapshot versions (rank 0 at " + std::to_string(inw[2]) +
                                                ", rank " + std::to_string(p) + " at " + std::to_string(inw[3 * p + 2]) +
                                                "): apply every write to every part before a routed batch"};
        const uint64_t m = std::accumulate(in.begin(), in.end(), 0ull);
        // the exchange buffers are allocated inside the agreement: a rank whose allocation fails still
        // meets its peers, and every rank returns that rank's code instead of waiting in the all-to-all
        uint64_t *d_words = nullptr, *d_in = nullptr;
        mine.run([&] {
            injected(*c, "roots_alloc");
            d_words = c->a.get<uint64_t>(std::max<uint64_t>(words.size(), 1));
            d_in = c->b.get<uint64_t>(std::max<uint64_t>(m, 1));
            if (!words.empty())
                HIP_OK(hipMemcpyAsync(d_words, words.data(), words.size() * 8, hipMemcpyHostToDevice, c->stream));
        });
        agree(*c, mine);
        c->t->alltoallv(d_words, sb, d_in, rb, c->stream);
        std::vector<uint64_t> got(m);
        if (m) HIP_OK(hipMemcpyAsync(got.data(), d_in, m * 8, hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        // expand the roots this part owns for the other ranks; pack the trees per origin rank
        std::vector<uint64_t> pack, pb(P, 0);            // 8-B words: {status | nodes << 8}, nodes...
        mine.run([&] {
            if (!m) return;
            injected(*c, "owner");
            Snapshot& S = *Sp;
            std::vector<uint32_t> root(m), flags(m, 1u), vid(m), rrow(m);
            std::vector<int32_t> depth(m);
            for (uint64_t k = 0; k < m; ++k) {
                const uint32_t r = (uint32_t)got[k];
                if (r >= S.n_rows() || !S.present(r)) throw Error{KETO_E_INVALID, "a routed expand root is not on its owner part"};
                root[k] = S.handle(r);
                vid[k] = S.vid_of_row(r);
                rrow[k] = r;
                depth[k] = (int32_t)(uint32_t)(got[k] >> 32);
            }
            ExpandResult er;
            device_expand(S, root, flags, vid, depth, global_max_depth, nullptr, er, nullptr, &rrow);
            uint64_t k = 0;
            for (int p = 0; p < P; ++p) {
                const uint64_t w0 = pack.size();
                for (uint64_t j = 0; j < in[p]; ++j, ++k) {
                    const uint64_t nn = er.status[k] == KETO_EXPAND_TREE ? er.offset[k + 1] - er.offset[k] : 0;
                    pack.push_back((uint64_t)er.status[k] | (nn << 8));
                    const keto_tree_node* nd = er.nodes.data() + er.offset[k];
                    for (uint64_t q = 0; q < nn; ++q) pack.push_back((uint64_t)nd[q].subject | ((uint64_t)nd[q].info << 32));
                }
                pb[p] = (pack.size() - w0) * 8;
            }
        });
        std::vector<uint64_t> bw(2ull * P);
        for (int p = 0; p < P; ++p) {
            bw[2 * p] = mine.code == KETO_OK ? pb[p] : 0;
            bw[2 * p + 1] = (uint64_t)(int64_t)mine.code;
        }
        const std::vector<uint64_t> backw = c->t->alltoall_u64(bw, 2, c->stream);
        std::vector<uint64_t> back(P);
        for (int p = 0; p < P; ++p) {
            back[p] = backw[2 * p];
            codes[p] = (int64_t)backw[2 * p + 1];
        }
        settle(*c, mine, codes);
        const uint64_t tot = std::accumulate(back.begin(), back.end(), 0ull);
        uint64_t *d_pack = nullptr, *d_back = nullptr;
        mine.run([&] {
            injected(*c, "trees_alloc");
            d_pack = c->d.get<uint64_t>(std::max<uint64_t>(pack.size(), 1));
            d_back = c->g.get<uint64_t>(std::max<uint64_t>(tot / 8, 1));
            if (!pack.empty())
                HIP_OK(hipMemcpyAsync(d_pack, pack.data(), pack.size() * 8, hipMemcpyHostToDevice, c->stream));
        });
        agree(*c, mine);
        c->t->alltoallv(d_pack, pb, d_back, back, c->stream);
        std::vector<uint64_t> trees(tot / 8);
        if (tot) HIP_OK(hipMemcpyAsync(trees.data(), d_back, tot, hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        // one arena in request order: the local trees, and the routed ones from their owners
        ExpandResult& L = local->r;
        ExpandResult R;
        R.status.resize(n);
        R.offset.assign((uint64_t)n + 1, 0);
        std::vector<uint64_t> at(n, ~0ull);               // a routed tree's header word in `trees`
        uint64_t w = 0;
        for (int p = 0; p < P; ++p) {
            const uint64_t end = w + back[p] / 8;
            for (uint32_t i : to[p]) {
                if (w >= end) throw Error{KETO_E_HIP, "expand trees missing from part " + std::to_string(p)};
                at[i] = w;
                w += 1 + (trees[w] >> 8);
            }
            if (w != end) throw Error{KETO_E_HIP, "expand trees from part " + std::to_string(p) + " do not match"};
        }
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t nn = routed[i] ? (trees[at[i]] >> 8) : L.offset[i + 1] - L.offset[i];
            R.status[i] = routed[i] ? (uint8_t)(trees[at[i]] & 0xFF) : L.status[i];
            R.offset[i + 1] = R.offset[i] + nn;
        }
        R.nodes.resize(R.offset[n]);
        for (uint32_t i = 0; i < n; ++i) {
            keto_tree_node* dst = R.nodes.data() + R.offset[i];
            const uint64_t nn = R.offset[i + 1] - R.offset[i];
            if (!routed[i]) {
                if (nn) std::memcpy(dst, L.nodes.data() + L.offset[i], nn * sizeof(keto_tree_node));
                continue;
            }
            for (uint64_t q = 0; q < nn; ++q) {
                const uint64_t x = trees[at[i] + 1 + q];
                dst[q].subject = (uint32_t)x;
                dst[q].info = (uint32_t)(x >> 32);
            }
        }
        local->r = std::move(R);
        *out = local.release();
        return KETO_OK;
    });
}

// A migrating partition's closure-filter exchange (collective; every rank calls it): rounds of
// "ask each stub's owner for its filter, OR the answers in, re-close locally" until no filter changes
// anywhere, then the signatures.  Used after the upload (keto_comm_close_filters) and again before a
// routed batch when writes laid a part out afresh.
void close_filters(keto_comm* c, keto_snapshot* h, uint32_t* rounds_out) {
    const int P = c->n;
    Local mine;
    Snapshot* Sp = nullptr;
    std::vector<uint32_t> stubs;
    std::vector<uint64_t> cnt(P, 0);
    mine.run([&] {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        Sp = h->s.get();
        if (Sp->part_mode != PART_MIGRATE || (int)Sp->n_parts != c->n || (int)Sp->part != c->rank)
            throw Error{KETO_E_INVALID, "not this rank's migrating part"};
        // this part's stubs, grouped by owner; the owners learn once which of their rows to answer for
        for (uint32_t r = 0; r < Sp->n_rows(); ++r)
            if (!Sp->stub.empty() && Sp->stub[r]) stubs.push_back(r);
        std::vector<std::vector<uint32_t>> by(P);
        for (uint32_t r : stubs) by[Sp->root_owner(r, P)].push_back(r);
        stubs.clear();
        for (int p = 0; p < P; ++p) {
            cnt[p] = by[p].size();
            stubs.insert(stubs.end(), by[p].begin(), by[p].end());
        }
    });
    std::vector<uint64_t> cw(2ull * P);
    for (int p = 0; p < P; ++p) {
        cw[2 * p] = mine.code == KETO_OK ? cnt[p] : 0;
        cw[2 * p + 1] = (uint64_t)(int64_t)mine.code;
    }
    const std::vector<uint64_t> inw = c->t->alltoall_u64(cw, 2, c->stream);
    std::vector<int64_t> codes(P);
    std::vector<uint64_t> in(P);
    for (int p = 0; p < P; ++p) {
        in[p] = inw[2 * p];
        codes[p] = (int64_t)inw[2 * p + 1];
    }
    settle(*c, mine, codes);
    Snapshot& S = *Sp;
    const uint64_t m = std::accumulate(in.begin(), in.end(), 0ull);
    uint32_t *d_stubs = nullptr, *d_asked = nullptr, *d_ans = nullptr, *d_got = nullptr;
    std::vector<uint32_t> asked(m), ans(m * CF_WORDS), got(stubs.size() * CF_WORDS);
    mine.run([&] {
        d_stubs = c->a.get<uint32_t>(std::max<uint64_t>(stubs.size(), 1));
        d_asked = c->b.get<uint32_t>(std::max<uint64_t>(m, 1));
        d_ans = c->c.get<uint32_t>(std::max<uint64_t>(ans.size(), 1));
        d_got = c->d.get<uint32_t>(std::max<uint64_t>(got.size(), 1));
        HIP_OK(hipMemcpyAsync(d_stubs, stubs.data(), stubs.size() * 4, hipMemcpyHostToDevice, c->stream));
    });
    agree(*c, mine);
    std::vector<uint64_t> sb(P), rb(P);
    for (int p = 0; p < P; ++p) {
        sb[p] = cnt[p] * 4;
        rb[p] = in[p] * 4;
    }
    c->t->alltoallv(d_stubs, sb, d_asked, rb, c->stream);
    HIP_OK(hipMemcpyAsync(asked.data(), d_asked, m * 4, hipMemcpyDeviceToHost, c->stream));
    sync(*c);
    for (int p = 0; p < P; ++p) {
        sb[p] = in[p] * 4 * CF_WORDS;        // answers go back to the askers
        rb[p] = cnt[p] * 4 * CF_WORDS;
    }
    uint64_t changed = 1;
    uint32_t rounds = 0;
    while (changed && rounds < 256) {
        mine.run([&] {
            injected(*c, "filters");
            part_filters(S, asked.data(), m, ans.data());
            HIP_OK(hipMemcpyAsync(d_ans, ans.data(), ans.size() * 4, hipMemcpyHostToDevice, c->stream));
        });
        agree(*c, mine);
        c->t->alltoallv(d_ans, sb, d_got, rb, c->stream);
        uint64_t mine_changed = 0;
        mine.run([&] {
            HIP_OK(hipMemcpyAsync(got.data(), d_got, got.size() * 4, hipMemcpyDeviceToHost, c->stream));
            sync(*c);
            mine_changed = part_close(S, stubs.data(), stubs.size(), got.data());
        });
        const std::vector<uint64_t> all = c->t->allgather_u64({(uint64_t)(int64_t)mine.code, mine_changed}, c->stream);
        changed = 0;
        for (int p = 0; p < P; ++p) {
            codes[p] = (int64_t)all[2 * p];
            changed += all[2 * p + 1];
        }
        settle(*c, mine, codes);
        ++rounds;
    }
    part_closure_done(S, changed == 0);
    if (rounds_out) *rounds_out = rounds;
}

int keto_comm_close_filters(keto_comm* c, keto_snapshot* h, uint32_t* rounds_out) {
    return guarded([&] {
        if (!c) throw Error{KETO_E_INVALID, "NULL communicator"};
        HIP_OK(hipSetDevice(c->device));
        // the exchange rewrites this part's filters: no batch on the part runs meanwhile
        std::unique_lock<RwGate> xl;
        if (h) xl = std::unique_lock<RwGate>(h->s->rw);
        close_filters(c, h, rounds_out);
        return KETO_OK;
    });
}

}  // extern "C"
