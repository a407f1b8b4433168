// Multi-GPU check batches over RCCL (xGMI), behind the C-ABI: one process per GPU, the exchanges
// keto_amd/multi.py runs over torch.distributed, here in the library so that a caller without
// Python -- the Go server, one process per GPU (internal/driver/daemon.go:62-69) -- can use every
// multi-GPU mode:
//
//   keto_check_batch_sharded    replicated snapshot: rank r checks the r-th contiguous shard of the
//                               batch, one all-gather returns every decision to every rank
//   keto_check_batch_routed     edge-partitioned snapshot (keto_snapshot_upload_part_mode): every
//                               rank's own batch is routed to the parts owning the requests' rows
//                               (one all-to-all), decided there, and the decisions come back (a
//                               second all-to-all); on a migrating partition the owners run the
//                               continuation-record rounds (an all-reduce and all-to-alls a round)
//   keto_comm_close_filters     a migrating partition's closure-filter exchange after upload
//
// All collectives run on the communicator's own stream with device buffers that are kept across
// calls.  The reference serves each check on one goroutine against one database
// (internal/check/handler.go:108-184); batching across GPUs is this engine's.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
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

}  // namespace

struct keto_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, n = 1, device = 0;
    hipStream_t stream = nullptr;
    // device buffers, kept across calls: a requests, b their order, c routing workspace / output,
    // d routed requests out, e / f small collectives, g routed requests in, h their decisions,
    // i decisions back, k / l the migrating rounds' records and offsets
    DBuf a, b, c, d, e, f, g, h, i, k, l;
    // owner part per row id (int16, -1 = every part) of the last routed snapshot
    const Snapshot* owner_of = nullptr;
    uint64_t owner_version = ~0ull;
    DBuf owner;
    ~keto_comm() {
        (void)hipSetDevice(device);
        if (comm) (void)ncclCommDestroy(comm);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

void sync(keto_comm& c) { HIP_OK(hipStreamSynchronize(c.stream)); }

// variable all-to-all of bytes: send[sdisp[p], +scount[p]) to rank p, receive recv[rdisp[p], +rcount[p])
void alltoallv(keto_comm& c, const void* send, const std::vector<uint64_t>& scount, void* recv,
               const std::vector<uint64_t>& rcount) {
    uint64_t so = 0, ro = 0;
    NCCL_OK(ncclGroupStart());
    for (int p = 0; p < c.n; ++p) {
        if (scount[p]) NCCL_OK(ncclSend(static_cast<const uint8_t*>(send) + so, scount[p], ncclUint8, p, c.comm, c.stream));
        if (rcount[p]) NCCL_OK(ncclRecv(static_cast<uint8_t*>(recv) + ro, rcount[p], ncclUint8, p, c.comm, c.stream));
        so += scount[p];
        ro += rcount[p];
    }
    NCCL_OK(ncclGroupEnd());
}

// every rank's `k` 64-bit words to every rank: out[p * k + j] = rank p's in[j]... per destination:
// in[p * k + j] goes to rank p, arriving as out[src * k + j]
std::vector<uint64_t> alltoall_u64(keto_comm& c, const std::vector<uint64_t>& in, int k) {
    uint64_t* d_in = c.e.get<uint64_t>((uint64_t)c.n * k * 2);
    uint64_t* d_out = d_in + (uint64_t)c.n * k;
    HIP_OK(hipMemcpyAsync(d_in, in.data(), in.size() * 8, hipMemcpyHostToDevice, c.stream));
    NCCL_OK(ncclGroupStart());
    for (int p = 0; p < c.n; ++p) {
        NCCL_OK(ncclSend(d_in + (uint64_t)p * k, k, ncclUint64, p, c.comm, c.stream));
        NCCL_OK(ncclRecv(d_out + (uint64_t)p * k, k, ncclUint64, p, c.comm, c.stream));
    }
    NCCL_OK(ncclGroupEnd());
    std::vector<uint64_t> out((uint64_t)c.n * k);
    HIP_OK(hipMemcpyAsync(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    return out;
}

uint64_t allreduce_sum(keto_comm& c, uint64_t v) {
    uint64_t* d = c.f.get<uint64_t>(1);
    HIP_OK(hipMemcpyAsync(d, &v, 8, hipMemcpyHostToDevice, c.stream));
    NCCL_OK(ncclAllReduce(d, d, 1, ncclUint64, ncclSum, c.comm, c.stream));
    HIP_OK(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    return v;
}

void shard(uint32_t n, int rank, int world, uint32_t& lo, uint32_t& hi) {
    const uint32_t base = n / world, extra = n % world;
    lo = rank * base + std::min<uint32_t>(rank, extra);
    hi = lo + base + ((uint32_t)rank < extra ? 1u : 0u);
}

const int16_t* owner_table(keto_comm& c, const Snapshot& S) {
    if (c.owner_of != &S || c.owner_version != S.version) {
        const uint32_t R = S.n_rows();
        std::vector<int16_t> own(std::max<uint32_t>(R, 1), -1);
        for (uint32_t r = 0; r < R; ++r) own[r] = (int16_t)S.row_owner(r, S.n_parts);
        int16_t* d = c.owner.get<int16_t>(own.size());
        HIP_OK(hipMemcpy(d, own.data(), own.size() * 2, hipMemcpyHostToDevice));
        c.owner_of = &S;
        c.owner_version = S.version;
    }
    return static_cast<const int16_t*>(c.owner.p);
}

// the migrating partition's record rounds for the requests routed to this part (decisions into
// d_dec, in routed order); every rank calls it collectively
void mig_rounds(keto_comm& c, Snapshot& S, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_dec) {
    MigOut out{};
    mig_begin(S, d_reqs, n, gmd, d_dec, c.stream, out);
    const int P = c.n;
    for (uint32_t rounds = 0;; ++rounds) {
        uint64_t mine = 0;
        for (int q = 0; q < P; ++q) mine += out.records[q];
        if (allreduce_sum(c, mine) == 0) return;
        if (rounds >= (1u << 20)) throw Error{KETO_E_RANGE, "migrating check did not finish in 2^20 rounds"};
        std::vector<uint64_t> cnt((uint64_t)P * 2);
        for (int q = 0; q < P; ++q) {
            cnt[2 * q] = out.units[q];
            cnt[2 * q + 1] = out.records[q];
        }
        const std::vector<uint64_t> in = alltoall_u64(c, cnt, 2);
        std::vector<uint64_t> su(P), sr(P), ru(P), rr(P);
        std::vector<uint32_t> in_recs(MIG_MAX_PARTS, 0);
        std::vector<uint64_t> in_units(MIG_MAX_PARTS, 0);
        uint64_t tu = 0, tr = 0;
        for (int q = 0; q < P; ++q) {
            su[q] = out.units[q] * 16;
            sr[q] = (uint64_t)out.records[q] * 4;
            ru[q] = in[2 * q] * 16;
            rr[q] = in[2 * q + 1] * 4;
            in_units[q] = in[2 * q];
            in_recs[q] = (uint32_t)in[2 * q + 1];
            tu += in[2 * q];
            tr += in[2 * q + 1];
        }
        uint8_t* rbuf = c.k.get<uint8_t>(tu * 16);
        uint32_t* roff = c.l.get<uint32_t>(tr);
        alltoallv(c, out.d_buf, su, rbuf, ru);
        alltoallv(c, out.d_off, sr, roff, rr);
        sync(c);
        out = MigOut{};
        mig_round(S, rbuf, roff, in_recs.data(), in_units.data(), c.stream, out);
    }
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
        if (n_ranks < 1 || rank < 0 || rank >= n_ranks || n_ranks > (int32_t)MIG_MAX_PARTS)
            throw Error{KETO_E_INVALID, "bad rank / rank count"};
        HIP_OK(hipSetDevice(device));
        auto c = std::make_unique<keto_comm>();
        c->rank = rank;
        c->n = n_ranks;
        c->device = device;
        HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, KETO_COMM_ID_BYTES);
        NCCL_OK(ncclCommInitRank(&c->comm, n_ranks, uid, rank));
        *out = c.release();
        return KETO_OK;
    });
}

void keto_comm_free(keto_comm* c) { delete c; }

int keto_check_batch_sharded(keto_comm* c, keto_snapshot* h, const keto_check_req* reqs, uint32_t n,
                             int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!c || !h || (n && (!reqs || !allowed_out || !status_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        if (h->s->n_parts > 1) throw Error{KETO_E_INVALID, "a partitioned snapshot: keto_check_batch_routed"};
        HIP_OK(hipSetDevice(c->device));
        uint32_t lo, hi, w0, w1;
        shard(n, c->rank, c->n, lo, hi);
        shard(n, 0, c->n, w0, w1);
        const uint32_t width = w1 - w0;          // the largest shard; every shard is padded to it
        std::vector<uint8_t> mine(2ull * std::max<uint32_t>(width, 1), 0);
        if (hi > lo) {
            const int rc = keto_check_batch(h, reqs + lo, hi - lo, global_max_depth, mine.data(), mine.data() + width);
            if (rc != KETO_OK) return rc;
        }
        // decisions and statuses of every shard, all-gathered as [allowed (width) | status (width)]
        uint8_t* d_send = c->a.get<uint8_t>(2ull * std::max<uint32_t>(width, 1));
        uint8_t* d_recv = c->b.get<uint8_t>(2ull * std::max<uint32_t>(width, 1) * c->n);
        HIP_OK(hipMemcpyAsync(d_send, mine.data(), 2ull * width, hipMemcpyHostToDevice, c->stream));
        if (width) NCCL_OK(ncclAllGather(d_send, d_recv, 2ull * width, ncclUint8, c->comm, c->stream));
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

int keto_check_batch_routed(keto_comm* c, keto_snapshot* h, const keto_check_req* reqs, uint32_t n,
                            int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!c || !h || (n && (!reqs || !allowed_out || !status_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        Snapshot& S = *h->s;
        std::shared_lock<std::shared_mutex> lk(S.rw);
        if ((int)S.n_parts != c->n || (int)S.part != c->rank)
            throw Error{KETO_E_INVALID, "the snapshot is not this rank's part (keto_snapshot_upload_part_mode with part = "
                                            "rank and n_parts = ranks)"};
        HIP_OK(hipSetDevice(c->device));
        // names -> row ids (routing needs rows, not this part's handles)
        std::vector<keto_check_ids> ids(std::max<uint32_t>(n, 1));
        const auto wild = resolve_all(S, reqs, n, ids.data(), status_out, true);
        if (!wild.empty())
            throw Error{KETO_E_INVALID, "request " + std::to_string(wild[0].i) +
                                            " is a wildcard query that no stored subject set uses: not routable on a "
                                            "partitioned snapshot"};
        keto_check_ids* d_reqs = c->a.get<keto_check_ids>(n);
        HIP_OK(hipMemcpyAsync(d_reqs, ids.data(), (uint64_t)n * sizeof(keto_check_ids), hipMemcpyHostToDevice, c->stream));
        const int16_t* d_owner = owner_table(*c, S);
        const uint64_t wb = route_work_bytes(n, c->n);
        uint8_t* work = c->c.get<uint8_t>(wb);
        keto_check_ids* d_send = c->d.get<keto_check_ids>(n);
        uint32_t* d_order = c->b.get<uint32_t>(n);
        std::vector<uint32_t> cs(c->n);
        route_rows(d_reqs, n, d_owner, S.n_rows(), c->rank, c->n, work, wb, d_send, d_order, cs.data(), c->stream);
        // counts, then the requests, to their owners
        std::vector<uint64_t> cnt(cs.begin(), cs.end());
        const std::vector<uint64_t> in = alltoall_u64(*c, cnt, 1);
        const uint64_t m = std::accumulate(in.begin(), in.end(), 0ull);
        if (m >= 0xFFFFFFFFull) throw Error{KETO_E_RANGE, "more than 2^32 - 1 requests routed to one part"};
        keto_check_ids* d_recv = c->g.get<keto_check_ids>(std::max<uint64_t>(m, 1));
        std::vector<uint64_t> sb(c->n), rb(c->n);
        for (int p = 0; p < c->n; ++p) {
            sb[p] = cnt[p] * sizeof(keto_check_ids);
            rb[p] = in[p] * sizeof(keto_check_ids);
        }
        alltoallv(*c, d_send, sb, d_recv, rb);
        sync(*c);
        uint8_t* d_dec = c->h.get<uint8_t>(std::max<uint64_t>(m, 1));
        if (S.part_mode == PART_MIGRATE) mig_rounds(*c, S, d_recv, (uint32_t)m, global_max_depth, d_dec);
        else device_check_rows(S, d_recv, (uint32_t)m, global_max_depth, d_dec, c->stream);
        // decisions back to their origins, in the origin's order
        uint8_t* d_back = c->i.get<uint8_t>(std::max<uint32_t>(n, 1));
        std::vector<uint64_t> sb2(in.begin(), in.end()), rb2(cnt.begin(), cnt.end());
        alltoallv(*c, d_dec, sb2, d_back, rb2);
        uint8_t* d_out = c->c.get<uint8_t>(std::max<uint64_t>(wb, n));
        unroute_rows(d_back, d_order, n, d_out, c->stream);
        if (n) HIP_OK(hipMemcpyAsync(allowed_out, d_out, n, hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        for (uint32_t i = 0; i < n; ++i)
            if (allowed_out[i] > 1) {            // KETO_UNDECIDED (and the migrating kernel's unset 255)
                allowed_out[i] = 0;
                if (status_out[i] == KETO_CHECK_OK) status_out[i] = KETO_CHECK_UNDECIDED;
            }
        return KETO_OK;
    });
}

int keto_comm_close_filters(keto_comm* c, keto_snapshot* h, uint32_t* rounds_out) {
    return guarded([&] {
        if (!c || !h) throw Error{KETO_E_INVALID, "NULL argument"};
        Snapshot& S = *h->s;
        if (S.part_mode != PART_MIGRATE || (int)S.n_parts != c->n || (int)S.part != c->rank)
            throw Error{KETO_E_INVALID, "not this rank's migrating part"};
        HIP_OK(hipSetDevice(c->device));
        // this part's stubs, grouped by owner; the owners learn once which of their rows to answer for
        std::vector<uint32_t> stubs;
        for (uint32_t r = 0; r < S.n_rows(); ++r)
            if (!S.stub.empty() && S.stub[r]) stubs.push_back(r);
        const int P = c->n;
        std::vector<uint64_t> cnt(P, 0);
        std::vector<std::vector<uint32_t>> by(P);
        for (uint32_t r : stubs) by[S.root_owner(r, P)].push_back(r);
        stubs.clear();
        for (int p = 0; p < P; ++p) {
            cnt[p] = by[p].size();
            stubs.insert(stubs.end(), by[p].begin(), by[p].end());
        }
        const std::vector<uint64_t> in = alltoall_u64(*c, cnt, 1);
        const uint64_t m = std::accumulate(in.begin(), in.end(), 0ull);
        uint32_t* d_stubs = c->a.get<uint32_t>(std::max<uint64_t>(stubs.size(), 1));
        uint32_t* d_asked = c->b.get<uint32_t>(std::max<uint64_t>(m, 1));
        HIP_OK(hipMemcpyAsync(d_stubs, stubs.data(), stubs.size() * 4, hipMemcpyHostToDevice, c->stream));
        std::vector<uint64_t> sb(P), rb(P);
        for (int p = 0; p < P; ++p) {
            sb[p] = cnt[p] * 4;
            rb[p] = in[p] * 4;
        }
        alltoallv(*c, d_stubs, sb, d_asked, rb);
        std::vector<uint32_t> asked(m);
        HIP_OK(hipMemcpyAsync(asked.data(), d_asked, m * 4, hipMemcpyDeviceToHost, c->stream));
        sync(*c);
        std::vector<uint32_t> ans(m * CF_WORDS), got(stubs.size() * CF_WORDS);
        uint32_t* d_ans = c->c.get<uint32_t>(std::max<uint64_t>(ans.size(), 1));
        uint32_t* d_got = c->d.get<uint32_t>(std::max<uint64_t>(got.size(), 1));
        for (int p = 0; p < P; ++p) {
            sb[p] = in[p] * 4 * CF_WORDS;        // answers go back to the askers
            rb[p] = cnt[p] * 4 * CF_WORDS;
        }
        uint64_t changed = 1;
        uint32_t rounds = 0;
        while (changed && rounds < 256) {
            part_filters(S, asked.data(), m, ans.data());
            HIP_OK(hipMemcpyAsync(d_ans, ans.data(), ans.size() * 4, hipMemcpyHostToDevice, c->stream));
            alltoallv(*c, d_ans, sb, d_got, rb);
            HIP_OK(hipMemcpyAsync(got.data(), d_got, got.size() * 4, hipMemcpyDeviceToHost, c->stream));
            sync(*c);
            changed = allreduce_sum(*c, part_close(S, stubs.data(), stubs.size(), got.data()));
            ++rounds;
        }
        part_closure_done(S, changed == 0);
        if (rounds_out) *rounds_out = rounds;
        return KETO_OK;
    });
}

}  // extern "C"
