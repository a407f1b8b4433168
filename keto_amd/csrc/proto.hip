// acl.SubjectTree protobuf encoding of expand trees on the GPU (keto_tree_proto_all_device): the
// bytes proto.Marshal gives for Tree.ToProto() (internal/expand/tree.go:165-188;
// proto/ory/keto/acl/v1alpha1/expand_service.proto, acl.proto), the same bytes as the host encoder
// keto_tree_proto_all (capi.cpp), from the node arena and the snapshot's strings resident on the
// device.  SURVEY.md 8(f) row 3: "expand tree materialization to proto directly from the GPU".
//
// A tree is pre-order nodes {subject, leaf | n_children}.  Its encoding is every node's header in
// pre-order -- [children tag 0x1A + varint(subtree size), except the root] [node_type 0x08, 1 union |
// 4 leaf] [subject tag 0x12 + varint(subject size)] [subject] -- so
//   1. per node (parallel): the subject's encoded size;
//   2. per tree (one lane, reverse pre-order with a stack kept in the tree's own slice of a
//      scratch array): every union node's subtree size.  Leaves (most nodes: a group's members)
//      are sized in parallel; a run of consecutive leaves is one step and one stack entry of the
//      serial pass, its children-field bytes a difference of prefix sums -- so a hub tree costs
//      its union nodes and leaf runs, not its leaves;
//   3. per node: its header length; one exclusive scan over all nodes gives every node's byte
//      offset, the trees' offsets included;
//   4. per node (parallel): write the header and the subject's strings.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t err__ = (x);                                                                     \
        if (err__ != hipSuccess)                                                                    \
            throw Error{KETO_E_HIP, std::string(#x) + ": " + hipGetErrorString(err__)};             \
    } while (0)

namespace {

constexpr uint32_t NONE_STR = 0xFFFFFFFFu;     // an absent (empty) field of a subject

template <class T>
T* palloc(uint64_t n) {
    void* p = nullptr;
    if (n == 0) n = 1;
    const hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw Error{KETO_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    return (T*)p;
}
struct PBuf {                     // a grow-only device buffer, freed with its owner
    void* p = nullptr;
    uint64_t cap = 0;
    PBuf() = default;
    PBuf(const PBuf&) = delete;
    PBuf& operator=(const PBuf&) = delete;
    template <class T>
    T* get(uint64_t n) {
        const uint64_t want = std::max<uint64_t>(1, n * sizeof(T));
        if (want > cap) {
            release();
            const uint64_t c = std::max<uint64_t>(want, cap + cap / 4);   // some headroom for the next call
            p = palloc<uint8_t>(c);
            cap = c;
        }
        return (T*)p;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    ~PBuf() { release(); }
};

// the strings a subject can name: snapshot strings, namespace names, the arena's extra strings
struct StrTab {
    const uint8_t* bytes;
    const uint64_t* off;          // n + 1
    uint32_t n;
};
struct Tables {
    StrTab strs, ns, extra;
    const int32_t* row_ns;        // namespace config index of a row, -1 = none ("")
    const uint32_t* row_obj;      // string id or ANY
    const uint32_t* row_rel;
    uint32_t n_rows;
    const int32_t* ov_ns;         // the arena's overlay rows (batch-local wildcard roots)
    const uint32_t* ov_obj;
    const uint32_t* ov_rel;
    uint32_t ov_base, n_ov;
    uint32_t extra_base;
};

struct Sub {                      // a subject's strings: (table, index) pairs; index NONE = ""
    bool set;
    const StrTab* t[3];
    uint32_t i[3];
};

__device__ inline uint32_t slen_of(const StrTab* t, uint32_t i) {
    return (t && i < t->n) ? (uint32_t)(t->off[i + 1] - t->off[i]) : 0u;
}

__device__ inline Sub subject_of(const Tables& T, uint32_t ref) {
    Sub s;
    s.set = (ref & EDGE_SET) != 0;
    const uint32_t v = ref & EDGE_VAL;
    if (!s.set) {
        s.t[0] = (v >= T.extra_base && v - T.extra_base < T.extra.n) ? &T.extra : &T.strs;
        s.i[0] = (v >= T.extra_base && v - T.extra_base < T.extra.n) ? v - T.extra_base : v;
        s.t[1] = s.t[2] = nullptr;
        s.i[1] = s.i[2] = NONE_STR;
        return s;
    }
    int32_t ns;
    uint32_t obj, rel;
    if (v >= T.ov_base && v - T.ov_base < T.n_ov) {
        ns = T.ov_ns[v - T.ov_base];
        obj = T.ov_obj[v - T.ov_base];
        rel = T.ov_rel[v - T.ov_base];
    } else if (v < T.n_rows) {
        ns = T.row_ns[v];
        obj = T.row_obj[v];
        rel = T.row_rel[v];
    } else {
        ns = -1;
        obj = rel = ANY;
    }
    s.t[0] = &T.ns;
    s.i[0] = ns < 0 ? NONE_STR : (uint32_t)ns;
    s.t[1] = &T.strs;
    s.i[1] = obj == ANY ? NONE_STR : obj;
    s.t[2] = &T.strs;
    s.i[2] = rel == ANY ? NONE_STR : rel;
    return s;
}

__host__ __device__ inline uint32_t vlen(uint64_t v) {
    uint32_t k = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++k;
    }
    return k;
}
__host__ __device__ inline uint64_t flen(uint64_t n) { return 1 + vlen(n) + n; }

// bytes of the Subject message (oneof id, present even when "" | set {namespace, object, relation;
// empty strings omitted})
__device__ inline uint64_t subject_len(const Sub& s) {
    if (!s.set) return flen(slen_of(s.t[0], s.i[0]));
    uint64_t in = 0;
    for (int f = 0; f < 3; ++f) {
        const uint32_t l = slen_of(s.t[f], s.i[f]);
        if (l) in += flen(l);
    }
    return flen(in);
}

// per node: the subject's size; a leaf's subtree size and its children-field bytes (leafw); the
// node's own position if it is a union node, else -1 (max-scanned into "last union at or before")
__global__ void __launch_bounds__(256) proto_slen(const keto_tree_node* __restrict__ nd, uint64_t n, Tables T,
                                                  uint64_t* __restrict__ slen, uint64_t* __restrict__ size,
                                                  uint64_t* __restrict__ leafw, int64_t* __restrict__ uni) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t l = subject_len(subject_of(T, nd[k].subject));
    slen[k] = l;
    const bool leaf = (nd[k].info & 0x80000000u) != 0;
    const uint64_t z = 2 + flen(l);
    size[k] = z;                                          // final for leaves; unions: proto_sizes
    leafw[k] = leaf ? flen(z) : 0;
    uni[k] = leaf ? -1 : (int64_t)k;
}

// one lane per tree: union nodes' subtree sizes in reverse pre-order.  Stack entries (2 words in
// the tree's slice of `st`): a finished union child {UNION, size}, or a run of leaf children
// {first, end} whose children-field bytes are lp[end] - lp[first] (lp = exclusive prefix of leafw);
// last_union[j] = the last union node at or before j (runs end there)
constexpr uint64_t ST_UNION = ~0ull;
__global__ void __launch_bounds__(256) proto_sizes(const keto_tree_node* __restrict__ nd,
                                                   const uint64_t* __restrict__ toff, uint32_t n_trees,
                                                   const uint64_t* __restrict__ lp,
                                                   const int64_t* __restrict__ last_union,
                                                   uint64_t* __restrict__ size, uint64_t* __restrict__ st) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_trees) return;
    const uint64_t b = toff[t], e = toff[t + 1];
    uint64_t* const stack = st + 2 * b;
    uint64_t sp = 0;
    uint64_t k = e;
    while (k > b) {
        --k;
        if (nd[k].info & 0x80000000u) {                   // the run of leaves ending at k
            const int64_t u = last_union[k];
            const uint64_t first = (u < 0 || (uint64_t)u < b) ? b : (uint64_t)u + 1;
            stack[2 * sp] = first;
            stack[2 * sp + 1] = k + 1;
            ++sp;
            k = first;
            continue;
        }
        uint32_t need = nd[k].info & 0x7FFFFFFFu;
        uint64_t z = size[k];                             // 2 + the subject field
        while (need > 0 && sp > 0) {
            uint64_t* top = stack + 2 * (sp - 1);
            if (top[0] == ST_UNION) {
                z += flen(top[1]);
                --need;
                --sp;
                continue;
            }
            const uint64_t m = top[1] - top[0], take = m < need ? m : need;   // the first `take` leaves
            z += lp[top[0] + take] - lp[top[0]];
            need -= (uint32_t)take;
            top[0] += take;
            if (top[0] == top[1]) --sp;
        }
        size[k] = z;
        stack[2 * sp] = ST_UNION;
        stack[2 * sp + 1] = z;
        ++sp;
    }
}

// header bytes of every node (tree roots have no children-field prefix)
__global__ void __launch_bounds__(256) proto_hdr(const uint64_t* __restrict__ slen, const uint64_t* __restrict__ size,
                                                 const uint8_t* __restrict__ is_root, uint64_t n,
                                                 uint64_t* __restrict__ hdr) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    hdr[k] = (is_root[k] ? 0u : 1u + vlen(size[k])) + 2u + flen(slen[k]);
}

__global__ void __launch_bounds__(256) proto_roots(const uint64_t* __restrict__ toff, uint32_t n_trees,
                                                   uint8_t* __restrict__ is_root) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n_trees && toff[t] < toff[t + 1]) is_root[toff[t]] = 1;
}

__device__ inline uint8_t* put_varint(uint8_t* p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    *p++ = (uint8_t)v;
    return p;
}
__device__ inline uint8_t* put_str(uint8_t* p, uint8_t tag, const StrTab* t, uint32_t i) {
    const uint32_t l = slen_of(t, i);
    *p++ = tag;
    p = put_varint(p, l);
    if (l) {
        const uint8_t* s = t->bytes + t->off[i];
        for (uint32_t c = 0; c < l; ++c) p[c] = s[c];
    }
    return p + l;
}

__global__ void __launch_bounds__(256) proto_write(const keto_tree_node* __restrict__ nd, uint64_t n, Tables T,
                                                   const uint64_t* __restrict__ slen, const uint64_t* __restrict__ size,
                                                   const uint8_t* __restrict__ is_root, const uint64_t* __restrict__ pos,
                                                   uint8_t* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint8_t* p = out + pos[k];
    if (!is_root[k]) {
        *p++ = 0x1A;
        p = put_varint(p, size[k]);
    }
    *p++ = 0x08;
    *p++ = (nd[k].info & 0x80000000u) ? 4 : 1;
    *p++ = 0x12;
    p = put_varint(p, slen[k]);
    const Sub s = subject_of(T, nd[k].subject);
    if (!s.set) {
        put_str(p, 0x0A, s.t[0], s.i[0]);
        return;
    }
    uint64_t in = 0;
    for (int f = 0; f < 3; ++f) {
        const uint32_t l = slen_of(s.t[f], s.i[f]);
        if (l) in += flen(l);
    }
    *p++ = 0x12;
    p = put_varint(p, in);
    const uint8_t tags[3] = {0x0A, 0x12, 0x1A};
    for (int f = 0; f < 3; ++f)
        if (slen_of(s.t[f], s.i[f])) p = put_str(p, tags[f], s.t[f], s.i[f]);
}

__global__ void __launch_bounds__(256) proto_tree_offsets(const uint64_t* __restrict__ toff, uint32_t n_trees,
                                                          const uint64_t* __restrict__ pos, uint64_t total,
                                                          uint64_t n_nodes, uint64_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n_trees) return;
    out[t] = toff[t] < n_nodes ? pos[toff[t]] : total;
}

// a string table on the device from host strings (its buffers are reused by the next upload)
struct DevStrs {
    PBuf b_bytes, b_off;
    uint8_t* bytes = nullptr;
    uint64_t* off = nullptr;
    uint32_t n = 0;
    template <class Get>
    void upload(uint32_t count, Get get) {
        std::vector<uint64_t> o(count + 1, 0);
        for (uint32_t i = 0; i < count; ++i) o[i + 1] = o[i] + get(i).size();
        std::vector<uint8_t> b(std::max<uint64_t>(1, o[count]));
        for (uint32_t i = 0; i < count; ++i) {
            const std::string_view s = get(i);
            if (!s.empty()) std::memcpy(b.data() + o[i], s.data(), s.size());
        }
        bytes = b_bytes.get<uint8_t>(b.size());
        off = b_off.get<uint64_t>(o.size());
        HIP_OK(hipMemcpy(bytes, b.data(), b.size(), hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(off, o.data(), o.size() * 8, hipMemcpyHostToDevice));
        n = count;
    }
    void release() {
        b_bytes.release();
        b_off.release();
        bytes = nullptr;
        off = nullptr;
        n = 0;
    }
    StrTab view() const { return StrTab{bytes, off, n}; }
};

// device_tree_proto's per-call buffers, kept across calls (one call at a time: the snapshot lock)
struct ProtoWork {
    DevStrs ex;
    PBuf ons, oobj, orel, nodes, toff, slen, size, st, root, hdr, pos, out, to, tmp, tmp3, lw, lp, uni, lu;
};

}  // namespace

// The snapshot's strings and row keys on the device (uploaded on first use, again after a write).
struct ProtoState {
    int device = 0;
    uint64_t version = ~0ull;
    DevStrs strs, ns;
    int32_t* row_ns = nullptr;
    uint32_t* row_obj = nullptr;
    uint32_t* row_rel = nullptr;
    uint32_t n_rows = 0;
    // two pinned bounce chunks for the output's D2H (d2h_staged)
    uint8_t* pin[2] = {nullptr, nullptr};
    uint64_t pin_bytes = 0;
    ProtoWork work;
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    void release_rows() {
        if (row_ns) (void)hipFree(row_ns);
        if (row_obj) (void)hipFree(row_obj);
        if (row_rel) (void)hipFree(row_rel);
        row_ns = nullptr;
        row_obj = row_rel = nullptr;
    }
    ~ProtoState() {
        (void)hipSetDevice(device);
        strs.release();
        ns.release();
        release_rows();
        for (int i = 0; i < 2; ++i) {
            if (pin[i]) (void)hipHostFree(pin[i]);
            if (pin_ev[i]) (void)hipEventDestroy(pin_ev[i]);
        }
    }
};

void ProtoStateDeleter::operator()(ProtoState* p) const { delete p; }

namespace {
ProtoState& proto_state(Snapshot& S, int device) {
    if (!S.proto) {
        S.proto.reset(new ProtoState);
        S.proto->device = device;
    }
    ProtoState& P = *S.proto;
    if (P.version == S.version) return P;
    P.strs.upload((uint32_t)S.strs.size(), [&](uint32_t i) { return std::string_view(S.strs[i]); });
    P.ns.upload((uint32_t)S.ns_names.size(), [&](uint32_t i) { return std::string_view(S.ns_names[i]); });
    const uint32_t R = S.n_rows();
    std::vector<int32_t> rns(R);
    std::vector<uint32_t> robj(R), rrel(R);
    for (uint32_t r = 0; r < R; ++r) {
        const RowKey& k = S.row_key[r];
        int32_t ci = -1;
        if (k.ns != ANY_NS) {
            auto it = S.ns_by_id.find((int32_t)k.ns);
            if (it != S.ns_by_id.end()) ci = it->second;
        }
        rns[r] = ci;
        robj[r] = k.obj;
        rrel[r] = k.rel;
    }
    P.release_rows();
    P.row_ns = palloc<int32_t>(R);
    P.row_obj = palloc<uint32_t>(R);
    P.row_rel = palloc<uint32_t>(R);
    HIP_OK(hipMemcpy(P.row_ns, rns.data(), (uint64_t)R * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(P.row_obj, robj.data(), (uint64_t)R * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(P.row_rel, rrel.data(), (uint64_t)R * 4, hipMemcpyHostToDevice));
    P.n_rows = R;
    P.version = S.version;
    return P;
}
}  // namespace

// D2H of the encoded bytes into the caller's buffer.  A pinned buffer takes one DMA.  A pageable
// one (the usual case: a fresh numpy / std::vector buffer) goes through two pinned bounce chunks:
// the DMA of chunk i + 1 overlaps the host threads' copy of chunk i out of its bounce buffer, which
// also takes the first-touch page faults of the caller's buffer in parallel (a plain pageable
// hipMemcpy ran at 16.8 GB/s on config #5's 36 MB).
// KETO_PROTO_PIN_CHUNK (bytes, tests): a smaller chunk, so small outputs take the staged path.
static void d2h_staged(ProtoState& P, uint8_t* buf, const uint8_t* d_src, uint64_t total, hipStream_t st) {
    uint64_t PIN_CHUNK = 8ull << 20;
    if (const char* e = getenv("KETO_PROTO_PIN_CHUNK")) PIN_CHUNK = std::max(1ll, atoll(e));
    hipPointerAttribute_t at{};
    const bool pinned = hipPointerGetAttributes(&at, buf) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();                       // pageable pointers report an error here
    if (pinned || total <= std::min<uint64_t>(1ull << 20, PIN_CHUNK)) {
        HIP_OK(hipMemcpyAsync(buf, d_src, total, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        return;
    }
    if (P.pin_bytes != PIN_CHUNK) {
        for (int i = 0; i < 2; ++i) {
            if (P.pin[i]) HIP_OK(hipHostFree(P.pin[i]));
            P.pin[i] = nullptr;
        }
        P.pin_bytes = PIN_CHUNK;
    }
    for (int i = 0; i < 2; ++i) {
        if (!P.pin[i]) HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&P.pin[i]), PIN_CHUNK, hipHostMallocDefault));
        if (!P.pin_ev[i]) HIP_OK(hipEventCreateWithFlags(&P.pin_ev[i], hipEventDisableTiming));
    }
    const uint64_t n_ch = (total + PIN_CHUNK - 1) / PIN_CHUNK;
    auto issue = [&](uint64_t c) {
        const uint64_t off = c * PIN_CHUNK, len = std::min(PIN_CHUNK, total - off);
        HIP_OK(hipMemcpyAsync(P.pin[c & 1], d_src + off, len, hipMemcpyDeviceToHost, st));
        HIP_OK(hipEventRecord(P.pin_ev[c & 1], st));
    };
    issue(0);
    if (n_ch > 1) issue(1);
    const unsigned th = std::min(8u, build_threads());
    for (uint64_t c = 0; c < n_ch; ++c) {
        HIP_OK(hipEventSynchronize(P.pin_ev[c & 1]));
        const uint64_t off = c * PIN_CHUNK, len = std::min(PIN_CHUNK, total - off);
        const uint8_t* src = P.pin[c & 1];
        par_chunks(len, th, 1ull << 20, [&](uint64_t b, uint64_t e, unsigned) { memcpy(buf + off + b, src + b, e - b); });
        if (c + 2 < n_ch) issue(c + 2);
    }
}

uint64_t device_tree_proto(Snapshot& S, const keto_tree_node* nodes, uint64_t n_nodes, const uint64_t* tree_off,
                           uint32_t n_trees, uint32_t ov_base, const std::vector<RowKey>& ov_keys, uint32_t extra_base,
                           const std::vector<std::string>& extra, uint8_t* buf, uint64_t cap, uint64_t* offsets) {
    const DevView dv = device_view(S);
    HIP_OK(hipSetDevice(dv.device));
    std::lock_guard<std::mutex> lk(S.mu);
    // KETO_PROTO_TRACE=1: phase times on stderr (tooling)
    const bool trace = getenv("KETO_PROTO_TRACE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[proto] %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    ProtoState& P = proto_state(S, dv.device);
    const hipStream_t st = 0;
    // the arena's overlay rows and extra strings
    ProtoWork& W = P.work;
    DevStrs& ex = W.ex;
    ex.upload((uint32_t)extra.size(), [&](uint32_t i) { return std::string_view(extra[i]); });
    const uint32_t n_ov = (uint32_t)ov_keys.size();
    std::vector<int32_t> ons(n_ov);
    std::vector<uint32_t> oobj(n_ov), orel(n_ov);
    for (uint32_t i = 0; i < n_ov; ++i) {
        int32_t ci = -1;
        if (ov_keys[i].ns != ANY_NS) {
            auto it = S.ns_by_id.find((int32_t)ov_keys[i].ns);
            if (it != S.ns_by_id.end()) ci = it->second;
        }
        ons[i] = ci;
        oobj[i] = ov_keys[i].obj;
        orel[i] = ov_keys[i].rel;
    }
    int32_t* d_ons = W.ons.get<int32_t>(n_ov);
    uint32_t* d_oobj = W.oobj.get<uint32_t>(n_ov);
    uint32_t* d_orel = W.orel.get<uint32_t>(n_ov);
    if (n_ov) {
        HIP_OK(hipMemcpy(d_ons, ons.data(), n_ov * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(d_oobj, oobj.data(), n_ov * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(d_orel, orel.data(), n_ov * 4, hipMemcpyHostToDevice));
    }
    Tables T{P.strs.view(), P.ns.view(), ex.view(), P.row_ns, P.row_obj, P.row_rel, P.n_rows, d_ons, d_oobj, d_orel,
             ov_base, n_ov, extra_base};
    keto_tree_node* d_nodes = W.nodes.get<keto_tree_node>(n_nodes);
    uint64_t* d_toff = W.toff.get<uint64_t>(n_trees + 1ull);
    HIP_OK(hipMemcpy(d_nodes, nodes, n_nodes * sizeof(keto_tree_node), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_toff, tree_off, (n_trees + 1ull) * 8, hipMemcpyHostToDevice));
    lap("upload");
    uint64_t* d_slen = W.slen.get<uint64_t>(n_nodes);
    uint64_t* d_size = W.size.get<uint64_t>(n_nodes);
    uint64_t* d_st = W.st.get<uint64_t>(2 * n_nodes);
    uint64_t* d_lw = W.lw.get<uint64_t>(n_nodes + 1);
    uint64_t* d_lp = W.lp.get<uint64_t>(n_nodes + 1);
    int64_t* d_uni = W.uni.get<int64_t>(n_nodes);
    int64_t* d_lu = W.lu.get<int64_t>(n_nodes);
    uint8_t* d_root = W.root.get<uint8_t>(n_nodes);
    uint64_t* d_hdr = W.hdr.get<uint64_t>(n_nodes + 1);
    uint64_t* d_pos = W.pos.get<uint64_t>(n_nodes + 1);
    uint64_t* d_to = W.to.get<uint64_t>(n_trees + 1ull);
    const auto g = [](uint64_t n) { return dim3((unsigned)std::max<uint64_t>(1, (n + 255) / 256)); };
    lap("alloc");
    HIP_OK(hipMemsetAsync(d_root, 0, std::max<uint64_t>(1, n_nodes), st));
    HIP_OK(hipMemsetAsync(d_hdr + n_nodes, 0, 8, st));
    HIP_OK(hipMemsetAsync(d_lw + n_nodes, 0, 8, st));
    size_t tmp_bytes = 0, tb2 = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_lw, d_lp, n_nodes + 1, st));
    HIP_OK(hipcub::DeviceScan::InclusiveScan(nullptr, tb2, d_uni, d_lu, hipcub::Max(), std::max<uint64_t>(1, n_nodes), st));
    tmp_bytes = std::max(tmp_bytes, tb2);
    if (n_nodes) {
        hipLaunchKernelGGL(proto_slen, g(n_nodes), dim3(256), 0, st, d_nodes, n_nodes, T, d_slen, d_size, d_lw, d_uni);
        lap("slen");
        void* d_t0 = W.tmp.get<uint8_t>(tmp_bytes);
        HIP_OK(hipcub::DeviceScan::ExclusiveSum(d_t0, tmp_bytes, d_lw, d_lp, n_nodes + 1, st));
        HIP_OK(hipcub::DeviceScan::InclusiveScan(d_t0, tb2, d_uni, d_lu, hipcub::Max(), n_nodes, st));
        hipLaunchKernelGGL(proto_sizes, g(n_trees), dim3(256), 0, st, d_nodes, d_toff, n_trees, d_lp, d_lu, d_size, d_st);
        lap("sizes");
        hipLaunchKernelGGL(proto_roots, g(n_trees), dim3(256), 0, st, d_toff, n_trees, d_root);
        hipLaunchKernelGGL(proto_hdr, g(n_nodes), dim3(256), 0, st, d_slen, d_size, d_root, n_nodes, d_hdr);
        HIP_OK(hipGetLastError());
    }
    lap("hdr");
    // exclusive scan over n_nodes + 1 entries (the last is 0): pos[n_nodes] = total
    size_t tb3 = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, d_hdr, d_pos, n_nodes + 1, st));
    void* d_tmp = W.tmp3.get<uint8_t>(tb3);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb3, d_hdr, d_pos, n_nodes + 1, st));
    uint64_t total = 0;
    HIP_OK(hipMemcpyAsync(&total, d_pos + n_nodes, 8, hipMemcpyDeviceToHost, st));
    hipLaunchKernelGGL(proto_tree_offsets, g(n_trees + 1ull), dim3(256), 0, st, d_toff, n_trees, d_pos, total, n_nodes,
                       d_to);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(st));
    // proto_tree_offsets ran before total was known on the device side: fix the tail entries
    HIP_OK(hipMemcpy(offsets, d_to, (n_trees + 1ull) * 8, hipMemcpyDeviceToHost));
    for (uint32_t t = 0; t <= n_trees; ++t)
        if (tree_off[t] >= n_nodes) offsets[t] = total;
    lap("scan");
    if (!buf || cap < total || total == 0) return total;
    uint8_t* d_out = W.out.get<uint8_t>(total);
    hipLaunchKernelGGL(proto_write, g(n_nodes), dim3(256), 0, st, d_nodes, n_nodes, T, d_slen, d_size, d_root, d_pos,
                       d_out);
    HIP_OK(hipGetLastError());
    lap("write");
    d2h_staged(P, buf, d_out, total, st);
    lap("d2h");
    return total;
}

}  // namespace keto
