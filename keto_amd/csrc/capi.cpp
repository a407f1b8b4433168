// C-ABI of the engine (include/keto_mi355x.h): request resolution (names -> snapshot ids, the
// role of whereQuery in internal/persistence/sql/relationtuples.go:178-198), batch dispatch to the
// device engine, and the expand tree arena with its JSON codec (internal/expand/tree.go:85-163).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include "capi_internal.hpp"
#include "parallel.hpp"
#include "snapshot.hpp"

using namespace keto;


thread_local std::string keto::g_err;

namespace {

inline std::string_view sv(const keto_str& s) { return std::string_view(s.p ? s.p : "", s.n); }

void json_escape(std::string& o, std::string_view s) {
    // encoding/json's HTMLEscape-compatible string encoding
    static const char* hex = "0123456789abcdef";
    o.push_back('"');
    for (size_t i = 0; i < s.size();) {
        unsigned char c = (unsigned char)s[i];
        if (c < 0x80) {
            if (c == '"' || c == '\\') {
                o.push_back('\\');
                o.push_back((char)c);
            } else if (c == '\n') {
                o += "\\n";
            } else if (c == '\r') {
                o += "\\r";
            } else if (c == '\t') {
                o += "\\t";
            } else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                o += "\\u00";
                o.push_back(hex[c >> 4]);
                o.push_back(hex[c & 15]);
            } else {
                o.push_back((char)c);
            }
            ++i;
            continue;
        }
        // multi-byte UTF-8; invalid sequences become U+FFFD like encoding/json
        int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        bool ok = len && i + len <= s.size();
        uint32_t cp = 0;
        if (ok) {
            cp = c & (0x7F >> len);
            for (int k = 1; k < len; ++k) {
                unsigned char cc = (unsigned char)s[i + k];
                if ((cc >> 6) != 2) { ok = false; break; }
                cp = (cp << 6) | (cc & 0x3F);
            }
            if (ok && ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
                       (cp >= 0xD800 && cp <= 0xDFFF)))
                ok = false;
        }
        if (!ok) {
            o += "\\ufffd";
            ++i;
            continue;
        }
        if (cp == 0x2028 || cp == 0x2029) {
            o += cp == 0x2028 ? "\\u2028" : "\\u2029";
        } else {
            o.append(s.substr(i, len));
        }
        i += len;
    }
    o.push_back('"');
}

struct SubjectFields {
    bool set;
    std::string id, ns, obj, rel;
};

SubjectFields fields_of(const Snapshot& S, const keto_tree_arena* a, uint32_t ref) {
    SubjectFields f;
    f.set = (ref & EDGE_SET) != 0;
    uint32_t v = ref & EDGE_VAL;
    if (!f.set) {
        if (a && v >= a->extra_base && v - a->extra_base < a->extra.size()) f.id = a->extra[v - a->extra_base];
        else if (v < S.strs.size()) f.id = S.strs[v];
        return f;
    }
    if (a && v >= a->ov_base && v - a->ov_base < a->ov_keys.size()) {
        const RowKey& k = a->ov_keys[v - a->ov_base];
        if (k.ns != ANY_NS) {
            auto it = S.ns_by_id.find((int32_t)k.ns);
            if (it != S.ns_by_id.end()) f.ns = S.ns_names[it->second];
        }
        if (k.obj != ANY) f.obj = S.strs[k.obj];
        if (k.rel != ANY) f.rel = S.strs[k.rel];
        return f;
    }
    f.ns = S.row_field_ns(v);
    f.obj = S.row_field(v, 1);
    f.rel = S.row_field(v, 2);
    return f;
}

// ---- acl.SubjectTree protobuf (proto/ory/keto/acl/v1alpha1/expand_service.proto, acl.proto), the
// bytes proto.Marshal gives for Tree.ToProto() (internal/expand/tree.go:165-188): node_type = 1
// (varint; UNION 1, LEAF 4), subject = 2 (Subject: oneof id = 1 | set = 2 {namespace 1, object 2,
// relation 3; empty strings omitted}, emitted even when empty), children = 3 (repeated, in order).
uint64_t varint_len(uint64_t v) {
    uint64_t k = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++k;
    }
    return k;
}
// the subject's strings as views into the snapshot / arena (no copies)
struct SubjectViews {
    bool set;
    std::string_view id, ns, obj, rel;
};
SubjectViews views_of(const Snapshot& S, const keto_tree_arena* a, uint32_t ref) {
    SubjectViews f{(ref & EDGE_SET) != 0, {}, {}, {}, {}};
    const uint32_t v = ref & EDGE_VAL;
    auto str = [&](uint32_t x) { return x == ANY || x >= S.strs.size() ? std::string_view() : std::string_view(S.strs[x]); };
    auto nsv = [&](int64_t ns) {
        if (ns == ANY_NS) return std::string_view();
        auto it = S.ns_by_id.find((int32_t)ns);
        return it == S.ns_by_id.end() ? std::string_view() : std::string_view(S.ns_names[it->second]);
    };
    if (!f.set) {
        if (a && v >= a->extra_base && v - a->extra_base < a->extra.size()) f.id = a->extra[v - a->extra_base];
        else f.id = str(v);
        return f;
    }
    const RowKey& k = (a && v >= a->ov_base && v - a->ov_base < a->ov_keys.size()) ? a->ov_keys[v - a->ov_base] : S.row_key[v];
    f.ns = nsv(k.ns);
    f.obj = str(k.obj);
    f.rel = str(k.rel);
    return f;
}
void subject_json(const Snapshot& S, const keto_tree_arena* a, uint32_t ref, std::string& o) {
    const SubjectViews f = views_of(S, a, ref);
    if (!f.set) {
        o += ",\"subject_id\":";
        json_escape(o, f.id);
    } else {
        o += ",\"subject_set\":{\"namespace\":";
        json_escape(o, f.ns);
        o += ",\"object\":";
        json_escape(o, f.obj);
        o += ",\"relation\":";
        json_escape(o, f.rel);
        o.push_back('}');
    }
    o.push_back('}');
}

// One tree's JSON (Tree.MarshalJSON, internal/expand/tree.go:85-163: type, children, then the
// subject) from its pre-order nodes, without recursion: a tree is as deep as its max-depth (up to
// 65535 levels).  `left` holds the children still to write of every open union; a union's subject
// and closing brace follow its last child.  A truncated node list closes what is open.
void tree_json(const Snapshot& S, const keto_tree_arena* a, const keto_tree_node* nd, uint64_t n, std::string& o) {
    if (n == 0) return;
    std::vector<uint32_t> left, subj;
    uint64_t pos = 0;
    for (;;) {
        const keto_tree_node x = nd[pos++];
        const bool leaf = (x.info & 0x80000000u) != 0;
        const uint32_t nc = x.info & 0x7FFFFFFFu;
        o += leaf ? "{\"type\":\"leaf\"" : "{\"type\":\"union\"";
        if (!leaf && nc) {
            o += ",\"children\":[";
            if (pos < n) {                       // its first child is the next node
                left.push_back(nc);
                subj.push_back(x.subject);
                continue;
            }
            o.push_back(']');
        }
        subject_json(S, a, x.subject, o);
        // a node is complete: go on with its parent's next child, or close the parent
        bool more = false;
        while (!left.empty()) {
            if (--left.back() > 0 && pos < n) {
                o.push_back(',');
                more = true;
                break;
            }
            o.push_back(']');
            subject_json(S, a, subj.back(), o);
            left.pop_back();
            subj.pop_back();
        }
        if (!more) return;
    }
}

inline uint64_t field_len(uint64_t n) { return 1 + varint_len(n) + n; }
// bytes of the Subject message: oneof id (present even when "") | set {namespace, object,
// relation; empty strings omitted}
uint64_t subject_len(const SubjectViews& f) {
    if (!f.set) return field_len(f.id.size());
    const uint64_t in = (f.ns.empty() ? 0 : field_len(f.ns.size())) + (f.obj.empty() ? 0 : field_len(f.obj.size())) +
                        (f.rel.empty() ? 0 : field_len(f.rel.size()));
    return field_len(in);
}
inline char* put_varint(char* p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = (char)(v | 0x80);
        v >>= 7;
    }
    *p++ = (char)v;
    return p;
}
inline char* put_field(char* p, uint32_t tag, std::string_view b) {
    *p++ = (char)tag;
    p = put_varint(p, b.size());
    std::memcpy(p, b.data(), b.size());
    return p + b.size();
}
char* put_subject(char* p, const SubjectViews& f) {
    if (!f.set) return put_field(p, 0x0A, f.id);
    const uint64_t in = (f.ns.empty() ? 0 : field_len(f.ns.size())) + (f.obj.empty() ? 0 : field_len(f.obj.size())) +
                        (f.rel.empty() ? 0 : field_len(f.rel.size()));
    *p++ = (char)0x12;
    p = put_varint(p, in);
    if (!f.ns.empty()) p = put_field(p, 0x0A, f.ns);
    if (!f.obj.empty()) p = put_field(p, 0x12, f.obj);
    if (!f.rel.empty()) p = put_field(p, 0x1A, f.rel);
    return p;
}
// one tree (pre-order nodes) -> SubjectTree bytes appended to o: subtree sizes bottom-up (reverse
// pre-order with a stack of finished children), then one forward pass writes every node behind its
// children-field tag and length, straight into o's buffer
void tree_proto(const Snapshot& S, const keto_tree_arena* a, const keto_tree_node* nd, uint64_t n, std::string& o) {
    std::vector<uint64_t> size(n), slen(n);
    std::vector<uint64_t> st;
    for (uint64_t k = n; k-- > 0;) {
        slen[k] = subject_len(views_of(S, a, nd[k].subject));
        const bool leaf = (nd[k].info & 0x80000000u) != 0;
        const uint32_t nc = leaf ? 0 : nd[k].info & 0x7FFFFFFFu;
        uint64_t z = 2 + field_len(slen[k]);
        for (uint32_t c = 0; c < nc && !st.empty(); ++c) {
            const uint64_t cz = st.back();
            st.pop_back();
            z += field_len(cz);
        }
        size[k] = z;
        st.push_back(z);
    }
    if (!n) return;
    uint64_t total = size[0];
    for (uint64_t k = 1; k < n; ++k) total += 1 + varint_len(size[k]);
    const uint64_t at = o.size();
    o.resize(at + total);
    char* p = &o[at];
    for (uint64_t k = 0; k < n; ++k) {
        if (k) {
            *p++ = (char)0x1A;
            p = put_varint(p, size[k]);
        }
        *p++ = (char)0x08;
        *p++ = (nd[k].info & 0x80000000u) ? (char)4 : (char)1;
        *p++ = (char)0x12;
        p = put_varint(p, slen[k]);
        p = put_subject(p, views_of(S, a, nd[k].subject));
    }
    o.resize((uint64_t)(p - o.data()));
}

int64_t copy_out(const std::string& s, char* buf, uint64_t cap) {
    if (buf && cap) {
        uint64_t k = std::min<uint64_t>(cap - 1, s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int64_t)s.size();
}

}  // namespace

// resolve_checks over a whole batch on host threads (the first error wins); the wildcard requests
// come back in request order
std::vector<WildReq> keto::resolve_all(const Snapshot& S, const keto_check_req* reqs, uint32_t n, keto_check_ids* ids,
                                       uint8_t* st, bool by_row) {
    std::atomic<bool> failed{false};
    Error first{KETO_OK, ""};
    std::mutex emu;
    const unsigned th = n >= 65536 ? build_threads() : 1u;
    std::vector<std::vector<WildReq>> wild(th);
    par_chunks(n, th, 4096, [&](uint64_t b, uint64_t e, unsigned t) {
        if (failed) return;
        try {
            resolve_checks(S, reqs, b, e, ids, st, wild[t], by_row);
        } catch (const Error& x) {
            std::lock_guard<std::mutex> lk(emu);
            if (!failed.exchange(true)) first = x;
        }
    });
    if (failed) throw first;
    std::vector<WildReq> all;
    for (auto& w : wild) all.insert(all.end(), w.begin(), w.end());
    std::sort(all.begin(), all.end(), [](const WildReq& a, const WildReq& b) { return a.i < b.i; });
    return all;
}

namespace keto {
// keto_check_batch's body (the caller holds the snapshot's lock shared); comm.cpp answers a
// partitioned batch's wildcard requests with it
void check_named(Snapshot& S, const keto_check_req* reqs, uint32_t n, int32_t global_max_depth, uint8_t* allowed_out,
                 uint8_t* status_out) {
    const auto t0 = std::chrono::steady_clock::now();
    // resolution (whereQuery on the snapshot) on host threads into uninitialized buffers (every
    // entry is written); wildcard requests that need a batch-local overlay row are materialized
    // afterwards, in request order
    std::vector<keto_check_ids, NoInitAlloc<keto_check_ids>> ids(n);
    std::vector<uint8_t, NoInitAlloc<uint8_t>> st(status_out ? 0 : n);
    uint8_t* status = status_out ? status_out : st.data();
    Overlay ov;
    ov.base = S.n_rows();
    for (const WildReq& w : resolve_all(S, reqs, n, ids.data(), status))
        ids[w.i].row = handle_of(S, &ov, overlay_row(S, ov, w.key));
    S.last_resolve_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    device_check_host(S, ids.data(), n, global_max_depth, allowed_out, FORM_HANDLES, 0, &ov);
    if (status_out)
        for (uint32_t i = 0; i < n; ++i)
            if (allowed_out[i] == KETO_UNDECIDED) {
                allowed_out[i] = 0;
                status_out[i] = KETO_CHECK_UNDECIDED;
            }
}
}  // namespace keto

extern "C" {

int keto_abi_version(void) { return KETO_ABI_VERSION; }
static_assert(KETO_ARENA_MAX_BYTES == keto::ARENA_MAX_WORDS * 4, "the header's arena cap is the engine's");

const char* keto_last_error(void) { return g_err.c_str(); }

int keto_snapshot_build(const keto_namespace* namespaces, uint32_t n_namespaces, const keto_tuple* tuples,
                        uint64_t n_tuples, const keto_snapshot_opts* opts, keto_snapshot** out) {
    return guarded([&] {
        if (!out) throw Error{KETO_E_INVALID, "out == NULL"};
        *out = nullptr;
        keto_snapshot_opts o = opts ? *opts : keto_snapshot_opts{100, 0, 0};
        auto h = std::make_unique<keto_snapshot>();
        h->s = build_snapshot(namespaces, n_namespaces, tuples, n_tuples, o.page_size);
        if (o.device >= 0) device_upload(*h->s, o.device);
        *out = h.release();
        return KETO_OK;
    });
}

int keto_snapshot_from_csr(const keto_namespace* namespaces, uint32_t n_namespaces, uint32_t n_rows,
                           const int32_t* row_ns, const uint32_t* row_obj, const uint32_t* row_rel,
                           const uint64_t* row_ptr, const uint32_t* edges, const keto_str* strings,
                           uint32_t n_strings, const keto_snapshot_opts* opts, keto_snapshot** out) {
    return guarded([&] {
        if (!out) throw Error{KETO_E_INVALID, "out == NULL"};
        *out = nullptr;
        keto_snapshot_opts o = opts ? *opts : keto_snapshot_opts{100, 0, 0};
        auto h = std::make_unique<keto_snapshot>();
        h->s = build_snapshot_csr(namespaces, n_namespaces, n_rows, row_ns, row_obj, row_rel, row_ptr, edges, strings,
                                  n_strings, o.page_size);
        if (o.device >= 0) device_upload(*h->s, o.device);
        *out = h.release();
        return KETO_OK;
    });
}

int keto_snapshot_clone(const keto_snapshot* src, int32_t device, keto_snapshot** out) {
    return guarded([&] {
        if (!src || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        *out = nullptr;
        auto h = std::make_unique<keto_snapshot>();
        {
            std::shared_lock<RwGate> lk(src->s->rw);      // one version: no apply copies under us
            h->s = clone_host(*src->s);
        }
        if (device >= 0) device_upload(*h->s, device);
        *out = h.release();
        return KETO_OK;
    });
}

int keto_snapshot_save(const keto_snapshot* s, const char* path, uint64_t tag) {
    return guarded([&] {
        if (!s || !path) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(s->s->rw);        // one version: no apply under us
        save_snapshot(*s->s, path, tag);
        return KETO_OK;
    });
}

int keto_snapshot_load(const char* path, int32_t device, keto_snapshot** out, uint64_t* tag_out) {
    return guarded([&] {
        if (!path || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        *out = nullptr;
        auto h = std::make_unique<keto_snapshot>();
        h->s = load_snapshot(path, tag_out);
        if (device >= 0) device_upload(*h->s, device);
        *out = h.release();
        return KETO_OK;
    });
}

void keto_snapshot_release(keto_snapshot* s) { delete s; }

int keto_snapshot_get_stats(const keto_snapshot* h, keto_snapshot_stats* out) {
    return guarded([&] {
        if (!h || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        const Snapshot& S = *h->s;
        out->n_tuples = S.n_tuples;
        out->n_edges = S.edges.size();
        out->n_rows = S.n_rows();
        out->n_real_rows = S.n_real_rows;
        out->n_wildcard_rows = S.n_wild_rows;
        out->n_seq_rows = S.n_seq_rows;
        out->n_poisoned_rows = S.n_poisoned_rows;
        out->n_strings = (uint32_t)S.strs.size();
        out->n_collision_keys = S.n_coll_keys;
        out->device_bytes = device_bytes(S);
        return KETO_OK;
    });
}

int keto_resolve_checks(const keto_snapshot* h, const keto_check_req* reqs, uint32_t n, keto_check_ids* out,
                        uint8_t* status_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        std::vector<uint8_t, NoInitAlloc<uint8_t>> st(status_out ? 0 : n);
        const auto wild = resolve_all(*h->s, reqs, n, out, status_out ? status_out : st.data());
        if (!wild.empty())
            throw Error{KETO_E_INVALID, "request " + std::to_string(wild[0].i) +
                                            " is a wildcard query that no stored subject set uses; "
                                            "pass it to keto_check_batch"};
        return KETO_OK;
    });
}


int keto_check_batch(keto_snapshot* h, const keto_check_req* reqs, uint32_t n, int32_t global_max_depth,
                     uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        check_named(*h->s, reqs, n, global_max_depth, allowed_out, status_out);
        return KETO_OK;
    });
}

int keto_check_batch_packed(keto_snapshot* h, const char* blob, uint64_t blob_len, const keto_check_packed* reqs,
                            uint32_t n, int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !allowed_out)) || (blob_len && !blob)) throw Error{KETO_E_INVALID, "NULL argument"};
        if (blob_len >= (1ull << 32)) throw Error{KETO_E_RANGE, "a packed batch's strings must stay below 4 GiB"};
        lock_trace("packed: waiting for rw shared");
        std::shared_lock<RwGate> lk(h->s->rw);
        lock_trace("packed: rw shared");
        Snapshot& S = *h->s;
        if (n == 0) return KETO_OK;
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<uint8_t> st_local(status_out ? 0 : n);
        uint8_t* status = status_out ? status_out : st_local.data();
        std::vector<uint32_t> host;
        device_check_packed(S, reinterpret_cast<const uint8_t*>(blob), blob_len, reqs, n, global_max_depth,
                            allowed_out, status, host);
        if (!host.empty()) {
            // wildcard queries: the host path (keto_check_batch), which may need batch-local rows
            std::vector<keto_check_req> q(host.size());
            for (size_t k = 0; k < host.size(); ++k) {
                const keto_check_packed& p = reqs[host[k]];
                const char* f = blob + p.off;
                keto_check_req& r = q[k];
                std::memset(&r, 0, sizeof r);
                r.namespace_ = keto_str{f, p.len[0]};
                r.object = keto_str{f + p.len[0], p.len[1]};
                r.relation = keto_str{f + p.len[0] + p.len[1], p.len[2]};
                const char* g = f + p.len[0] + p.len[1] + p.len[2];
                if (p.kind == 0) {
                    r.subject.kind = 0;
                    r.subject.id = keto_str{g, p.len[3]};
                } else {
                    r.subject.kind = 1;
                    r.subject.set_namespace = keto_str{g, p.len[3]};
                    r.subject.set_object = keto_str{g + p.len[3], p.len[4]};
                    r.subject.set_relation = keto_str{g + p.len[3] + p.len[4], p.len[5]};
                }
                r.max_depth = p.max_depth;
            }
            std::vector<uint8_t> a(host.size()), st(host.size());
            check_named(S, q.data(), (uint32_t)q.size(), global_max_depth, a.data(), st.data());
            for (size_t k = 0; k < host.size(); ++k) {
                allowed_out[host[k]] = a[k];
                status[host[k]] = st[k];
            }
        }
        S.last_resolve_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return KETO_OK;
    });
}

int keto_check_batch_ids(keto_snapshot* h, const keto_check_ids* reqs, uint32_t n, int32_t global_max_depth,
                         uint8_t* allowed_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check_host(*h->s, reqs, n, global_max_depth, allowed_out, FORM_HANDLES, 0, nullptr);
        return KETO_OK;
    });
}

int keto_check_batch_rows(keto_snapshot* h, const keto_check_ids* reqs, uint32_t n, int32_t global_max_depth,
                          uint8_t* allowed_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check_host(*h->s, reqs, n, global_max_depth, allowed_out, FORM_ROWS, 0, nullptr);
        return KETO_OK;
    });
}

int keto_check_batch_pairs(keto_snapshot* h, const keto_check_pair* reqs, uint32_t n, int32_t max_depth,
                           int32_t global_max_depth, uint8_t* allowed_out) {
    return guarded([&] {
        if (!h || (n && (!reqs || !allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check_host(*h->s, reqs, n, global_max_depth, allowed_out, FORM_PAIRS, max_depth, nullptr);
        return KETO_OK;
    });
}

int keto_host_alloc(uint64_t bytes, void** out) {
    return guarded([&] {
        if (!out) throw Error{KETO_E_INVALID, "NULL argument"};
        *out = host_alloc(bytes);
        return KETO_OK;
    });
}

void keto_host_free(void* p) { host_free(p); }

int keto_check_batch_device(keto_snapshot* h, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                            uint8_t* d_allowed_out, void* stream) {
    return guarded([&] {
        if (!h || (n && (!d_reqs || !d_allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check(*h->s, d_reqs, n, global_max_depth, d_allowed_out, stream);
        return KETO_OK;
    });
}

int keto_row_handles(const keto_snapshot* h, const uint32_t* rows, uint64_t n, uint32_t* out) {
    return guarded([&] {
        if (!h || (n && (!rows || !out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        const Snapshot& S = *h->s;
        for (uint64_t i = 0; i < n; ++i) {
            if (rows[i] == KETO_NO_ROW) { out[i] = KETO_NO_ROW; continue; }
            if (rows[i] >= S.n_rows()) throw Error{KETO_E_INVALID, "row id out of range"};
            if (!S.present(rows[i])) throw Error{KETO_E_INVALID, "row " + std::to_string(rows[i]) + " is owned by another part"};
            out[i] = S.handle(rows[i]);
        }
        return KETO_OK;
    });
}

int keto_last_batch_timing(const keto_snapshot* h, keto_batch_timing* out) {
    return guarded([&] {
        if (!h || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        *out = device_last_timing(*h->s);
        out->resolve_ms = h->s->last_resolve_ms;
        return KETO_OK;
    });
}

const char* keto_check_kernel_name(int32_t global_max_depth) { return device_check_kernel_name(global_max_depth); }

int keto_check_batch_rows_device(keto_snapshot* h, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                                 uint8_t* d_allowed_out, void* stream) {
    return guarded([&] {
        if (!h || (n && (!d_reqs || !d_allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check_rows(*h->s, d_reqs, n, global_max_depth, d_allowed_out, stream);
        return KETO_OK;
    });
}

extern "C++" {
namespace keto {
void lock_trace(const char* what) {
    static const bool on = getenv("KETO_TRACE_LOCKS") != nullptr;
    if (!on) return;
    const auto t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    fprintf(stderr, "[lk %.3f %zx] %s\n", t, std::hash<std::thread::id>{}(std::this_thread::get_id()) & 0xFFFFFF, what);
}
}  // namespace keto
}  // extern "C++"

int keto_snapshot_apply(keto_snapshot* h, const keto_tuple* inserts, uint64_t n_inserts, const keto_tuple* deletes,
                        uint64_t n_deletes, uint64_t* version_out) {
    return guarded([&] {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        Snapshot& S = *h->s;
        // writes one at a time; a transaction is staged (parsed, merged into its rows' current edges,
        // collision and wildcard effects found -- reads only) under the shared lock, so batches keep
        // running, and committed to the host tables and the device arena under the exclusive one
        std::lock_guard<std::mutex> wl(S.apply_mu);
        lock_trace("apply: apply_mu");
        std::shared_lock<RwGate> rl(S.rw);
        lock_trace("apply: rw shared");
        std::unique_lock<RwGate> xl(S.rw, std::defer_lock);
        // on every exit (a HIP error or KETO_E_REBUILD after the swap included): release the exclusive
        // lock, then free the tables the commit replaced -- apply_mu is still held, retired is ours
        struct Retire {
            Snapshot& S;
            std::unique_lock<RwGate>& xl;
            ~Retire() {
                if (xl.owns_lock()) xl.unlock();
                S.retired.clear();
            }
        } retire{S, xl};
        const auto t0 = std::chrono::steady_clock::now();
        auto t1 = t0;
        apply_writes(S, inserts, n_inserts, deletes, n_deletes, [&] {
            t1 = std::chrono::steady_clock::now();
            rl.unlock();
            lock_trace("apply: staged, waiting for rw exclusive");
            xl.lock();
            lock_trace("apply: rw exclusive");
        });
        const auto t2 = std::chrono::steady_clock::now();
        device_apply(S);
        lock_trace("apply: device_apply done");
        if (getenv("KETO_APPLY_TRACE"))             // tooling: staged (shared lock), then the exclusive part
            fprintf(stderr, "[apply] staged %.3f ms, lock wait %.3f ms, host commit + device %.3f ms\n",
                    std::chrono::duration<double, std::milli>(t1 - t0).count(),
                    std::chrono::duration<double, std::milli>(t2 - t1).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
        if (version_out) *version_out = S.version;
        return KETO_OK;
    });
}

uint64_t keto_snapshot_version(const keto_snapshot* h) { return h ? h->s->version.load() : 0; }

namespace {
int upload_part(keto_snapshot* h, uint32_t part, uint32_t n_parts, int32_t device, uint32_t mode, uint64_t hot_bytes) {
    return guarded([&] {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        Snapshot& S = *h->s;
        if (S.dev) throw Error{KETO_E_INVALID, "snapshot is already on a device (build it with device = -1)"};
        if (n_parts == 0 || part >= n_parts) throw Error{KETO_E_INVALID, "bad part"};
        if (mode != KETO_PART_SHARED && mode != KETO_PART_MIGRATE) throw Error{KETO_E_INVALID, "bad partition mode"};
        if (mode == KETO_PART_MIGRATE && n_parts > KETO_MIG_MAX_PARTS)
            throw Error{KETO_E_INVALID, "a migrating partition has at most 30 parts"};
        S.part = part;
        S.n_parts = n_parts;
        S.part_mode = (int)mode;
        S.hot_bytes = mode == KETO_PART_MIGRATE ? hot_bytes : 0;
        compute_layout(S);
        device_upload(S, device);
        return KETO_OK;
    });
}
}  // namespace

int keto_snapshot_upload_part_mode(keto_snapshot* h, uint32_t part, uint32_t n_parts, int32_t device, uint32_t mode) {
    return upload_part(h, part, n_parts, device, mode, 0);
}

int keto_snapshot_upload_part_migrate(keto_snapshot* h, uint32_t part, uint32_t n_parts, int32_t device,
                                      uint64_t hot_bytes) {
    return upload_part(h, part, n_parts, device, KETO_PART_MIGRATE, hot_bytes);
}

int keto_snapshot_upload_part(keto_snapshot* h, uint32_t part, uint32_t n_parts, int32_t device) {
    return keto_snapshot_upload_part_mode(h, part, n_parts, device, KETO_PART_SHARED);
}

int keto_snapshot_part_stats_mode(keto_snapshot* h, uint32_t part, uint32_t n_parts, uint32_t mode,
                                  keto_part_stats* out) {
    return guarded([&] {
        if (!h || !out || n_parts == 0 || part >= n_parts) throw Error{KETO_E_INVALID, "bad argument"};
        if (mode != KETO_PART_SHARED && mode != KETO_PART_MIGRATE) throw Error{KETO_E_INVALID, "bad partition mode"};
        if (mode == KETO_PART_MIGRATE && n_parts > KETO_MIG_MAX_PARTS)
            throw Error{KETO_E_INVALID, "a migrating partition has at most 30 parts"};
        Snapshot& S = *h->s;
        // lays the snapshot out for the part and back: no other call may read the layout meanwhile
        std::unique_lock<RwGate> xl(S.rw);
        if (S.dev) throw Error{KETO_E_INVALID, "part statistics need a host-only snapshot (device = -1)"};
        const uint32_t p0 = S.part, n0 = S.n_parts;
        const int m0 = S.part_mode;
        S.part = part;
        S.n_parts = n_parts;
        S.part_mode = (int)mode;
        compute_layout(S);
        out->arena_bytes = S.n_words * 4;
        out->shared_bytes = mode == KETO_PART_SHARED ? S.shared_words * 4 : 0;
        out->rows = 0;
        out->shared_rows = 0;
        out->root_rows = 0;
        for (uint32_t r = 0; r < S.n_rows(); ++r) {
            if (!S.present(r)) continue;
            ++out->rows;
            if (S.is_root[r]) ++out->root_rows;
            else if (mode == KETO_PART_SHARED) ++out->shared_rows;
        }
        out->stub_rows = S.n_stubs;
        if (mode == KETO_PART_MIGRATE) {                 // the replicated hot prefix
            out->shared_rows = (uint32_t)S.hot_rows;
            out->shared_bytes = (uint64_t)S.hot_units * HDR_WORDS * 4;
        }
        S.part = p0;
        S.n_parts = n0;
        S.part_mode = m0;
        compute_layout(S);
        return KETO_OK;
    });
}

int keto_snapshot_part_stats(keto_snapshot* h, uint32_t part, uint32_t n_parts, keto_part_stats* out) {
    return keto_snapshot_part_stats_mode(h, part, n_parts, KETO_PART_SHARED, out);
}

int64_t keto_part_stubs(const keto_snapshot* h, uint32_t* rows_out, uint64_t cap) {
    return guarded([&]() -> int64_t {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        const Snapshot& S = *h->s;
        if (S.part_mode != PART_MIGRATE || S.stub.empty()) return 0;
        uint64_t k = 0;
        for (uint32_t r = 0; r < S.n_rows(); ++r) {
            if (!S.stub[r]) continue;
            if (rows_out && k < cap) rows_out[k] = r;
            ++k;
        }
        return (int64_t)k;
    });
}

int keto_part_filters(keto_snapshot* h, const uint32_t* rows, uint64_t n, uint32_t* filters_out) {
    return guarded([&] {
        if (!h || (n && (!rows || !filters_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        part_filters(*h->s, rows, n, filters_out);
        return KETO_OK;
    });
}

int keto_part_close(keto_snapshot* h, const uint32_t* stub_rows, uint64_t n, const uint32_t* filters,
                    uint64_t* changed_out) {
    return guarded([&] {
        if (!h || (n && (!stub_rows || !filters))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::unique_lock<RwGate> xl(h->s->rw);          // rewrites the part's filters
        const uint64_t c = part_close(*h->s, stub_rows, n, filters);
        if (changed_out) *changed_out = c;
        return KETO_OK;
    });
}

int keto_part_closure_done(keto_snapshot* h, int converged) {
    return guarded([&] {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        std::unique_lock<RwGate> xl(h->s->rw);
        if (h->s->part_mode != PART_MIGRATE) throw Error{KETO_E_INVALID, "not a migrating part"};
        part_closure_done(*h->s, converged != 0);
        return KETO_OK;
    });
}

namespace {
void copy_out(const MigOut& m, keto_mig_out* out) {
    for (uint32_t p = 0; p < KETO_MIG_MAX_PARTS; ++p) {
        out->units[p] = m.units[p];
        out->records[p] = m.records[p];
    }
    out->d_records = m.d_buf;
    out->d_offsets = m.d_off;
    out->decided = m.decided;
    out->undecided = m.undecided;
    out->processed = m.processed;
    out->reruns = m.reruns;
}
}  // namespace

int keto_mig_begin(keto_snapshot* h, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                   uint8_t* d_allowed_out, void* stream, keto_mig_out* out) {
    return guarded([&] {
        if (!h || !out) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        MigOut m{};
        mig_begin(*h->s, d_reqs, n, global_max_depth, d_allowed_out, stream, m);
        copy_out(m, out);
        return KETO_OK;
    });
}

int keto_device_memory(int32_t device, uint64_t* free_out, uint64_t* total_out) {
    return guarded([&] {
        if (!free_out || !total_out) throw Error{KETO_E_INVALID, "NULL argument"};
        if (device < 0) throw Error{KETO_E_INVALID, "no device " + std::to_string(device)};
        device_memory(device, *free_out, *total_out);
        return KETO_OK;
    });
}

int keto_device_copy(void* dst, const void* src, uint64_t bytes, void* stream) {
    return guarded([&] {
        if (bytes && (!dst || !src)) throw Error{KETO_E_INVALID, "NULL argument"};
        device_copy(dst, src, bytes, stream);
        return KETO_OK;
    });
}

int keto_mig_round(keto_snapshot* h, const void* d_records, const uint32_t* d_offsets, const uint32_t* in_records,
                   const uint64_t* in_units, void* stream, keto_mig_out* out) {
    return guarded([&] {
        if (!h || !out || !in_records || !in_units) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        MigOut m{};
        mig_round(*h->s, d_records, d_offsets, in_records, in_units, stream, m);
        copy_out(m, out);
        return KETO_OK;
    });
}

uint64_t keto_route_work_bytes(uint32_t n, uint32_t n_parts) { return route_work_bytes(n, n_parts); }

int keto_route_rows_device(const keto_check_ids* d_reqs, uint32_t n, const int16_t* d_owner, uint32_t n_rows,
                           uint32_t self_part, uint32_t n_parts, void* d_work, uint64_t work_bytes,
                           keto_check_ids* d_send, uint32_t* d_order, uint32_t* counts_out, void* stream) {
    return guarded([&] {
        if (!counts_out || (n && (!d_reqs || !d_owner || !d_work || !d_send || !d_order)))
            throw Error{KETO_E_INVALID, "NULL argument"};
        route_rows(d_reqs, n, d_owner, n_rows, self_part, n_parts, d_work, work_bytes, d_send, d_order, counts_out,
                   stream);
        return KETO_OK;
    });
}

int keto_unroute_device(const uint8_t* d_back, const uint32_t* d_order, uint32_t n, uint8_t* d_out, void* stream) {
    return guarded([&] {
        if (n && (!d_back || !d_order || !d_out)) throw Error{KETO_E_INVALID, "NULL argument"};
        unroute_rows(d_back, d_order, n, d_out, stream);
        return KETO_OK;
    });
}

int keto_row_owner(const keto_snapshot* h, const uint32_t* rows, uint64_t n, uint32_t n_parts, int32_t* out) {
    return guarded([&] {
        if (!h || (n && (!rows || !out)) || n_parts == 0) throw Error{KETO_E_INVALID, "bad argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        const Snapshot& S = *h->s;
        for (uint64_t i = 0; i < n; ++i) {
            if (rows[i] == KETO_NO_ROW) { out[i] = -1; continue; }
            if (rows[i] >= S.n_rows()) throw Error{KETO_E_INVALID, "row id out of range"};
            out[i] = S.row_owner(rows[i], n_parts);
        }
        return KETO_OK;
    });
}

int keto_check_work_device(keto_snapshot* h, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                           uint8_t* d_allowed_out, uint64_t out[KETO_WORK_SLOTS]) {
    return guarded([&] {
        if (!h || !out || (n && (!d_reqs || !d_allowed_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        device_check(*h->s, d_reqs, n, global_max_depth, d_allowed_out, nullptr, out);
        return KETO_OK;
    });
}

int keto_check_steps_device(keto_snapshot* h, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                            uint8_t* d_allowed_out, uint32_t* d_steps) {
    return guarded([&] {
        if (!h || (n && (!d_reqs || !d_allowed_out || !d_steps))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        uint64_t w[KETO_WORK_SLOTS];
        device_check(*h->s, d_reqs, n, global_max_depth, d_allowed_out, nullptr, w, d_steps);
        return KETO_OK;
    });
}

extern "C++" {
namespace keto {
// keto_expand_batch's body (the caller holds the snapshot's lock shared); skip[i] != 0: request i is
// answered elsewhere (comm.cpp routes it to the part owning its root row) and gets an empty slot
void expand_named(Snapshot& S, const keto_expand_req* reqs, uint32_t n, int32_t global_max_depth, keto_tree_arena& A,
                  const uint8_t* skip) {
    keto_tree_arena* a = &A;
    Overlay ov;
    ov.base = S.n_rows();
    a->ov_base = ov.base;
    a->extra_base = (uint32_t)S.strs.size();
    std::vector<uint32_t> root(n), flags(n), vid(n, 0), rrow(n, KETO_NO_ROW);
    std::vector<int32_t> depth(n);
    std::vector<uint8_t> not_found(n, 0);
    std::vector<std::pair<uint32_t, uint32_t>> remote;                  // (request, row) of other parts
    for (uint32_t i = 0; i < n; ++i) {
        const keto_subject& sj = reqs[i].subject;
        depth[i] = reqs[i].max_depth;
        if (skip && skip[i]) {                                          // answered on another part
            root[i] = KETO_NO_ROW;
            flags[i] = 1;
            continue;
        }
        if (sj.kind == 0) {                                             // SubjectID -> Leaf
            int64_t sid = S.lookup_str(sv(sj.id));
            if (sid < 0) {
                sid = a->extra_base + a->extra.size();
                a->extra.emplace_back(sv(sj.id));
            }
            root[i] = (uint32_t)sid;
            flags[i] = 0;
            continue;
        }
        flags[i] = 1;
        RowKey k;
        int64_t r = S.resolve_query(sv(sj.set_namespace), sv(sj.set_object), sv(sj.set_relation), &k);
        if (r == -2) {
            not_found[i] = 1;
            root[i] = KETO_NO_ROW;
        } else if (r == -1) {
            root[i] = KETO_NO_ROW;
        } else if (r == -3) {
            root[i] = handle_of(S, &ov, overlay_row(S, ov, k));
            std::string key = std::string(sv(sj.set_namespace)) + ":" + std::string(sv(sj.set_object)) + "#" +
                              std::string(sv(sj.set_relation));
            vid[i] = S.vid_of_key(key);
        } else if (!S.present((uint32_t)r)) {
            // another part's row: a migrating part copies it in (device_expand); a shared-rows part
            // routes it to its owner (keto_expand_batch_routed) and never gets here with it
            if (!(S.part_mode == PART_MIGRATE && S.n_parts > 1))
                throw Error{KETO_E_INVALID, "expand root is owned by another part"};
            remote.emplace_back(i, (uint32_t)r);
            root[i] = KETO_NO_ROW;
        } else {
            root[i] = S.handle((uint32_t)r);
            vid[i] = S.vid_of_row((uint32_t)r);
            rrow[i] = (uint32_t)r;
        }
    }
    a->ov_keys = ov.keys;
    device_expand(S, root, flags, vid, depth, global_max_depth, &ov, a->r, &remote, &rrow);
    for (uint32_t i = 0; i < n; ++i)
        if (not_found[i]) a->r.status[i] = KETO_EXPAND_NOT_FOUND;
}
}  // namespace keto
}  // extern "C++"

int keto_expand_batch(keto_snapshot* h, const keto_expand_req* reqs, uint32_t n, int32_t global_max_depth,
                      keto_tree_arena** out) {
    return guarded([&] {
        if (!h || !out || (n && !reqs)) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        *out = nullptr;
        auto a = std::make_unique<keto_tree_arena>();
        expand_named(*h->s, reqs, n, global_max_depth, *a, nullptr);
        *out = a.release();
        return KETO_OK;
    });
}

int keto_expand_batch_ids(keto_snapshot* h, const uint32_t* roots, const int32_t* max_depth, uint32_t n,
                          int32_t global_max_depth, keto_tree_arena** out) {
    return guarded([&] {
        if (!h || !out || (n && (!roots || !max_depth))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        *out = nullptr;
        Snapshot& S = *h->s;
        auto a = std::make_unique<keto_tree_arena>();
        a->extra_base = (uint32_t)S.strs.size();
        std::vector<uint32_t> root(n), flags(n), vid(n, 0), rrow(n, KETO_NO_ROW);
        std::vector<int32_t> depth(max_depth, max_depth + n);
        for (uint32_t i = 0; i < n; ++i) {
            const bool set = (roots[i] & EDGE_SET) != 0;
            root[i] = roots[i] & EDGE_VAL;
            flags[i] = set ? 1u : 0u;
            if (set) {
                if (root[i] >= S.n_rows()) throw Error{KETO_E_INVALID, "root row out of range"};
                if (!S.present(root[i])) throw Error{KETO_E_INVALID, "expand root is owned by another part"};
                vid[i] = S.vid_of_row(root[i]);
                rrow[i] = root[i];
                root[i] = S.handle(root[i]);
            }
        }
        device_expand(S, root, flags, vid, depth, global_max_depth, nullptr, a->r, nullptr, &rrow);
        *out = a.release();
        return KETO_OK;
    });
}

void keto_tree_arena_free(keto_tree_arena* a) { delete a; }

uint32_t keto_tree_count(const keto_tree_arena* a) { return a ? (uint32_t)a->r.status.size() : 0; }

int keto_tree_status(const keto_tree_arena* a, uint32_t i) {
    if (!a || i >= a->r.status.size()) return KETO_E_INVALID;
    return a->r.status[i];
}

const keto_tree_node* keto_tree_nodes(const keto_tree_arena* a, uint32_t i, uint64_t* n_nodes) {
    if (n_nodes) *n_nodes = 0;
    if (!a || i >= a->r.status.size() || a->r.status[i] != KETO_EXPAND_TREE) return nullptr;
    uint64_t b = a->r.offset[i], e = a->r.offset[i + 1];
    if (n_nodes) *n_nodes = e - b;
    return a->r.nodes.data() + b;
}

// The tree encoders read the snapshot's strings and row keys, which keto_snapshot_apply extends
// (push_back may reallocate): they hold the snapshot's lock shared, like the batch calls.
int64_t keto_tree_json(const keto_snapshot* h, const keto_tree_arena* a, uint32_t i, char* buf, uint64_t cap) {
    return guarded([&]() -> int64_t {
        if (!h || !a || i >= a->r.status.size()) throw Error{KETO_E_INVALID, "bad argument"};
        if (a->r.status[i] == KETO_EXPAND_NOT_FOUND) throw Error{KETO_E_INVALID, "Unknown namespace"};
        if (a->r.status[i] == KETO_EXPAND_UNDECIDED)
            throw Error{KETO_E_RANGE, "the tree exceeds the engine's limits (KETO_EXPAND_UNDECIDED)"};
        std::string o;
        if (a->r.status[i] != KETO_EXPAND_TREE) {
            o = "null";
        } else {
            std::shared_lock<RwGate> lk(h->s->rw);
            const uint64_t b = a->r.offset[i], e = a->r.offset[i + 1];
            tree_json(*h->s, a, a->r.nodes.data() + b, e - b, o);
        }
        return copy_out(o, buf, cap);
    });
}

extern "C++" {
// Every tree of the arena encoded on host threads by `one(i, out)`, into buf at offsets (see
// keto_tree_json_all / keto_tree_proto_all).  A call whose buf cannot take the total keeps the
// encodings in the arena for the next call of the same kind on the same snapshot version.
template <class One>
int64_t encode_all(const keto_snapshot* h, const keto_tree_arena* a, int kind, char* buf, uint64_t cap,
                   uint64_t* offsets, One one) {
    const uint32_t n = (uint32_t)a->r.status.size();
    const unsigned th = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::shared_lock<RwGate> rlk(h->s->rw);      // before enc_mu: apply takes rw alone
    std::lock_guard<std::mutex> lk(a->enc_mu);
    std::vector<std::string>& enc = a->enc;
    if (!(a->enc_kind == kind && a->enc_uid == h->s->uid && a->enc_version == h->s->version && enc.size() == n)) {
        enc.assign(n, std::string());
        std::vector<std::thread> ts;
        std::atomic<uint32_t> next{0};
        for (unsigned t = 0; t < th; ++t)
            ts.emplace_back([&] {
                for (;;) {
                    const uint32_t k = next.fetch_add(64);
                    if (k >= n) break;
                    for (uint32_t i = k; i < std::min(n, k + 64); ++i) one(i, enc[i]);
                }
            });
        for (auto& x : ts) x.join();
    }
    offsets[0] = 0;
    for (uint32_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + enc[i].size();
    const int64_t total = (int64_t)offsets[n];
    if (buf && cap >= offsets[n]) {
        par_chunks(n, offsets[n] >= (8u << 20) ? th : 1u, 256, [&](uint64_t b, uint64_t e, unsigned) {
            for (uint64_t i = b; i < e; ++i) std::memcpy(buf + offsets[i], enc[i].data(), enc[i].size());
        });
        std::vector<std::string>().swap(enc);          // written: drop the cache
        a->enc_kind = 0;
    } else {
        a->enc_kind = kind;
        a->enc_uid = h->s->uid;
        a->enc_version = h->s->version;
    }
    return total;
}
}  // extern "C++"

int64_t keto_tree_json_all(const keto_snapshot* h, const keto_tree_arena* a, char* buf, uint64_t cap,
                           uint64_t* offsets) {
    return guarded([&]() -> int64_t {
        if (!h || !a || !offsets) throw Error{KETO_E_INVALID, "NULL argument"};
        return encode_all(h, a, 1, buf, cap, offsets, [&](uint32_t i, std::string& o) {
            const int st = a->r.status[i];
            if (st == KETO_EXPAND_TREE) {
                const uint64_t b = a->r.offset[i], e = a->r.offset[i + 1];
                tree_json(*h->s, a, a->r.nodes.data() + b, e - b, o);
            } else if (st != KETO_EXPAND_NOT_FOUND && st != KETO_EXPAND_UNDECIDED) {
                o = "null";
            }
        });
    });
}

int64_t keto_tree_proto(const keto_snapshot* h, const keto_tree_arena* a, uint32_t i, uint8_t* buf, uint64_t cap) {
    return guarded([&]() -> int64_t {
        if (!h || !a || i >= a->r.status.size()) throw Error{KETO_E_INVALID, "bad argument"};
        const int st = a->r.status[i];
        if (st == KETO_EXPAND_NOT_FOUND) throw Error{KETO_E_INVALID, "Unknown namespace"};
        if (st == KETO_EXPAND_UNDECIDED) throw Error{KETO_E_RANGE, "the tree exceeds the engine's limits"};
        if (st != KETO_EXPAND_TREE) return 0;                     // nil tree: no message
        std::string o;
        {
            std::shared_lock<RwGate> lk(h->s->rw);
            const uint64_t b = a->r.offset[i], e = a->r.offset[i + 1];
            tree_proto(*h->s, a, a->r.nodes.data() + b, e - b, o);
        }
        if (buf && cap) std::memcpy(buf, o.data(), std::min<uint64_t>(cap, o.size()));
        return (int64_t)o.size();
    });
}

int64_t keto_tree_proto_all(const keto_snapshot* h, const keto_tree_arena* a, uint8_t* buf, uint64_t cap,
                            uint64_t* offsets) {
    return guarded([&]() -> int64_t {
        if (!h || !a || !offsets) throw Error{KETO_E_INVALID, "NULL argument"};
        return encode_all(h, a, 2, reinterpret_cast<char*>(buf), cap, offsets, [&](uint32_t i, std::string& o) {
            if (a->r.status[i] == KETO_EXPAND_TREE) {
                const uint64_t b = a->r.offset[i], e = a->r.offset[i + 1];
                tree_proto(*h->s, a, a->r.nodes.data() + b, e - b, o);
            }
        });
    });
}

int64_t keto_tree_proto_all_device(keto_snapshot* h, const keto_tree_arena* a, uint8_t* buf, uint64_t cap,
                                   uint64_t* offsets) {
    return guarded([&]() -> int64_t {
        if (!h || !a || !offsets) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> rlk(h->s->rw);    // strings / row keys (before S.mu)
        const uint32_t n = (uint32_t)a->r.status.size();
        // the nodes of the trees (other statuses have none), tree t = [toff[t], toff[t + 1])
        std::vector<uint64_t> toff(n + 1, 0);
        bool all = true;
        for (uint32_t i = 0; i < n; ++i) {
            const bool tree = a->r.status[i] == KETO_EXPAND_TREE;
            all &= tree || a->r.offset[i] == a->r.offset[i + 1];
        }
        std::vector<keto_tree_node> sel;
        const keto_tree_node* nodes = a->r.nodes.data();
        uint64_t n_nodes = a->r.nodes.size();
        if (all) {
            for (uint32_t i = 0; i <= n; ++i) toff[i] = a->r.offset[i];
        } else {
            for (uint32_t i = 0; i < n; ++i) {
                toff[i] = sel.size();
                if (a->r.status[i] == KETO_EXPAND_TREE)
                    sel.insert(sel.end(), a->r.nodes.begin() + a->r.offset[i], a->r.nodes.begin() + a->r.offset[i + 1]);
            }
            toff[n] = sel.size();
            nodes = sel.data();
            n_nodes = sel.size();
        }
        return (int64_t)device_tree_proto(*h->s, nodes, n_nodes, toff.data(), n, a->ov_base, a->ov_keys, a->extra_base,
                                          a->extra, buf, cap, offsets);
    });
}

int64_t keto_subject_fields(const keto_snapshot* h, const keto_tree_arena* a, const uint32_t* subjects, uint64_t n,
                            char* buf, uint64_t cap, uint32_t* lens_out) {
    return guarded([&]() -> int64_t {
        if (!h || (n && (!subjects || !lens_out))) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        const Snapshot& S = *h->s;
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t ref = subjects[i];
            if ((ref & EDGE_SET) && (ref & EDGE_VAL) >= S.n_rows() &&
                !(a && (ref & EDGE_VAL) >= a->ov_base && (ref & EDGE_VAL) - a->ov_base < a->ov_keys.size()))
                throw Error{KETO_E_INVALID, "subject reference " + std::to_string(i) + " names no row"};
            const SubjectViews f = views_of(S, a, ref);
            if (!f.set) {
                lens_out[3 * i] = (uint32_t)f.id.size();
                lens_out[3 * i + 1] = lens_out[3 * i + 2] = 0;
                total += f.id.size();
            } else {
                lens_out[3 * i] = (uint32_t)f.ns.size();
                lens_out[3 * i + 1] = (uint32_t)f.obj.size();
                lens_out[3 * i + 2] = (uint32_t)f.rel.size();
                total += f.ns.size() + f.obj.size() + f.rel.size();
            }
        }
        if (buf && cap >= total) {
            char* p = buf;
            auto put = [&](std::string_view v) {
                std::memcpy(p, v.data(), v.size());
                p += v.size();
            };
            for (uint64_t i = 0; i < n; ++i) {
                const SubjectViews f = views_of(S, a, subjects[i]);
                if (!f.set) {
                    put(f.id);
                } else {
                    put(f.ns);
                    put(f.obj);
                    put(f.rel);
                }
            }
        }
        return (int64_t)total;
    });
}

int64_t keto_subject_string(const keto_snapshot* h, uint32_t subject, char* buf, uint64_t cap) {
    return guarded([&]() -> int64_t {
        if (!h) throw Error{KETO_E_INVALID, "NULL argument"};
        std::shared_lock<RwGate> lk(h->s->rw);
        SubjectFields f = fields_of(*h->s, nullptr, subject);
        return copy_out(f.set ? f.ns + ":" + f.obj + "#" + f.rel : f.id, buf, cap);
    });
}

}  // extern "C"
