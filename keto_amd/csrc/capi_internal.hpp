// Shared by the C-ABI translation units (capi.cpp, comm.cpp): the opaque snapshot handle, the
// per-thread last error behind keto_last_error, and the exception guard every entry point runs in.
#pragma once

#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "snapshot.hpp"

struct keto_snapshot {
    std::unique_ptr<keto::Snapshot> s;
};

struct keto_tree_arena {
    keto::ExpandResult r;
    uint32_t ov_base = 0xFFFFFFFFu;
    std::vector<keto::RowKey> ov_keys;     // overlay roots (wildcard queries)
    uint32_t extra_base = 0;               // subject-id strings not in the snapshot
    std::vector<std::string> extra;
    // keto_tree_json_all / keto_tree_proto_all: the encodings of a sizing call (buf too small), kept
    // for the filling call that follows it, so a size-then-fill pair encodes once
    mutable std::mutex enc_mu;
    mutable int enc_kind = 0;              // 0 none, 1 JSON, 2 protobuf
    mutable uint64_t enc_uid = 0;          // the snapshot the encodings were made with (Snapshot::uid)
    mutable uint64_t enc_version = 0;
    mutable std::vector<std::string> enc;
};

namespace keto {

extern thread_local std::string g_err;   // keto_last_error

// runs an entry point's body: keto::Error -> its code, bad_alloc -> KETO_E_NOMEM, other exceptions
// -> KETO_E_INVALID, with the message kept for keto_last_error; nothing crosses the C boundary
template <class F>
auto guarded(F&& f) -> decltype(f()) {
    try {
        g_err.clear();
        return f();
    } catch (const Error& e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return KETO_E_NOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return KETO_E_INVALID;
    }
}

// resolve_checks over a whole batch on host threads (capi.cpp); by_row as in resolve_checks
std::vector<WildReq> resolve_all(const Snapshot& S, const keto_check_req* reqs, uint32_t n, keto_check_ids* ids,
                                 uint8_t* st, bool by_row = false);

// keto_check_batch's body, the caller holding the snapshot's lock shared (capi.cpp)
void check_named(Snapshot& S, const keto_check_req* reqs, uint32_t n, int32_t global_max_depth, uint8_t* allowed_out,
                 uint8_t* status_out);

// keto_expand_batch's body, the caller holding the snapshot's lock shared (capi.cpp); skip[i] != 0:
// request i is answered by another part (an empty slot here)
void expand_named(Snapshot& S, const keto_expand_req* reqs, uint32_t n, int32_t global_max_depth, keto_tree_arena& a,
                  const uint8_t* skip);

}  // namespace keto
