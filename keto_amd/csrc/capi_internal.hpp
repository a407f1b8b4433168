// Shared by the C-ABI translation units (capi.cpp, comm.cpp): the opaque snapshot handle, the
// per-thread last error behind keto_last_error, and the exception guard every entry point runs in.
#pragma once

#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "snapshot.hpp"

struct keto_snapshot {
    std::unique_ptr<keto::Snapshot> s;
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

}  // namespace keto
