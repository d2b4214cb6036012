// nrc_guard.h — error plumbing shared by the C-ABI translation units: exceptions never cross the ABI;
// guarded() maps them to nrc_status and keeps the message for nrc_last_error() (thread-local).
#pragma once

#include <stdexcept>
#include <string>

#include <hip/hip_runtime_api.h>

#include "nrc/nrc_c.h"

namespace nrc_amd {

inline thread_local std::string g_last_error;

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct ApiError : std::runtime_error {
    nrc_status code;
    ApiError(nrc_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            throw HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " (" + __FILE__ + ":" + \
                           std::to_string(__LINE__) + ")");                                          \
    } while (0)

template <class F>
nrc_status guarded(F&& f) {
    try {
        f();
        g_last_error.clear();
        return NRC_OK;
    } catch (const ApiError& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const HipError& e) {
        g_last_error = e.what();
        return NRC_ERR_HIP;
    } catch (const std::bad_alloc& e) {
        g_last_error = "out of host memory";
        return NRC_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return NRC_ERR_INTERNAL;
    } catch (...) {
        g_last_error = "unknown error";
        return NRC_ERR_INTERNAL;
    }
}

}  // namespace nrc_amd
