// gpad_abi.h -- the host runtime's C-ABI boundary helper (gpad_host.cpp, gpad_group.cpp,
// gpad_io.cpp).
#pragma once

#include <exception>
#include <new>
#include <string>

#include "../../include/gpad.h"
#include "gpad_internal.h"

namespace gpad {

// Every int-returning C-ABI entry point runs its body through abi_guard: no C++ exception (a
// std::bad_alloc of a host buffer sized from caller dims or a corrupted data file, a
// std::length_error) crosses the extern "C" boundary -- it becomes GPAD_ERR_NOMEM / GPAD_ERR_INVALID
// with the reason in gpad_last_error() instead of std::terminate.
template <class F>
int abi_guard(const char* where, F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return set_last_error(GPAD_ERR_NOMEM, std::string(where) + ": host allocation failed");
    } catch (const std::exception& e) {
        return set_last_error(GPAD_ERR_INVALID, std::string(where) + ": " + e.what());
    } catch (...) {
        return set_last_error(GPAD_ERR_INVALID, std::string(where) + ": unknown C++ exception");
    }
}

}  // namespace gpad
