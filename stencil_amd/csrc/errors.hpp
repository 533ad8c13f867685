// errors.hpp -- the library's per-thread error state (include/stencil_hip.h's
// stencil_last_error / stencil_last_error_message), HIP-free so that host-only
// code (slab_core.hpp and its CPU test build) can report errors the same way.
#pragma once

#include "stencil_hip.h"

namespace stencil {

// Record an error for stencil_last_error_message(); returns `code`.
int set_error(int code, const char* fmt, ...);
// Clear the per-thread error state (success).
void clear_error();

}  // namespace stencil
