// knobs.cpp -- environment knobs of libstencil_hip.so (see common.hpp).
//
// Compiled twice: into the product library without STENCIL_DEBUG_KNOBS, where
// knob() ignores the environment (the library runs AUTO's plan and nothing
// else), and with it into libstencil_hip_debug.so, the build the shape-sweep
// parity tests and the A/B tools load to select workgroup shapes, forced
// z-chunks and kernel families.  api_knob() reads the variables
// include/stencil_hip.h documents in both.
#include <cstdlib>

#include "common.hpp"

namespace stencil {

static int env_or(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return s && *s ? std::atoi(s) : dflt;
}

int knob(const char* name, int dflt) {
#ifdef STENCIL_DEBUG_KNOBS
    return env_or(name, dflt);
#else
    (void)name;
    return dflt;
#endif
}

int api_knob(const char* name, int dflt) { return env_or(name, dflt); }

#ifndef STENCIL_DEBUG_KNOBS
// The box code-generation probe (kernels_boxk_probe.hip, debug cfgs 95RRNN /
// 96RRNN) is linked into the debug library only; the product library gets
// these stubs, which its AUTO plan never reaches.
int launch_boxk_probe_slp(const stencil_layout&, const void*, void*, int64_t, int64_t, int, int, hipStream_t) {
    return set_error(STENCIL_EUNSUPPORTED, "the box probe shapes are in libstencil_hip_debug.so only");
}
int launch_boxk_probe_noslp(const stencil_layout&, const void*, void*, int64_t, int64_t, int, int, hipStream_t) {
    return set_error(STENCIL_EUNSUPPORTED, "the box probe shapes are in libstencil_hip_debug.so only");
}
int launch_tkstrip_probe(const stencil_layout&, const void*, void*, int64_t, int64_t, int, hipStream_t) {
    return set_error(STENCIL_EUNSUPPORTED, "the strip probe shapes are in libstencil_hip_debug.so only");
}
#endif

}  // namespace stencil

// which build this is (tests: the shape-sweep tests must run on the debug one)
extern "C" int stencil_debug_knobs(void) {
#ifdef STENCIL_DEBUG_KNOBS
    return 1;
#else
    return 0;
#endif
}
