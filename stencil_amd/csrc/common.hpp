// common.hpp -- shared device/host definitions for libstencil_hip.so (gfx950).
//
// Everything here is internal to the library; the public boundary is
// include/stencil_hip.h.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <functional>

#include "errors.hpp"
#include "stencil_hip.h"

namespace stencil {

// Geometry handed to kernels by value (SGPR-resident).
struct Geom {
    int64_t nx, ny, nz;  // interior extents (nz = 1 for 2D)
    int64_t row;         // row stride (elements)
    int64_t plane;       // plane stride (elements)
    int64_t origin;      // element offset of interior (0,0,0)
};

inline Geom geom_of(const stencil_layout& l) {
    return Geom{l.prob.nx, l.prob.ny, l.prob.nz, l.row, l.plane, l.origin};
}

// Workgroup slots of `kern` (launched with `threads` threads) on the CURRENT
// device: CUs x resident workgroups per CU (one_per_cu: CUs only).  Cached
// per (device, kernel) under a lock -- one process may drive several GPUs
// from several threads (stencil_set_device is per thread).
int resident_slots(const void* kern, int threads, bool one_per_cu, int* slots);
template <typename F>
inline int resident_slots(F* kern, int threads, int* slots) {
    return resident_slots(reinterpret_cast<const void*>(kern), threads, false, slots);
}

#define STENCIL_HIP_CHECK(expr)                                                              \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return ::stencil::set_error(STENCIL_EHIP, "%s failed: %s (%s:%d)", #expr,        \
                                        hipGetErrorString(e_), __FILE__, __LINE__);          \
    } while (0)

#define STENCIL_LAUNCH_CHECK()                                                               \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess)                                                                \
            return ::stencil::set_error(STENCIL_EHIP, "kernel launch failed: %s (%s:%d)",    \
                                        hipGetErrorString(e_), __FILE__, __LINE__);          \
    } while (0)

// Averaging weight, computed on the host in the element type so the IEEE
// division is the same correctly-rounded one the reference performs
// (stencil.cpp:85-86: 1.f / float((bw + bh) * 2)).
template <typename T>
inline T avg_weight(const stencil_problem& p) {
    if (p.shape == STENCIL_BOX) {
        int64_t w = 2 * int64_t(p.radius) + 1, n = w * w;
        if (p.dims == 3) n *= w;
        return T(1) / T(n - 1);
    }
    return T(1) / T(2 * p.dims * p.radius);
}

// Launch geometry of the K-step strip kernel, filled instead of launching
// while a LaunchInfo is installed for the calling thread
// (stencil_sweepk_geometry).
struct LaunchInfo {
    int64_t workgroups = 0;
    int zchunk = 0;   // planes per z-chunk; 0 = one balanced share per workgroup
    int packed = 0;   // 0 equal chunks, 1 packed (measured faster), 2 packed by the model, not yet measured
    int steps = 0;
    int slots = 0;    // resident workgroups of the kernel on the device (one round)
};
extern thread_local LaunchInfo* tl_dry_launch;

// Jobs long enough to run at the package power limit (the C2
// job's launches slow by ~7 % once the limiter engages, ~20 ms into
// continuous load) take the energy-saving work orders: the packed z-chunk
// tables in XCD patches (fewer fabric bytes per cell, slower by ~1 % below
// the limit, faster at it).  stencil_iterate and stencil_slab_run set the
// hint for the calling thread when a call covers kSustainedSweeps or more.
constexpr uint32_t kSustainedSweeps = 256;
extern thread_local bool tl_sustained;
struct SustainedScope {
    bool prev;
    explicit SustainedScope(bool on) : prev(tl_sustained) { tl_sustained = on; }
    ~SustainedScope() { tl_sustained = prev; }
};

// A face-signalled slab launch's geometry (a dry launch: nothing runs):
// x-y tiles, workgroups and one round's resident slots.  slab.hip confines a
// job's exchange to a few CUs when the launch beside it takes several rounds
// of workgroups (slab_core.hpp).
int signal_launch_geometry(const stencil_layout& l, int64_t begin, int64_t end, int steps, int64_t* tiles,
                           int64_t* workgroups, int* slots);

// The packed longest-first z-chunk schedule (kernels_strip.hip): for a grid of
// few tiles, chunks of Lc planes per tile (the last one shorter) dispatched
// longest first, Lc chosen by simulating the dispatcher with `fill` steps of
// pipeline fill per chunk; a device table of {tile, first plane, planes} per
// workgroup when it beats equal chunks of zc planes, else *sched untouched.
// The cache is keyed by the kernel itself (one instantiation: dtype and shape)
// and the device.  *verdict (when asked for) points at the shape's measured
// choice: kPackUntested until pick_schedule has timed both grids on this
// device, then kPackPacked or kPackEqual.  The table is searched on the host
// and uploaded on the first real launch on `s` (stream-ordered, one host
// wait); `dry` (stencil_sweepk_geometry) and launches into a capturing stream
// upload nothing -- a capturing launch runs equal chunks -- and a dry call
// reports a table that would be used through *sched = kDrySchedule.
enum { kPackUntested = 0, kPackPacked = 1, kPackEqual = 2 };
extern const int* const kDrySchedule;
// faces_out (face-signalled slab launches): each tile's first full chunk
// starts at plane 0 marching up and its last full chunk ends at the top
// marching down (planes < 0 in the table), the short remainder in between,
// so both faces lie in chunks of the first dispatch round; no table unless a
// tile has at least 3 chunks.
// xcd_w > 0 (tiles_x: the tile grid's width): within every generation of
// equal chunks (same length and first plane) the table's entries are
// reordered so that the workgroups the dispatcher deals to one XCD
// (workgroup i -> XCD i % 8) hold a compact 2D patch of tiles -- column
// strips of xcd_w tiles cut into 8 runs -- and neighbouring tiles' shared
// halo lines become hits in that XCD's L2 (xcd_patch_order).  Same lengths
// at the same positions: the same makespan.
int packed_schedule(const void* kern, int dev, int64_t tiles, int64_t nz, int K, int fill, int slots, int zc,
                    hipStream_t s, bool dry, const int** sched, int64_t* nb, std::atomic<int>** verdict = nullptr,
                    bool faces_out = false, int64_t tiles_x = 0, int xcd_w = 0);

// The dispatcher model behind packed_schedule mispredicts some shapes badly
// (measured: 504 x 512 x 512 fp64 packed 0.555 vs equal 0.450 ms per launch,
// 256^3 -17 %, 448^3 -7 %, while 512^3 gains 8 %; profiles/r02gg_pack.log),
// so the first launch of a shape times both grids on the caller's stream and
// keeps the faster one.  launch(packed) enqueues ONE launch of the same
// sweep (same in, same out: every trial writes identical bits).  Runs
// 3 x (packed, equal) launches, blocks the host once for the events, records
// the verdict.  On a capturing stream nothing is timed: the model's choice
// is launched once (*launched = true either way unless an error is returned).
int pick_schedule(std::atomic<int>* verdict, hipStream_t s, const std::function<hipError_t(bool)>& launch);
// STENCIL_TK_PACK / STENCIL_BOXK_PACK: 0 = equal chunks, 1 = measured choice
// (default), 2 = the model's choice without measuring

// Environment knobs.  api_knob: the few include/stencil_hip.h documents
// (STENCIL_TK_STEPS, STENCIL_BOX_STEPS, STENCIL_TK_PACK, STENCIL_BOXK_PACK,
// STENCIL_SLAB_SIGNAL), read in every build.  knob: the experiment selectors
// (workgroup shapes, forced z-chunks and kernel families, diagnostics) -- read
// only by the debug library (knobs.cpp built with -DSTENCIL_DEBUG_KNOBS into
// stencil_amd/libstencil_hip_debug.so, which the shape-sweep tests load); in
// the product library knob() returns `dflt`, so it runs AUTO's plan and
// nothing else.
int knob(const char* name, int dflt);
int api_knob(const char* name, int dflt);

// ---- kernel entry points (defined in kernels_*.hip) ----------------------
int launch_direct(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                  hipStream_t s);
int launch_zmarch(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                  hipStream_t s);
int launch_temporal2(const stencil_layout& l, const void* in, void* out, int64_t begin,
                     int64_t end, hipStream_t s);
// The two-tier 7-point launch (kernels_strip.hip TIER): 8
// sweeps per launch, the intermediate grid through a ring of plane slots.
struct TierJob {
    void* mem = nullptr;  // slots + flags + fail counter (stream-ordered allocation)
    int64_t tiles = 0;
    struct Args {
        void* slots = nullptr;
        uint32_t* prod = nullptr;
        uint32_t* cons = nullptr;
        unsigned* fail = nullptr;
        uint32_t base = 0;
        int rmask = 0;
    } a;
};
bool tier_eligible(const stencil_layout& l);
int tier_begin(const stencil_layout& l, hipStream_t s, TierJob* j);
int tier_launch(const stencil_layout& l, const void* in, void* out, TierJob* j, hipStream_t s);
int tier_end(TierJob* j, hipStream_t s, bool* failed);
int launch_temporalk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                     int steps, hipStream_t s);
int launch_tkstrip(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                   int cfg, hipStream_t s);
// kernels_strip_ilp.hip: the fp64 K = 4 and fp32 K = 5 default strip shapes built under the gcn-max-ilp
// machine scheduler (launch_tkstrip routes the shapes measured faster that way)
int launch_tkstrip_ilp(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                       hipStream_t s);
// kernels_strip_probe.hip (debug library only; the product links knobs.cpp's stub): the max-ILP shapes
// built as a compile-time variant, debug cfg 97
int launch_tkstrip_probe(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                         hipStream_t s);
// The halo gate of a face-signalled launch (stencil_sweepk_signal_gated):
// the workgroups whose z range reaches a halo plane first wait until *word
// (the slab's exchange-completion word, stencil_exchange_done) has reached
// `need` (wrap-safe), or until *release != 0 (a failed job), or 10 s (then
// it sets *release: the job reports the timeout).  A null word: no gate.
struct StripGate {
    const uint32_t* word = nullptr;
    uint32_t* release = nullptr;
    uint32_t need = 0;
};
int launch_tkstrip_signal(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                          unsigned* sig, unsigned long long* fsig, int* nsig, hipStream_t s,
                          const StripGate& gate = StripGate{});
int launch_boxk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                hipStream_t s);
int launch_boxk_signal(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                       unsigned* sig, unsigned long long* fsig, int* nsig, hipStream_t s);
bool zmarch_supports(const stencil_problem& p);
bool temporal2_supports(const stencil_problem& p);
int launch_box27(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                 int steps, hipStream_t s);
bool box27_supports(const stencil_problem& p);
// the fp32 one-cell-per-lane box strip shapes (cfg RRNN), compiled with and
// without SLP vectorisation (kernels_boxk_probe.hip; debug cfgs 95RRNN / 96RRNN)
int launch_boxk_probe_slp(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                          int cfg, hipStream_t s);
int launch_boxk_probe_noslp(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                            int cfg, hipStream_t s);
int launch_tb2d(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s);
// the whole 2D job as one persistent launch (kernels_tb2dp.hip); EUNSUPPORTED
// when the tiles do not all fit on the GPU at once
int launch_tb2dp(const stencil_layout& l, void* a, void* b, uint32_t iterations, hipStream_t s, int* final_in_b);
bool tb2dp_supports(const stencil_problem& p);
bool tb2dp_fits(const stencil_layout& l);  // queries the current device
int tb2dp_steps(const stencil_problem& p);
bool tb2d_supports(const stencil_problem& p);
int tb2d_max_steps(const stencil_problem& p);
int tb2d_steps(const stencil_layout& l, uint32_t iterations);  // sweeps per launch (queries the device)
// a 2D grid small enough for one workgroup's LDS: the whole job in one launch
bool tb2d1_fits(const stencil_layout& l);
int launch_tb2d1(const stencil_layout& l, const void* in, void* out, uint32_t iterations, hipStream_t s);

// Kernel-family coverage: the z-marching single-sweep family (7-point star
// and 27-point box, r = 1) and the fused two-step family (same stencils).
inline bool march_supported(const stencil_problem& p) { return zmarch_supports(p) || box27_supports(p); }
inline bool fused_supported(const stencil_problem& p) { return temporal2_supports(p) || box27_supports(p); }

}  // namespace stencil
