// kernels_boxk_probe.hip -- code-generation probe for the box strip kernel.
//
// Round 2 found the fp32 one-cell-per-lane box strip shapes (ext_vector_type(1)
// floats) wrong in some shapes -- rows 4-7 of 8-row strips, up to 4 % off from
// the first fused sweep -- while the same code in fp64 is bitwise right.  In
// fp32 with one cell per lane the SLP vectoriser pairs the scalar adds of two
// rows into v_pk_add_f32 (fp64 has no packed add; the two-cell fp32 shapes use
// packed adds within one row).  This file re-instantiates those shapes from
// kernels_boxk.hip twice: as is (launch_boxk_probe_slp) and, built with
// -fno-slp-vectorize (Makefile: PROBE_NOSLP), without packed adds
// (launch_boxk_probe_noslp).  Debug cfgs 95RRNN / 96RRNN reach them
// (tools/box_v1_diff.py); the product never does.
#define BOXK_PROBE_TU
#include "kernels_boxk.hip"

namespace stencil {

#ifdef PROBE_NOSLP
#define PROBE_FN launch_boxk_probe_noslp
#else
#define PROBE_FN launch_boxk_probe_slp
#endif

int PROBE_FN(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps, int cfg,
             hipStream_t s) {
    switch (steps * 10000 + cfg) {
    case 30808: return launch_bk<float, 1, 8, 8, 3, false, true>(l, in, out, begin, end, s);
    case 30408: return launch_bk<float, 1, 4, 8, 3, false, true>(l, in, out, begin, end, s);
    case 10808: return launch_bk<float, 1, 8, 8, 1, false, true>(l, in, out, begin, end, s);
    case 20808: return launch_bk<float, 1, 8, 8, 2, false, true>(l, in, out, begin, end, s);
    case 40408: return launch_bk<float, 1, 4, 8, 4, false, true>(l, in, out, begin, end, s);
    default: return set_error(STENCIL_EINVAL, "box probe: no shape %d for %d steps", cfg, steps);
    }
}

}  // namespace stencil
