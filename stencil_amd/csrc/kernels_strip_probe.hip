// kernels_strip_probe.hip -- the max-ILP strip shapes (kernels_strip_ilp.hip)
// a third time, as a compile-time variant to time beside the default build in
// ONE process (debug cfg 97: STENCIL_TK_STRIP=97, tools/ab.py): separate
// library builds timed in separate processes also differ in where the grids
// land in physical memory, which moves the fp32 strip by up to 7 % with
// bit-identical kernel code.  Linked into the debug library
// only.  Now a control (the same code as kernels_strip_ilp.hip); round 6 built
// it with TK_PROBE_NOBAR, TK_PROBE_SPLIT(64), TK_SST, TK_XRING8 and under the
// gcn-iterative-ilp scheduler (profiles/r06/r06q_* .. r06w_*).
#define STRIP_ILP_TU
#define STRIP_ILP_FN launch_tkstrip_probe
#define TK_ILP_NS32 4
#include "kernels_strip.hip"
