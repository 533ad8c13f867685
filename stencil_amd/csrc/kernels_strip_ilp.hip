// kernels_strip_ilp.hip -- the 7-point strip kernel (kernels_strip.hip) a
// second time, compiled under LLVM's gcn-max-ilp machine scheduler (Makefile:
// per-file flags), for the two default shapes measured faster that way:
// the fp64 K = 4 strip on grids of at most 2 tiles per CU slot (the packed
// schedule, with its interior fast path) and the fp32 K = 5 strip.  Same
// source, same sums: bitwise the default build.
#define STRIP_ILP_TU
#include "kernels_strip.hip"
