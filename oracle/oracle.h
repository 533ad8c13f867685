/*
 * oracle.h -- CPU restatement of the reference's naive Jacobi sweep.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (stencil_amd/, the CLI,
 * libstencil_hip.so) includes, links or calls this.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load liboracle.so,
 * and only as the checker / the CPU baseline, never as a compute path.
 *
 * What it restates (all citations into the read-only reference tree):
 *   - Stencil::check_result, src/stencil/stencil.cpp:75-131   (naive order)
 *   - Stencil::generate_initialized_matrix, stencil.cpp:190-207 and
 *     BoundaryMatrix::fill_boundary, include/stencil/boundary_matrix.hpp:129-170
 *   - ping-pong parity, stencil.cpp:88-92,129-134
 *   - neighbor1_impl::stencil_iterate_dma arithmetic,
 *     src/stencil/slave/stencil_dma.cpp:431-444            ("dma" order, r = 1)
 *   - neighbors_impl::stencil_iterate_dma arithmetic,
 *     src/stencil/slave/stencil_dma.cpp:636-650,700-720    ("dma" order, r > 1)
 *
 * Pinning: oracle/ref/build.sh compiles the reference's OWN naive loop
 * (stencil.cpp:77-131) and initial condition (190-207) from /root/reference
 * with its real headers into oracle/_ref/ref_naive (the lines are piped into
 * g++; no stand-in header: the athread include, stencil.cpp:2, is outside the
 * slice).  tests/golden/make_ref_golden.py records its outputs; the 2D naive
 * restatement here equals them bit for bit in fp32 (and in fp64 against the
 * same lines with float -> double), C1 included (tests/test_oracle_golden.py).
 * The reference's CPE kernels (DMA order) need the Sunway athread SDK and are
 * pinned by the deviation statistics SURVEY.md §8c recorded from its probe.
 * 3D and box shapes have no reference code ("parity unpinned" -- DESIGN.md §4).
 *
 * Layout: a dense ghost-padded array, x fastest.  Extents with ghosts are
 *   sx = nx + 2r, sy = ny + 2r, sz = (dims == 3 ? nz + 2r : 1).
 * The "slow axis" is z for 3D and y for 2D; sweeps take a [begin, end) range
 * of interior indices along it (used by the slab tests).
 */
#ifndef STENCIL_ORACLE_H
#define STENCIL_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_F32 = 0, ORACLE_F64 = 1 };
enum { ORACLE_STAR = 0, ORACLE_BOX = 1 };
/* ORACLE_ORDER_LEX: the box's round-1 definition (26 terms added in
 * lexicographic (dz, dy, dx) order), kept only to show the separable order
 * (the box's definition, oracle_impl.inc) agrees with it to ~1e-15 relative. */
enum { ORACLE_ORDER_NAIVE = 0, ORACLE_ORDER_DMA = 1, ORACLE_ORDER_LEX = 2 };
enum { ORACLE_INIT_REFERENCE = 0, ORACLE_INIT_RANDOM = 1 };

typedef struct {
    int32_t dims;   /* 2 or 3 */
    int32_t dtype;  /* ORACLE_F32 / ORACLE_F64 */
    int32_t shape;  /* ORACLE_STAR / ORACLE_BOX */
    int32_t radius; /* >= 1 */
    int32_t order;  /* ORACLE_ORDER_NAIVE / ORACLE_ORDER_DMA (2D star only) / ORACLE_ORDER_LEX (box only) */
    int32_t reserved;
    int64_t nx, ny, nz; /* interior extents; nz ignored for 2D */
} oracle_problem;

/* Number of elements of the ghost-padded dense array. */
int64_t oracle_elems(const oracle_problem* p);

/* 0 if the problem is valid, else a negative code. */
int oracle_check(const oracle_problem* p);

/* Fill with the reference initial condition (ORACLE_INIT_REFERENCE: interior 0,
 * ghost columns x < r and x >= nx + r are 1 at every y/z, every other ghost 0)
 * or with splitmix64(seed + interior linear index) uniform [0,1) in the
 * interior and the same ghosts (ORACLE_INIT_RANDOM). */
int oracle_init(const oracle_problem* p, int init_kind, uint64_t seed, void* buf);

/* One sweep: out = S(in) on interior slow-axis indices [begin, end). Ghost
 * cells of `out` are not touched. nthreads <= 1 runs single-threaded; the
 * per-cell arithmetic does not depend on it. */
int oracle_sweep(const oracle_problem* p, const void* in, void* out, int64_t begin, int64_t end,
                 int nthreads);

/* `iterations` ping-pong sweeps starting from `a`; returns 0 when the final
 * grid is in `a`, 1 when it is in `b` (parity rule of stencil.cpp:88-92,134),
 * negative on error. */
int oracle_run(const oracle_problem* p, uint32_t iterations, void* a, void* b, int nthreads);

/* FNV-1a-64 over the interior bytes in row-major order (x fastest). */
uint64_t oracle_fnv1a64_interior(const oracle_problem* p, const void* buf);

/* Sum of the interior in row-major order, accumulated in double. */
double oracle_sum_interior(const oracle_problem* p, const void* buf);

/* Copy the interior out densely (nx*ny[*nz] elements). */
int oracle_copy_interior(const oracle_problem* p, const void* buf, void* dst);

#ifdef __cplusplus
}
#endif

#endif /* STENCIL_ORACLE_H */
