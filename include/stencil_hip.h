/*
 * stencil_hip.h -- the C-ABI boundary of the MI355X stencil engine
 * (libstencil_hip.so, built from the .hip sources in stencil_amd/csrc for gfx950).
 *
 * Plain C: pointers, sizes and opaque stream handles only (a stream is a
 * hipStream_t passed as void*; NULL = the default stream).  No HIP, torch or
 * C++ types cross this boundary; the host CLI (stencil_amd/csrc/host) is
 * compiled with plain g++ against this header alone.
 *
 * Two layers:
 *
 *  1. The reference's own kernel ABI, layout-compatible and name-identical
 *     (drop-in for src/stencil/slave/stencil_slave.hpp:13-46):
 *        void stencil_iterate_dma(StencilArguments*);                 (:28)
 *        void stencil_iterate_dma_static_unroll(StencilArguments*);   (:33)
 *        void stencil_iterate_dma_slave_pack(StencilArguments*);      (:41)
 *        void stencil_iterate_rma(StencilArguments*);                 (:44)
 *     In the reference these run on the 64 CPEs via
 *     athread_spawn(SLAVE_FUN(fn), &args); athread_join()
 *     (src/stencil/stencil.cpp:34-53).  Here the call runs the whole job on
 *     the current GPU and returns when the parity-selected host buffer holds
 *     the result.  Arithmetic order follows each reference variant so results
 *     are bit-identical to what that variant computes.
 *
 *  2. The native engine API (device-resident grids, fp32/fp64, 2D/3D, star
 *     and box shapes, any radius, slab sweeps for multi-GPU).  The reference
 *     has no counterpart; it generalises Stencil::run
 *     (src/stencil/stencil.cpp:23-57) and BoundaryMatrix
 *     (include/stencil/boundary_matrix.hpp:31-238).
 *
 * Errors: native calls return STENCIL_OK (0) or a negative STENCIL_E* code;
 * stencil_last_error_message() describes the most recent failure on the
 * calling thread.  The reference-ABI entry points return void like the
 * reference (stencil_slave.hpp:26-46) and report through
 * stencil_last_error() (0 = success).
 */
#ifndef STENCIL_HIP_H
#define STENCIL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
#define STENCIL_OK 0
#define STENCIL_EINVAL (-1)      /* bad argument / unsupported combination */
#define STENCIL_EHIP (-2)        /* a HIP runtime call failed */
#define STENCIL_ENOMEM (-3)      /* device allocation failed */
#define STENCIL_ENODEV (-4)      /* no usable gfx950 device */
#define STENCIL_EUNSUPPORTED (-5)
#define STENCIL_ETIMEOUT (-6)      /* a slab job's device wait passed its deadline (a peer stopped answering) */

const char* stencil_strerror(int code);
const char* stencil_last_error_message(void);
int stencil_last_error(void);
/* 0 in libstencil_hip.so (the product: AUTO's plan, the environment knobs
 * below only); 1 in libstencil_hip_debug.so, which also reads the experiment
 * knobs (STENCIL_*_CFG workgroup shapes, forced z-chunks and kernel families)
 * the shape-sweep tests and A/B tools use.  Documented knobs, read by both:
 * STENCIL_TK_STEPS (3..5) / STENCIL_BOX_STEPS (3, 4) fused sweeps per launch,
 * STENCIL_TK_PACK / STENCIL_BOXK_PACK (0 equal z-chunks, 1 measured choice,
 * 2 the model's), STENCIL_SLAB_SIGNAL=0 (slab rounds without face signals),
 * STENCIL_SLAB_CPWAIT=1 (face-signalled slab rounds wait for the faces in the
 * command processor, hipStreamWaitValue64, instead of a polling wait kernel),
 * STENCIL_SLAB_SERIAL=1 (every full slab round as one plain launch, then the
 * exchange: nothing runs beside the launch), STENCIL_SLAB_XCU=c (default 1:
 * a face-signalled job whose launch takes several rounds of workgroups runs
 * its exchange confined to c CUs of every XCD and its launches off them;
 * 0 = never confined) and STENCIL_SLAB_XCU_EXCL=0 (the launches may use the
 * exchange's CUs too),
 * STENCIL_SLAB_PLACEMENTS=n (default 1 = the first allocation; n > 1: a
 * two-grid slab tries n placements of its grids at creation and keeps the
 * fastest -- the same launch runs 4-8 % apart in short bursts depending on
 * the grids' physical pages, 0.8 % over C2's 1000 sweeps.  Cost at
 * stencil_slab_create*: up to n candidate grid pairs allocated at once,
 * within a quarter of the free HBM, and about 6 timed K-step launches per
 * candidate; bench.py opts in with its --placements, default 16),
 * STENCIL_SLAB_TIMEOUT_MS (a slab job's deadline for any device wait,
 * default 60000: stencil_slab_set_timeout), STENCIL_SLAB_ROLLING_OVERLAP=0
 * (rolling slab rounds exchange after the pass instead of beside it),
 * STENCIL_SLAB_STAGED=0 (slabs whose launch takes several rounds of
 * workgroups run face-signalled rounds instead of staged ones),
 * STENCIL_SLAB_GATE=0 (face-signalled rounds wait for the exchange stream's
 * event before each launch instead of gating the launch's halo-reading
 * workgroups on the exchange-completion word: stencil_slab_round_info). */
int stencil_debug_knobs(void);

/* --------------------------------------------- 1. reference-compatible ABI */

/* Layout-identical to detail::BoundaryMatrix<float,false>
 * (include/stencil/boundary_matrix.hpp:225-237 field order, LP64: 40 bytes). */
typedef struct StencilMatrixView {
    size_t actual_width;      /* width + 2*boundary_width  (_actual_width)  */
    size_t actual_height;     /* height + 2*boundary_height (_actual_height) */
    unsigned boundary_width;  /* _boundary_width  (= radius) */
    unsigned boundary_height; /* _boundary_height (= radius) */
    size_t data_stride;       /* _data_stride, elements per row */
    float* data;              /* _data, row-major incl. ghost ring, HOST memory */
} StencilMatrixView;

/* Layout-identical to struct Arguments (stencil_slave.hpp:13-24): 88 bytes. */
typedef struct StencilArguments {
    unsigned block_size; /* accepted for compatibility; the GPU picks its own tiling */
    unsigned iterations;
    StencilMatrixView input;  /* both buffers hold the initial grid + ghosts */
    StencilMatrixView output; /* final grid: output if iterations odd, else input */
} StencilArguments;

void stencil_iterate_dma(StencilArguments* args);
void stencil_iterate_dma_static_unroll(StencilArguments* args);
void stencil_iterate_dma_slave_pack(StencilArguments* args);
void stencil_iterate_rma(StencilArguments* args);

/* ------------------------------------------------------ 2. native engine */

enum { STENCIL_F32 = 0, STENCIL_F64 = 1 };
enum { STENCIL_STAR = 0, STENCIL_BOX = 1 };
/* Sum order. NAIVE = Stencil::check_result (stencil.cpp:104-125) and
 * DMAStaticUnroll; DMA = stencil_dma.cpp (r=1: 431-444, r>1: 636-650).
 * DMA order exists for 2D star only. */
enum { STENCIL_ORDER_NAIVE = 0, STENCIL_ORDER_DMA = 1 };
/* Kernel family. AUTO picks the fastest one that supports the problem. */
enum {
    STENCIL_KERNEL_AUTO = 0,
    STENCIL_KERNEL_DIRECT = 1,    /* one cell per lane, neighbours via L1/L2 */
    STENCIL_KERNEL_ZMARCH = 2,    /* 2.5D: LDS plane + z register queue */
    STENCIL_KERNEL_TEMPORAL2 = 3, /* ZMARCH with 2 fused time steps per launch */
    STENCIL_KERNEL_TEMPORALK = 4, /* 3D 7-point star: K = 3..5 fused steps per launch
                                     (K = env STENCIL_TK_STEPS, default 4) */
    STENCIL_KERNEL_PERSISTENT = 5 /* 2D star r <= 2: the whole job in one launch, one
                                     resident workgroup per tile, K-cell rings exchanged
                                     through the grid with neighbour-only flags every
                                     K sweeps (K = env STENCIL_TB2DP_K, default 8/r);
                                     grids whose tiles do not all fit at once use
                                     TEMPORAL2 */
};
enum { STENCIL_INIT_REFERENCE = 0, STENCIL_INIT_RANDOM = 1 };
/* stencil_problem.flags: which z faces of this grid are halos filled by a
 * neighbouring slab (multi-GPU) rather than Dirichlet ghosts.  Only the fused
 * two-step kernel cares: it must advance halo planes to t+1, and must keep
 * Dirichlet ghost planes fixed. */
enum { STENCIL_HALO_LO = 1, STENCIL_HALO_HI = 2 };

typedef struct stencil_problem {
    int32_t dims;   /* 2 or 3 */
    int32_t dtype;  /* STENCIL_F32 / STENCIL_F64 */
    int32_t shape;  /* STENCIL_STAR / STENCIL_BOX */
    int32_t radius; /* >= 1 (reference -r) */
    int32_t order;  /* STENCIL_ORDER_* */
    int32_t kernel; /* STENCIL_KERNEL_* */
    int32_t halo;   /* 3D: ghost planes per z side, >= radius (0 = radius); 2 for fused slabs */
    int32_t flags;  /* STENCIL_HALO_* */
    int64_t nx, ny, nz; /* interior extents (reference: width = height = -s); nz = 1 for 2D */
} stencil_problem;

/* Device layout: x fastest, ghost ring of width `radius` on x and y and of
 * `zghost` planes on z (3D), rows padded so interior x = 0 of every row is
 * 128-byte aligned.
 * Element (x, y, z) of the interior (ghosts at -r..-1 and n..n+r-1) is at
 *   base[origin + z*plane + y*row + x]    (z = 0 for 2D). */
typedef struct stencil_layout {
    stencil_problem prob;
    int64_t row;    /* elements between consecutive rows (y) */
    int64_t plane;  /* elements between consecutive planes (z); rows*row */
    int64_t planes; /* allocated planes (nz + 2*zghost for 3D, 1 for 2D) */
    int64_t zghost; /* ghost/halo planes per z side (3D; 0 for 2D) */
    int64_t rows;   /* allocated rows per plane (ny + 2r) */
    int64_t origin; /* element offset of interior (0,0,0) */
    int64_t elems;  /* elements to allocate */
    int64_t bytes;  /* elems * sizeof(element) */
} stencil_layout;

int stencil_layout_init(const stencil_problem* prob, stencil_layout* out);

/* Extent of the slow axis (z for 3D, y for 2D): sweeps and slabs range over it. */
int64_t stencil_slow_extent(const stencil_layout* l);

int stencil_device_count(int* count);
int stencil_set_device(int device);
int stencil_synchronize(void* stream);
int stencil_alloc(const stencil_layout* l, void** dev);
int stencil_free(void* dev);

/* Initial condition on the device (interior + ghosts), see DESIGN.md §Init:
 * REFERENCE = stencil.cpp:190-207 (x-ghosts 1, every other cell 0);
 * RANDOM    = interior splitmix64(seed + linear index) in [0,1). */
int stencil_fill_initial(const stencil_layout* l, void* dev, int init_kind, uint64_t seed,
                         void* stream);

/* Host <-> device copies of the whole ghost-padded grid. The host array is
 * dense: row stride host_row elements, host_rows rows per plane (the
 * reference's BoundaryMatrix has host_row = n + 2r). Asynchronous on
 * `stream` (host memory should be pinned for true overlap). */
int stencil_upload(const stencil_layout* l, void* dev, const void* host, int64_t host_row,
                   int64_t host_rows, void* stream);
int stencil_download(const stencil_layout* l, const void* dev, void* host, int64_t host_row,
                     int64_t host_rows, void* stream);
/* Copy `count` planes (slow-axis units, ghost rows/planes included, indices
 * relative to the interior: -g .. n+g-1 with g = zghost in 3D, radius in 2D)
 * between two device grids. */
int stencil_copy_planes(const stencil_layout* l, const void* src, int64_t src_first,
                        void* dst, int64_t dst_first, int64_t count, void* stream);

/* One Jacobi sweep out = S(in) over slow-axis interior indices [begin, end).
 * Ghost cells are read, never written. */
int stencil_sweep(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                  void* stream);

/* Two fused sweeps (TEMPORAL2 family): out = S(S(in)) on [begin, end), using
 * `in`'s ghost/halo planes (2r deep) for the redundant halo compute. `out`
 * must differ from `in`; no scratch grid is needed. */
int stencil_sweep2(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                   void* stream);

/* K fused sweeps, out = S^K(in) on [begin, end): steps 1 = stencil_sweep,
 * 2 = stencil_sweep2, 3..5 = the TEMPORALK kernel (3D 7-point star), 3..4 =
 * the K-step box kernel (3D 27-point box; kernels_boxk.hip, which also serves
 * the box's 2-step sweep2).
 * With HALO_LO/HI flags the grid needs halo >= steps. */
int stencil_sweepk(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                   int32_t steps, void* stream);

/* Launch geometry of stencil_sweepk's K-step kernel (3D r=1 7-point star,
 * steps 3..5) on [begin, end), computed as the launch would, without
 * launching: workgroups, planes per z-chunk (0 = balanced shares) and
 * whether the packed longest-first chunk schedule is used (it is built and
 * uploaded on first use).  Queries the current device. */
int stencil_sweepk_geometry(const stencil_layout* l, int64_t begin, int64_t end, int32_t steps, int64_t* workgroups,
                            int32_t* zchunk, int32_t* packed);

/* Multi-GPU slabs: stencil_sweepk over [begin, end) (3D 7-point star, steps
 * 3..5; 27-point box, steps 2..4) as ONE launch whose workgroups add 1 to counters[0] as soon as the
 * low face planes [begin, begin+steps) are stored and to counters[1] for
 * [end-steps, end) (the last z-chunk marches downward, so both faces come
 * first); *signals_per_face = adds per face per launch.  counters: two
 * uint32 in device memory, zeroed by the caller, accumulating over launches.
 * face_signal (optional, from stencil_face_signal_create): the workgroup
 * that completes a face's count for this launch also adds 1 to it, so it
 * grows by 2 per launch once both faces are stored.
 * stencil_wait_counters queues on `stream` a one-lane kernel that returns
 * when counters[0] >= target_lo and counters[1] >= target_hi -- what is
 * queued behind it (the halo send) waits for the faces, not for the whole
 * launch.  After 10 s it sets *timeout_flag and returns instead; a wait that
 * finds *timeout_flag already set returns at once (a lost peer costs one
 * timeout, and the slab job's run() reports it).
 * stencil_wait_face_signal queues the same wait on the command processor
 * (hipStreamWaitValue64, *face_signal >= target): no kernel, no timeout. */
int stencil_sweepk_signal(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                          int32_t steps, uint32_t* counters, uint64_t* face_signal, int32_t* signals_per_face,
                          void* stream);
int stencil_wait_counters(const uint32_t* counters, uint32_t target_lo, uint32_t target_hi, uint32_t* timeout_flag,
                          void* stream);
/* The halo-gated form (the 7-point star only; the box: STENCIL_EUNSUPPORTED):
 * as stencil_sweepk_signal, and the workgroups whose z range reaches a halo
 * plane (z < 0 with STENCIL_HALO_LO, z >= nz with STENCIL_HALO_HI) first wait
 * until counters[3] >= gate_need (uint32, wrap-safe), until *release_flag != 0
 * (host-coherent, as stencil_wait_counters' timeout flag; may be NULL), or
 * 10 s (then they set *release_flag and go on with stale halos: the caller
 * must treat the launch as failed).  A slab round then queues its launch right behind the previous
 * round's launch, with no event wait for the exchange that fills its halos
 * (DESIGN.md §7): the halo planes are the only bytes that exchange writes.
 * stencil_exchange_done queues on `stream` (behind the exchange's transfers)
 * one lane storing counters[3] = value. */
int stencil_sweepk_signal_gated(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                                int32_t steps, uint32_t* counters, uint64_t* face_signal, uint32_t gate_need,
                                uint32_t* release_flag, int32_t* signals_per_face, void* stream);
int stencil_exchange_done(uint32_t* counters, uint32_t value, void* stream);
/* face signals: 8 bytes of HIP signal memory (hipExtMallocWithFlags,
 * hipMallocSignalMemory) holding a uint64 count */
int stencil_face_signal_create(uint64_t** face_signal);
int stencil_face_signal_destroy(uint64_t* face_signal);
int stencil_face_signal_reset(uint64_t* face_signal, void* stream);   /* queued: *face_signal = 0 */
int stencil_face_signal_read(const uint64_t* face_signal, uint64_t* value);  /* synchronous */
int stencil_wait_face_signal(const uint64_t* face_signal, uint64_t target, void* stream);

/* Whole job: `iterations` ping-pong sweeps starting from grid `a` (grid `b`
 * must hold the same ghosts). *final_in_b = 1 when the result is in `b`
 * (iterations odd), 0 when in `a` (parity rule, stencil.cpp:88-92,134).
 * With prob.kernel == TEMPORAL2, pairs of iterations run as one launch;
 * with TEMPORALK, K-tuples (remainder as a pair and/or a single sweep).
 * If elapsed_ms is non-NULL the call brackets its launches with hipEvents on
 * `stream`, synchronises, and stores the elapsed device time. */
int stencil_iterate(const stencil_layout* l, void* a, void* b, uint32_t iterations, void* stream,
                    int* final_in_b, float* elapsed_ms);

/* Settle stencil_iterate's one-time, per-shape choices before a timed run:
 * the first fused launch of the job (K-step 7-point star or box) from `a`
 * into `b`, which on a shape's first use times the packed and equal z-chunk
 * grids (blocking once) and keeps the faster.  `a` is not changed; `b` is
 * overwritten (its ghost cells are not).  Then the same launch again for
 * about 25 ms of device time (at most 2048 launches): after the GPU has idled
 * its clock needs that long to settle (the first launches run up to 1.45x
 * slower), so a timed run that follows measures the settled state.  2D jobs
 * of K-step launches settle the same way (they have no per-shape choice).
 * Blocks the host once.  A no-op for jobs without a K-step launch.  No
 * reference counterpart (the reference has no per-shape state). */
int stencil_prepare(const stencil_layout* l, const void* a, void* b, void* stream);
/* The same, reporting what ran before the caller's timed region: the kernel
 * launches (the schedule trial's included) and their device time, estimated
 * from the one timed settle launch. */
int stencil_prepare2(const stencil_layout* l, const void* a, void* b, void* stream, int64_t* settle_launches,
                     float* settle_ms);

/* One resident grid instead of two (3D, no slab flags): for jobs whose two
 * ping-pong grids do not fit the GPU -- BASELINE config 3, 4096^3 fp32, is
 * 2 x 279 GB; one grid plus a few hundred spare planes fits 288 GiB.  The
 * reference swaps two owner buffers every sweep (src/stencil/stencil.cpp:
 * 14-21, 88-92; include/stencil/boundary_matrix.hpp:59); here a pass of K
 * fused sweeps writes plane z of the new grid into the slot D planes below
 * (down pass) or back (up pass), in launches over z-ranges of D - K*r planes
 * ordered so that no launch writes a slot any later read needs (D >= K*r + 1;
 * K = the sweeps of one pass, r = the radius).  Results
 * are bitwise those of stencil_iterate.
 *   allocation: stencil_rolling_bytes(l, D, &bytes, &K) bytes at `base`;
 *   the grid at home (position 0) is the layout's grid at base + D*plane*esz,
 *   shifted (position 1) at base.  Fill / upload the home grid as usual,
 *   then stencil_rolling_init_margin copies its top ghost plane into the D
 *   spare slots (the x/y ghost ring must be the same in every plane and the
 *   z ghost planes alike, as in the reference initial condition).
 *   stencil_rolling_iterate: `iterations` sweeps from *position (updated);
 *   launches = kernel launches issued; elapsed_ms as stencil_iterate. */
int stencil_rolling_bytes(const stencil_layout* l, int64_t shift_planes, int64_t* bytes, int32_t* sweeps_per_pass);
int stencil_rolling_init_margin(const stencil_layout* l, void* base, int64_t shift_planes, void* stream);
int stencil_rolling_iterate(const stencil_layout* l, void* base, int64_t shift_planes, uint32_t iterations,
                            int32_t* position, void* stream, int64_t* launches, float* elapsed_ms);

/* The dispatcher model behind the packed z-chunk schedule, on the host (no
 * GPU needed): `tiles` x-y tiles of `planes` planes on `slots` one-workgroup
 * CU slots, `fill` planes of pipeline fill per chunk (2K for the 7-point
 * K-step kernel, 3K for the box), equal chunks of `zchunk` planes as the
 * alternative.  Returns the simulated makespans (plane steps) of the equal
 * chunks and of the best packed grid, and the packed grid's workgroups (0 when
 * it would not be used: it must beat equal chunks by 2 %).  stencil_iterate
 * then times both grids on a shape's first launch (STENCIL_TK_PACK=1). */
int stencil_pack_plan(int64_t tiles, int64_t planes, int32_t fill, int32_t slots, int32_t zchunk,
                      int64_t* equal_steps, int64_t* packed_steps, int64_t* workgroups);
/* The packed grid itself (host only): {tile, first plane, planes} per
 * workgroup in dispatch order, for a tile grid `tiles_x` wide; xcd_width > 0
 * reorders every generation of equal chunks into XCD patches of that width
 * (the dispatcher deals workgroup i to XCD i % 8); -1: the width with the most
 * same-XCD x/y neighbour tiles, as long jobs (>= 256 sweeps per call of
 * stencil_iterate / stencil_slab_run) launch it.  Writes at most
 * `capacity` triples into `table` (may be NULL) and the count to
 * *workgroups (0: no packed grid). */
int stencil_pack_table(int64_t tiles, int64_t tiles_x, int64_t planes, int32_t fill, int32_t slots, int32_t zchunk,
                       int32_t xcd_width, int32_t* table, int64_t capacity, int64_t* workgroups);

/* Launch plan of stencil_iterate for `iterations`: number of kernel launches
 * and the kernel family AUTO resolves to. */
int stencil_plan(const stencil_layout* l, uint32_t iterations, int64_t* launches,
                 int32_t* kernel);

/* Device-side checksums of the interior: per-plane sums (double, ascending
 * x, y order within the plane) written to `plane_sums` (slow_extent
 * entries, device or host pointer) -- the "checksum of checksums" used by
 * the full-size property tests. */
int stencil_plane_sums(const stencil_layout* l, const void* dev, double* plane_sums_host,
                       void* stream);

/* A plain device copy kernel (read n bytes, write n bytes) used by bench.py to
 * calibrate attainable HBM bandwidth on the box. */
int stencil_copy_bandwidth(void* dst, const void* src, int64_t bytes, int reps, void* stream,
                           float* elapsed_ms);

/* ------------------------------------------------ 3. multi-GPU z-slab jobs
 *
 * The reference runs its whole decomposed job behind one call: 64 CPEs own
 * 8x8 blocks and exchange halo strips every iteration (athread_spawn/join,
 * src/stencil/stencil.cpp:34-53; stencil_dma.cpp:236-247, stencil_rma.cpp:
 * 198-255).  A slab job does the same across GPUs from ONE host thread: the
 * global 3D grid is cut into contiguous z-slabs (remainder planes to the
 * lowest slabs), slab i lives on devices[i] with K ghost planes per shared
 * face (K = the sweeps stencil_iterate fuses into one launch for `global`),
 * and every round of K fused sweeps exchanges K whole planes with each
 * neighbour: the boundary planes first on a high-priority stream with the
 * exchange behind them, the interior on a second stream.  Results are bitwise
 * those of one grid.  Exchange: RCCL ncclSend/ncclRecv (ncclCommInitAll over
 * the devices, one slab per GPU; librccl is loaded on first use) or device
 * copies (hipMemcpyPeerAsync; slabs may share a GPU).  PERIODIC joins the
 * two z ends into a ring (a rehearsal mode: one slab exchanges with itself). */
enum { STENCIL_EXCHANGE_RCCL = 0, STENCIL_EXCHANGE_COPY = 1 };
/* PERIODIC: the z ends form a ring.  ROLLING: each slab keeps ONE resident
 * grid plus a margin of spare planes instead of two grids (the scheme of
 * stencil_rolling_*, per slab): a round is a pass of ceil(n / S) z-range
 * launches (S = margin - K*radius), then the exchange -- for slabs whose two
 * grids do not fit one GPU, e.g. the north star's 4096^3 fp64 on 2 GPUs (one
 * 278 GB grid each).  Bitwise the two-grid job; no face-signalled rounds.
 * No sweep writes a ghost cell, and a pass lands each plane in a slot whose
 * x/y ghost ring came from another plane, so a ROLLING job needs the same
 * x/y ghost ring in every plane and equal bottom ghost planes (the reference
 * initial condition has both): stencil_slab_upload checks a host grid for
 * this and returns STENCIL_EINVAL otherwise. */
enum { STENCIL_SLAB_PERIODIC = 1, STENCIL_SLAB_ROLLING = 2 };
typedef struct stencil_slab_job stencil_slab_job;

/* global: a 3D problem with halo = 0 and flags = 0; devices: ngpus ordinals
 * (NULL = 0 .. ngpus-1).  Every slab must own at least K planes. */
int stencil_slab_create(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange,
                        int32_t flags, stencil_slab_job** job);
/* The same with the rolling margin: margin_planes > 0 spare planes per slab
 * (at least K*radius + 1), 0 = as deep as each device's free memory allows
 * beside its grid (less a 4 GiB reserve for RCCL), at most 512.  Ignored
 * without STENCIL_SLAB_ROLLING. */
int stencil_slab_create2(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange,
                         int32_t flags, int64_t margin_planes, stencil_slab_job** job);
/* Rank mode: one process per GPU, as the reference's MPI-style launch and
 * torch.distributed.run give it.  Rank 0 makes an RCCL id
 * (stencil_slab_unique_id, STENCIL_SLAB_ID_BYTES bytes) and hands it to every
 * rank by its own channel (a torch.distributed broadcast, MPI_Bcast, a file);
 * each rank then calls stencil_slab_create_rank with the same global problem
 * and builds only its slab (z split as above, slab = rank) on `device`, joined
 * by ncclCommInitRank -- a collective: every rank must call it (a rank that
 * does not within STENCIL_SLAB_TIMEOUT_MS fails the others' calls with
 * STENCIL_ETIMEOUT; RCCL's bootstrap thread for the abandoned attempt then
 * stays blocked until the process exits).  The job then
 * holds ONE slab (stencil_slab_info slab 0) and every call below is
 * per-rank and collective over the ranks (run: every rank the same
 * iterations).  Host arrays keep the global shape: upload reads and download /
 * plane_sums write only this rank's planes (download: plus the global ghost
 * planes at the two ends).  Exchange is always RCCL. */
enum { STENCIL_SLAB_ID_BYTES = 128 };
int stencil_slab_unique_id(void* id, int64_t bytes);
int stencil_slab_create_rank(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device,
                             const void* id, int64_t id_bytes, int32_t flags, stencil_slab_job** job);
int stencil_slab_create_rank2(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device,
                              const void* id, int64_t id_bytes, int32_t flags, int64_t margin_planes,
                              stencil_slab_job** job);
int stencil_slab_destroy(stencil_slab_job* job);
int stencil_slab_info(const stencil_slab_job* job, int32_t slab, int64_t* first_plane, int64_t* planes,
                      int32_t* device, int32_t* sweeps_per_round);
/* Rolling slabs: the margin (0: two grids per slab) and the most z-range
 * launches one pass makes on a slab of this process. */
int stencil_slab_rolling_info(const stencil_slab_job* job, int64_t* margin_planes, int64_t* launches_per_pass);
/* Initial condition of the global grid (global linear indices for the random
 * interior, as stencil_fill_initial on one grid), halos exchanged. */
int stencil_slab_fill_initial(stencil_slab_job* job, int32_t init_kind, uint64_t seed);
/* The global grid from / to a dense host array with ghosts (x fastest,
 * host_row elements per row, host_rows rows per plane, nz + 2r planes).
 * ROLLING jobs: see the ghost-ring condition above. */
int stencil_slab_upload(stencil_slab_job* job, const void* host, int64_t host_row, int64_t host_rows);
int stencil_slab_download(stencil_slab_job* job, void* host, int64_t host_row, int64_t host_rows);
/* `iterations` sweeps of the whole job (rounds of K, the remainder as one
 * shorter round); synchronous.  elapsed_ms: host wall time of the rounds,
 * all devices synchronised at both ends. */
int stencil_slab_run(stencil_slab_job* job, uint32_t iterations, float* elapsed_ms);
/* Per-plane interior sums of the current global grid (nz doubles, host). */
int stencil_slab_plane_sums(stencil_slab_job* job, double* sums);
/* Kernel timing for roofline figures: with timing on, every round records
 * hipEvents around slab 0's compute launch (the whole slab in face-signalled
 * rounds, its interior launch in boundary + interior rounds, the pass's
 * z-range launches in rolling rounds) on that launch's stream.  kernel_time
 * synchronises and returns the summed device time, the spans timed, the
 * interior cells one span covers and whether the rounds are face-signalled
 * (1) or not (0); stencil_slab_round_form gives the form (a staged round's
 * span is its face launches and its middle launch).  Enabling (or
 * disabling) drops earlier records. */
int stencil_slab_kernel_timing(stencil_slab_job* job, int32_t enable);
int stencil_slab_kernel_time(stencil_slab_job* job, float* total_ms, int64_t* launches, int64_t* cells_per_launch,
                             int32_t* signalled);
/* With kernel timing on, every timed round also records its exchange on slab
 * 0's exchange stream: from the end of what precedes the transfers there (the
 * face wait of a face-signalled round; a rolling round's face launches) to
 * the end of the RCCL send/recv (or copies).  exchange_time synchronises and
 * returns the summed transfer time, the part of it that ran while the same
 * round's timed launch span ran (the overlap the round form is for; ~0 for
 * serial rounds), and the exchanges counted.  Over xGMI this is the wire
 * time of K planes per shared face plus RCCL's own latency. */
int stencil_slab_exchange_time(stencil_slab_job* job, float* transfer_ms, float* beside_ms, int64_t* exchanges);
/* The form of the job's full rounds (kernel_time's `signalled` is 1 for
 * face-signalled rounds, 0 otherwise). */
enum {
    STENCIL_SLAB_FORM_BOUNDARY_INTERIOR = 0, /* boundary planes on one stream, the interior on another */
    STENCIL_SLAB_FORM_SIGNALLED = 1,         /* one face-signalled launch, the exchange as the faces land */
    STENCIL_SLAB_FORM_ROLLING = 2,           /* one grid + a margin: a pass of z-range launches */
    STENCIL_SLAB_FORM_SERIAL = 3,            /* one launch of the whole slab, then the exchange */
    STENCIL_SLAB_FORM_STAGED = 4             /* the face quarters, then the middle beside the exchange */
};
int stencil_slab_round_form(const stencil_slab_job* job, int32_t* form);
/* How the job's full rounds run beyond their form (each output may be NULL):
 * *gated = 1 when face-signalled launches gate their halo-reading workgroups
 * on the exchange-completion word instead of waiting for the exchange stream
 * (stencil_sweepk_signal_gated; STENCIL_SLAB_GATE=0: never), *confined = 1
 * when the exchange runs on a few CUs of its own (STENCIL_SLAB_XCU). */
int stencil_slab_round_info(const stencil_slab_job* job, int32_t* form, int32_t* gated, int32_t* confined);
/* The exchange's CU budget (staged rounds with a confined exchange, slab 0):
 * CUs per XCD in use, the alternative budget the tuning rounds tried (0:
 * none; STENCIL_SLAB_XCU_ALT, default 4), and the timed tuning round with the
 * default (STENCIL_SLAB_XCU) and with the alternative budget, ms (0: not run:
 * the alternative is tried only when the exchange ran at least 0.8x as long
 * as the middle launch beside it).  The faster is kept (the alternative only
 * when 2 % faster); the face span is then tuned from that round. */
int stencil_slab_exchange_budget(const stencil_slab_job* job, int32_t* cus, int32_t* alt_cus, float* round_ms,
                                 float* alt_round_ms);
/* Bounded-time failure.  Every wait of the job for its devices (the end of
 * run(), fill, upload, download, plane sums, and -- while run() issues
 * rounds -- the exchange of the round kInflight = 8 rounds back) gives up
 * after `timeout_ms` (default 60000, or the STENCIL_SLAB_TIMEOUT_MS knob at
 * creation); so does an asynchronous RCCL error, polled meanwhile
 * (ncclCommGetAsyncError).  The job then aborts its communicators
 * (ncclCommAbort: RCCL's kernels waiting for a peer that stopped posting
 * return), releases its queued face waits, and the call returns
 * STENCIL_ETIMEOUT (or the error); every later call on the job fails, and
 * stencil_slab_destroy frees it.  The reference has no counterpart: its
 * never-waited reply (stencil_rma.cpp:334-338) hangs instead. */
int stencil_slab_set_timeout(stencil_slab_job* job, int64_t timeout_ms);

#ifdef __cplusplus
}
#endif

#endif /* STENCIL_HIP_H */
