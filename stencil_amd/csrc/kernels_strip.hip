// kernels_strip.hip -- K fused Jacobi sweeps per launch for the 3D 7-point
// star (r = 1, naive order) with every wave owning a STRIP of consecutive
// rows: the "strip" layout of the K-step z-march of kernels_temporalk.hip.
//
// Why.  In kernels_temporalk.hip a wave owns rows w, w+NW, ... of the
// region, so every y-neighbour and every centre comes from LDS: per plane
// and wave 3*RY reads and RY writes of 1 KiB per stage, two barriers per
// plane.  On MI355X a ds_write_b128 costs ~13 LDS cycles and a ds_read_b128
// 4, which at 16 waves/CU is ~2400 LDS cycles per plane step -- as long as
// the VALU work, and the kernel does not speed up when its HBM bytes drop
// (DESIGN.md §5).  Here wave w owns region rows [w*RY, w*RY + RY):
//   * centre, y-neighbours inside the strip and z-neighbours come from the
//     lane's own registers, x-neighbours from DPP lane shifts;
//   * only the strip's first and last rows go through LDS (the row above /
//     below the strip is the neighbour wave's last / first row): 2 writes
//     and 2 reads per stage and wave;
//   * the boundary-row buffers are double-buffered by plane parity, so one
//     barrier per plane suffices (a wave that passed barrier p has every
//     wave's reads of plane p-1's buffer behind it).
//
// Pipeline (as kernels_temporalk.hip): at plane step p stage s computes
// t_s(p-s) from t_{s-1}(p-s-1) (z-), t_{s-1}(p-s) (centre + x/y) and
// t_{s-1}(p-s+1) (z+, stage s-1's result of this step; stage 1: in(p)).
// Per lane and stage the two older planes live in a 2-slot register history
// H (slot = plane parity), the input in a 4-slot ring (in(p-2) .. in(p+1),
// loads issued two planes ahead).  t_K(p-K) goes to HBM (nontemporal).
//
// Per step:
//   barrier
//   read phase   boundary rows of t_{s-1}(p-s) from buffer (p-1)&1,
//                stages 1..K, store t_K(p-K)
//   write phase  boundary rows of in(p), t_1(p-1) .. t_{K-1}(p-K+1) into
//                buffer p&1; request in(p+2)
//
// Arithmetic is the single sweep's (0 + x- + x+ + y- + y+ + z- + z+) * avg
// with the "0 +" folded into fma(sum, avg, +0) exactly as in
// kernels_temporalk.hip; intermediate planes keep ghost cells at their input
// value; slab-halo planes (HALO_LO/HI) are advanced.  Bitwise equal to K
// plain sweeps (tests/test_gpu_parity.py).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.hpp"

#ifndef TK_FAST_PATH
#define TK_FAST_PATH 1
#endif
#ifndef TK_PACK2
#define TK_PACK2 1
#endif
// TK_SEG_FAST: a segment (tile, z-chunk) whose region lies inside the grid
// in x and y and whose stage planes that reach the output lie inside in z
// runs an instantiation of the plane loop with no ghost-cell selects at all;
// the choice is made once per segment, so the two loops never share live
// registers (the per-step choice, kFast, duplicates the step inside the loop).
// fp64 shapes of the default build (wide-plane grids, slab launches):
// 2048^2 x 512 +1 % in one process (profiles/r06/r06i_*)
#ifndef TK_SEG_FAST
#define TK_SEG_FAST 1
#endif
// TK_ILP_NS32: the input-plane ring of the max-ILP fp32 K = 5 strip (4: loads
// two planes ahead)
#ifndef TK_ILP_NS32
#define TK_ILP_NS32 4
#endif
// TK_PROBE_NOBAR (kernels_strip_probe.hip only, timing experiment: results
// wrong): the plain launches' per-step workgroup barrier left out -- the upper
// bound of what a barrier-free plane step could gain
#ifndef TK_PROBE_NOBAR
#define TK_PROBE_NOBAR 0
#endif
// TK_SST (kernels_strip_probe.hip only, an experiment): the fp32 two-cells-per-
// lane strip stores its output planes as 16-B lane vectors staged through an
// LDS image of the wave's own rows (ds_write_b64 per row, ds_read_b128 per row
// pair: lanes 0..31 row 2i, 32..63 row 2i+1), with an 8-cell x ring so every
// stored lane vector is whole inside the tile
#ifndef TK_SST
#define TK_SST 0
#endif
// TK_XRING8 (kernels_strip_probe.hip only, an experiment): the fp32 two-cells-
// per-lane strip with an 8-cell x ring (TX = 112), so regions start on a 32-B
// boundary
#ifndef TK_XRING8
#define TK_XRING8 0
#endif

namespace stencil {
namespace {

template <typename T, int V>
struct VecS {
    typedef T type __attribute__((ext_vector_type(V)));
};

__device__ __forceinline__ float sfma0(float s, float a) { return __builtin_fmaf(s, a, 0.0f); }
__device__ __forceinline__ double sfma0(double s, double a) { return __builtin_fma(s, a, 0.0); }

template <int CTRL>
__device__ __forceinline__ float sdpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ double sdpp(double v) {
    const int2 b = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_mov_dpp(b.x, CTRL, 0xf, 0xf, true),
                                                 __builtin_amdgcn_mov_dpp(b.y, CTRL, 0xf, 0xf, true)));
}
constexpr int kSShr1 = 0x138, kSShl1 = 0x130;  // wave_shr:1 / wave_shl:1
// the kernel's `fast` bits (STENCIL_TK_FAST, debug library): kFastStep = the
// per-step choice (kFast shapes), kFastSeg = the per-segment choice
// (TK_SEG_FAST), kFastAll = every tile taken as inside (timing only: wrong ghost cells)
constexpr int kFastStep = 1, kFastAll = 2, kFastSeg = 4;

// The plane loop unrolled N steps (compile-time step index), and the tail of
// fewer than N steps.
template <int I, int N, typename F>
__device__ __forceinline__ void unroll_steps(F& f, int p) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{}, p + I);
        unroll_steps<I + 1, N>(f, p);
    }
}
template <int I, int N, typename F>
__device__ __forceinline__ void tail_steps(F& f, int p, int plast) {
    if constexpr (I < N) {
        if (p + I <= plast) f(std::integral_constant<int, I>{}, p + I);
        tail_steps<I + 1, N>(f, p, plast);
    }
}

// SPLIT: each wave holds TWO strips, one per half-wave (lanes 0..31 strip w,
// lanes 32..63 strip NW + w), so a strip row is 32 lanes x V cells: with V = 4
// fp32 every plane load / store is a 16-B lane vector (half the memory
// instructions of the 8-B V = 2 shape for the same region width), while the
// y-neighbours stay in the lane's registers.  The x lane shifts cross the
// half boundary (lane 32 reads lane 31) only inside the x ring.
template <typename T, int V, int RY, int NW, int K, bool DB, bool SPLIT = false>
struct StripTile {
    static constexpr int LW = SPLIT ? 32 : 64;       // lanes per strip row
    static constexpr int NSTR = SPLIT ? 2 * NW : NW; // strips per region
    static constexpr bool SSTS = TK_SST && sizeof(T) == 4 && V == 2 && !SPLIT;  // TK_SST staged stores
    static constexpr bool XR8 = (SSTS || TK_XRING8) && sizeof(T) == 4 && V == 2 && !SPLIT;
    static constexpr int XR = XR8 ? 8 / V : (K + V - 1) / V;  // ring vectors per x side
    static constexpr int RW = LW * V;           // region width
    static constexpr int TX = RW - 2 * XR * V;  // output tile width
    static constexpr int RH = NSTR * RY;        // region height
    static constexpr int TY = RH - 2 * K;       // output tile height
    static constexpr int NB = DB ? 2 : 1;       // boundary-row buffers (plane parity)
    // boundary rows: [buffer][stage input][strip][top, bottom][RW]
    static constexpr size_t lds_bytes = size_t(NB) * K * NSTR * 2 * RW * sizeof(T);
};

// TIER (the two-tier job): a launch of 2 x tiles
// workgroups does 2K sweeps.  Workgroups [0, tiles) are PRODUCERS: the K-step
// march of their tile over the whole z range, storing t_K (the grid after K
// sweeps) -- output tile plus the region's ghost cells -- into a ring of R
// plane slots instead of the output grid.  Workgroups [tiles, 2 tiles) are
// CONSUMERS: the same march over the slots (their neighbours' outputs give the
// region's ring; the fixed z-ghost planes come from `in`), storing t_2K to
// `out`.  Only `in` and `out` travel to HBM; the slots (R x one plane) stay in
// the Infinity Cache.  Hand-off per plane (MI355X_MICROARCH.md, inter-workgroup
// visibility, hand-off table row 1): slot stores and loads are `sc1`; a
// producer publishes "planes stored" once every wave's counted vmcnt shows its
// stores of the previous step done and a barrier has joined the waves; a
// consumer publishes "planes loaded" the same way; a consumer's wave 0 checks
// its <= 9 producers before the step that loads a plane, a producer's its <= 9
// consumers before reusing a slot.  The checks read flags PREFETCHED one step
// earlier (issued before that step's plane loads, so the counted wait the step
// does anyway covers them -- wave 0's loads stay pipelined); only a flag still
// short spins, with a budget: a wait that gives up counts in `fail` and the
// host reports the job as failed.  All 2 x tiles workgroups must be resident
// at once (one per CU): the host launches it only when they fit.
// (TierJob::Args, common.hpp): slots = R plane slots in the grid's plane
// layout (plane z -> slot z & rmask, R a power of two); prod / cons = per
// tile, one 128-B line each, the planes stored / loaded by every wave (+ base,
// this launch's flag origin: flags run on across launches); fail = waits
// that gave up
using TierArgs = TierJob::Args;
constexpr int kTierFlagStride = 32;  // uint32 per flag line

__device__ __forceinline__ uint32_t tier_poll(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tier_publish(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tier_ge(uint32_t a, uint32_t b) { return int32_t(a - b) >= 0; }
// spin until *p >= need (wrap-safe), a tenth of a second at most; once any
// wait of the launch has given up, every later one returns at once, so a
// broken hand-off ends the launch quickly (with a wrong grid the host reports)
__device__ __forceinline__ void tier_spin(const uint32_t* p, uint32_t need, unsigned* fail) {
    for (int it = 0; !tier_ge(tier_poll(p), need); ++it) {
        if (it > (1 << 22) || (it % 1024 == 0 && tier_poll(fail) != 0)) {
            atomicAdd(fail, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// The halo gate (SIG, StripGate): one lane polls the exchange-completion
// word with relaxed agent-scope loads (they bypass L1) until it reaches
// `need`, the host releases it (a failed job) or 10 s of s_memrealtime
// (100 MHz) pass (then it sets the release flag, the job's timeout flag, so
// run() reports the failure); then ONE agent acquire and its vmcnt wait, before the
// workgroup barrier behind which every wave loads the halo planes
// (MI355X_MICROARCH.md §visibility, the consumer recipe).  The word is written
// by a one-lane kernel queued behind the exchange's transfers on their stream
// (stencil_exchange_done), so the transfers' kernels have ended -- and
// released their writes -- before it.
__device__ __forceinline__ void gate_wait(const StripGate& g) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (int32_t(__hip_atomic_load(g.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - g.need) < 0) {
        if (g.release && __hip_atomic_load(g.release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > uint64_t(1000) * 1000 * 1000) {
            // the halos this chunk reads are stale: fail the job (as a face-counter wait does)
            if (g.release) __hip_atomic_store(g.release, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename VT>
__device__ __forceinline__ VT sc1_load(const void* p) {
    static_assert(sizeof(VT) == 8, "tier hand-offs move 8-byte lane vectors");
    return __builtin_bit_cast(VT, __hip_atomic_load(static_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT));
}
template <typename VT>
__device__ __forceinline__ void sc1_store(void* p, const VT& v) {
    static_assert(sizeof(VT) == 8, "tier hand-offs move 8-byte lane vectors");
    __hip_atomic_store(static_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// DIAG (timing experiments only, results are wrong): 1 = no loads after the
// first two planes, 2 = no arithmetic (t_s = centre), 3 = no stores
// SIG: face signalling for multi-GPU slabs (stencil_sweepk_signal): the
// last z-chunk of every tile marches DOWNWARD, so the K planes of both faces
// of the range are among the first planes stored, and the workgroup that
// stores a face signals sig[0] (low face) / sig[1] (high face) right after
// (release, then one agent-scope add: MI355X_MICROARCH.md §visibility).  A
// stream waits for the counts (stencil_wait_counters) and sends the faces
// while the rest of the launch runs.  With fsig (HIP signal memory), the
// workgroup whose add completes a face's count for this launch (the counts
// run on across launches: every tiles_x*tiles_y-th add) also adds 1 to
// *fsig, so the command processor can gate the exchange stream on it
// (hipStreamWaitValue64) with no wait kernel resident during the launch.
// NS: input planes in registers -- in(p-2) .. in(p+NS-3): loads are issued
// NS-2 planes ahead (4: two planes).
// HL: stage 1's two history planes t_1(q) live in LDS instead of registers --
// each wave's own rows only (no barrier: a wave reads back what it wrote), so
// LDS serves as per-wave register space: 28 VGPRs per lane fewer at RY = 7,
// for 7 ds_write_b64 + 28 ds_read_b64 per wave and step, which pays for one
// more fused sweep (K = 5) at the same 7-row strips.
template <typename T, int V, int RY, int NW, int K, bool DB, int DIAG = 0, bool SIG = false, int NS = 4, bool FP = true,
          bool HL = false, bool TIER = false, bool SPLIT = false>
__global__ void __launch_bounds__(64 * NW)
    tkstrip_7pt(const T* __restrict__ in, T* __restrict__ out, Geom g, int zbeg, int zend, int zchunk,
                int tiles_x, int tiles_y, int halo_lo, int halo_hi, T avg, unsigned* __restrict__ sig,
                unsigned long long* __restrict__ fsig, const int* __restrict__ sched, int fast, int xcd_pw,
                TierArgs tier, StripGate gate) {
    using Tl = StripTile<T, V, RY, NW, K, DB, SPLIT>;
    using VT = typename VecS<T, V>::type;
    constexpr int XR = Tl::XR, TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, RW = Tl::RW, NB = Tl::NB;
    constexpr int LW = Tl::LW, NSTR = Tl::NSTR;
    static_assert(!SPLIT || !TIER, "SPLIT: plain or face-signalled launches");
    constexpr bool SST = Tl::SSTS && !SIG && !TIER && !HL;
    constexpr int NI = (RY + 1) / 2;  // SST: row pairs per strip
    typedef T V4T __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) T IMG[SST ? RH : 1][SST ? RW : 1];
    static_assert(TY > 0 && TX > 0, "tile too small for K");
    static_assert(RY >= 2, "a strip needs a first and a last row");
    static_assert(!HL || K >= 2, "HL keeps stage 1's history");
    __shared__ __attribute__((aligned(16))) T L[NB][K][NSTR][2][RW];
    // HL: t_1 history [plane parity][region row][x], each wave its own rows
    __shared__ __attribute__((aligned(16))) T HLs[HL ? 2 : 1][HL ? RH : 1][HL ? RW : 1];

    // Work = the linearised (tile, z) space of the range, tile-major: units
    // [lo, hi) of it per workgroup.  zchunk > 0: fixed chunks of every tile;
    // zchunk == 0: one equal share per workgroup (the grid is one workgroup
    // per slot), walked as one segment per tile it touches -- no partial last
    // round, at the price of one extra pipeline fill per segment boundary.
    const int nzr = zend - zbeg;
    const int64_t tiles = int64_t(tiles_x) * tiles_y;
    int64_t lo, hi;
    bool rev = false;  // this workgroup's chunk marches down (SIG: the last chunk)
    static_assert(!TIER || (!SIG && sizeof(T) * V == 8), "TIER: plain launches of 8-byte lane vectors");
    const bool tprod = TIER && int64_t(blockIdx.x) < tiles;  // TIER: producer (else consumer)
    if constexpr (TIER) {  // one segment per workgroup: its tile, the whole z range
        const int64_t t = tprod ? int64_t(blockIdx.x) : int64_t(blockIdx.x) - tiles;
        lo = t * nzr;
        hi = lo + nzr;
    } else if (sched) {
        // packed schedule (STENCIL_TK_PACK): {tile, first plane, planes}; on
        // face-signalled launches planes < 0 marks the chunk that ends at the
        // top face and marches down (packed_schedule's faces_out tables)
        const int* e = sched + 3 * int64_t(blockIdx.x);
        lo = int64_t(e[0]) * nzr + e[1];
        hi = lo + (e[2] < 0 ? -e[2] : e[2]);
        rev = SIG && e[2] < 0;
    } else if (zchunk > 0) {
        int64_t t = blockIdx.x % tiles, c = blockIdx.x / tiles;
        if (!SIG && xcd_pw > 0) {
            // XCD patches (experiment, STENCIL_TK_XCD = patch width; as the box
            // kernel's): XCD b % 8 walks its own run of (chunk, tile) units in
            // column strips of xcd_pw tiles, so the workgroups resident on one
            // XCD at a time form a 2D patch whose shared halo lines are L2 hits
            const int64_t nch = (nzr + zchunk - 1) / zchunk, total = tiles * nch, per = (total + 7) / 8;
            const int64_t u = int64_t(blockIdx.x % 8) * per + blockIdx.x / 8;
            if (u >= total) return;  // whole workgroup, before any barrier
            c = u / tiles;
            const int64_t tt = u - c * tiles;
            const int64_t strip = tt / (int64_t(xcd_pw) * tiles_y), rem = tt - strip * xcd_pw * tiles_y;
            const int64_t sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
            t = rem / sw * tiles_x + strip * xcd_pw + rem % sw;
        }
        const int64_t nch = (nzr + zchunk - 1) / zchunk;
        // face-signalled launches of several chunks per tile: the two face
        // chunks (the first, marching up, and the last, marching down) are
        // dispatched as the first two generations, the middle chunks after
        // them, so the faces are stored early even when the grid takes many
        // rounds of workgroups
        if (SIG && nch >= 3) c = c == 0 ? 0 : c == 1 ? nch - 1 : c - 1;
        lo = t * nzr + c * zchunk;
        hi = lo + (zchunk < nzr - c * zchunk ? zchunk : nzr - c * zchunk);
        rev = SIG && nch >= 2 && c == nch - 1;
    } else {
        const int64_t units = tiles * nzr;
        lo = units * blockIdx.x / gridDim.x;
        hi = units * (blockIdx.x + 1) / gridDim.x;
    }

    const int lane = threadIdx.x, w = threadIdx.y;
    // this lane's strip (vw) and its lane within the strip row (hl)
    const int vw = SPLIT ? (lane >> 5) * NW + w : w;
    const int hl = SPLIT ? (lane & 31) : lane;
    const int nz = int(g.nz);
    const int64_t plane = g.plane;
    // Addresses are a uniform per-plane base (SGPRs) + a non-negative 32-bit
    // byte offset per row (one VGPR, shared by loads and stores): the
    // saddr form of global_load/store.  bias moves the lowest offset (row -1,
    // x = -XR*V) to >= 0.
    const int64_t bias = g.row + XR * V;
    const char* __restrict__ src = reinterpret_cast<const char*>(in + g.origin - bias);
    char* __restrict__ dst = reinterpret_cast<char*>(out + g.origin - bias);

    {
        constexpr int N16 = int(Tl::lds_bytes / 16);
        VT* l16 = reinterpret_cast<VT*>(&L[0][0][0][0][0]);
        for (int i = threadIdx.y * 64 + threadIdx.x; i < N16; i += 64 * NW) l16[i] = VT{};
    }

    const int xl = hl * V;
    // neighbour strips (the first / last wave reads its own: those rows are ring rows)
    const int wa = vw > 0 ? vw - 1 : 0, wb = vw < NSTR - 1 ? vw + 1 : NSTR - 1;

    // the tile's whole region inside the grid in x and y (fast & kFastAll: every
    // tile -- a timing experiment of the edge tiles' select cost, wrong ghost
    // cells; STENCIL_TK_FAST, debug library)
    auto region_inner = [&](int bx, int by, int on) -> bool {
        return (fast & kFastAll) ||
               (on && int64_t(bx) * TX - XR * V >= 0 && int64_t(bx) * TX - XR * V + RW <= g.nx &&
                int64_t(by) * TY - K >= 0 && int64_t(by) * TY - K + RH <= g.ny);
    };
    // the next segment (units [lo, hi)) needs no ghost-cell select: its region
    // is inside in x and y, and for every intermediate stage s the planes
    // whose t_s reaches the output -- [za - (K - s), zb + K - s) -- are inside
    // in z (a halo side: the slab's halo planes count as inside).  The planes
    // the pipeline's fill and drain compute beyond them are never read.
    auto seg_fast = [&]() -> bool {
        if (!(fast & kFastSeg)) return false;
        const int t = int(lo / nzr);
        const int za = zbeg + int(lo - int64_t(t) * nzr);
        const int zb = za + (hi - lo < int64_t(zend - za) ? int(hi - lo) : zend - za);
        if (!region_inner(t % tiles_x, t / tiles_x, 1)) return false;
        // strongest at s = 1 (the widest reach): [za - K + 1, zb + K - 1)
        return za - (K - 1) >= (halo_lo ? -(K - 1) : 0) && zb + K - 1 <= (halo_hi ? nz + K - 1 : nz);
    };
    auto segment = [&](auto REV_, auto PROD_, auto SFAST_) {  // one segment: tile t, planes [za, zb)
    constexpr bool REV = decltype(REV_)::value;
    constexpr bool SFAST = decltype(SFAST_)::value;  // the whole segment without ghost-cell selects
    constexpr bool PROD = TIER && decltype(PROD_)::value;  // TIER producer (stores t_K into the slots)
    constexpr bool CONS = TIER && !PROD;                   // TIER consumer (reads the slots)
    const int t = int(lo / nzr);
    const int za = zbeg + int(lo - int64_t(t) * nzr);
    const int zb = za + (hi - lo < int64_t(zend - za) ? int(hi - lo) : zend - za);
    lo += zb - za;
    const int bx = t % tiles_x;
    const int by = t / tiles_x;
    const int64_t x = int64_t(bx) * TX - XR * V + int64_t(hl) * V;
    const int64_t y0 = int64_t(by) * TY - K + int64_t(vw) * RY;  // this strip's first row

    // Unconditional loads from clamped addresses (kernels_temporalk.hip): the
    // plane wait is then a counted vmcnt, not vmcnt(0).
    uint32_t off[RY];  // byte offset of this lane's vector in row k, from the biased plane base
    bool yin[RY], st[RY];
    const int64_t xmax = g.nx / V * V;
    const int64_t xc = x < xmax ? x : xmax;
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = vw * RY + k;
        const int64_t y = y0 + k;
        const int64_t yc = y < -1 ? -1 : (y > g.ny ? g.ny : y);
        off[k] = uint32_t((yc * g.row + xc + bias) * int64_t(sizeof(T)));
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= K && rr < RH - K && y < g.ny && hl >= XR && hl < LW - XR;
    }
    // SST: the 16-B store lanes (cells 4(l%32) .. +3 of strip row 2i + l/32)
    uint32_t soff[SST ? NI : 1];
    bool sfull[SST ? NI : 1], spart[SST ? NI : 1];
    const int64_t xs = int64_t(bx) * TX - XR * V + 4 * int64_t(lane & 31);
    if constexpr (SST) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int kk = 2 * i + (lane >> 5);
            const int rr = w * RY + kk;
            const int64_t y = y0 + kk;
            const bool ok = kk < RY && rr >= K && rr < RH - K && y < g.ny && 4 * (lane & 31) >= XR * V &&
                            4 * (lane & 31) < RW - XR * V;
            const int64_t yc = y < 0 ? 0 : (y > g.ny ? g.ny : y);
            const int64_t xc = xs < 0 ? 0 : (xs > g.nx ? g.nx : xs);
            soff[i] = uint32_t((yc * g.row + xc + bias) * int64_t(sizeof(T)));
            sfull[i] = ok && xs + 3 < g.nx;
            spart[i] = ok && xs < g.nx && xs + 3 >= g.nx;
        }
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    // TIER producer: the slot cells this lane stores per row -- its output
    // tile's, and the region's ghost cells (x in {-1, nx} or y in {-1, ny}:
    // ghost cells never change, and the consumers' regions read them from the
    // slots); V = 1
    // (ghost cells: x in {-1, nx} with y in [-1, ny], or y in {-1, ny} with x
    // in [-1, nx]; the x part per lane, the y part per row, uniform)
    const bool xghost = PROD && (x == -1 || x == g.nx);
    const bool xspan = PROD && x >= -1 && x <= g.nx;
    int tnb = -1;  // TIER: the neighbour tile (3 x 3, lanes 0..8 of wave 0) whose flag this lane watches
    if constexpr (TIER) {
        const int nbx = bx + lane % 3 - 1, nby = by + lane / 3 - 1;
        if (w == 0 && lane < 9 && nbx >= 0 && nbx < tiles_x && nby >= 0 && nby < tiles_y) tnb = nby * tiles_x + nbx;
    }
    uint32_t* const tier_mine = TIER ? (PROD ? tier.prod : tier.cons) + int64_t(t) * kTierFlagStride : nullptr;
    const uint32_t* const tier_flags = TIER ? (PROD ? tier.cons : tier.prod) : nullptr;  // + the watched tile's line
    // slot z's plane base (biased like src / dst)
    const char* const slots = TIER ? static_cast<const char*>(tier.slots) +
                                         (g.origin - (g.origin / plane) * plane - bias) * int64_t(sizeof(T))
                                   : nullptr;
    uint32_t tier_pv = 0;  // the prefetched flag
    // the whole region inside the grid in x and y: intermediate stages need no
    // ghost-cell select on steps whose stage planes are all inside in z
    const bool xy_inner = region_inner(bx, by, fast & kFastStep);
    const int ld_lo = halo_lo ? -K : -1;
    const int ld_hi = halo_hi ? nz + K - 1 : nz;
    const int zfirst = za - K > ld_lo ? za - K : ld_lo;
    const int zlast = zb + K - 1 < ld_hi ? zb + K - 1 : ld_hi;
    // march index m -> plane: the chunk is walked upward, or downward (REV)
    auto zr = [&](int m) { return REV ? za + zb - 1 - m : m; };
    // (the box kernels make each use of off[k] opaque to get the saddr +
    // 32-bit voffset form; here that costs the fp64 fast-path shape its
    // register fit -- 9 spilled VGPRs, 910 vs 1212 Gcell/s at 512^3 -- so the
    // hoisted 64-bit offsets stay, profiles/r02p_ab_saddr_fast.log)
    auto load_plane = [&](VT (&d)[RY], int m) {
        const int z = zr(m);
        const int zz = z < zfirst ? zfirst : (z > zlast ? zlast : z);
        if constexpr (CONS) {
            // consumer: every plane from the slots (sc1): plane z in slot z & rmask,
            // the fixed z-ghost planes -1 / nz in slots R / R + 1
            const int slot = zz < 0 ? tier.rmask + 1 : (zz >= nz ? tier.rmask + 2 : (zz & tier.rmask));
            const char* base = slots + int64_t(slot) * plane * int64_t(sizeof(T));
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = sc1_load<VT>(base + off[k]);
            return;
        }
        const char* base = src + int64_t(zz) * plane * int64_t(sizeof(T));
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(base + off[k]);
    };

    // TIER producer: one plane's output-tile and ghost cells into a slot
    auto tier_store_plane = [&](const VT (&d)[RY], int slot) {
        if constexpr (PROD) {
            char* base = const_cast<char*>(slots) + int64_t(slot) * plane * int64_t(sizeof(T));
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const int64_t y = y0 + k;
                const bool yghost = y == -1 || y == g.ny, yspan = y >= -1 && y <= g.ny;
                if ((st[k] && xin[0]) || (yghost && xspan) || (xghost && yspan)) sc1_store<VT>(base + off[k], d[k]);
            }
        }
    };
    static_assert(NS >= 4, "the input ring holds in(p-2) .. in(p+1) at least");
    constexpr int LCM = NS % 2 == 0 ? NS : 2 * NS;  // steps until ring slot and H parity repeat
    const int p0 = za - K;
    VT vin[NS][RY];                 // slot (q - p0) % NS holds in(q)
    VT H[K > 1 ? K - 1 : 1][2][RY]; // H[s-1][(q - p0) & 1] holds t_s(q), s < K (HL: s >= 2 only)
    // t_s(q) of parity `par`, row k: stage 1 from LDS with HL, else registers
    auto hget = [&](int s, int par, int k) -> VT {
        if (HL && s == 1) return *reinterpret_cast<const VT*>(&HLs[par][vw * RY + k][xl]);
        return H[s - 1][par][k];
    };
    auto hset = [&](int s, int par, int k, const VT& v) {
        if (HL && s == 1) *reinterpret_cast<VT*>(&HLs[par][vw * RY + k][xl]) = v;
        else H[s - 1][par][k] = v;
    };
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int k = 0; k < RY; ++k) vin[i][k] = VT{};
#pragma unroll
    for (int s = 0; s < (K > 1 ? K - 1 : 1); ++s)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int k = 0; k < RY; ++k) H[s][b][k] = VT{};
    if constexpr (CONS) {
        // the first loads read slot R (the bottom z-ghost plane): wait until
        // every producer in reach has stored it (and plane 0)
        if (tnb >= 0) tier_spin(tier_flags + tnb * kTierFlagStride, tier.base + 1u, tier.fail);
        __syncthreads();
    }
    if constexpr (SIG) {
        // halo gate: a chunk whose loads reach a halo plane waits for the
        // exchange that filled it (the launch follows the previous round's
        // launch on its queue, with no event wait for that exchange)
        if (gate.word && ((halo_lo && zfirst < 0) || (halo_hi && zlast >= nz))) {
            if (threadIdx.x == 0 && threadIdx.y == 0) gate_wait(gate);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < NS - 2; ++i) load_plane(vin[i], p0 + i);
    if constexpr (PROD) {  // the bottom z-ghost plane (p0 clamps to -1) into slot R
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tier_store_plane(vin[0], tier.rmask + 1);
    }


    auto stepb = [&](auto S_, int p, auto FAST_) {
        constexpr int S = decltype(S_)::value;  // (p - p0) % LCM
        constexpr bool FAST = decltype(FAST_)::value;  // no ghost-cell selects this step
        // fp32 two cells per lane (four: SPLIT): packed math (-DTK_PACK2=0 builds keep the scalar loop)
        constexpr bool kPack2 = TK_PACK2 && sizeof(T) == 4 && (V == 2 || (V == 4 && SPLIT));
        constexpr int P = DB ? (S & 1) : 0;  // buffer written this step
        constexpr int PR = DB ? (P ^ 1) : 0; // buffer read this step
        if constexpr (TIER) {
            // this step's input plane and the previous step's stores are done
            // (only plane p+1's RY loads, issued after them, may be in flight);
            // the flag prefetched last step is then in too
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
            if (tnb >= 0) {
                // producer: slot of plane p-K free (its consumers loaded plane
                // p-K-R); consumer: plane p+2, loaded at the end of this step, stored
                const int need = PROD ? p - K - tier.rmask : (p + 3 <= nz ? p + 3 : nz + 1);
                if (need > 0 && !tier_ge(tier_pv, tier.base + uint32_t(need)))
                    tier_spin(tier_flags + tnb * kTierFlagStride, tier.base + uint32_t(need), tier.fail);
            }
        }
        if constexpr (!(TK_PROBE_NOBAR && !SIG && !TIER)) __syncthreads();  // boundary rows of step p-1 are visible
        if constexpr (TIER) {
            // every wave's wait above is behind the barrier: publish the planes
            // stored (producer: t_K up to p-K-1) / loaded (consumer: up to p)
            const int done = PROD ? p - K : p + 1;
            if (threadIdx.x == 0 && threadIdx.y == 0 && done > 0 && done <= nz)
                tier_publish(tier_mine, tier.base + uint32_t(done));
        }
        // Row-major order: for each row k all K stages, so only one result per
        // stage is live at a time (stage s+1 of row k needs stage s of row k
        // only as z+; its y-neighbours are the previous step's planes in H).
        // Stage s's result then replaces, in H, the z- plane that stage s+1 of
        // this row has just consumed.
        // the neighbour strips' boundary rows, read where used (row 0 / RY-1)
#define STRIP_ABOVE(s) (*reinterpret_cast<const VT*>(&L[PR][s][wa][1][xl]))
#define STRIP_BELOW(s) (*reinterpret_cast<const VT*>(&L[PR][s][wb][0][xl]))
        bool zin[K];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            const int z = zr(p - s);
            const int lo_s = halo_lo ? -(K - s) : 0;
            const int hi_s = halo_hi ? nz + (K - s) : nz;
            zin[s - 1] = z >= lo_s && z < hi_s;
        }
        const int zo = p - K;  // t_K(p-K) -> HBM
        const bool do_store = DIAG != 3 && zo >= za && zo < zb;
        char* obase = dst + int64_t(zr(zo)) * plane * int64_t(sizeof(T));
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            VT prev{};  // this row's result of the previous stage
            auto stage = [&](auto s_) {
                constexpr int s = decltype(s_)::value;
                // t_{s-1} planes p-s (centre), p-s-1 (z-), p-s+1 (z+)
                VT c, zm, zp, up, dn;
                if constexpr (s == 1) {
                    c = vin[(S + NS - 1) % NS][k];
                    zm = vin[(S + NS - 2) % NS][k];
                    zp = vin[S % NS][k];
                    up = k == 0 ? STRIP_ABOVE(0) : vin[(S + NS - 1) % NS][k == 0 ? 0 : k - 1];
                    dn = k == RY - 1 ? STRIP_BELOW(0) : vin[(S + NS - 1) % NS][k == RY - 1 ? 0 : k + 1];
                } else {
                    c = hget(s - 1, (S - s + 4) & 1, k);
                    zm = hget(s - 1, (S - s + 5) & 1, k);
                    zp = prev;
                    up = k == 0 ? STRIP_ABOVE(s - 1) : hget(s - 1, (S - s + 4) & 1, k == 0 ? 0 : k - 1);
                    dn = k == RY - 1 ? STRIP_BELOW(s - 1) : hget(s - 1, (S - s + 4) & 1, k == RY - 1 ? 0 : k + 1);
                }
                const T wl = sdpp<kSShr1>(c[V - 1]);
                const T er = sdpp<kSShl1>(c[0]);
                VT o;
                if constexpr (kPack2) {
                    // fp32 pairs: the same sums as the loop below, the x
                    // pair scalar (its lane shifts fold into v_add_f32_dpp),
                    // the rest in packed math (v_pk_add_f32 / v_pk_fma_f32:
                    // both cells of the lane per instruction, each
                    // IEEE-rounded as the scalar op)
                    VT sum;
                    if constexpr (V == 2) sum = VT{wl + c[1], c[0] + er};
                    else sum = VT{wl + c[1], c[0] + c[2], c[1] + c[3], c[2] + er};
                    sum += up;
                    sum += dn;
                    sum += REV ? zp : zm;
                    sum += REV ? zm : zp;
                    o = DIAG == 2 ? c : __builtin_elementwise_fma(sum, (VT)(avg), VT{});
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        if (s < K && !FAST) o[j] = (zin[s - 1] && yin[k] && xin[j]) ? o[j] : c[j];
                        if (PROD && s == K && !FAST) o[j] = (yin[k] && xin[j]) ? o[j] : c[j];
                    }
                } else {
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    T sum = (j == 0 ? wl : c[j - 1]) + (j == V - 1 ? er : c[j + 1]);
                    sum += up[j];
                    sum += dn[j];
                    // the reference adds the lower plane first; marching down,
                    // the march's z+ is the lower one
                    sum += REV ? zp[j] : zm[j];
                    sum += REV ? zm[j] : zp[j];
                    o[j] = DIAG == 2 ? c[j] : sfma0(sum, avg);
                    if (s < K && !FAST) o[j] = (zin[s - 1] && yin[k] && xin[j]) ? o[j] : c[j];
                    // TIER producer: t_K keeps the ghost cells too (they go to the slots)
                    if (PROD && s == K && !FAST) o[j] = (yin[k] && xin[j]) ? o[j] : c[j];
                }
                }
                // t_{s-1}(p-s+1) takes the slot of t_{s-1}(p-s-1), consumed just now
                if constexpr (s >= 2) hset(s - 1, (S - s + 5) & 1, k, prev);
                prev = o;
            };
            stage(std::integral_constant<int, 1>{});
            stage(std::integral_constant<int, 2>{});
            if constexpr (K >= 3) stage(std::integral_constant<int, (K >= 3 ? 3 : 1)>{});
            if constexpr (K >= 4) stage(std::integral_constant<int, (K >= 4 ? 4 : 1)>{});
            if constexpr (K >= 5) stage(std::integral_constant<int, (K >= 5 ? 5 : 1)>{});
            if constexpr (K >= 6) stage(std::integral_constant<int, (K >= 6 ? 6 : 1)>{});
            static_assert(K >= 2 && K <= 6, "K = 2..6");
            if constexpr (PROD) {
                const int64_t y = y0 + k;
                const bool yghost = y == -1 || y == g.ny, yspan = y >= -1 && y <= g.ny;
                if (do_store && ((st[k] && xin[0]) || (yghost && xspan) || (xghost && yspan)))
                    sc1_store<VT>(const_cast<char*>(slots) + int64_t(zo & tier.rmask) * plane * int64_t(sizeof(T)) +
                                      off[k], prev);
                continue;
            }
            if constexpr (SST) {
                if (do_store) *reinterpret_cast<VT*>(&IMG[w * RY + k][xl]) = prev;
                continue;
            }
            if (do_store && st[k]) {
                T* q = reinterpret_cast<T*>(obase + off[k]);
                if (xst[V - 1]) {
                    __builtin_nontemporal_store(prev, reinterpret_cast<VT*>(q));
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j)
                        if (xst[j]) q[j] = prev[j];
                }
            }
        }
        if constexpr (SST) {
            // the wave's own image rows back as 16-B lane vectors (LDS ops of one
            // wave execute in order; the asm keeps the compiler from moving them)
            if (do_store) {
                asm volatile("" ::: "memory");
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const int kk = 2 * i + (lane >> 5) < RY ? 2 * i + (lane >> 5) : RY - 1;
                    const V4T v = *reinterpret_cast<const V4T*>(&IMG[w * RY + kk][4 * (lane & 31)]);
                    T* q = reinterpret_cast<T*>(obase + soff[i]);
                    if (sfull[i]) {
                        __builtin_nontemporal_store(v, reinterpret_cast<V4T*>(q));
                    } else if (spart[i]) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (xs + j < g.nx) q[j] = v[j];
                    }
                }
                asm volatile("" ::: "memory");
            }
        }
        // boundary rows for step p+1: stage 1's centre is in(p), stage s's is t_{s-1}(p-s+1)
        if constexpr (!DB) __syncthreads();  // single buffer: every read of it is done
        *reinterpret_cast<VT*>(&L[P][0][vw][0][xl]) = vin[S % NS][0];
        *reinterpret_cast<VT*>(&L[P][0][vw][1][xl]) = vin[S % NS][RY - 1];
#pragma unroll
        for (int s = 2; s <= K; ++s) {  // t_{s-1}(p-s+1), now in H
            *reinterpret_cast<VT*>(&L[P][s - 1][vw][0][xl]) = hget(s - 1, (S - s + 5) & 1, 0);
            *reinterpret_cast<VT*>(&L[P][s - 1][vw][1][xl]) = hget(s - 1, (S - s + 5) & 1, RY - 1);
        }
        if constexpr (SIG) {
            // right after the store of a face's last plane (the host makes
            // every chunk at least K planes long): the low face is planes
            // [zbeg, zbeg+K) of the first chunk, the high face [zend-K, zend)
            // of the last one, walked down (REV) so they come first.  Uniform
            // condition: every wave drains its stores, then one lane releases
            // and adds.
            const bool lo_here = !REV && za == zbeg && zo == za + K - 1;
            const bool hi_here = zb == zend && zo == (REV ? za + K - 1 : zb - 1);
            if (lo_here || hi_here) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0 && threadIdx.y == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const unsigned ntiles = unsigned(tiles_x) * unsigned(tiles_y);
                    // faces this workgroup completed (0, 1 or 2: a one-chunk
                    // slab of K planes stores both faces at the same step)
                    unsigned long long done = 0;
                    if (lo_here)
                        done += (__hip_atomic_fetch_add(&sig[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (hi_here)
                        done += (__hip_atomic_fetch_add(&sig[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (fsig && done) {
                        // every add of this face came after its workgroup's release
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        __hip_atomic_fetch_add(fsig, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
        }
        if constexpr (TIER) {  // read at the next step, behind its counted wait
            if (tnb >= 0) tier_pv = tier_poll(tier_flags + tnb * kTierFlagStride);
        }
        if constexpr (DIAG != 1) load_plane(vin[(S + NS - 2) % NS], p + NS - 2);  // slot of in(p-2), consumed above
    };
    auto step = [&](auto S_, int p) {
        if constexpr (SFAST) {
            stepb(S_, p, std::true_type{});
            return;
        }
        // compiled for the fp64 one-cell-per-lane shapes only: duplicating the
        // step costs the fp32 / signalled shapes their register fit
        constexpr bool kFast = TK_FAST_PATH && FP && sizeof(T) == 8 && V == 1 && !SIG && DIAG == 0;
        if constexpr (!kFast) {
            stepb(S_, p, std::false_type{});
            return;
        }
        bool all_in = xy_inner;
#pragma unroll
        for (int s = 1; s < K; ++s) {
            const int z = zr(p - s);
            all_in = all_in && z >= (halo_lo ? -(K - s) : 0) && z < (halo_hi ? nz + (K - s) : nz);
        }
        if (all_in) stepb(S_, p, std::true_type{});
        else stepb(S_, p, std::false_type{});
    };

    const int plast = zb + K - 1;
    int p = p0;
    for (; p + LCM - 1 <= plast; p += LCM) unroll_steps<0, LCM>(step, p);
    tail_steps<0, LCM - 1>(step, p, plast);
    if constexpr (TIER) {
        if constexpr (PROD) {
            // the top z-ghost plane into slot R + 1: the ring's last loads
            // were clamped to plane nz
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            tier_store_plane(vin[0], tier.rmask + 2);
        }
        // the last stores / loads are done: the whole range (+ the ghost slot)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && threadIdx.y == 0) tier_publish(tier_mine, tier.base + uint32_t(nz + 1));
    }
    };  // segment
    // fp64 shapes of the default build only: the fp32 K = 5 strip runs its
    // select-free loop no faster (4096^2 x 256: 2441 vs 2441 Gcell/s in one
    // process with 24 % fewer instructions per step), and the
    // packed-regime fp64 grids (max-ILP build) have the per-step choice
#ifdef STRIP_ILP_TU
    constexpr bool kSegFast = false;
#else
    constexpr bool kSegFast = TK_SEG_FAST && FP && DIAG == 0 && !TIER && sizeof(T) == 8;
#endif
    using F = std::false_type;
    using Tr = std::true_type;
    while (lo < hi) {
        if constexpr (TIER) {
            if (tprod) segment(F{}, Tr{}, F{});
            else segment(F{}, F{}, F{});
        } else if constexpr (kSegFast) {
            const bool sf = seg_fast();
            if (SIG && rev) {
                if (sf) segment(Tr{}, F{}, Tr{});
                else segment(Tr{}, F{}, F{});
            } else {
                if (sf) segment(F{}, F{}, Tr{});
                else segment(F{}, F{}, F{});
            }
        } else if constexpr (SIG) {
            if (rev) segment(Tr{}, F{}, F{});
            else segment(F{}, F{}, F{});
        } else {
            segment(F{}, F{}, F{});
        }
    }
}

int senv_int(const char* name, int dflt) { return knob(name, dflt); }

template <typename T, int V, int RY, int NW, int K, bool DB = true, int DIAG = 0, bool SIG = false, int NS = 4,
          bool FP = true, bool HL = false, bool SPLIT = false>
int launch_st(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, hipStream_t s,
              unsigned* sig = nullptr, int* nsig = nullptr, unsigned long long* fsig = nullptr,
              const StripGate& gate = StripGate{}) {
    using Tl = StripTile<T, V, RY, NW, K, DB, SPLIT>;
    static_assert(Tl::lds_bytes + (HL ? size_t(2) * Tl::RH * Tl::RW * sizeof(T) : 0) <= 160 * 1024, "LDS budget");
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    if ((g.plane + g.row + 64) * int64_t(sizeof(T)) >= (int64_t(1) << 32) || g.nz + 2 * K >= (int64_t(1) << 30))
        return set_error(STENCIL_EINVAL, "plane too large for tkstrip (4 GiB per plane, 2^30 planes)");
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    auto kern = tkstrip_7pt<T, V, RY, NW, K, DB, DIAG, SIG, NS, FP, HL, false, SPLIT>;
    const int64_t tiles = gx * gy;
    int dev = 0, slots = 0;
    STENCIL_HIP_CHECK(hipGetDevice(&dev));
    if (const int rc = resident_slots(kern, 64 * NW, &slots)) return rc;
    int zc = senv_int("STENCIL_TK_ZCHUNK", 0);
    int64_t nb = 0;
    if (zc > 0) {
        nb = tiles * ((nz + zc - 1) / zc);  // fixed chunks (tests: seams, short chunks)
    } else {
        if (!SIG && senv_int("STENCIL_TK_BALANCE", 0)) {
            // one equal share of the (tile, z) units per slot, each share at
            // least 4K planes long (a segment costs 2K planes of pipeline fill).
            // Measured 20-30 % SLOWER than whole chunks on MI355X (512^3 fp64
            // 902 vs 1120 Gcell/s, 2048^2 x 512 984 vs 1386): the shares start
            // at scattered z, so x/y-neighbour tiles no longer read their
            // shared halo lines at about the same time and those re-reads miss
            // L2 / Infinity Cache.  Chunk rounds keep all tiles of a chunk in
            // z lock-step.
            nb = std::max<int64_t>(1, std::min<int64_t>(slots, tiles * nz / (4 * K)));
            zc = 0;  // one equal share per workgroup (the kernel's zchunk == 0 mode); never packed
        } else {
            // whole chunks: the count minimising rounds x (chunk + 2K)
            int64_t best_c = 1, best = INT64_MAX;
            for (int64_t c = 1; c <= nz; ++c) {
                const int64_t z = (nz + c - 1) / c;
                if (c > 1 && z < 2 * K) break;
                const int64_t cost = ((tiles * c + slots - 1) / slots) * (z + 2 * K);
                if (cost <= best) best = cost, best_c = c;
            }
            // A slab of a multi-GPU job (halo flags): its halo exchange runs
            // kernels (RCCL P2P, or the face wait) beside this launch, and a
            // grid that fills every CU for several rounds loses a whole round
            // of balance to one busy CU: 512^3 fp64 K=4, 990 workgroups
            // 0.50 -> 0.565 ms with a 1-wave kernel resident on another queue
            // (tools/sig_time.py), 220 workgroups (2 chunks) 0.48 either way.
            // So: the most chunks that still fit one round with a CU per XCD
            // to spare, when the tiles fit at all.
            if (l.prob.flags & (STENCIL_HALO_LO | STENCIL_HALO_HI)) {
                const int64_t room = slots - slots / 32;
                for (int64_t c = 1; tiles * c <= room && c <= nz; ++c) {
                    if (c > 1 && (nz + c - 1) / c < 2 * K) break;
                    best_c = c;
                }
                // a face-signalled grid of several rounds (4096^2 planes: ~6400
                // tiles): at least 4 chunks per tile, whose two face chunks the
                // kernel dispatches first, so the faces are stored about halfway
                // through the launch instead of in its last round (+2 % plane
                // steps for the extra chunk fills)
                if (SIG && tiles > room) {
                    int64_t want = senv_int("STENCIL_TK_SIG_CHUNKS", 4);
                    while (want > 1 && (nz + want - 1) / want < 2 * K) --want;
                    best_c = std::max(best_c, want);
                }
            }
            zc = int((nz + best_c - 1) / best_c);
            nb = tiles * ((nz + zc - 1) / zc);
        }
    }
    if constexpr (SIG) {
        // every chunk at least K planes (a face lies inside one chunk)
        int64_t nch = (nz + zc - 1) / zc;
        auto last = [&](int64_t c) { return nz - (c - 1) * ((nz + c - 1) / c); };
        while (nch > 1 && ((nz + nch - 1) / nch < K || last(nch) < K)) --nch;
        zc = int((nz + nch - 1) / nch);
        nb = tiles * nch;
        if (nsig) *nsig = int(tiles);
    }
    const int* sched = nullptr;
    std::atomic<int>* verdict = nullptr;
    const int64_t nb_equal = nb;
    // default: the packed longest-first schedule where the model predicts a
    // gain AND the first launch measured it faster (pick_schedule; 512^3 fp64
    // 1173 vs 1105 Gcell/s, tools/pack_ab.sh); not for slabs of a multi-GPU
    // job, whose one-round grid above is deliberate
    const int pack_mode = api_knob("STENCIL_TK_PACK", 1);
    const bool halo = l.prob.flags & (STENCIL_HALO_LO | STENCIL_HALO_HI);
    if (zc > 0 && pack_mode && senv_int("STENCIL_TK_ZCHUNK", 0) <= 0 && (!halo || SIG) &&
        (!SIG || knob("STENCIL_TK_PACK_SIG", 1))) {
        // face-signalled slab launches: the model for one CU per XCD spared
        // (the exchange's kernels run beside the launch), faces in the first
        // round's chunks, and no timing trial (its extra launches would add to
        // the face counters the exchange waits on): the model's choice
        // STENCIL_TK_SIG_SPARE (debug library): CUs per XCD the packed
        // face-signalled schedule leaves to the exchange (default 1)
        const int pslots = SIG ? slots - slots / 32 * senv_int("STENCIL_TK_SIG_SPARE", 1) : slots;
        // the packed table's generations in XCD patches for long jobs (the
        // width with the most same-XCD neighbour tiles; C2: 5 of 10 tiles,
        // reads 1.81x -> 1.46x compulsory, +1-1.5 % at the power limit, -1.5 %
        // below it: DESIGN.md §5.1), tile-major otherwise; STENCIL_TK_PACK_XCD
        // (debug library): that width always (0: tile-major)
        const int pack_xcd = senv_int("STENCIL_TK_PACK_XCD", tl_sustained ? -1 : 0);
        const int rc = packed_schedule(reinterpret_cast<const void*>(kern), dev, gx * gy, nz, K, 2 * K, pslots, zc, s,
                                       tl_dry_launch != nullptr, &sched, &nb, &verdict, SIG, gx, pack_xcd);
        if (rc != STENCIL_OK) return rc;
        if (pack_mode != 1 || SIG) verdict = nullptr;  // 2: the model's choice, unmeasured
        if (verdict && verdict->load() == kPackEqual) sched = nullptr, nb = nb_equal, verdict = nullptr;
    }
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for tkstrip");
    // interior steps without ghost-cell selects, per step (fp64 one-cell-per-lane
    // shapes): by default only where the packed schedule runs -- few tiles,
    // 512^3 fp64 1212 vs 1175 Gcell/s -- since on large planes the duplicated
    // step loses (2048^2 x 512 1357 vs 1384, 2048^3 1310 vs 1365;
    // profiles/r02o_ab_tk_fast.log); per segment (TK_SEG_FAST) wherever compiled
    const int fast_env = senv_int("STENCIL_TK_FAST", -1);
    auto fast_of = [&](bool packed) { return fast_env >= 0 ? fast_env : (packed ? kFastStep : 0) | kFastSeg; };
    if (senv_int("STENCIL_TK_VERBOSE", 0)) {
        int per_cu = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, 0);
        std::fprintf(stderr, "tkstrip K=%d V=%d RY=%d NW=%d: tiles %lldx%lld, zchunk %d, %lld workgroups, %d per CU\n", K,
                     V, RY, NW, (long long)gx, (long long)gy, zc, (long long)nb, per_cu);
    }
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if ((lo || hi) && l.zghost < K)
        return set_error(STENCIL_EINVAL, "%d fused steps across a slab halo need halo >= %d (got %lld)", K, K,
                         (long long)l.zghost);
    if (LaunchInfo* info = tl_dry_launch) {  // stencil_sweepk_geometry: describe, do not launch
        info->workgroups = nb;
        info->zchunk = zc;
        info->packed = sched == nullptr ? 0 : (verdict && verdict->load() == kPackUntested ? 2 : 1);
        info->steps = K;
        info->slots = slots;
        return STENCIL_OK;
    }
    // XCD-patch work order (STENCIL_TK_XCD = patch width, the box kernel's
    // map) for grids of more than two rounds of tiles: fp32 16 tiles wide --
    // 4096^2 x 256 fp32 K = 5 reads 32.1 -> 21.6 GB per launch (1.87x ->
    // 1.25x compulsory) and runs 3 % faster, C3 2612 -> 2722 Gcell/s; fp64 8
    // wide on launches of a whole grid -- reads 1.76x -> 1.19x at 2048^2 x
    // 512, NS 2048^3 1317 -> 1373 Gcell/s over three alternating sustained
    // runs -- but not on slab launches (halo planes: the staged rounds ran
    // 3.5 % slower, NS4096 rank of 4 1292 vs 1340) nor on z-range launches
    // (rolling C4: 1262 vs 1351)
    const bool whole = !halo && begin == 0 && end == g.nz;
    const int xcd_dflt = tiles > 2 * int64_t(slots) ? (sizeof(T) == 4 ? 16 : (whole ? 8 : 0)) : 0;
    const int xcd_pw = !SIG && zc > 0 ? senv_int("STENCIL_TK_XCD", xcd_dflt) : 0;
    auto launch = [&](bool packed) {
        const int64_t n = packed ? nb : (xcd_pw > 0 ? (nb_equal + 7) / 8 * 8 : nb_equal);
        hipLaunchKernelGGL(kern, dim3(unsigned(n)), dim3(64, NW, 1), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(out), g, int(begin), int(end), zc, int(gx),
                           int(gy), int(lo), int(hi), avg_weight<T>(l.prob), sig, fsig, packed ? sched : nullptr,
                           fast_of(packed), packed ? 0 : xcd_pw, TierArgs{}, SIG ? gate : StripGate{});
        return hipGetLastError();
    };
    if (sched && verdict && verdict->load() == kPackUntested) return pick_schedule(verdict, s, launch);
    if (const hipError_t e = launch(sched != nullptr); e != hipSuccess)
        return set_error(STENCIL_EHIP, "kernel launch failed: %s (tkstrip)", hipGetErrorString(e));
    return STENCIL_OK;
}

// ---- the two-tier launch (TIER, above): host side --------------------------
#ifndef STRIP_ILP_TU
using TierKernelShape = StripTile<double, 1, 7, 8, 4, true>;
constexpr int kTierSlots = 16;  // R: plane slots of the producer -> consumer ring (2.2 MB each at 512^2 fp64)

int tier_tiles(const stencil_layout& l, int64_t* tiles) {
    const Geom g = geom_of(l);
    *tiles = ((g.nx + TierKernelShape::TX - 1) / TierKernelShape::TX) * ((g.ny + TierKernelShape::TY - 1) / TierKernelShape::TY);
    return STENCIL_OK;
}
#endif

}  // namespace

#ifndef STRIP_ILP_TU
// Can the grid run the two-tier launch?  The fp64 7-point star, K = 4 strip
// shape, a single grid (no slab halos), at least 2K planes, and both tiers'
// workgroups resident at once (2 x tiles <= the device's workgroup slots).
bool tier_eligible(const stencil_layout& l) {
    if (l.prob.dtype != STENCIL_F64 || !temporal2_supports(l.prob)) return false;
    if (l.prob.flags & (STENCIL_HALO_LO | STENCIL_HALO_HI)) return false;
    if (l.prob.nz < 8 || l.prob.nx < 1 || l.prob.ny < 1) return false;
    int64_t tiles = 0;
    tier_tiles(l, &tiles);
    int slots = 0;
    if (resident_slots(tkstrip_7pt<double, 1, 7, 8, 4, true, 0, false, 4, false, true, true>, 64 * 8, &slots) !=
        STENCIL_OK)
        return false;
    return 2 * tiles <= slots;
}

// The slots + flags live in one device buffer per GPU, kept for the process
// (allocated on first use, grown when a larger plane needs it) and held by
// one job at a time: a job that finds it taken (another stream of the same
// process in the middle of a two-tier job) gets STENCIL_EUNSUPPORTED and the
// caller runs the K = 4 launches instead.
namespace {
struct TierBuffer {
    void* mem = nullptr;
    size_t bytes = 0;
    bool busy = false;
};
std::mutex g_tier_mu;
std::map<int, TierBuffer> g_tier_buf;
}  // namespace

int tier_begin(const stencil_layout& l, hipStream_t s, TierJob* j) {
    *j = TierJob{};
    int64_t tiles = 0;
    tier_tiles(l, &tiles);
    // R slots for the ring + 2 for the fixed z-ghost planes
    const size_t slot_bytes = size_t(kTierSlots + 2) * size_t(l.plane) * sizeof(double) + 256;
    const size_t flag_bytes = size_t(2 * tiles) * kTierFlagStride * sizeof(uint32_t);
    const size_t bytes = slot_bytes + flag_bytes + 256;
    int dev = 0;
    STENCIL_HIP_CHECK(hipGetDevice(&dev));
    void* mem = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_tier_mu);
        TierBuffer& b = g_tier_buf[dev];
        if (b.busy) return set_error(STENCIL_EUNSUPPORTED, "the two-tier buffer of device %d is in use", dev);
        if (b.bytes < bytes) {
            if (b.mem) {
                (void)hipDeviceSynchronize();  // an earlier job's launches may still read it
                (void)hipFree(b.mem);
                b.mem = nullptr;
                b.bytes = 0;
            }
            if (hipMalloc(&b.mem, bytes) != hipSuccess) {
                (void)hipGetLastError();
                b.mem = nullptr;
                return set_error(STENCIL_ENOMEM, "two-tier buffer of %zu bytes", bytes);
            }
            b.bytes = bytes;
        }
        b.busy = true;
        mem = b.mem;
    }
    char* m = static_cast<char*>(mem);
    if (hipMemsetAsync(m + slot_bytes, 0, flag_bytes + 256, s) != hipSuccess) {
        std::lock_guard<std::mutex> lock(g_tier_mu);
        g_tier_buf[dev].busy = false;
        return set_error(STENCIL_EHIP, "two-tier flag reset failed");
    }
    j->mem = mem;
    j->tiles = tiles;
    j->a.slots = m;
    j->a.prod = reinterpret_cast<uint32_t*>(m + slot_bytes);
    j->a.cons = j->a.prod + tiles * kTierFlagStride;
    j->a.fail = reinterpret_cast<unsigned*>(m + slot_bytes + flag_bytes);
    j->a.base = 0;
    j->a.rmask = kTierSlots - 1;
    return STENCIL_OK;
}

// One launch: 2K = 8 sweeps of the whole grid, in -> out.
int tier_launch(const stencil_layout& l, const void* in, void* out, TierJob* j, hipStream_t s) {
    const Geom g = geom_of(l);
    const int64_t gx = (g.nx + TierKernelShape::TX - 1) / TierKernelShape::TX;
    const int64_t gy = (g.ny + TierKernelShape::TY - 1) / TierKernelShape::TY;
    if ((g.plane + g.row + 64) * int64_t(sizeof(double)) >= (int64_t(1) << 32) || g.nz >= (int64_t(1) << 30))
        return set_error(STENCIL_EINVAL, "plane too large for the two-tier launch");
    auto kern = tkstrip_7pt<double, 1, 7, 8, 4, true, 0, false, 4, false, true, true>;
    const int fast = 1;  // few tiles: the interior fast path pays (as the packed regime)
    hipLaunchKernelGGL(kern, dim3(unsigned(2 * j->tiles)), dim3(64, 8, 1), 0, s, static_cast<const double*>(in),
                       static_cast<double*>(out), g, 0, int(g.nz), 0, int(gx), int(gy), 0, 0,
                       avg_weight<double>(l.prob), nullptr, nullptr, nullptr, fast, 0, j->a, StripGate{});
    STENCIL_LAUNCH_CHECK();
    j->a.base += uint32_t(g.nz + 1);  // the flags end at base + nz + 1: the next launch's origin
    return STENCIL_OK;
}

// Free the job's memory (stream-ordered) and report whether any hand-off wait
// gave up (then the grid is wrong): one host wait on `s`.
int tier_end(TierJob* j, hipStream_t s, bool* failed) {
    *failed = false;
    if (!j->mem) return STENCIL_OK;
    unsigned f = 0;
    hipError_t e = hipMemcpyAsync(&f, j->a.fail, sizeof f, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the job's launches are done: the buffer is free
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lock(g_tier_mu);
        g_tier_buf[dev].busy = false;
    }
    j->mem = nullptr;
    if (e != hipSuccess) return set_error(STENCIL_EHIP, "two-tier job: %s", hipGetErrorString(e));
    *failed = f != 0;
    return STENCIL_OK;
}
#endif  // !STRIP_ILP_TU

#ifdef STRIP_ILP_TU
// kernels_strip_ilp.hip: the two default shapes measured faster when this file is compiled under LLVM's
// gcn-max-ilp machine scheduler: the fp64 K = 4 strip on grids of at most 2 tiles per
// CU slot (the packed schedule with its interior fast path: 512^3 +1.5 %) and the fp32 K = 5 strip (C3).
// (kernels_strip_probe.hip builds this TU a third time, as launch_tkstrip_probe: a compile-time variant)
#ifndef STRIP_ILP_FN
#define STRIP_ILP_FN launch_tkstrip_ilp
#endif
int STRIP_ILP_FN(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                 hipStream_t s) {
#ifdef TK_PROBE_SPLIT64
    if (l.prob.dtype == STENCIL_F64 && steps == 4)
        return launch_st<double, 2, TK_PROBE_SPLIT64, 8, 4, false, 0, false, 4, true, true, true>(l, in, out, begin, end, s);
#endif
    if (l.prob.dtype == STENCIL_F64 && steps == 4) return launch_st<double, 1, 7, 8, 4>(l, in, out, begin, end, s);
#ifdef TK_PROBE_SPLIT
    if (l.prob.dtype == STENCIL_F32 && steps == 5)
        return launch_st<float, 4, TK_PROBE_SPLIT, 8, 5, false, 0, false, 4, true, true, true>(l, in, out, begin, end, s);
#endif
    if (l.prob.dtype == STENCIL_F32 && steps == 5)
        return launch_st<float, 2, 5, 8, 5, true, 0, false, TK_ILP_NS32>(l, in, out, begin, end, s);
    return set_error(STENCIL_EINVAL, "no max-ILP strip shape for %d steps", steps);
}
#else
// Makespan (in plane steps) of workgroups of the given plane counts on
// `slots` one-workgroup CU slots: workgroup i goes to XCD i % 8 (the
// dispatcher's round robin), and inside an XCD to the slot that frees first
// (in-order dispatch); a chunk of n planes costs n + fill steps (pipeline fill:
// 2K for the 7-point strip kernel, 3K for the box's).
static int64_t simulate_makespan(const std::vector<int>& len, int fill, int slots) {
    constexpr int kXcd = 8;
    const int per = std::max(1, slots / kXcd);
    std::vector<std::vector<int64_t>> free_at(kXcd, std::vector<int64_t>(per, 0));
    int64_t span = 0;
    for (size_t i = 0; i < len.size(); ++i) {
        auto& f = free_at[i % kXcd];
        auto it = std::min_element(f.begin(), f.end());
        *it += len[i] + fill;
        span = std::max(span, *it);
    }
    return span;
}

// The dispatcher-model search behind packed_schedule (host only): chunks of
// Lc planes per tile, longest first, for every Lc in [max(fill, nz/16), nz];
// *base = the simulated makespan of equal chunks of zc planes, *best the best
// packed one (force_lc > 0: that Lc, *best = -1), *tab its {tile, first
// plane, planes} table (empty when no Lc beats equal chunks).
static void pack_search(int64_t tiles, int64_t nz, int fill, int slots, int zc, int force_lc, std::vector<int>* tab_out,
                        int64_t* base_out, int64_t* best_out) {
    auto build = [&](int64_t lc, std::vector<int>& tab) {
        lc = std::max<int64_t>(1, lc);
        struct Item { int len, c, t, z; };
        std::vector<Item> items;
        for (int64_t t = 0; t < tiles; ++t)
            for (int64_t z = 0, c = 0; z < nz; z += lc, ++c)
                items.push_back({int(std::min<int64_t>(lc, nz - z)), int(c), int(t), int(z)});
        std::stable_sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
            return a.len != b.len ? a.len > b.len : (a.c != b.c ? a.c < b.c : a.t < b.t);
        });
        std::vector<int> len;
        tab.clear();
        for (const Item& it : items) {
            len.push_back(it.len);
            tab.insert(tab.end(), {it.t, it.z, it.len});
        }
        return simulate_makespan(len, fill, slots);
    };
    std::vector<int> tab, best_tab;
    const int64_t base = build(zc, tab);
    int64_t best = base;
    for (int64_t lc = std::max<int64_t>(fill, nz / 16); lc <= nz && force_lc <= 0; lc += std::max<int64_t>(1, nz / 256)) {
        const int64_t m = build(lc, tab);
        if (m < best) best = m, best_tab = tab;
    }
    if (force_lc > 0) {
        build(force_lc, best_tab);
        best = -1;  // always used
    }
    *tab_out = std::move(best_tab);
    *base_out = base;
    *best_out = best;
}

const int* const kDrySchedule = reinterpret_cast<const int*>(uintptr_t(16));

// STENCIL_TK_PACK (default 1; 0 = equal chunks): chunks of Lc planes per tile (the last one
// shorter), longest first -- every tile's full chunks start in z lock-step,
// the short remainders fill the CUs the full chunks leave idle.  Lc is the
// one with the shortest simulated makespan; used only when it beats the
// equal-chunk grid (zc planes per chunk) by 2 %.  The table is built once per
// shape and kept for the process.
// The table lives in the memory of the device it was built on: the cache is
// keyed by kernel and device ordinal and guarded (a process may drive several
// GPUs from several threads: stencil_set_device is per thread).
// Rewrite a packed table so that each tile's faces lie in full chunks: its
// first full chunk at plane 0 (up), its last full chunk ending at nz
// (planes < 0: down), the short remainder between them.  Same lengths per
// tile, so the same dispatch order and makespan.  False (no table) when a
// tile has fewer than 3 chunks.
static bool faces_outward(std::vector<int>& tab, int64_t nz) {
    std::map<int, std::vector<size_t>> by_tile;  // entry indices of each tile, in table order
    int lc = 0;
    for (size_t i = 0; i < tab.size(); i += 3) {
        by_tile[tab[i]].push_back(i);
        lc = std::max(lc, tab[i + 2]);
    }
    for (auto& [t, idx] : by_tile) {
        if (idx.size() < 3) return false;
        int64_t z = 0;
        size_t full_seen = 0, full = 0;
        for (size_t i : idx) full += tab[i + 2] == lc;
        for (size_t i : idx) {  // full chunks bottom-up, the last one at the top; the remainder after the others
            if (tab[i + 2] != lc) continue;
            if (++full_seen == full) {
                tab[i + 1] = int(nz - lc);
                tab[i + 2] = -lc;
            } else {
                tab[i + 1] = int(z);
                z += lc;
            }
        }
        for (size_t i : idx)
            if (tab[i + 2] > 0 && tab[i + 2] != lc) tab[i + 1] = int(z), z += tab[i + 2];
        if (z != nz - lc) return false;  // the lengths do not tile the range as expected
    }
    return true;
}

// Reorder a packed table's generations into XCD patches (packed_schedule's
// xcd_w, common.hpp).  A generation is a run of entries with the same
// length and first plane (the tiles' same chunk, dispatched together).
static void xcd_patch_order(std::vector<int>& tab, int64_t tiles_x, int w) {
    constexpr int kXcd = 8;
    const size_t n = tab.size() / 3;
    for (size_t g0 = 0; g0 < n;) {
        size_t g1 = g0 + 1;
        while (g1 < n && tab[3 * g1 + 1] == tab[3 * g0 + 1] && tab[3 * g1 + 2] == tab[3 * g0 + 2]) ++g1;
        // the generation's tiles in patch order: column strips of w tiles,
        // row-major inside a strip
        std::vector<int> t;
        for (size_t i = g0; i < g1; ++i) t.push_back(tab[3 * i]);
        std::stable_sort(t.begin(), t.end(), [&](int a, int b) {
            const int64_t sa = (a % tiles_x) / w, sb = (b % tiles_x) / w;
            return sa != sb ? sa < sb : a < b;
        });
        // XCD x takes the next cnt[x] tiles of that order, into its positions
        std::vector<size_t> pos[kXcd];
        for (size_t i = g0; i < g1; ++i) pos[i % kXcd].push_back(i);
        size_t k = 0;
        for (int x = 0; x < kXcd; ++x)
            for (size_t i : pos[x]) tab[3 * i] = t[k++];
        g0 = g1;
    }
}

// Same-XCD x/y neighbour pairs of a table (workgroup i -> XCD i % 8, per
// generation), and the patch width in [2, min(tiles_x, 16)] that maximises
// them (the smallest on ties; 0 when no width beats tile-major).
static int64_t same_xcd_pairs(const std::vector<int>& tab, int64_t tiles_x) {
    constexpr int kXcd = 8;
    std::map<std::tuple<int, int, int>, int> where;  // (tile, first plane, planes) -> XCD
    for (size_t i = 0; i < tab.size() / 3; ++i) where[{tab[3 * i], tab[3 * i + 1], tab[3 * i + 2]}] = int(i % kXcd);
    int64_t pairs = 0;
    for (const auto& [k, x] : where) {
        const int t = std::get<0>(k);
        for (int nb : {t + 1, t + int(tiles_x)}) {
            if (nb == t + 1 && (t + 1) % tiles_x == 0) continue;
            auto it = where.find({nb, std::get<1>(k), std::get<2>(k)});
            pairs += it != where.end() && it->second == x;
        }
    }
    return pairs;
}
static int best_patch_width(const std::vector<int>& tab, int64_t tiles_x) {
    int best_w = 0;
    int64_t best = same_xcd_pairs(tab, tiles_x);
    for (int w = 2; w <= std::min<int64_t>(tiles_x, 16); ++w) {
        std::vector<int> t = tab;
        xcd_patch_order(t, tiles_x, w);
        const int64_t p = same_xcd_pairs(t, tiles_x);
        if (p > best) best = p, best_w = w;
    }
    return best_w;
}

int packed_schedule(const void* kern, int dev, int64_t tiles, int64_t nz, int K, int fill, int slots, int zc,
                    hipStream_t s, bool dry, const int** sched, int64_t* nb, std::atomic<int>** verdict,
                    bool faces_out, int64_t tiles_x, int xcd_w) {
    // Only grids of few tiles: with more than 2 tiles per slot the equal
    // chunks already fill the rounds (2048^2 x 512 fp64: packed 1312 vs 1315
    // Gcell/s), and the search would cost host time at the first launch.
    if (tiles > 2 * int64_t(slots)) return STENCIL_OK;
    if (zc <= 0) return STENCIL_OK;  // no equal-chunk grid to compare with (balanced split)
    // The first real launch of a shape builds and uploads BOTH work orders'
    // tables (tile-major and the long jobs' XCD patches): a long call that
    // follows short ones -- a slab job's untimed settle rounds, then its timed
    // run -- then finds its table ready instead of searching and uploading
    // (a host sync) inside its timed rounds.
    static thread_local bool sibling = false;
    if (!dry && !sibling && tiles_x > 0 && (xcd_w == 0 || xcd_w == -1)) {
        sibling = true;
        const int* d = nullptr;
        int64_t n = 0;
        const int rc = packed_schedule(kern, dev, tiles, nz, K, fill, slots, zc, s, false, &d, &n, nullptr, faces_out,
                                       tiles_x, xcd_w == 0 ? -1 : 0);
        sibling = false;
        if (rc != STENCIL_OK) return rc;
    }
    struct Entry {
        std::vector<int> host;  // {tile, first plane, planes} per workgroup; empty: not used
        int* table = nullptr;   // its device copy, uploaded on the first real launch
        int64_t workgroups = 0;
        std::atomic<int> verdict{kPackUntested};
    };
    static std::mutex mu;
    // map nodes never move: the verdict's address stays valid for the process
    static std::map<std::tuple<const void*, int, int64_t, int64_t, int, int, int, int>, Entry> cache;
    std::unique_lock<std::mutex> lock(mu);
    // STENCIL_TK_PACK_LC (experiments): chunks of exactly this many planes,
    // used whatever the model says
    const int force_lc = senv_int("STENCIL_TK_PACK_LC", 0);
    if (tiles_x <= 0) xcd_w = 0;
    int xcd_w_used = xcd_w;  // xcd_w < 0: chosen below (best_patch_width)
    const auto key = std::make_tuple(kern, dev, tiles, nz, K, slots, force_lc, xcd_w);
    auto hit = cache.find(key);
    if (hit == cache.end()) {
        std::vector<int> best_tab;
        int64_t base = 0, best = 0;
        pack_search(tiles, nz, fill, slots, zc, force_lc, &best_tab, &base, &best);
        hit = cache.try_emplace(key).first;
        if (faces_out && !best_tab.empty() && !faces_outward(best_tab, nz)) best_tab.clear();
        if (xcd_w < 0 && !best_tab.empty()) xcd_w_used = best_patch_width(best_tab, tiles_x);
        if (xcd_w_used > 0 && !best_tab.empty()) xcd_patch_order(best_tab, tiles_x, xcd_w_used);
        if (!best_tab.empty() && (best * 50 < base * 49 || force_lc > 0)) {
            hit->second.workgroups = int64_t(best_tab.size() / 3);
            hit->second.host = std::move(best_tab);
        }
        if (senv_int("STENCIL_TK_VERBOSE", 0))
            std::fprintf(stderr, "pack: equal chunks %lld steps, packed %lld steps (%lld workgroups, XCD patches %d wide)%s\n",
                         (long long)base, (long long)best, (long long)hit->second.workgroups, xcd_w_used,
                         hit->second.host.empty() ? " -- not used" : "");
    }
    Entry& e = hit->second;
    if (e.host.empty()) return STENCIL_OK;
    if (dry) {  // geometry query: no upload, no GPU work
        *sched = kDrySchedule;
        *nb = e.workgroups;
        if (verdict) *verdict = &e.verdict;
        return STENCIL_OK;
    }
    if (!e.table) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
            (void)hipGetLastError();
            cap = hipStreamCaptureStatusActive;
        }
        if (cap != hipStreamCaptureStatusNone) return STENCIL_OK;  // no allocation inside a capture: equal chunks
        // Upload on a private stream of the caller's device, outside the
        // lock: the host waits for this copy only -- not for the work queued
        // on `s` (a slab round's counter wait and exchange) -- and other
        // threads / devices are not held behind it.  The entry's host table
        // never changes once built (map nodes do not move).
        const std::vector<int>& host = e.host;
        lock.unlock();
        int* d = nullptr;
        hipStream_t up = nullptr;
        hipError_t err = hipMalloc(&d, host.size() * sizeof(int));
        if (err == hipSuccess) err = hipStreamCreateWithFlags(&up, hipStreamNonBlocking);
        if (err == hipSuccess)
            err = hipMemcpyAsync(d, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice, up);
        if (err == hipSuccess) err = hipStreamSynchronize(up);  // landed before any launch reads it
        if (up) (void)hipStreamDestroy(up);
        if (err != hipSuccess) {
            if (d) (void)hipFree(d);
            return set_error(STENCIL_EHIP, "packed schedule upload failed: %s", hipGetErrorString(err));
        }
        lock.lock();
        if (e.table) (void)hipFree(d);  // another thread uploaded it meanwhile
        else e.table = d;
    }
    *sched = e.table;
    *nb = e.workgroups;
    if (verdict) *verdict = &e.verdict;
    return STENCIL_OK;
}

int pick_schedule(std::atomic<int>* verdict, hipStream_t s, const std::function<hipError_t(bool)>& launch) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
        (void)hipGetLastError();  // status unknown: do not block, launch untimed
        cap = hipStreamCaptureStatusActive;
    }
    if (cap != hipStreamCaptureStatusNone) {  // no host sync inside a capture: the model's choice
        STENCIL_HIP_CHECK(launch(true));
        return STENCIL_OK;
    }
    constexpr int kRounds = 3;
    hipEvent_t ev[2 * kRounds + 1] = {};
    hipError_t err = hipSuccess;
    for (auto& e : ev)
        if (err == hipSuccess) err = hipEventCreate(&e);
    if (err == hipSuccess) err = hipEventRecord(ev[0], s);
    for (int i = 0; i < 2 * kRounds && err == hipSuccess; ++i) {
        err = launch(i % 2 == 0);  // packed, equal, packed, ...
        if (err == hipSuccess) err = hipEventRecord(ev[i + 1], s);
    }
    if (err == hipSuccess) err = hipEventSynchronize(ev[2 * kRounds]);
    float best[2] = {1e30f, 1e30f};
    for (int i = 0; i < 2 * kRounds && err == hipSuccess; ++i) {
        float ms = 0.f;
        err = hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
        best[i % 2] = std::min(best[i % 2], ms);
    }
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    if (err != hipSuccess)
        return set_error(STENCIL_EHIP, "schedule trial failed: %s", hipGetErrorString(err));
    // The model predicted packing (a table exists only for a predicted gain of
    // 2 % or more): keep it unless the trial finds it clearly slower (3 %),
    // so noisy timings -- a profiler's counter passes, a busy GPU -- do not
    // flip the choice between processes; the mispredictions measured were
    // 7-20 %
    const bool packed = best[0] <= best[1] * 1.03f;
    verdict->store(packed ? kPackPacked : kPackEqual);
    if (senv_int("STENCIL_TK_VERBOSE", 0))
        std::fprintf(stderr, "schedule trial: packed %.4f ms, equal chunks %.4f ms -> %s\n", best[0], best[1],
                     packed ? "packed" : "equal chunks");
    return STENCIL_OK;
}


// Whether launch_st would consider the packed schedule for this shape (a
// single grid of at most 2 tiles per CU slot: packed_schedule's own test).
template <typename T, int V, int RY, int NW, int K>
static bool packed_regime(const stencil_layout& l) {
    using Tl = StripTile<T, V, RY, NW, K, true>;
    if (l.prob.flags & (STENCIL_HALO_LO | STENCIL_HALO_HI)) return false;
    const Geom g = geom_of(l);
    const int64_t tiles = ((g.nx + Tl::TX - 1) / Tl::TX) * ((g.ny + Tl::TY - 1) / Tl::TY);
    int slots = 0;
    if (resident_slots(tkstrip_7pt<T, V, RY, NW, K, true>, 64 * NW, &slots) != STENCIL_OK) return false;
    return tiles <= 2 * int64_t(slots);
}

// cfg = RY*100 + NW (rows per wave x waves); 0 = default shape.
int launch_tkstrip(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                   int cfg, hipStream_t s) {
    if (!temporal2_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "tkstrip supports the 3D r=1 naive 7-point star only");
    // debug cfg 97: the max-ILP shapes from kernels_strip_probe.hip (debug library only)
    if (cfg == 97) return launch_tkstrip_probe(l, in, out, begin, end, steps, s);
    if (l.prob.dtype == STENCIL_F32) {
        if (steps == 3) {
            switch (cfg) {
            case 416: return launch_st<float, 4, 4, 16, 3, false>(l, in, out, begin, end, s);
            case 808: return launch_st<float, 4, 8, 8, 3>(l, in, out, begin, end, s);
            case 20808: return launch_st<float, 2, 8, 8, 3>(l, in, out, begin, end, s);
            case 20608: return launch_st<float, 2, 6, 8, 3>(l, in, out, begin, end, s);
            default: return launch_st<float, 4, 4, 8, 3>(l, in, out, begin, end, s);
            }
        }
        if (steps == 4) {
            switch (cfg) {
            case 20808: return launch_st<float, 2, 8, 8, 4>(l, in, out, begin, end, s);
            case 404: return launch_st<float, 4, 4, 8, 4>(l, in, out, begin, end, s);
            default: return launch_st<float, 2, 7, 8, 4>(l, in, out, begin, end, s);
            }
        }
    } else {
        if (steps == 3) {
            switch (cfg) {
            case 416: return launch_st<double, 2, 4, 16, 3, false>(l, in, out, begin, end, s);
            case 10408: return launch_st<double, 2, 4, 8, 3, false>(l, in, out, begin, end, s);
            case 608: return launch_st<double, 2, 6, 8, 3>(l, in, out, begin, end, s);
            case 216: return launch_st<double, 2, 2, 16, 3, false>(l, in, out, begin, end, s);
            case 10808: return launch_st<double, 1, 8, 8, 3>(l, in, out, begin, end, s);
            case 10608: return launch_st<double, 1, 6, 8, 3>(l, in, out, begin, end, s);
#ifdef STENCIL_DIAG
            // timing experiments only, results wrong on purpose: never in the product build
            case 91: return launch_st<double, 2, 4, 8, 3, true, 1>(l, in, out, begin, end, s);
            case 92: return launch_st<double, 2, 4, 8, 3, true, 2>(l, in, out, begin, end, s);
            case 93: return launch_st<double, 2, 4, 8, 3, true, 3>(l, in, out, begin, end, s);
#endif
            default: return launch_st<double, 2, 4, 8, 3>(l, in, out, begin, end, s);
            }
        }
        if (steps == 4) {
            switch (cfg) {
            case 10808: return launch_st<double, 1, 8, 8, 4>(l, in, out, begin, end, s);
            // the default shape from this file's build whatever the grid (AUTO takes the max-ILP build on
            // packed-regime grids)
            case 10708: return launch_st<double, 1, 7, 8, 4>(l, in, out, begin, end, s);
            case 10608: return launch_st<double, 1, 6, 8, 4>(l, in, out, begin, end, s);
            case 404: return launch_st<double, 2, 4, 8, 4>(l, in, out, begin, end, s);
            case 510708: return launch_st<double, 1, 7, 8, 4, true, 0, false, 5>(l, in, out, begin, end, s);
            // the default shape without the interior fast path (no duplicated step)
            case 710708: return launch_st<double, 1, 7, 8, 4, true, 0, false, 4, false>(l, in, out, begin, end, s);
            case 510608: return launch_st<double, 1, 6, 8, 4, true, 0, false, 5>(l, in, out, begin, end, s);
            case 610608: return launch_st<double, 1, 6, 8, 4, true, 0, false, 6>(l, in, out, begin, end, s);
            case 610508: return launch_st<double, 1, 5, 8, 4, true, 0, false, 6>(l, in, out, begin, end, s);
            // stage 1's history in LDS (HL): 8-row strips at K = 4
            case 810808: return launch_st<double, 1, 8, 8, 4, true, 0, false, 4, true, true>(l, in, out, begin, end, s);
            case 810708: return launch_st<double, 1, 7, 8, 4, true, 0, false, 4, true, true>(l, in, out, begin, end, s);
            // SPLIT (two strips per wave, 32 lanes x 2 cells: 16-B lane loads): 64 x 64 / 64 x 48 regions
            case 1020408: return launch_st<double, 2, 4, 8, 4, true, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1020308: return launch_st<double, 2, 3, 8, 4, true, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1820408: return launch_st<double, 2, 4, 8, 4, false, 0, false, 4, true, true, true>(l, in, out, begin, end, s);
            // 9-row strips without the fast path: 72 rows for 64 output rows (512 = 8 x 64)
            case 820908: return launch_st<double, 1, 9, 8, 4, true, 0, false, 4, false, true>(l, in, out, begin, end, s);
            default:
                // grids of at most 2 tiles per CU slot (packed schedule, fast path): the max-ILP build
                if (packed_regime<double, 1, 7, 8, 4>(l)) return launch_tkstrip_ilp(l, in, out, begin, end, 4, s);
                return launch_st<double, 1, 7, 8, 4>(l, in, out, begin, end, s);
            }
        }
    }
    if (steps == 5) {
        if (l.prob.dtype == STENCIL_F32) {
            switch (cfg) {
            case 20608: return launch_st<float, 2, 6, 8, 5>(l, in, out, begin, end, s);
            // stage 1's history in LDS (HL): 6-row strips (226 VGPRs); 7 rows with one boundary buffer (254)
            case 820608: return launch_st<float, 2, 6, 8, 5, true, 0, false, 4, true, true>(l, in, out, begin, end, s);
            case 830708: return launch_st<float, 2, 7, 8, 5, false, 0, false, 4, true, true>(l, in, out, begin, end, s);
            // the default shape from this file's build (AUTO takes the max-ILP build)
            case 20508: return launch_st<float, 2, 5, 8, 5>(l, in, out, begin, end, s);
            // input planes loaded 3 / 4 planes ahead (NS = 5 / 6) instead of 2
            case 520508: return launch_st<float, 2, 5, 8, 5, true, 0, false, 5>(l, in, out, begin, end, s);
            case 620508: return launch_st<float, 2, 5, 8, 5, true, 0, false, 6>(l, in, out, begin, end, s);
            // 4 cells per lane (256-wide regions: 16-B lane loads), one boundary-row buffer (80 KB of LDS)
            case 40408: return launch_st<float, 4, 4, 8, 5, false>(l, in, out, begin, end, s);
            case 840408: return launch_st<float, 4, 4, 8, 5, false, 0, false, 4, true, true>(l, in, out, begin, end, s);
            // SPLIT (two strips per wave, 32 lanes x 4 cells: 16-B lane loads): 128 x 32 / 128 x 48 regions
            case 1040208: return launch_st<float, 4, 2, 8, 5, true, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1040308: return launch_st<float, 4, 3, 8, 5, true, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1030308: return launch_st<float, 4, 3, 8, 5, false, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1030212: return launch_st<float, 4, 2, 12, 5, false, 0, false, 4, true, false, true>(l, in, out, begin, end, s);
            case 1830308: return launch_st<float, 4, 3, 8, 5, false, 0, false, 4, true, true, true>(l, in, out, begin, end, s);
            case 1830408: return launch_st<float, 4, 4, 8, 5, false, 0, false, 4, true, true, true>(l, in, out, begin, end, s);
            // the same, 5-row strips with stage 1's history in LDS (160 KB)
            case 840508: return launch_st<float, 4, 5, 8, 5, false, 0, false, 4, true, true>(l, in, out, begin, end, s);
            default: return launch_tkstrip_ilp(l, in, out, begin, end, 5, s);
            }
        }
        switch (cfg) {
        case 10608: return launch_st<double, 1, 6, 8, 5>(l, in, out, begin, end, s);
        // stage 1's history in LDS (HL): 7- and 8-row strips at K = 5
        case 810708: return launch_st<double, 1, 7, 8, 5, true, 0, false, 4, true, true>(l, in, out, begin, end, s);
        case 810608: return launch_st<double, 1, 6, 8, 5, true, 0, false, 4, true, true>(l, in, out, begin, end, s);
        // + one boundary-row buffer (a second barrier per step) and no fast path: 7 rows fit (254 VGPRs)
        case 830708: return launch_st<double, 1, 7, 8, 5, false, 0, false, 4, false, true>(l, in, out, begin, end, s);
        default: return launch_st<double, 1, 5, 8, 5>(l, in, out, begin, end, s);
        }
    }
    return set_error(STENCIL_EINVAL, "tkstrip steps must be 3, 4 or 5 (got %d)", steps);
}

// The default shapes with face signalling (stencil_sweepk_signal).
int launch_tkstrip_signal(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                          unsigned* sig, unsigned long long* fsig, int* nsig, hipStream_t s, const StripGate& gate) {
    if (!temporal2_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "face-signalled sweeps cover the 3D r=1 naive 7-point star only");
    if (l.prob.dtype == STENCIL_F32) {
        switch (steps) {
        case 3: return launch_st<float, 4, 4, 8, 3, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        case 4: return launch_st<float, 2, 7, 8, 4, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        case 5: return launch_st<float, 2, 5, 8, 5, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        default: break;
        }
    } else {
        switch (steps) {
        case 3: return launch_st<double, 2, 4, 8, 3, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        case 4: return launch_st<double, 1, 7, 8, 4, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        case 5: return launch_st<double, 1, 5, 8, 5, true, 0, true>(l, in, out, begin, end, s, sig, nsig, fsig, gate);
        default: break;
        }
    }
    return set_error(STENCIL_EINVAL, "face-signalled sweeps: steps must be 3, 4 or 5 (got %d)", steps);
}

#endif  // STRIP_ILP_TU

}  // namespace stencil

#ifndef STRIP_ILP_TU
// The packed-schedule model on the host, without a GPU (tests, tools): see
// include/stencil_hip.h.
int stencil_pack_plan(int64_t tiles, int64_t planes, int32_t fill, int32_t slots, int32_t zchunk, int64_t* equal_steps,
                      int64_t* packed_steps, int64_t* workgroups) {
    using namespace stencil;
    if (tiles <= 0 || planes <= 0 || fill < 0 || slots <= 0 || zchunk <= 0 || planes > (int64_t(1) << 30) ||
        tiles * ((planes + zchunk - 1) / zchunk) > (int64_t(1) << 26))
        return set_error(STENCIL_EINVAL, "pack plan: tiles, planes, slots, zchunk > 0, fill >= 0, at most 2^26 chunks");
    std::vector<int> tab;
    int64_t base = 0, best = 0;
    pack_search(tiles, planes, fill, slots, zchunk, 0, &tab, &base, &best);
    if (equal_steps) *equal_steps = base;
    if (packed_steps) *packed_steps = best;
    if (workgroups) *workgroups = (!tab.empty() && best * 50 < base * 49) ? int64_t(tab.size() / 3) : 0;
    clear_error();
    return STENCIL_OK;
}
int stencil_pack_table(int64_t tiles, int64_t tiles_x, int64_t planes, int32_t fill, int32_t slots, int32_t zchunk,
                       int32_t xcd_width, int32_t* table, int64_t capacity, int64_t* workgroups) {
    using namespace stencil;
    if (tiles <= 0 || tiles_x <= 0 || planes <= 0 || fill < 0 || slots <= 0 || zchunk <= 0 || xcd_width < -1 ||
        planes > (int64_t(1) << 30) || tiles * ((planes + zchunk - 1) / zchunk) > (int64_t(1) << 26))
        return set_error(STENCIL_EINVAL, "pack table: tiles, tiles_x, planes, slots, zchunk > 0, fill, xcd_width >= 0");
    std::vector<int> tab;
    int64_t base = 0, best = 0;
    pack_search(tiles, planes, fill, slots, zchunk, 0, &tab, &base, &best);
    if (tab.empty() || best * 50 >= base * 49) tab.clear();
    if (xcd_width < 0 && !tab.empty()) xcd_width = best_patch_width(tab, tiles_x);
    if (xcd_width > 0 && !tab.empty()) xcd_patch_order(tab, tiles_x, xcd_width);
    const int64_t n = int64_t(tab.size() / 3);
    if (table)
        for (int64_t i = 0; i < std::min(n, capacity) * 3; ++i) table[i] = tab[size_t(i)];
    if (workgroups) *workgroups = n;
    clear_error();
    return STENCIL_OK;
}
#endif  // STRIP_ILP_TU
