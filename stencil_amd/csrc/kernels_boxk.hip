// kernels_boxk.hip -- the 3D 27-point box stencil (r = 1, naive order):
// K = 1 .. 4 sweeps per launch, z-marching with SEPARABLE partial sums.
//
// Sum order (no reference code for the box; defined in DESIGN.md §3 and
// restated by oracle/oracle_impl.inc):
//     R(y')  = (in[x-1] + in[x]) + in[x+1]          row sum of row y'
//     P9(z') = (R(y-1) + R(y)) + R(y+1)              plane sum of plane z'
//     cell   = (((P9(z-1) + P9(z)) + P9(z+1)) - in[z,y,x]) * avg
// Row sums are shared by the three cells above / at / below a row, plane sums
// by the three cells below / at / above a plane: 8 VALU operations per cell
// and stage (round 2 summed the centre plane without its centre,
// ((P9(z-1) + C(z)) + P9(z+1)): 10, and the centre-row sum E = l + r live
// beside every row sum -- the order change cut 236 -> 144 VGPRs at 3 x 8 rows,
// K = 4) instead of the 26 dependent additions of a
// lexicographic order.
//
// Pipeline (as the round-1 kernel: stage s lags stage s-1 by two planes).
// When plane q of t_{s-1} is "in LDS", stage s
//     finishes t_s(q-1) = ((A(q-1) + P9(q)) - centre(q-1)) * avg
//     continues        A(q)  = P9(q-1) + P9(q)
// with A and P9 carried in registers from plane to plane.  What LDS holds of
// plane q is only its row sums R (the rows y-1, y, y+1: three LDS reads); the
// lane keeps the plane's values themselves (the centre, also the value of
// the ghost cells of intermediate planes).  Per stage and
// row a lane carries 4 vectors (centre of q and q-1, A, P9; the last stage 3),
// so 8 waves x 4 rows fit 256 VGPRs.
//
// Per step p (one workgroup barrier; the LDS row-sum planes are double-
// buffered by step parity, so a wave past barrier p has every wave's reads of
// the buffer it is about to overwrite behind it):
//   barrier
//   read phase   for s = 1..K: plane q = p-2s+1 of t_{s-1}: finish t_s(p-2s),
//                continue A; intermediate planes keep ghost cells at their
//                input value, slab-halo planes (HALO_LO/HI) are advanced;
//                t_K(p-2K) -> HBM (nontemporal)
//   write phase  row sums of in(p) and of t_s(p-2s), s < K, into buffer p&1;
//                the lane keeps the planes' values; request in(p+2)
// Bitwise equal to K sweeps of the oracle's box (tests/test_gpu_parity.py).
#include <cstdlib>

#include "common.hpp"

// The interior fast path (no ghost selects on steps whose region lies inside
// the grid) is compiled out: with it the 2048^2 x 256 box ran 24-28 % slower
// (fp64 K = 4 695 -> 530, fp32 K = 3 1398 -> 1011 Gcell/s,
// profiles/r03/r03h_ab_box*.txt), a second copy of the step body the
// compiler schedules worse.  -DBOX_FAST_PATH=1 builds it (debug knob
// STENCIL_BOXK_FAST then selects it).
#ifndef BOX_FAST_PATH
#define BOX_FAST_PATH 0
#endif

namespace stencil {
namespace {

// A per-row 32-bit offset made opaque at each use: the zero extension then
// sits next to the address add in the loop body, so instruction selection
// forms saddr + 32-bit voffset (global_load v, voff, s[base]) instead of a
// 64-bit VGPR address built by v_lshl_add_u64 from a hoisted zext (2 VGPRs
// per row held across the loop, one VALU op per access).
__device__ __forceinline__ uint32_t row_off(uint32_t o) {
    asm volatile("" : "+v"(o));
    return o;
}

template <typename T, int V>
struct VecB {
    typedef T type __attribute__((ext_vector_type(V)));
};

template <int CTRL>
__device__ __forceinline__ float bdpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ double bdpp(double v) {
    const int2 b = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_mov_dpp(b.x, CTRL, 0xf, 0xf, true),
                                                 __builtin_amdgcn_mov_dpp(b.y, CTRL, 0xf, 0xf, true)));
}
constexpr int kShr1 = 0x138, kShl1 = 0x130;  // wave_shr:1 / wave_shl:1

template <typename T, int V, int RY, int NW, int K>
struct BKTile {
    static constexpr int XR = (K + V - 1) / V;  // ring vectors per x side
    static constexpr int RW = 64 * V;           // region width
    static constexpr int TX = RW - 2 * XR * V;  // output tile width
    static constexpr int RH = NW * RY;          // region height
    static constexpr int TY = RH - 2 * K;       // output tile height
    static constexpr int LY = RH + 2;           // row-sum planes: one zero pad row each side
    static constexpr size_t lds_bytes = size_t(2) * K * LY * RW * sizeof(T);
};

// Rows: wave w owns region rows w, w + NW, ... (RY of them).
// SIG: face signalling for multi-GPU slabs (stencil_sweepk_signal, as
// kernels_strip.hip): the last z-chunk of every tile marches DOWNWARD, so the
// K planes of both faces are among the first stored, and the workgroup that
// stores a face adds to sig[0] / sig[1] (release, then one agent-scope add).
// Marching down, plane z's sum ((P9(z-1) + P9(z)) + P9(z+1)) - centre needs the
// NEWEST plane sum first, so the down-march carries the two previous plane
// sums instead of the pre-added A: same additions, same order, bitwise equal.
template <typename T, int V, int RY, int NW, int K, bool SIG = false>
__global__ void __launch_bounds__(64 * NW)
    box27_sep(const T* __restrict__ in, T* __restrict__ out, Geom g, int zbeg, int zend, int zchunk, int tiles_x,
              int tiles_y, int halo_lo, int halo_hi, int ld_lo, int ld_hi, T avg, unsigned* __restrict__ sig,
              unsigned long long* __restrict__ fsig, const int* __restrict__ sched, int /*xcd_pw: strip only*/,
              int /*fast: strip only*/) {
    using Tl = BKTile<T, V, RY, NW, K>;
    using VT = typename VecB<T, V>::type;
    constexpr int XR = Tl::XR, TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LY = Tl::LY, RW = Tl::RW;
    static_assert(TY > 0 && TX > 0, "tile too small for K");
    __shared__ __attribute__((aligned(16))) T L[2][K][LY][RW];

    const int t = blockIdx.x;
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int nch = (zend - zbeg + zchunk - 1) / zchunk;
    int bz = t / (tiles_x * tiles_y);
    // face-signalled launches: the two face chunks dispatched first (kernels_strip.hip)
    if (SIG && nch >= 3) bz = bz == 0 ? 0 : bz == 1 ? nch - 1 : bz - 1;
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - XR * V + int64_t(lane) * V;
    const int64_t y0 = int64_t(by) * TY - K;
    const int za = zbeg + bz * zchunk;
    const int zb = za + zchunk < zend ? za + zchunk : zend;
    const bool rev = SIG && nch >= 2 && bz == nch - 1;  // this workgroup's chunk marches down
    const int nz = int(g.nz);
    const int64_t plane = g.plane;
    // uniform per-plane base + one non-negative 32-bit byte offset per row
    // (the saddr form of global_load/store, as kernels_strip.hip)
    const int64_t bias = g.row + XR * V;
    const char* __restrict__ src = reinterpret_cast<const char*>(in + g.origin - bias);
    char* __restrict__ dst = reinterpret_cast<char*>(out + g.origin - bias);

    {  // zero everything once: the pad rows must read as 0 (ring cells only)
        constexpr int N = int(Tl::lds_bytes / sizeof(VT));
        VT* l = reinterpret_cast<VT*>(&L[0][0][0][0]);
        for (int i = threadIdx.y * 64 + threadIdx.x; i < N; i += 64 * NW) l[i] = VT{};
    }

    // unconditional loads from clamped addresses (the plane wait is a counted
    // vmcnt, kernels_temporalk.hip)
    uint32_t off[RY];
    bool yin[RY], st[RY];
    const int64_t xmax = g.nx / V * V;
    const int64_t xc = x < xmax ? x : xmax;
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w + NW * k;
        const int64_t y = y0 + rr;
        const int64_t yc = y < -1 ? -1 : (y > g.ny ? g.ny : y);
        off[k] = uint32_t((yc * g.row + xc + bias) * int64_t(sizeof(T)));
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= K && rr < RH - K && y < g.ny && lane >= XR && lane < 64 - XR;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    // R = (l + c) + r of a row vector v (x-neighbours from the adjacent lanes)
    auto row_sum = [&](const VT& v) {
        const T wl = bdpp<kShr1>(v[V - 1]);
        const T er = bdpp<kShl1>(v[0]);
        VT o;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const T l = j == 0 ? wl : v[j == 0 ? 0 : j - 1];
            const T r = j == V - 1 ? er : v[j == V - 1 ? 0 : j + 1];
            o[j] = (l + v[j]) + r;
        }
        return o;
    };
    const int xl = lane * V;
    __syncthreads();  // LDS zeroed

    auto segment = [&](auto REV_) {  // the chunk [za, zb), marched up or (REV) down
    constexpr bool REV = decltype(REV_)::value;
    const int zfirst = za - K > ld_lo ? za - K : ld_lo;
    const int zlast = zb + K - 1 < ld_hi ? zb + K - 1 : ld_hi;
    // march index m -> plane
    auto zr = [&](int m) { return REV ? za + zb - 1 - m : m; };
    auto load_plane = [&](VT (&d)[RY], int m) {
        const int z = zr(m);
        const int zz = z < zfirst ? zfirst : (z > zlast ? zlast : z);
        const char* base = src + int64_t(zz) * plane * int64_t(sizeof(T));
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(base + row_off(off[k]));
    };

    // Registers, per row.  The lane's own values of the stages' input planes
    // are read in place: in(m) in the input ring vin[(m - p0) % 4] (in(p-2) ..
    // in(p+1) at step p; loads issued two planes ahead into the slot just
    // consumed), t_s(m) in H[s-1][(m - p0) & 1] -- no copies, so no load result
    // is ever moved (a move would wait for the load).  Steps are unrolled 4 at
    // a time (ring slot and parity are compile-time).
    const int p0 = za - K;
    VT vin[4][RY];
    VT H[K > 1 ? K - 1 : 1][2][RY];
    // per stage, carried from plane to plane: up-march A(q-1) and P9(q-1);
    // down-march (REV) P9(q-1), P9(q-2) (march order)
    VT A[K][RY], P9p[K][RY], P9q[REV ? K : 1][RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
#pragma unroll
        for (int s = 0; s < K; ++s) A[s][k] = P9p[s][k] = VT{};
#pragma unroll
        for (int s = 0; s < (REV ? K : 1); ++s) P9q[s][k] = VT{};
#pragma unroll
        for (int s = 0; s < (K > 1 ? K - 1 : 1); ++s) H[s][0][k] = H[s][1][k] = VT{};
        vin[2][k] = vin[3][k] = VT{};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) load_plane(vin[i], p0 + i);

    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;  // (p - p0) % 4
        constexpr int PW = S & 1, PR = PW ^ 1;  // LDS buffer written / read this step
        __syncthreads();
        VT res[K][RY];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            const int m = zr(p - 2 * s);  // plane of t_s finished now
            const int lo_s = halo_lo ? -(K - s) : 0;
            const int hi_s = halo_hi ? nz + (K - s) : nz;
            const bool zin = m >= lo_s && m < hi_s;
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const int yy = w + NW * k + 1;
                const VT up = *reinterpret_cast<const VT*>(&L[PR][s - 1][yy - 1][xl]);
                const VT own = *reinterpret_cast<const VT*>(&L[PR][s - 1][yy][xl]);
                const VT dn = *reinterpret_cast<const VT*>(&L[PR][s - 1][yy + 1][xl]);
                // plane q - 1 of t_{s-1} (the centre of the plane finished now): s = 1 -> in(p-2)
                const VT& cq1 = s == 1 ? vin[(S + 2) % 4][k] : H[s >= 2 ? s - 2 : 0][S & 1][k];
                VT o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const T p9 = (up[j] + own[j]) + dn[j];
                    T fin;
                    if constexpr (!REV) {  // plane q-1: ((P9(q-2) + P9(q-1)) + P9(q)) - centre
                        fin = (A[s - 1][k][j] + p9) - cq1[j];
                        A[s - 1][k][j] = P9p[s - 1][k][j] + p9;
                        P9p[s - 1][k][j] = p9;
                    } else {  // plane zr(q-1): ((P9(zr(q)) + P9(zr(q-1))) + P9(zr(q-2))) - centre
                        fin = ((p9 + P9p[s - 1][k][j]) + P9q[REV ? s - 1 : 0][k][j]) - cq1[j];
                        P9q[REV ? s - 1 : 0][k][j] = P9p[s - 1][k][j];
                        P9p[s - 1][k][j] = p9;
                    }
                    o[j] = fin * avg;
                    if (s < K) o[j] = (zin && yin[k] && xin[j]) ? o[j] : cq1[j];
                }
                res[s - 1][k] = o;
#ifdef BOXK_SB
                __builtin_amdgcn_sched_barrier(0);
#endif
            }
        }
        // t_K(p-2K) -> HBM
        const int zo = p - 2 * K;
        if (zo >= za && zo < zb) {
            char* obase = dst + int64_t(zr(zo)) * plane * int64_t(sizeof(T));
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                if (st[k]) {
                    T* q = reinterpret_cast<T*>(obase + row_off(off[k]));
                    if (xst[V - 1]) {
                        __builtin_nontemporal_store(res[K - 1][k], reinterpret_cast<VT*>(q));
                    } else {
#pragma unroll
                        for (int j = 0; j < V; ++j)
                            if (xst[j]) q[j] = res[K - 1][k][j];
                    }
                }
            }
        }
        if constexpr (SIG) {
            // right after the store of a face's last plane (every chunk is at
            // least K planes): the low face is [zbeg, zbeg+K) of the first
            // chunk, the high face [zend-K, zend) of the last, walked down
            // (REV) so it comes first -- as kernels_strip.hip
            const bool lo_here = !REV && za == zbeg && zo == za + K - 1;
            const bool hi_here = zb == zend && zo == (REV ? za + K - 1 : zb - 1);
            if (lo_here || hi_here) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0 && threadIdx.y == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const unsigned ntiles = unsigned(tiles_x) * unsigned(tiles_y);
                    unsigned long long done = 0;  // faces completed here: 0, 1 or 2
                    if (lo_here)
                        done += (__hip_atomic_fetch_add(&sig[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (hi_here)
                        done += (__hip_atomic_fetch_add(&sig[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (fsig && done) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        __hip_atomic_fetch_add(fsig, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
        }
        // write phase: row sums of in(p) (stage 1's next input plane) and of
        // t_s(p-2s) (stage s+1's), s < K
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                // in(p) / t_s(p-2s) -> H[s-1][(p - p0) & 1] (its old content,
                // t_s(p-2s-2), was stage s+1's plane q-1, read above)
                if (s > 0) H[s > 0 ? s - 1 : 0][S & 1][k] = res[s > 0 ? s - 1 : 0][k];
                const VT& v = s == 0 ? vin[S][k] : H[s > 0 ? s - 1 : 0][S & 1][k];
                *reinterpret_cast<VT*>(&L[PW][s][yy][xl]) = row_sum(v);
            }
        }
        load_plane(vin[(S + 2) % 4], p + 2);  // the slot of in(p-2), read above
    };

    const int plast = zb - 1 + 2 * K;
    int p = p0;
    for (; p + 3 <= plast; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    if (p <= plast) step(std::integral_constant<int, 0>{}, p);
    if (p + 1 <= plast) step(std::integral_constant<int, 1>{}, p + 1);
    if (p + 2 <= plast) step(std::integral_constant<int, 2>{}, p + 2);
    };  // segment
    if constexpr (SIG) {
        if (rev) segment(std::true_type{});
        else segment(std::false_type{});
    } else {
        segment(std::false_type{});
    }
}

// The STRIP layout of the same pipeline (kernels_strip.hip did this for the
// 7-point star): wave w owns CONSECUTIVE region rows [w*RY, w*RY + RY), so a
// row's y-neighbour row sums come from the lane's own registers and only the
// strip's first and last row sums go through LDS (2 writes + 2 reads per
// stage and wave instead of RY writes + 3*RY reads).  The freed LDS traffic
// and the res[K][RY] staging of box27_sep (stages now run K .. 1, so stage s
// writes t_s straight into the history slot stage s+1 has just read) pay for
// taller regions: 8 waves x 6 rows = 48 rows for 42 output rows (y over-fetch
// 1.14) instead of 24 for 18 (1.33).  Same sums, same order, same pipeline
// (stage s lags two planes per stage), bitwise equal to box27_sep.
//
// Per step p (one barrier; boundary row sums double-buffered by step parity):
//   barrier
//   stage K     plane q = p-2K+1 of t_{K-1}: finish t_K(p-2K) -> HBM
//   stage s<K   finish t_s(p-2s) into H[s-1] (the slot stage s+1 read),
//               its first / last row sums -> LDS buffer p&1
//   row sums of in(p)'s first / last rows -> LDS buffer p&1; request in(p+2)
template <typename T, int V, int RY, int NW, int K, bool SIG = false>
__global__ void __launch_bounds__(64 * NW)
    box27_strip(const T* __restrict__ in, T* __restrict__ out, Geom g, int zbeg, int zend, int zchunk, int tiles_x,
                int tiles_y, int halo_lo, int halo_hi, int ld_lo, int ld_hi, T avg, unsigned* __restrict__ sig,
                unsigned long long* __restrict__ fsig, const int* __restrict__ sched, int xcd_pw, int fast) {
    using Tl = BKTile<T, V, RY, NW, K>;
    using VT = typename VecB<T, V>::type;
    constexpr int XR = Tl::XR, TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, RW = Tl::RW;
    static_assert(TY > 0 && TX > 0, "tile too small for K");
    static_assert(RY >= 2, "a strip needs a first and a last row");
    // boundary row sums: [step parity][stage input][wave][first, last row][RW]
    __shared__ __attribute__((aligned(16))) T L[2][K][NW][2][RW];

    // work: tile (bx, by) and planes [za, zb) -- equal z-chunks, or one entry
    // {tile, first plane, planes} of the packed schedule (few-tile grids;
    // never on the face-signalled launches)
    int t = blockIdx.x, za, zb;
    int64_t nch = 1;
    if (!SIG && sched) {
        const int* e = sched + 3 * int64_t(blockIdx.x);
        t = e[0];
        za = zbeg + e[1];
        zb = za + e[2];
    } else {
        nch = (zend - zbeg + zchunk - 1) / zchunk;
        if (!SIG && xcd_pw > 0) {
            // XCD patches (default 4 tiles wide; STENCIL_BOXK_XCD = width): blocks
            // b and b + 8 share an XCD (round-robin dispatch; speed only, the
            // map is a bijection either way), so XCD b % 8 walks its own
            // contiguous run of (chunk, tile) units in column strips of xcd_pw
            // tiles -- the workgroups resident on one XCD at a time form a
            // 2D patch whose shared halo rows / columns are L2 hits
            const int64_t tiles = int64_t(tiles_x) * tiles_y, total = tiles * nch;
            const int64_t per = (total + 7) / 8;
            const int64_t u = int64_t(blockIdx.x % 8) * per + blockIdx.x / 8;
            if (u >= total) return;  // whole workgroup, before any barrier
            const int64_t c = u / tiles, tt = u - c * tiles;
            const int64_t strip = tt / (int64_t(xcd_pw) * tiles_y);
            const int64_t rem = tt - strip * xcd_pw * tiles_y;
            const int64_t sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
            t = int(rem / sw * tiles_x + strip * xcd_pw + rem % sw);
            za = zbeg + int(c) * zchunk;
        } else {
            const int bz = t / (tiles_x * tiles_y);
            t -= bz * tiles_x * tiles_y;
            // face-signalled launches: the two face chunks dispatched first (kernels_strip.hip)
            za = zbeg + (SIG && nch >= 3 ? (bz == 0 ? 0 : bz == 1 ? nch - 1 : bz - 1) : bz) * zchunk;
        }
        zb = za + zchunk < zend ? za + zchunk : zend;
    }
    const int bx = t % tiles_x;
    const int by = t / tiles_x;
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - XR * V + int64_t(lane) * V;
    const int64_t y0 = int64_t(by) * TY - K + int64_t(w) * RY;  // this wave's first row
    const bool rev = SIG && nch >= 2 && zb == zend;  // this workgroup's chunk (the last) marches down
    const int nz = int(g.nz);
    const int64_t plane = g.plane;
    const int64_t bias = g.row + XR * V;
    const char* __restrict__ src = reinterpret_cast<const char*>(in + g.origin - bias);
    char* __restrict__ dst = reinterpret_cast<char*>(out + g.origin - bias);

    {  // the first step reads a buffer nobody wrote (ring cells only): zero it
        constexpr int N = int(sizeof(L) / sizeof(VT));
        VT* l = reinterpret_cast<VT*>(&L[0][0][0][0][0]);
        for (int i = threadIdx.y * 64 + threadIdx.x; i < N; i += 64 * NW) l[i] = VT{};
    }

    uint32_t off[RY];
    bool yin[RY], st[RY];
    const int64_t xmax = g.nx / V * V;
    const int64_t xc = x < xmax ? x : xmax;
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w * RY + k;
        const int64_t y = y0 + k;
        const int64_t yc = y < -1 ? -1 : (y > g.ny ? g.ny : y);
        off[k] = uint32_t((yc * g.row + xc + bias) * int64_t(sizeof(T)));
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= K && rr < RH - K && y < g.ny && lane >= XR && lane < 64 - XR;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    // the whole region inside the grid in x and y (the fast path's condition)
    const bool xy_inner = fast && int64_t(bx) * TX - XR * V >= 0 && int64_t(bx) * TX - XR * V + RW <= g.nx &&
                          int64_t(by) * TY - K >= 0 && int64_t(by) * TY - K + RH <= g.ny;
    // R = (l + c) + r of a row vector (x-neighbours by DPP)
    auto rsum = [&](const VT& v) {
        const T wl = bdpp<kShr1>(v[V - 1]);
        const T er = bdpp<kShl1>(v[0]);
        VT R;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const T l = j == 0 ? wl : v[j == 0 ? 0 : j - 1];
            const T r = j == V - 1 ? er : v[j == V - 1 ? 0 : j + 1];
            R[j] = (l + v[j]) + r;
        }
        return R;
    };
    const int xl = lane * V;
    // neighbour strips (the first / last wave reads its own: ring rows)
    const int wa = w > 0 ? w - 1 : 0, wb = w < NW - 1 ? w + 1 : NW - 1;
    __syncthreads();  // LDS zeroed

    auto segment = [&](auto REV_) {
    constexpr bool REV = decltype(REV_)::value;
    const int zfirst = za - K > ld_lo ? za - K : ld_lo;
    const int zlast = zb + K - 1 < ld_hi ? zb + K - 1 : ld_hi;
    auto zr = [&](int m) { return REV ? za + zb - 1 - m : m; };
    auto load_plane = [&](VT (&d)[RY], int m) {
        const int z = zr(m);
        const int zz = z < zfirst ? zfirst : (z > zlast ? zlast : z);
        const char* base = src + int64_t(zz) * plane * int64_t(sizeof(T));
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(base + row_off(off[k]));
    };

    // in(m) in vin[(m - p0) % 4], t_s(m) in H[s-1][(m - p0) & 1] (read in
    // place); per stage the carried A(q-1) / P9(q-1) (REV: P9(q-1), P9(q-2))
    const int p0 = za - K;
    VT vin[4][RY];
    VT H[K > 1 ? K - 1 : 1][2][RY];
    VT A[K][RY], P9p[K][RY], P9q[REV ? K : 1][RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
#pragma unroll
        for (int s = 0; s < K; ++s) A[s][k] = P9p[s][k] = VT{};
#pragma unroll
        for (int s = 0; s < (REV ? K : 1); ++s) P9q[s][k] = VT{};
#pragma unroll
        for (int s = 0; s < (K > 1 ? K - 1 : 1); ++s) H[s][0][k] = H[s][1][k] = VT{};
        vin[2][k] = vin[3][k] = VT{};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) load_plane(vin[i], p0 + i);

    auto stepb = [&](auto S_, int p, auto FAST_) {
        constexpr int S = decltype(S_)::value;  // (p - p0) % 4
        constexpr bool FAST = decltype(FAST_)::value;  // every stage plane and the region inside: no ghost selects
        constexpr int PW = S & 1, PR = PW ^ 1;  // LDS buffer written / read this step
        __syncthreads();
        const int zo = p - 2 * K;  // t_K(zo) -> HBM this step
        const bool do_store = zo >= za && zo < zb;
        char* obase = dst + int64_t(zr(zo)) * plane * int64_t(sizeof(T));
        auto stage = [&](auto s_) {
            constexpr int s = decltype(s_)::value;
            const int m = zr(p - 2 * s);  // plane of t_s finished now
            const int lo_s = halo_lo ? -(K - s) : 0;
            const int hi_s = halo_hi ? nz + (K - s) : nz;
            const bool zin = m >= lo_s && m < hi_s;
            // rows of plane q = p - 2s + 1 (centre) and q - 1 of t_{s-1}
            auto cq = [&](int k) -> const VT& { return s == 1 ? vin[(S + 3) % 4][k] : H[s >= 2 ? s - 2 : 0][(S + 1) & 1][k]; };
            auto cq1 = [&](int k) -> const VT& { return s == 1 ? vin[(S + 2) % 4][k] : H[s >= 2 ? s - 2 : 0][S & 1][k]; };
            VT Rm = *reinterpret_cast<const VT*>(&L[PR][s - 1][wa][1][xl]);  // row above the strip
            VT Rc = rsum(cq(0));
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const VT Rn = k == RY - 1 ? *reinterpret_cast<const VT*>(&L[PR][s - 1][wb][0][xl])  // row below
                                          : rsum(cq(k + 1 < RY ? k + 1 : k));
                VT o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const T p9 = (Rm[j] + Rc[j]) + Rn[j];
                    T fin;
                    if constexpr (!REV) {  // plane q-1: ((P9(q-2) + P9(q-1)) + P9(q)) - centre, A = P9(q-2) + P9(q-1)
                        fin = (A[s - 1][k][j] + p9) - cq1(k)[j];
                        A[s - 1][k][j] = P9p[s - 1][k][j] + p9;
                        P9p[s - 1][k][j] = p9;
                    } else {  // plane zr(q-1): ((P9(zr(q)) + P9(zr(q-1))) + P9(zr(q-2))) - centre
                        fin = ((p9 + P9p[s - 1][k][j]) + P9q[REV ? s - 1 : 0][k][j]) - cq1(k)[j];
                        P9q[REV ? s - 1 : 0][k][j] = P9p[s - 1][k][j];
                        P9p[s - 1][k][j] = p9;
                    }
                    o[j] = fin * avg;
                    if (s < K && !FAST) o[j] = (zin && yin[k] && xin[j]) ? o[j] : cq1(k)[j];
                }
                if constexpr (s == K) {
                    if (do_store && st[k]) {
                        T* qp = reinterpret_cast<T*>(obase + row_off(off[k]));
                        if (xst[V - 1]) {
                            __builtin_nontemporal_store(o, reinterpret_cast<VT*>(qp));
                        } else {
#pragma unroll
                            for (int j = 0; j < V; ++j)
                                if (xst[j]) qp[j] = o[j];
                        }
                    }
                } else {
                    // t_s(p-2s) takes the slot of t_s(p-2s-2), stage s+1's
                    // plane q-1, already read (stages run K .. 1)
                    H[s < K ? s - 1 : 0][S & 1][k] = o;
                    if (k == 0) *reinterpret_cast<VT*>(&L[PW][s][w][0][xl]) = rsum(o);
                    if (k == RY - 1) *reinterpret_cast<VT*>(&L[PW][s][w][1][xl]) = rsum(o);
                }
                Rm = Rc;
                Rc = Rn;
            }
        };
        stage(std::integral_constant<int, K>{});
        if constexpr (SIG) {
            // right after the store of a face's last plane (box27_sep)
            const bool lo_here = !REV && za == zbeg && zo == za + K - 1;
            const bool hi_here = zb == zend && zo == (REV ? za + K - 1 : zb - 1);
            if (lo_here || hi_here) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0 && threadIdx.y == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const unsigned ntiles = unsigned(tiles_x) * unsigned(tiles_y);
                    unsigned long long done = 0;  // faces completed here: 0, 1 or 2
                    if (lo_here)
                        done += (__hip_atomic_fetch_add(&sig[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (hi_here)
                        done += (__hip_atomic_fetch_add(&sig[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) %
                                    ntiles == 0;
                    if (fsig && done) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        __hip_atomic_fetch_add(fsig, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
        }
        // stages K-1 .. 1
        if constexpr (K >= 5) stage(std::integral_constant<int, (K >= 5 ? 4 : 1)>{});
        if constexpr (K >= 4) stage(std::integral_constant<int, (K >= 4 ? 3 : 1)>{});
        if constexpr (K >= 3) stage(std::integral_constant<int, (K >= 3 ? 2 : 1)>{});
        if constexpr (K >= 2) stage(std::integral_constant<int, 1>{});
        static_assert(K >= 1 && K <= 5, "K = 1..5");
        // stage 1's next input plane: in(p)
        *reinterpret_cast<VT*>(&L[PW][0][w][0][xl]) = rsum(vin[S][0]);
        *reinterpret_cast<VT*>(&L[PW][0][w][1][xl]) = rsum(vin[S][RY - 1]);
        load_plane(vin[(S + 2) % 4], p + 2);  // the slot of in(p-2), read above
    };

    // interior steps skip the intermediate stages' ghost-cell selects (as the
    // 7-point strip kernel's fast path): the region inside the grid in x and
    // y, every intermediate stage plane inside its computed z range
    auto step = [&](auto S_, int p) {
        if constexpr (!BOX_FAST_PATH || SIG) {
            stepb(S_, p, std::false_type{});
        } else {
            bool all_in = xy_inner;
#pragma unroll
            for (int s = 1; s < K; ++s) {
                const int m = zr(p - 2 * s);
                all_in = all_in && m >= (halo_lo ? -(K - s) : 0) && m < (halo_hi ? nz + (K - s) : nz);
            }
            if (all_in) stepb(S_, p, std::true_type{});
            else stepb(S_, p, std::false_type{});
        }
    };

    const int plast = zb - 1 + 2 * K;
    int p = p0;
    for (; p + 3 <= plast; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    if (p <= plast) step(std::integral_constant<int, 0>{}, p);
    if (p + 1 <= plast) step(std::integral_constant<int, 1>{}, p + 1);
    if (p + 2 <= plast) step(std::integral_constant<int, 2>{}, p + 2);
    };  // segment
    if constexpr (SIG) {
        if (rev) segment(std::true_type{});
        else segment(std::false_type{});
    } else {
        segment(std::false_type{});
    }
}

int env_int(const char* name, int dflt) { return knob(name, dflt); }

template <typename T, int V, int RY, int NW, int K, bool SIG = false, bool STRIP = false>
int launch_bk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, hipStream_t s,
              unsigned* sig = nullptr, int* nsig = nullptr, unsigned long long* fsig = nullptr) {
    using Tl = BKTile<T, V, RY, NW, K>;
    static_assert((STRIP ? size_t(2) * K * NW * 2 * Tl::RW * sizeof(T) : Tl::lds_bytes) <= 160 * 1024, "LDS budget");
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    if ((g.plane + g.row + 64) * int64_t(sizeof(T)) >= (int64_t(1) << 32) || g.nz + 4 * K >= (int64_t(1) << 30))
        return set_error(STENCIL_EINVAL, "plane too large for the box kernel (4 GiB per plane, 2^30 planes)");
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if (K > 1 && (lo || hi) && l.zghost < K)
        return set_error(STENCIL_EINVAL, "%d fused steps across a slab halo need halo >= %d (got %lld)", K, K,
                         (long long)l.zghost);
    // planes the launch may read: the ghost / halo planes its range needs
    // (single sweeps may cover slab-halo planes themselves: stencil_sweep)
    const int64_t ld_lo = std::min<int64_t>(lo ? -K : -1, begin - 1);
    const int64_t ld_hi = std::max<int64_t>(hi ? g.nz + K - 1 : g.nz, end);
    if (ld_lo < -l.zghost || ld_hi > g.nz + l.zghost - 1)
        return set_error(STENCIL_EINVAL, "box sweep of planes [%lld, %lld) reads past the %lld ghost planes",
                         (long long)begin, (long long)end, (long long)l.zghost);
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    const int64_t tiles = gx * gy;
    auto kern = [] {
        if constexpr (STRIP) return box27_strip<T, V, RY, NW, K, SIG>;
        else return box27_sep<T, V, RY, NW, K, SIG>;
    }();
    int zc = env_int("STENCIL_BOXK_ZCHUNK", 0);
    int slots = 0;
    if (zc <= 0) {
        // chunk count c minimising rounds x (chunk + 3K): a chunk's march
        // costs its planes plus the 3K-plane pipeline fill (kernels_strip.hip)
        if (const int rc = resident_slots(kern, 64 * NW, &slots)) return rc;
        int64_t best_c = 1, best = INT64_MAX;
        for (int64_t c = 1; c <= nz; ++c) {
            const int64_t z = (nz + c - 1) / c;
            if (c > 1 && z < 3 * K) break;
            const int64_t cost = ((tiles * c + slots - 1) / slots) * (z + 3 * K);
            if (cost <= best) best = cost, best_c = c;
        }
        if (SIG) {
            // face-signalled slab rounds: the most chunks that fit ONE round
            // with a CU per XCD to spare (the exchange runs beside the launch,
            // kernels_strip.hip); a grid of several rounds: at least 4 chunks,
            // whose two face chunks go first (the kernel's chunk order)
            const int64_t room = slots - slots / 32;
            for (int64_t c = 1; tiles * c <= room && c <= nz; ++c) {
                if (c > 1 && (nz + c - 1) / c < 3 * K) break;
                best_c = c;
            }
            if (tiles > room) {
                int64_t want = env_int("STENCIL_BOXK_SIG_CHUNKS", 4);
                while (want > 1 && (nz + want - 1) / want < 3 * K) --want;
                best_c = std::max(best_c, want);
            }
        }
        zc = int((nz + best_c - 1) / best_c);
    }
    if constexpr (SIG) {
        // every chunk at least K planes (a face lies inside one chunk)
        int64_t nch = (nz + zc - 1) / zc;
        auto last = [&](int64_t c) { return nz - (c - 1) * ((nz + c - 1) / c); };
        while (nch > 1 && ((nz + nch - 1) / nch < K || last(nch) < K)) --nch;
        zc = int((nz + nch - 1) / nch);
        if (nsig) *nsig = int(tiles);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    int64_t nb = tiles * gz;
    // few-tile grids: the packed longest-first schedule of the 7-point kernel
    // with the box's 3K-plane pipeline fill; not on slabs.  fp64 only by
    // default: 400^3 811 vs 755 Gcell/s, 512^3 796 vs 790, 640^2 x 320 equal;
    // in fp32 it loses (512^3 1012 vs 1389, 640^2 x 320 1262 vs 1400) although
    // the dispatcher model predicts 2-3 % fewer steps (profiles/r02dd_ab_box_pack.log)
    // (measured choice on the first launch of a shape: pick_schedule)
    const int* sched = nullptr;
    std::atomic<int>* verdict = nullptr;
    const int64_t nb_equal = nb;
    const int pack_mode = api_knob("STENCIL_BOXK_PACK", sizeof(T) == 8 ? 1 : 0);
    if (STRIP && !SIG && slots > 0 && pack_mode && !(lo || hi)) {
        int dev = 0;
        STENCIL_HIP_CHECK(hipGetDevice(&dev));
        if (const int rc = packed_schedule(reinterpret_cast<const void*>(kern), dev, tiles, nz, K, 3 * K, slots, zc, s,
                                           false, &sched, &nb, &verdict))
            return rc;
        if (pack_mode != 1) verdict = nullptr;  // 2: the model's choice, unmeasured
        if (verdict && verdict->load() == kPackEqual) sched = nullptr, nb = nb_equal, verdict = nullptr;
    }
    if (nb > (int64_t(1) << 31) - 8) return set_error(STENCIL_EINVAL, "grid too large for the box kernel");
    if (LaunchInfo* info = tl_dry_launch) {  // describe, do not launch
        if (slots == 0)
            if (const int rc = resident_slots(kern, 64 * NW, &slots)) return rc;
        info->workgroups = nb;
        info->zchunk = zc;
        info->packed = sched != nullptr;
        info->steps = K;
        info->slots = slots;
        return STENCIL_OK;
    }
    // XCD-patch work order for equal-chunk strip launches: 2048^2 x 256 fp64
    // K = 4 cuts L2-miss reads from 18.6 to 10.6 GB per launch (2.16x -> 1.23x
    // compulsory) and the launch time by 3 % (6.12 -> 5.93 ms; widths 2 / 8:
    // 6.01 / 5.96; profiles/r03/r03d_ab_box_xcd.txt) -- the kernel is bound by
    // its fp64 VALU work, not by those bytes
    const int xcd_pw = STRIP && !SIG ? env_int("STENCIL_BOXK_XCD", 4) : 0;
    auto launch = [&](bool packed) {
        const int64_t n = packed ? nb : (xcd_pw > 0 ? (nb_equal + 7) / 8 * 8 : nb_equal);
        hipLaunchKernelGGL(kern, dim3(unsigned(n)), dim3(64, NW, 1), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(out), g, int(begin), int(end), zc, int(gx),
                           int(gy), int(lo), int(hi), int(ld_lo), int(ld_hi), avg_weight<T>(l.prob), sig, fsig,
                           packed ? sched : nullptr, packed ? 0 : xcd_pw, env_int("STENCIL_BOXK_FAST", 1));
        return hipGetLastError();
    };
    if (sched && verdict && verdict->load() == kPackUntested) return pick_schedule(verdict, s, launch);
    if (const hipError_t e = launch(sched != nullptr); e != hipSuccess)
        return set_error(STENCIL_EHIP, "kernel launch failed: %s (box)", hipGetErrorString(e));
    return STENCIL_OK;
}

}  // namespace

#ifndef BOXK_PROBE_TU  // kernels_boxk_probe.hip re-includes the kernels above only
bool box27_supports(const stencil_problem& p) {
    return p.dims == 3 && p.shape == STENCIL_BOX && p.radius == 1 && p.order == STENCIL_ORDER_NAIVE;
}

// Workgroup shape cfg = RY*100 + NW (rows per wave x waves), STENCIL_BOXK_CFG.
int launch_boxk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                hipStream_t s) {
    if (!box27_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "the box kernel supports the 3D r=1 naive 27-point box only");
    const int cfg = env_int("STENCIL_BOXK_CFG", 0);
    // code-generation probe (debug library only): fp32 one cell
    // per lane, built with (95xxxx) and without (96xxxx) SLP vectorisation
    if (cfg >= 950000 && cfg < 970000 && l.prob.dtype == STENCIL_F32)
        return cfg < 960000 ? launch_boxk_probe_slp(l, in, out, begin, end, steps, cfg % 10000, s)
                            : launch_boxk_probe_noslp(l, in, out, begin, end, steps, cfg % 10000, s);
    // strip layout (box27_strip): cfg = 9VRRNN (V cells per lane, RR rows per wave, NN waves)
    if (cfg >= 900000) {
        if (l.prob.dtype == STENCIL_F32) {
            switch (steps * 1000000 + cfg) {
            case 3920408: return launch_bk<float, 2, 4, 8, 3, false, true>(l, in, out, begin, end, s);
            case 4920308: return launch_bk<float, 2, 3, 8, 4, false, true>(l, in, out, begin, end, s);
            case 4920408: return launch_bk<float, 2, 4, 8, 4, false, true>(l, in, out, begin, end, s);
            case 3920312: return launch_bk<float, 2, 3, 12, 3, false, true>(l, in, out, begin, end, s);
            case 2920408: return launch_bk<float, 2, 4, 8, 2, false, true>(l, in, out, begin, end, s);
            case 2920312: return launch_bk<float, 2, 3, 12, 2, false, true>(l, in, out, begin, end, s);
            case 2940208: return launch_bk<float, 4, 2, 8, 2, false, true>(l, in, out, begin, end, s);
            case 3920216: return launch_bk<float, 2, 2, 16, 3, false, true>(l, in, out, begin, end, s);
            case 1940408: return launch_bk<float, 4, 4, 8, 1, false, true>(l, in, out, begin, end, s);
            case 3920608: return launch_bk<float, 2, 6, 8, 3, false, true>(l, in, out, begin, end, s);
            case 4920508: return launch_bk<float, 2, 5, 8, 4, false, true>(l, in, out, begin, end, s);
            case 5920408: return launch_bk<float, 2, 4, 8, 5, false, true>(l, in, out, begin, end, s);
            case 5920508: return launch_bk<float, 2, 5, 8, 5, false, true>(l, in, out, begin, end, s);
            default: break;
            }
        } else {
            switch (steps * 1000000 + cfg) {
            case 3910408: return launch_bk<double, 1, 4, 8, 3, false, true>(l, in, out, begin, end, s);
            case 4910308: return launch_bk<double, 1, 3, 8, 4, false, true>(l, in, out, begin, end, s);
            case 4910408: return launch_bk<double, 1, 4, 8, 4, false, true>(l, in, out, begin, end, s);
            case 4910216: return launch_bk<double, 1, 2, 16, 4, false, true>(l, in, out, begin, end, s);
            case 3910312: return launch_bk<double, 1, 3, 12, 3, false, true>(l, in, out, begin, end, s);
            case 3910212: return launch_bk<double, 1, 2, 12, 3, false, true>(l, in, out, begin, end, s);
            case 3910308: return launch_bk<double, 1, 3, 8, 3, false, true>(l, in, out, begin, end, s);
            case 2910408: return launch_bk<double, 1, 4, 8, 2, false, true>(l, in, out, begin, end, s);
            case 2910312: return launch_bk<double, 1, 3, 12, 2, false, true>(l, in, out, begin, end, s);
            case 2910216: return launch_bk<double, 1, 2, 16, 2, false, true>(l, in, out, begin, end, s);
            case 3910216: return launch_bk<double, 1, 2, 16, 3, false, true>(l, in, out, begin, end, s);
            case 1920408: return launch_bk<double, 2, 4, 8, 1, false, true>(l, in, out, begin, end, s);
            case 3910608: return launch_bk<double, 1, 6, 8, 3, false, true>(l, in, out, begin, end, s);
            case 4910508: return launch_bk<double, 1, 5, 8, 4, false, true>(l, in, out, begin, end, s);
            case 5910408: return launch_bk<double, 1, 4, 8, 5, false, true>(l, in, out, begin, end, s);
            case 5910508: return launch_bk<double, 1, 5, 8, 5, false, true>(l, in, out, begin, end, s);
            default: break;
            }
        }
        // no strip shape for this (dtype, steps): the default shapes below
    }
    if (l.prob.dtype == STENCIL_F32) {
        switch (steps) {
        case 1:
            return launch_bk<float, 4, 2, 16, 1>(l, in, out, begin, end, s);
        case 2:
            switch (cfg) {
            case 216: return launch_bk<float, 4, 2, 16, 2>(l, in, out, begin, end, s);
            case 408: return launch_bk<float, 4, 4, 8, 2>(l, in, out, begin, end, s);
            case 208: return launch_bk<float, 4, 2, 8, 2>(l, in, out, begin, end, s);
            case 20116: return launch_bk<float, 2, 1, 16, 2>(l, in, out, begin, end, s);
            default: return launch_bk<float, 4, 1, 16, 2>(l, in, out, begin, end, s);
            }
        case 3:
            switch (cfg) {
            case 208: return launch_bk<float, 4, 2, 8, 3>(l, in, out, begin, end, s);
            case 20116: return launch_bk<float, 2, 1, 16, 3>(l, in, out, begin, end, s);
            case 20216: return launch_bk<float, 2, 2, 16, 3>(l, in, out, begin, end, s);
            case 416: return launch_bk<float, 4, 1, 16, 3>(l, in, out, begin, end, s);
            case 20308: return launch_bk<float, 2, 3, 8, 3>(l, in, out, begin, end, s);
            // strip layout, 8-B lanes, 4 rows x 8 waves: 2048^2 x 256 1504 vs 1012,
            // 512^3 1349 vs 879, 2048^3 1510 vs 1116 Gcell/s for the interleaved
            // 3 x 8 (profiles/r02j_ab_box_strip.log)
            default: return launch_bk<float, 2, 4, 8, 3, false, true>(l, in, out, begin, end, s);
            }
        default: break;
        }
    } else {
        switch (steps) {
        case 1:
            return launch_bk<double, 2, 2, 16, 1>(l, in, out, begin, end, s);
        case 2:
            switch (cfg) {
            case 216: return launch_bk<double, 2, 2, 16, 2>(l, in, out, begin, end, s);
            case 408: return launch_bk<double, 2, 4, 8, 2>(l, in, out, begin, end, s);
            case 308: return launch_bk<double, 2, 3, 8, 2>(l, in, out, begin, end, s);
            case 208: return launch_bk<double, 2, 2, 8, 2>(l, in, out, begin, end, s);
            case 10116: return launch_bk<double, 1, 1, 16, 2>(l, in, out, begin, end, s);
            case 10216: return launch_bk<double, 1, 2, 16, 2>(l, in, out, begin, end, s);
            default: return launch_bk<double, 2, 1, 16, 2>(l, in, out, begin, end, s);
            }
        case 3:
            switch (cfg) {
            case 308: return launch_bk<double, 2, 3, 8, 3>(l, in, out, begin, end, s);
            case 208: return launch_bk<double, 2, 2, 8, 3>(l, in, out, begin, end, s);
            case 10116: return launch_bk<double, 1, 1, 16, 3>(l, in, out, begin, end, s);
            case 10216: return launch_bk<double, 1, 2, 16, 3>(l, in, out, begin, end, s);
            case 10308: return launch_bk<double, 1, 3, 8, 3>(l, in, out, begin, end, s);
            case 10408: return launch_bk<double, 1, 4, 8, 3>(l, in, out, begin, end, s);
            case 216: return launch_bk<double, 2, 1, 16, 3>(l, in, out, begin, end, s);
            // strip layout, one cell per lane (profiles/r02j_ab_box_strip.log):
            // planes of < 1024^2 cells 4 rows x 8 waves (512^3 773 vs 578 Gcell/s
            // for the interleaved 3 x 8), larger planes 2 rows x 16 waves
            // (2048^2 x 256 759 vs 706, 2048^3 766 vs 739; 4 x 8 loses there)
            default:
                if (l.prob.nx * l.prob.ny < (int64_t(1) << 20))
                    return launch_bk<double, 1, 4, 8, 3, false, true>(l, in, out, begin, end, s);
                return launch_bk<double, 1, 2, 16, 3, false, true>(l, in, out, begin, end, s);
            }
        default: break;
        }
    }
    if (steps == 4) {
        // strip layout, 5 rows x 8 waves (40 rows for 32 output rows): fits
        // since round 3's box order (fp64 238 VGPRs, fp32 249); 2048^2 x 256
        // fp64 1108 vs 1057 (4 x 8) and 850 (3 x 8) Gcell/s, fp32 1997 vs
        // 1895 / 1763; 512^3 fp64 1096 vs 979 / 762 (profiles/r03/r03k_ab_box*.txt)
        if (l.prob.dtype == STENCIL_F32) return launch_bk<float, 2, 5, 8, 4, false, true>(l, in, out, begin, end, s);
        return launch_bk<double, 1, 5, 8, 4, false, true>(l, in, out, begin, end, s);
    }
    return set_error(STENCIL_EINVAL, "box kernel steps must be 1..4 (got %d; K = 5 shapes are debug configurations)",
                     steps);
}

// Face-signalled box launches for multi-GPU slab rounds (stencil_sweepk_signal):
// the default shapes of launch_boxk.
int launch_boxk_signal(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                       unsigned* sig, unsigned long long* fsig, int* nsig, hipStream_t s) {
    if (!box27_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "the box kernel supports the 3D r=1 naive 27-point box only");
    const int cfg = env_int("STENCIL_BOXK_SIG_CFG", 0);
    if (cfg >= 900000) {  // strip layout, as launch_boxk
        if (l.prob.dtype == STENCIL_F32) {
            switch (steps * 1000000 + cfg) {
            case 3920408: return launch_bk<float, 2, 4, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 3920308: return launch_bk<float, 2, 3, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4920408: return launch_bk<float, 2, 4, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4920508: return launch_bk<float, 2, 5, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            default: break;
            }
        } else {
            switch (steps * 1000000 + cfg) {
            case 3910408: return launch_bk<double, 1, 4, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 3910308: return launch_bk<double, 1, 3, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 3910312: return launch_bk<double, 1, 3, 12, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4910308: return launch_bk<double, 1, 3, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4910212: return launch_bk<double, 1, 2, 12, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4910216: return launch_bk<double, 1, 2, 16, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4910408: return launch_bk<double, 1, 4, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            case 4910508: return launch_bk<double, 1, 5, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            default: break;
            }
        }
    }
    if (l.prob.dtype == STENCIL_F32) {
        switch (steps) {
        case 2: return launch_bk<float, 4, 1, 16, 2, true>(l, in, out, begin, end, s, sig, nsig, fsig);
        case 3:
            if (cfg == 20308) return launch_bk<float, 2, 3, 8, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            if (cfg == 20208) return launch_bk<float, 2, 2, 8, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            if (cfg == 20116) return launch_bk<float, 2, 1, 16, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            // strip layout, 3 rows x 8 waves (4 rows spill with the down-march's carry)
            return launch_bk<float, 2, 3, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
        default: break;
        }
    } else {
        switch (steps) {
        case 2: return launch_bk<double, 2, 1, 16, 2, true>(l, in, out, begin, end, s, sig, nsig, fsig);
        case 3:
            if (cfg == 10308) return launch_bk<double, 1, 3, 8, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            if (cfg == 10208) return launch_bk<double, 1, 2, 8, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            if (cfg == 10116) return launch_bk<double, 1, 1, 16, 3, true>(l, in, out, begin, end, s, sig, nsig, fsig);
            // strip layout, 3 rows x 8 waves: 2048^3 interior rank 758 vs 659
            // Gcell/s for the interleaved 1 x 16 (profiles/r02k_bench_c5_loopback_sig*.json)
            return launch_bk<double, 1, 3, 8, 3, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
        default: break;
        }
    }
    if (steps == 4) {  // strip layout, 5 rows x 8 waves (as launch_boxk)
        if (l.prob.dtype == STENCIL_F32)
            return launch_bk<float, 2, 5, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
        return launch_bk<double, 1, 5, 8, 4, true, true>(l, in, out, begin, end, s, sig, nsig, fsig);
    }
    return set_error(STENCIL_EINVAL, "face-signalled box sweeps: steps must be 2..4 (got %d)", steps);
}

// Single sweeps and fused pairs of the box (stencil_sweep / stencil_sweep2).
int launch_box27(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                 hipStream_t s) {
    return launch_boxk(l, in, out, begin, end, steps, s);
}
#endif  // BOXK_PROBE_TU

}  // namespace stencil
