// kernels_temporalk.hip -- K = 3 or 4 fused Jacobi sweeps per launch for the
// 3D 7-point star (r = 1, naive order): deeper temporal blocking than
// kernels_temporal.hip.
//
// One launch reads grid t once and writes grid t+K once, so HBM traffic per
// update falls from ~9 B (K = 2, measured) to ~(8 * f + 8) / K with f the
// halo over-fetch of the tile.
//
// Why a different structure from temporal2_7pt_lc: that kernel double-buffers
// every stage's plane in LDS so that one barrier per plane suffices; with K
// stages this needs 2K region planes (K = 3: 215 KB, more than the 160 KB of a
// CU).  Here every stage owns ONE LDS plane and an iteration has two phases:
//
//   barrier A
//   read phase   for s = 1..K:  t_s(p-s) = S(t_{s-1}) with
//                  x/y neighbours and centre of t_{s-1}(p-s) from LDS plane s-1,
//                  z-  = t_{s-1}(p-s-1): this lane's own centre from the
//                        previous iteration, kept in registers,
//                  z+  = t_{s-1}(p-s+1): stage s-1's result of this iteration
//                        (stage 1: input plane p from the register ring)
//                t_K(p-K) -> HBM (nontemporal)
//   barrier B
//   write phase  LDS plane 0 <- in(p);  LDS plane s <- t_s(p-s), s < K
//                request in(p+R) into the ring slot in(p) just vacated
//
// so a launch needs K region planes of LDS (K = 3, 128 x 48 fp64 region:
// 158 KB) and (R + 2K) planes x RY rows of registers per lane.
//
// Tiles: the workgroup's lanes cover a region of 64V x NW*RY cells; stage s is
// exact on the region minus an s-cell ring, so the output tile is
// TX = 64V - 2V*ceil(K/V) by TY = NW*RY - 2K.  z is marched in chunks
// [za, zb); a chunk reads input planes za-K .. zb+K-1 and runs zb-za+2K
// iterations.  Intermediate planes t_s outside the domain (ghost cells) keep
// their input value (Dirichlet), as in a plain sweep.
//
// Arithmetic: every cell of every stage is the single-sweep expression
// (0 + x- + x+ + y- + y+ + z- + z+) * avg.  The leading "0 +" is folded into
// the multiply as fma(sum, avg, +0): the partial sums differ from the
// reference's only in the sign of an exact zero, and fma(+-0 * avg, +0) = +0
// equals the reference's (+0) * avg, while for sum != 0 fma(sum, avg, 0) is
// the correctly rounded product.  Results are bitwise equal to K plain
// sweeps (tests/test_gpu_parity.py, including a field of -0.0 cells).
#include <cstdlib>

#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int V>
struct VecK {
    typedef T type __attribute__((ext_vector_type(V)));
};

__device__ __forceinline__ float fma0(float s, float a) { return __builtin_fmaf(s, a, 0.0f); }
__device__ __forceinline__ double fma0(double s, double a) { return __builtin_fma(s, a, 0.0); }

// Whole-wave lane shifts (DPP wave_shr:1 / wave_shl:1): lane i receives
// lane i-1's (shr) or lane i+1's (shl) value; the lane without a source gets
// 0 (bound_ctrl: no "old" operand to initialise -- that lane is a ring lane
// whose value is never used).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f(double v) {
    const int2 b = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_mov_dpp(b.x, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(b.y, CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
constexpr int kWaveShr1 = 0x138, kWaveShl1 = 0x130;

template <typename T, int V, int RY, int NW, int K, bool AL = false, int XRO = 0>
struct TKTile {
    static constexpr int XR = XRO ? XRO : (K + V - 1) / V;  // ring vectors per x side
    static constexpr int RW = 64 * V;              // region width
    // output tile width; AL: a multiple of 128 B so every tile's output rows
    // start on a cache line (the lanes past TX/V + 2 XR then idle)
    static constexpr int AW = 128 / int(sizeof(T));
    static constexpr int TX = AL ? (RW - 2 * XR * V) / AW * AW : RW - 2 * XR * V;
    static constexpr int NL = TX / V + 2 * XR;     // lanes that load
    static constexpr int RH = NW * RY;             // region height
    static constexpr int TY = RH - 2 * K;          // output tile height
    static constexpr int LX = RW + 2 * V;          // LDS row: pad V | region | pad V
    static constexpr int LY = RH + 2;              // LDS rows: pad | region | pad
    static constexpr size_t lds_bytes = size_t(K) * LY * LX * sizeof(T);
};

template <typename T, int V, int RY, int NW, int K, int R, bool DPPX, bool AL, int XRO, int WPE, bool SB = false>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE)))
    temporalk_7pt(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
                  int zchunk, int tiles_x, int tiles_y, int halo_lo, int halo_hi, int remap, T avg) {
    using Tl = TKTile<T, V, RY, NW, K, AL, XRO>;
    using VT = typename VecK<T, V>::type;
    constexpr int XR = Tl::XR, TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LX = Tl::LX, LY = Tl::LY, NL = Tl::NL;
    static_assert(TY > 0 && TX > 0, "tile too small for K");
    static_assert(R >= 2 && R % 2 == 0, "ring size must be even (z- parity) and >= 2");
    __shared__ __attribute__((aligned(16))) T L[K][LY][LX];

    // Optional XCD-aware order: workgroups are dealt round-robin to the 8
    // XCDs, so give XCD j the j-th contiguous run of tiles (neighbours in x/y
    // then share halo lines in that XCD's L2); uneven shares allowed.
    int t = blockIdx.x;
    if (remap) {
        const int nb = gridDim.x, q = nb >> 3, r8 = nb & 7, j = t & 7;
        t = j * q + (j < r8 ? j : r8) + (t >> 3);
    }
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int bz = t / (tiles_x * tiles_y);

    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - XR * V + int64_t(lane) * V;
    const int64_t y0 = int64_t(by) * TY - K;
    const int64_t za = zbeg + int64_t(bz) * zchunk;
    const int64_t zb = za + zchunk < zend ? za + zchunk : zend;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;
    const int64_t plane = g.plane;

    // Zero all LDS planes (pads and not-yet-written rows feed ring cells only,
    // but keep them finite).
    {
        constexpr int N16 = int(Tl::lds_bytes / 16);
        VT* l16 = reinterpret_cast<VT*>(&L[0][0][0]);
        for (int i = threadIdx.y * 64 + threadIdx.x; i < N16; i += 64 * NW) l16[i] = VT{};
    }

    // Loads are issued unconditionally from clamped addresses (rows outside
    // [-1, ny], vectors past x = nx, idle lanes, planes outside the loaded
    // range re-read valid cells that only feed ring cells): with no branch
    // around them the compiler can wait for plane p with vmcnt(RY) instead of
    // vmcnt(0) -- a conditional load or store leaves a path with no younger
    // memory op, and vmcnt(0) also waits for the prefetched plane p+1.
    int off[RY];  // in-plane offsets (a plane has < 2^31 elements, checked at launch)
    bool yin[RY], st[RY];
    const int64_t xmax = g.nx / V * V;  // last vector start that stays inside the padded row
    const int64_t xl = lane < NL ? x : int64_t(bx) * TX - XR * V + int64_t(NL - 1) * V;
    const int64_t xc = xl < xmax ? xl : xmax;
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w + NW * k;
        const int64_t y = y0 + rr;
        const int64_t yc = y < -1 ? -1 : (y > g.ny ? g.ny : y);
        off[k] = int(yc * g.row + xc);
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= K && rr < RH - K && y < g.ny && lane >= XR && lane < NL - XR;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    // Loaded input planes: [ld_lo, zlast]; stage s is computed on planes
    // [lo_s, hi_s) and copied (Dirichlet ghost planes) elsewhere.
    const int64_t ld_lo = halo_lo ? -K : -1;
    const int64_t ld_hi = halo_hi ? g.nz + K - 1 : g.nz;
    const int64_t zlast = zb + K - 1 < ld_hi ? zb + K - 1 : ld_hi;

    auto load_plane = [&](VT (&d)[RY], int64_t z) {
        const int64_t zc = z < ld_lo ? ld_lo : (z > zlast ? zlast : z);
        const T* base = src + zc * plane;
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(base + int64_t(off[k]));
    };

    const int64_t p0 = za - K;
    VT vin[R][RY];   // ring: slot (q - p0) mod R holds in(q)
    VT hz[2][K][RY]; // z- of stage s+1: own centre of t_s read one iteration ago (parity-indexed)
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int k = 0; k < RY; ++k) vin[i][k] = VT{};
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < K; ++s)
#pragma unroll
            for (int k = 0; k < RY; ++k) hz[b][s][k] = VT{};
#pragma unroll
    for (int i = 0; i < R; ++i) load_plane(vin[i], p0 + i);

    const int xx = V + lane * V;

    auto step = [&](auto S_, int64_t p) {
        constexpr int S = decltype(S_)::value;
        constexpr int P = S & 1;  // hz[P] receives this iteration's centres, hz[P^1] holds z-
        __syncthreads();          // A: last write phase visible
        VT res[K][RY];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            const int64_t z = p - s;
            const int64_t lo_s = halo_lo ? -(K - s) : 0;
            const int64_t hi_s = halo_hi ? g.nz + (K - s) : g.nz;
            const bool zin = z >= lo_s && z < hi_s;
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const int yy = w + NW * k + 1;
                const T* cr = &L[s - 1][yy][xx];
                const VT c = *reinterpret_cast<const VT*>(cr);
                const VT up = *reinterpret_cast<const VT*>(&L[s - 1][yy - 1][xx]);
                const VT dn = *reinterpret_cast<const VT*>(&L[s - 1][yy + 1][xx]);
                T wl, er;
                if constexpr (DPPX) {  // x neighbours from the adjacent lanes' registers
                    wl = dpp_f<kWaveShr1>(c[V - 1]);
                    er = dpp_f<kWaveShl1>(c[0]);
                } else {
                    wl = cr[-1];
                    er = cr[V];
                }
                const VT zm = hz[P ^ 1][s - 1][k];
                const VT zp = s == 1 ? vin[S][k] : res[s - 2 < 0 ? 0 : s - 2][k];
                VT o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    T sum = (j == 0 ? wl : c[j - 1]) + (j == V - 1 ? er : c[j + 1]);
                    sum += up[j];
                    sum += dn[j];
                    sum += zm[j];
                    sum += zp[j];
                    o[j] = fma0(sum, avg);
                    if (s < K) o[j] = (zin && yin[k] && xin[j]) ? o[j] : c[j];
                }
                hz[P][s - 1][k] = c;
                res[s - 1][k] = o;
            }
            if constexpr (SB) __builtin_amdgcn_sched_barrier(0);  // no hoisting across stages
        }
        // t_K(p-K) -> HBM
        const int64_t zo = p - K;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                if (st[k]) {
                    T* q = dst + zo * plane + int64_t(off[k]);
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
        __syncthreads();  // B: every read of the old planes is done
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
            *reinterpret_cast<VT*>(&L[0][yy][xx]) = vin[S][k];
#pragma unroll
            for (int s = 1; s < K; ++s) *reinterpret_cast<VT*>(&L[s][yy][xx]) = res[s - 1][k];
        }
        load_plane(vin[S], p + R);
    };

    // Whole blocks of R steps unconditionally, then the tail: a conditional
    // step inside the loop would keep the previous z- planes live across the
    // back edge (twice the registers).
    const int64_t plast = zb + K - 1;
    int64_t p = p0;
    for (; p + R - 1 <= plast; p += R) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        if constexpr (R > 2) {
            step(std::integral_constant<int, 2 % R>{}, p + 2);
            step(std::integral_constant<int, 3 % R>{}, p + 3);
        }
    }
    if (p <= plast) step(std::integral_constant<int, 0>{}, p);
    if constexpr (R > 2) {
        if (p + 1 <= plast) step(std::integral_constant<int, 1>{}, p + 1);
        if (p + 2 <= plast) step(std::integral_constant<int, 2 % R>{}, p + 2);
    }
}

int env_int(const char* name, int dflt) { return knob(name, dflt); }

template <typename T, int V, int RY, int NW, int K, int R, bool DPPX = false, bool AL = false, int XRO = 0,
          int WPE = 1, bool SB = false>
int launch_tk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, hipStream_t s) {
    using Tl = TKTile<T, V, RY, NW, K, AL, XRO>;
    static_assert(Tl::lds_bytes <= 160 * 1024, "LDS budget");
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    auto kern = temporalk_7pt<T, V, RY, NW, K, R, DPPX, AL, XRO, WPE, SB>;
    if (g.plane >= (int64_t(1) << 31)) return set_error(STENCIL_EINVAL, "plane too large for temporalk (2^31 elements)");
    int zc = env_int("STENCIL_TK_ZCHUNK", 0);
    if (zc <= 0) {
        // Chunk count c minimising  ceil(tiles*c / slots) * (nz/c + 2K):
        // workgroups run in "rounds" of `slots` (one per CU here: the LDS
        // planes take 108 KB), each round costs one chunk march of nz/c + 2K
        // planes, and a last round that is mostly empty costs as much as a
        // full one (measured, 512^3 fp64: zc 103 / 52 -> 2 / 3.9 rounds
        // 885 Gcell/s, zc 64 / 128 -> 3.1 / 1.6 rounds 760-790).
        int slots = 0;
        if (const int rc = resident_slots(kern, 64 * NW, &slots)) return rc;
        const int64_t tiles = gx * gy;
        int64_t best_c = 1, best = INT64_MAX;
        for (int64_t c = 1; c <= nz; ++c) {
            const int64_t z = (nz + c - 1) / c;
            if (c > 1 && z < 2 * K) break;  // chunks shorter than their halo
            const int64_t cost = ((tiles * c + slots - 1) / slots) * (z + 2 * K);
            if (cost <= best) best = cost, best_c = c;
        }
        zc = int((nz + best_c - 1) / best_c);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    const int64_t nb = gx * gy * gz;
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for temporalk");
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if ((lo || hi) && l.zghost < K)
        return set_error(STENCIL_EINVAL, "%d fused steps across a slab halo need halo >= %d (got %lld)", K, K,
                         (long long)l.zghost);
    hipLaunchKernelGGL(kern, dim3(unsigned(nb)), dim3(64, NW, 1), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, begin, end, zc, int(gx), int(gy),
                       int(lo), int(hi), env_int("STENCIL_TK_REMAP", 0), avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

}  // namespace

int launch_temporalk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                     hipStream_t s) {
    if (!temporal2_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "TEMPORALK supports 3D star r=1 naive order only");
    // cfg = RY*100 + NW: rows per wave x waves (region 64V x RY*NW); default
    // x neighbours by DPP lane shifts (+6.6 % fp64 / +13 % fp32 over the LDS
    // reads of cfg 216, 512^3); 2xxxx / 3xxxx = DPP shapes (3xxxx: fp32, V = 2)
    const int cfg = env_int("STENCIL_TK_CFG", 0);
    // Default: the strip layout (kernels_strip.hip; +2-3 % at K = 3 and the
    // only layout whose K = 4 shapes fit the register file).  STENCIL_TK_STRIP
    // = 0 selects this file's interleaved-row layout, > 1 a strip cfg.
    if (const int strip = env_int("STENCIL_TK_STRIP", 1))
        return launch_tkstrip(l, in, out, begin, end, steps, strip == 1 ? 0 : strip, s);
    if (l.prob.dtype == STENCIL_F32) {
        if (steps == 3) {
            switch (cfg) {
            case 312: return launch_tk<float, 4, 3, 12, 3, 2>(l, in, out, begin, end, s);
            case 608: return launch_tk<float, 4, 6, 8, 3, 2>(l, in, out, begin, end, s);
            case 216: return launch_tk<float, 4, 2, 16, 3, 2>(l, in, out, begin, end, s);
            case 30216: return launch_tk<float, 2, 2, 16, 3, 2, true>(l, in, out, begin, end, s);
            case 40216: return launch_tk<float, 4, 2, 16, 3, 2, true, true>(l, in, out, begin, end, s);
            case 30316: return launch_tk<float, 2, 3, 16, 3, 2, true>(l, in, out, begin, end, s);
            default: return launch_tk<float, 4, 2, 16, 3, 2, true>(l, in, out, begin, end, s);
            }
        }
        if (steps == 4) {
            switch (cfg) {
            case 408: return launch_tk<float, 4, 4, 8, 4, 2>(l, in, out, begin, end, s);
            case 216: return launch_tk<float, 4, 2, 16, 4, 2>(l, in, out, begin, end, s);
            default: return launch_tk<float, 4, 2, 16, 4, 2, true>(l, in, out, begin, end, s);
            }
        }
    } else {
        if (steps == 3) {
            switch (cfg) {
            case 312: return launch_tk<double, 2, 3, 12, 3, 2>(l, in, out, begin, end, s);
            case 216: return launch_tk<double, 2, 2, 16, 3, 2>(l, in, out, begin, end, s);
            case 20312: return launch_tk<double, 2, 3, 12, 3, 2, true>(l, in, out, begin, end, s);
            case 20412: return launch_tk<double, 2, 4, 12, 3, 2, true>(l, in, out, begin, end, s);
            case 20408: return launch_tk<double, 2, 4, 8, 3, 2, true>(l, in, out, begin, end, s);
            case 20216 + 40000: return launch_tk<double, 2, 2, 16, 3, 4, true>(l, in, out, begin, end, s);
            case 40216: return launch_tk<double, 2, 2, 16, 3, 2, true, true>(l, in, out, begin, end, s);
            default: return launch_tk<double, 2, 2, 16, 3, 2, true>(l, in, out, begin, end, s);
            }
        }
        if (steps == 4) {
            switch (cfg) {
            case 408: return launch_tk<double, 2, 4, 8, 4, 2>(l, in, out, begin, end, s);
            case 20408: return launch_tk<double, 2, 4, 8, 4, 2, true>(l, in, out, begin, end, s);
            case 216: return launch_tk<double, 2, 2, 16, 4, 2>(l, in, out, begin, end, s);
            default: return launch_tk<double, 2, 2, 16, 4, 2, true>(l, in, out, begin, end, s);
            }
        }
    }
    return set_error(STENCIL_EINVAL, "the interleaved-row temporalk layout does %s steps; 3 or 4 only (got %d)",
                     steps == 5 ? "not do 5" : "not do these", steps);
}

}  // namespace stencil
