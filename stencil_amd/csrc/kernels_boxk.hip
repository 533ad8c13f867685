// kernels_boxk.hip -- K fused sweeps per launch of the 3D 27-point box
// stencil (r = 1, naive order), in the two-phase z-march of
// kernels_temporalk.hip.
//
// Sum order.  The reference adds the 26 neighbours lexicographically in
// (dz, dy, dx) with the centre skipped (oracle/oracle_impl.inc): the 9 terms
// of plane z-1, then the 8 of plane z, then the 9 of plane z+1.  So while
// plane q of t_{s-1} sits in LDS, stage s can, for every cell of its column,
//     finish   t_s(q-1)   (+ its 9 dz=+1 terms)   -> * avg
//     continue t_s(q)     (+ its 8 dz=0 terms)
//     start    t_s(q+1)   (its 9 dz=-1 terms)
// which is every cell's 26 additions in exactly that order, with two running
// sums per cell (t_s(q), t_s(q+1)) carried in registers between planes.
//
// Pipeline.  Stage s finishes plane q-1 at the iteration where its newest
// input plane is q = p - 2s + 1, and stage s+1 reads that plane one iteration
// later, so stage s lags stage s-1 by two planes and a chunk [za, zb) runs
// zb - za + 3K iterations over input planes za-K .. zb+K-1.  Per iteration:
//   barrier A
//   read phase   for s = 1..K: the 3x3 neighbourhood of the lane's cells in
//                LDS plane s-1 (3 vector reads, x neighbours by DPP lane
//                shifts); finish / continue / start as above.  Intermediate
//                planes keep ghost cells at their input value (the lane's own
//                centre of plane q-1, kept from the previous iteration);
//                slab-halo planes (HALO_LO/HI) are advanced like interior ones.
//                t_K(p-2K) -> HBM
//   barrier B
//   write phase  LDS plane 0 <- in(p); LDS plane s <- t_s(p-2s), s < K;
//                request in(p+R) (unconditional clamped loads, as in
//                kernels_temporalk.hip, so the plane wait is a counted vmcnt).
//
// Arithmetic: the leading "0 +" of the reference's sum is folded into
// fma(sum, avg, +0) exactly as in kernels_temporalk.hip (bit-identical; a
// -0.0 field is in tests/test_gpu_parity.py).
#include <cstdlib>

#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int V>
struct VecB {
    typedef T type __attribute__((ext_vector_type(V)));
};

__device__ __forceinline__ float bfma0(float s, float a) { return __builtin_fmaf(s, a, 0.0f); }
__device__ __forceinline__ double bfma0(double s, double a) { return __builtin_fma(s, a, 0.0); }

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
    static constexpr int RW = 64 * V;
    static constexpr int TX = RW - 2 * XR * V;
    static constexpr int RH = NW * RY;
    static constexpr int TY = RH - 2 * K;
    static constexpr int LX = RW + 2 * V;
    static constexpr int LY = RH + 2;
    static constexpr size_t lds_bytes = size_t(K) * LY * LX * sizeof(T);
};

// XD: x-neighbours by DPP lane shifts (true, default) or by two extra LDS
// reads per row (false; measured 11-13 % slower in fp64 although the DPP
// moves are ~18 % of the kernel's VALU instructions).
template <typename T, int V, int RY, int NW, int K, int R, bool XD>
__global__ void __launch_bounds__(64 * NW)
    boxk_27pt(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend, int zchunk,
              int tiles_x, int tiles_y, int halo_lo, int halo_hi, T avg) {
    using Tl = BKTile<T, V, RY, NW, K>;
    using VT = typename VecB<T, V>::type;
    constexpr int XR = Tl::XR, TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LX = Tl::LX, LY = Tl::LY;
    static_assert(TY > 0 && TX > 0, "tile too small for K");
    static_assert(R >= 2 && R % 2 == 0, "ring size must be even (register parity)");
    __shared__ __attribute__((aligned(16))) T L[K][LY][LX];

    const int t = blockIdx.x;
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int bz = t / (tiles_x * tiles_y);
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - XR * V + int64_t(lane) * V;
    const int64_t y0 = int64_t(by) * TY - K;
    // z in 32-bit scalars; addresses = uniform per-plane base + one
    // non-negative 32-bit byte offset per row (saddr form), as in
    // kernels_strip.hip
    const int za = int(zbeg) + bz * zchunk;
    const int zb = za + zchunk < int(zend) ? za + zchunk : int(zend);
    const int nz = int(g.nz);
    const int64_t plane = g.plane;
    const int64_t bias = g.row + XR * V;
    const char* __restrict__ src = reinterpret_cast<const char*>(in + g.origin - bias);
    char* __restrict__ dst = reinterpret_cast<char*>(out + g.origin - bias);

    {
        constexpr int N16 = int(Tl::lds_bytes / 16);
        VT* l16 = reinterpret_cast<VT*>(&L[0][0][0]);
        for (int i = threadIdx.y * 64 + threadIdx.x; i < N16; i += 64 * NW) l16[i] = VT{};
    }

    // unconditional loads from clamped addresses (see kernels_temporalk.hip)
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
    const int ld_lo = halo_lo ? -K : -1;
    const int ld_hi = halo_hi ? nz + K - 1 : nz;
    const int zlast = zb + K - 1 < ld_hi ? zb + K - 1 : ld_hi;
    auto load_plane = [&](VT (&d)[RY], int z) {
        const int zz = z < ld_lo ? ld_lo : (z > zlast ? zlast : z);
        const char* base = src + int64_t(zz) * plane * int64_t(sizeof(T));
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(base + off[k]);
    };

    const int p0 = za - K;
    VT vin[R][RY];
    VT part[2][K][RY];  // running sums, parity-indexed: [P^1] = t_s(q-1) (finish), [P] = t_s(q) (continue)
    VT cen[2][K][RY];   // own centre of the stage's input plane, parity-indexed ([P^1] = plane q-1)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < K; ++s)
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                part[b][s][k] = VT{};
                cen[b][s][k] = VT{};
            }
#pragma unroll
    for (int i = 0; i < R; ++i) load_plane(vin[i], p0 + i);
    const int xx = V + lane * V;

    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        constexpr int P = S & 1;
        __syncthreads();  // A
        VT res[K][RY];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            const int m = p - 2 * s;  // plane finished now
            const int lo_s = halo_lo ? -(K - s) : 0;
            const int hi_s = halo_hi ? nz + (K - s) : nz;
            const bool zin = m >= lo_s && m < hi_s;
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const int yy = w + NW * k + 1;
                // 3 x (V+2) neighbourhood of this lane's cells in plane q
                T nb[3][V + 2];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const VT c = *reinterpret_cast<const VT*>(&L[s - 1][yy - 1 + r][xx]);
                    if constexpr (XD) {
                        nb[r][0] = bdpp<kShr1>(c[V - 1]);
                    } else {
                        nb[r][0] = L[s - 1][yy - 1 + r][xx - 1];
                    }
#pragma unroll
                    for (int j = 0; j < V; ++j) nb[r][j + 1] = c[j];
                    if constexpr (XD) {
                        nb[r][V + 1] = bdpp<kShl1>(c[0]);
                    } else {
                        nb[r][V + 1] = L[s - 1][yy - 1 + r][xx + V];
                    }
                }
                VT fin, cont, start, o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    // finish t_s(q-1): + 9 terms (dz = +1)
                    T a = part[P ^ 1][s - 1][k][j];
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) a += nb[r][j + dx];
                    fin[j] = a;
                    // continue t_s(q): + 8 terms (dz = 0, centre skipped)
                    T b = part[P][s - 1][k][j];
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) b += nb[0][j + dx];
                    b += nb[1][j];
                    b += nb[1][j + 2];
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) b += nb[2][j + dx];
                    cont[j] = b;
                    // start t_s(q+1): 9 terms (dz = -1); "0 +" folded into the fma
                    T c0 = nb[0][j] + nb[0][j + 1];
                    c0 += nb[0][j + 2];
#pragma unroll
                    for (int r = 1; r < 3; ++r)
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) c0 += nb[r][j + dx];
                    start[j] = c0;
                    o[j] = bfma0(fin[j], avg);
                    if (s < K) o[j] = (zin && yin[k] && xin[j]) ? o[j] : cen[P ^ 1][s - 1][k][j];
                }
                part[P ^ 1][s - 1][k] = start;  // t_s(q+1) takes the finished slot
                part[P][s - 1][k] = cont;
                VT cc;
#pragma unroll
                for (int j = 0; j < V; ++j) cc[j] = nb[1][j + 1];
                cen[P][s - 1][k] = cc;
                res[s - 1][k] = o;
            }
#ifdef BOXK_SB
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
        // t_K(p-2K) -> HBM
        const int zo = p - 2 * K;
        if (zo >= za && zo < zb) {
            char* obase = dst + int64_t(zo) * plane * int64_t(sizeof(T));
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                if (st[k]) {
                    T* q = reinterpret_cast<T*>(obase + off[k]);
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
        __syncthreads();  // B
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
            *reinterpret_cast<VT*>(&L[0][yy][xx]) = vin[S][k];
#pragma unroll
            for (int s = 1; s < K; ++s) *reinterpret_cast<VT*>(&L[s][yy][xx]) = res[s - 1][k];
        }
        load_plane(vin[S], p + R);
    };

    const int plast = zb - 1 + 2 * K;
    int p = p0;
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

int env_int(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return s && *s ? std::atoi(s) : dflt;
}

template <typename T, int V, int RY, int NW, int K, int R, bool XD = true>
int launch_bk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, hipStream_t s) {
    using Tl = BKTile<T, V, RY, NW, K>;
    static_assert(Tl::lds_bytes <= 160 * 1024, "LDS budget");
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    if ((g.plane + g.row + 64) * int64_t(sizeof(T)) >= (int64_t(1) << 32) || g.nz + 4 * K >= (int64_t(1) << 30))
        return set_error(STENCIL_EINVAL, "plane too large for boxk (4 GiB per plane, 2^30 planes)");
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    auto kern = boxk_27pt<T, V, RY, NW, K, R, XD>;
    int zc = env_int("STENCIL_BOXK_ZCHUNK", 0);
    if (zc <= 0) {
        // as kernels_temporalk.hip, with the 3K-plane pipeline fill of this kernel
        int slots = 0;
        if (const int rc = resident_slots(kern, 64 * NW, &slots)) return rc;
        const int64_t tiles = gx * gy;
        int64_t best_c = 1, best = INT64_MAX;
        for (int64_t c = 1; c <= nz; ++c) {
            const int64_t z = (nz + c - 1) / c;
            if (c > 1 && z < 3 * K) break;
            const int64_t cost = ((tiles * c + slots - 1) / slots) * (z + 3 * K);
            if (cost <= best) best = cost, best_c = c;
        }
        zc = int((nz + best_c - 1) / best_c);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    const int64_t nb = gx * gy * gz;
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for boxk");
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if ((lo || hi) && l.zghost < K)
        return set_error(STENCIL_EINVAL, "%d fused steps across a slab halo need halo >= %d (got %lld)", K, K,
                         (long long)l.zghost);
    hipLaunchKernelGGL(kern, dim3(unsigned(nb)), dim3(64, NW, 1), 0, s, static_cast<const T*>(in),
                       static_cast<T*>(out), g, begin, end, zc, int(gx), int(gy), int(lo), int(hi),
                       avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

}  // namespace

int launch_boxk(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end, int steps,
                hipStream_t s) {
    if (!box27_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "BOXK supports the 3D r=1 naive 27-point box only");
    // cfg = RY*100 + NW
    const int cfg = env_int("STENCIL_BOXK_CFG", 0);
    if (l.prob.dtype == STENCIL_F32) {
        if (steps == 2) {
            switch (cfg) {
            case 408: return launch_bk<float, 4, 4, 8, 2, 2>(l, in, out, begin, end, s);
            case 208: return launch_bk<float, 4, 2, 8, 2, 2>(l, in, out, begin, end, s);
            case 116: return launch_bk<float, 4, 1, 16, 2, 2>(l, in, out, begin, end, s);
            case 1116: return launch_bk<float, 2, 1, 16, 2, 2, false>(l, in, out, begin, end, s);
            case 1416: return launch_bk<float, 4, 1, 16, 2, 2, false>(l, in, out, begin, end, s);
            case 1216: return launch_bk<float, 2, 1, 16, 2, 2>(l, in, out, begin, end, s);
            default:
                // measured (tools/box_ab.sh): 16-B lanes with LDS x-neighbours
                // on wide rows (2048^2 x 256: 735 vs 685 Gcell/s), 8-B lanes
                // with DPP on narrow ones (512^3: 582 vs 504)
                if (l.prob.nx >= 1024) return launch_bk<float, 4, 1, 16, 2, 2, false>(l, in, out, begin, end, s);
                return launch_bk<float, 2, 1, 16, 2, 2>(l, in, out, begin, end, s);
            }
        }
        if (steps == 3) {
            switch (cfg) {
            case 208: return launch_bk<float, 4, 2, 8, 3, 2>(l, in, out, begin, end, s);
            default: return launch_bk<float, 4, 1, 16, 3, 2>(l, in, out, begin, end, s);
            }
        }
    } else {
        if (steps == 2) {
            switch (cfg) {
            case 216: return launch_bk<double, 2, 2, 16, 2, 2>(l, in, out, begin, end, s);
            case 308: return launch_bk<double, 2, 3, 8, 2, 2>(l, in, out, begin, end, s);
            case 408: return launch_bk<double, 2, 4, 8, 2, 2>(l, in, out, begin, end, s);
            case 212: return launch_bk<double, 2, 2, 12, 2, 2>(l, in, out, begin, end, s);
            case 208: return launch_bk<double, 2, 2, 8, 2, 2>(l, in, out, begin, end, s);
            case 1116: return launch_bk<double, 2, 1, 16, 2, 2, false>(l, in, out, begin, end, s);
            default: return launch_bk<double, 2, 1, 16, 2, 2>(l, in, out, begin, end, s);
            }
        }
        if (steps == 3) {
            switch (cfg) {
            case 208: return launch_bk<double, 2, 2, 8, 3, 2>(l, in, out, begin, end, s);
            case 308: return launch_bk<double, 2, 3, 8, 3, 2>(l, in, out, begin, end, s);
            case 408: return launch_bk<double, 2, 4, 8, 3, 2>(l, in, out, begin, end, s);
            default: return launch_bk<double, 2, 1, 16, 3, 2>(l, in, out, begin, end, s);
            }
        }
    }
    return set_error(STENCIL_EINVAL, "boxk steps must be 2 or 3 (got %d)", steps);
}

}  // namespace stencil
