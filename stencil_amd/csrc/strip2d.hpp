// strip2d.hpp -- the register-strip 2D region update shared by the K-step
// launch kernel tb2ds (kernels_tb2d.hip) and the persistent kernel tb2dp
// (kernels_tb2dp.hip).
#pragma once

#include "common.hpp"

namespace stencil {
namespace strip2d {

// Strip variant (R <= V): each wave keeps RY consecutive rows of the region in
// registers (V cells per lane), x-neighbours come from the lane's own cells
// and DPP lane shifts, y-neighbours from its own rows; only the R top and R
// bottom rows of each wave's strip go through LDS (double-buffered by sweep
// parity: one barrier per sweep).  The LDS sweep of tb2d reads 4 LDS values
// per cell (measured 1.5 us per sweep on a 64 x 64 region); here a wave
// moves 2R rows through LDS per sweep.  Same arithmetic order as cell2d.
template <typename T, int V>
struct Vec2 {
    typedef T type __attribute__((ext_vector_type(V)));
};

template <int CTRL>
__device__ __forceinline__ float dpp2(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ double dpp2(double v) {
    const int2 b = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_mov_dpp(b.x, CTRL, 0xf, 0xf, true),
                                                 __builtin_amdgcn_mov_dpp(b.y, CTRL, 0xf, 0xf, true)));
}

// The reference's sums start from +0 (0 + a + b ...).  Dropping that first add
// changes only the sign of an all-zero sum: the chain without it ends at -0
// exactly when every term is -0, where the reference's ends at +0; every
// other value (zero or not) is the same.  fma(sum, avg, +0) rounds the exact
// product once, as sum * avg does, and turns -0 * avg into +0: so
// fma0(chain without the leading 0) == (chain with it) * avg, bit for bit,
// one VALU operation fewer per cell (the 3D strip's sfma0 is the same).
__device__ __forceinline__ float fma0(float s, float a) { return __builtin_fmaf(s, a, 0.0f); }
__device__ __forceinline__ double fma0(double s, double a) { return __builtin_fma(s, a, 0.0); }

template <typename T, int R, int V, int NW>
using Lds = T[2][NW][2][R][64 * V];  // [parity][wave][top, bottom][row][x]

// One region of tile (bx, by): load tile + H-cell ring from `in`, `steps`
// sweeps (steps * R <= H), store the tile to `out`.  Tiles are RW - 2H by
// RH - 2H cells.  BF: every cell's update is computed and the ghost cells'
// kept value chosen by a select (an empty asm pins the update, so the
// compiler cannot sink it under an exec-mask branch per row).
template <typename T, int ORDER, int R, int V, int RY, int NW, bool BF = false>
__device__ __forceinline__ void region(const T* __restrict__ in, T* __restrict__ out, const Geom& g, int steps,
                                       int H, int bx, int by, T avg, Lds<T, R, V, NW>& L) {
    static_assert(R <= V, "one DPP shift reaches R cells");
    static_assert(RY >= R, "a strip holds at least R rows");
    using VT = typename Vec2<T, V>::type;
    constexpr int RW = 64 * V, RH = NW * RY;
    const int TX = RW - 2 * H, TY = RH - 2 * H;
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - H + int64_t(lane) * V;
    const int64_t yw = int64_t(by) * TY - H + int64_t(w) * RY;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;

    bool xin[V], xld[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xld[j] = x + j >= -R && x + j < g.nx + R;
    }
    bool yin[RY];
    VT c0[RY], c1[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int64_t y = yw + k;
        yin[k] = y >= 0 && y < g.ny;
        const bool yld = y >= -R && y < g.ny + R;
#pragma unroll
        for (int j = 0; j < V; ++j) c0[k][j] = (yld && xld[j]) ? src[y * g.row + x + j] : T(0);
        c1[k] = c0[k];
    }
    const int wa = w > 0 ? w - 1 : 0, wb = w < NW - 1 ? w + 1 : NW - 1;
    const int xl = lane * V;

    // one sweep a -> b, boundary rows through LDS buffer P
    auto sweep = [&](const VT (&a)[RY], VT (&b)[RY], int P) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            *reinterpret_cast<VT*>(&L[P][w][0][i][xl]) = a[i];
            *reinterpret_cast<VT*>(&L[P][w][1][i][xl]) = a[RY - R + i];
        }
        __syncthreads();
        VT above[R], below[R];  // rows -R..-1 and RY..RY+R-1 of this strip
#pragma unroll
        for (int i = 0; i < R; ++i) {
            above[i] = *reinterpret_cast<const VT*>(&L[P][wa][1][i][xl]);
            below[i] = *reinterpret_cast<const VT*>(&L[P][wb][0][i][xl]);
        }
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            auto rowv = [&](int m) -> VT {  // strip row m in [-R, RY+R)
                if (m < 0) return above[m + R];
                if (m >= RY) return below[m - RY];
                return a[m];
            };
            const VT cv = a[k];
            // x-neighbour cells of this lane's V cells: [-R, V+R)
            T xs[V + 2 * R];
#pragma unroll
            for (int j = 0; j < V; ++j) xs[R + j] = cv[j];
#pragma unroll
            for (int i = 0; i < R; ++i) {
                xs[i] = dpp2<0x138>(cv[V - R + i]);   // wave_shr:1: lane-1's cells
                xs[R + V + i] = dpp2<0x130>(cv[i]);   // wave_shl:1: lane+1's cells
            }
            VT o;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                T r;
                if constexpr (ORDER == STENCIL_ORDER_DMA && R == 1) {
                    r = T(0.25) * (((rowv(k - 1)[j] + xs[R + j - 1]) + xs[R + j + 1]) + rowv(k + 1)[j]);
                } else if constexpr (ORDER == STENCIL_ORDER_DMA) {
                    // the reference's sum starts from 0; fma(sum, avg, +0) is the
                    // same bits with one add fewer (fma0 below)
                    T sum = xs[j];
#pragma unroll
                    for (int d = -R + 1; d <= R; ++d) sum += xs[R + j + d];
#pragma unroll
                    for (int d = -R; d <= R; ++d) sum += rowv(k + d)[j];
                    sum -= cv[j] + cv[j];
                    r = fma0(sum, avg);
                } else {
                    T sum = xs[j];  // d = R: the reference's 0 + x[-R], see fma0
#pragma unroll
                    for (int d = R - 1; d >= 1; --d) sum += xs[R + j - d];
#pragma unroll
                    for (int d = 1; d <= R; ++d) sum += xs[R + j + d];
#pragma unroll
                    for (int d = R; d >= 1; --d) sum += rowv(k - d)[j];
#pragma unroll
                    for (int d = 1; d <= R; ++d) sum += rowv(k + d)[j];
                    r = fma0(sum, avg);
                }
                if constexpr (BF) asm volatile("" : "+v"(r));
                o[j] = (xin[j] && yin[k]) ? r : cv[j];  // ghost cells keep their value
            }
            b[k] = o;
        }
    };
    int s = 0;
    for (; s + 2 <= steps; s += 2) {
        sweep(c0, c1, 0);
        sweep(c1, c0, 1);
    }
    if (s < steps) {
        sweep(c0, c1, 0);
#pragma unroll
        for (int k = 0; k < RY; ++k) c0[k] = c1[k];
    }
    // the tile: region columns [H, H + TX), rows [H, H + TY)
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w * RY + k;
        const int64_t y = yw + k;
        if (rr < H || rr >= H + TY || y >= g.ny) continue;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int cx = xl + j;
            if (cx >= H && cx < H + TX && x + j < g.nx) dst[y * g.row + x + j] = c0[k][j];
        }
    }
}

// NaN over the tile's interior cells (a persistent launch that gave up).
template <typename T, int R, int V, int RY, int NW>
__device__ __forceinline__ void poison(T* __restrict__ out, const Geom& g, int H, int bx, int by) {
    constexpr int RW = 64 * V, RH = NW * RY;
    const int TX = RW - 2 * H, TY = RH - 2 * H;
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = int64_t(bx) * TX - H + int64_t(lane) * V;
    const int64_t yw = int64_t(by) * TY - H + int64_t(w) * RY;
    for (int k = 0; k < RY; ++k) {
        const int rr = w * RY + k;
        const int64_t y = yw + k;
        if (rr < H || rr >= H + TY || y < 0 || y >= g.ny) continue;
        for (int j = 0; j < V; ++j) {
            const int cx = lane * V + j;
            if (cx >= H && cx < H + TX && x + j >= 0 && x + j < g.nx)
                out[g.origin + y * g.row + x + j] = __builtin_nan("");
        }
    }
}

}  // namespace strip2d
}  // namespace stencil
