// kernels_direct.hip -- the general sweep kernel: every dims / shape / radius /
// sum order / dtype the engine supports.  One output cell per lane, 64-lane
// rows along x (one wave = one coalesced 256/512-byte row segment), neighbour
// re-reads served by L1/L2.  It is the correctness baseline every specialised
// kernel is checked against and the fallback for shapes without one.
//
// Arithmetic follows the reference exactly (see oracle/oracle_impl.inc for the
// CPU restatement and its citations):
//   NAIVE: stencil.cpp:104-125  -- 0 + left[c-r..c-1] + right[c+1..c+r]
//          + up[r-r..r-1] + down[r+1..r+r] (+ z-, z+ in 3D), then * avg
//   DMA  : stencil_dma.cpp:431-444 (r = 1) -- 0.25 * (up + left + right + down)
//          stencil_dma.cpp:636-650 (r > 1) -- 0 + row window + column window
//          - (centre + centre), then * avg
//   BOX  : separable partial sums (no reference code; DESIGN.md §3,
//          oracle/oracle_impl.inc): row sums R, plane sums P; 3D
//          S = (P(-r) + .. + P(r)) - centre, 2D S = W + E (the centre row's
//          other rows W, centre row E), then * avg
// The library is compiled with -ffp-contract=off so no FMA changes rounding.
#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int DIMS, int SHAPE, int ORDER, int R>
__device__ __forceinline__ T cell(const T* __restrict__ c, int64_t row, int64_t plane, int rr,
                                  T avg) {
    const int r = R > 0 ? R : rr;
    T sum = T(0);
    if constexpr (SHAPE == STENCIL_BOX) {
        auto rowsum = [&](const T* q) {  // q -> the row's centre cell
            T a = q[-r];
            for (int dx = -r + 1; dx <= r; ++dx) a += q[dx];
            return a;
        };
        if constexpr (DIMS == 3) {  // (P(-r) + ... + P(r)) - centre
            for (int dz = -r; dz <= r; ++dz) {
                const T* pl = c + dz * plane;
                T term = rowsum(pl - r * row);
                for (int dy = -r + 1; dy <= r; ++dy) term += rowsum(pl + dy * row);
                sum = dz == -r ? term : sum + term;
            }
            return (sum - c[0]) * avg;
        } else {  // W + E
            T w = rowsum(c - r * row);
            for (int dy = -r + 1; dy <= r; ++dy)
                if (dy != 0) w += rowsum(c + dy * row);
            T e = c[-r];
            for (int dx = -r + 1; dx <= r; ++dx)
                if (dx != 0) e += c[dx];
            return (w + e) * avg;
        }
    } else if constexpr (ORDER == STENCIL_ORDER_DMA) {
        if (r == 1) return T(0.25) * (((c[-row] + c[-1]) + c[1]) + c[row]);
#pragma unroll
        for (int k = -r; k <= r; ++k) sum += c[k];
#pragma unroll
        for (int k = -r; k <= r; ++k) sum += c[k * row];
        sum -= c[0] + c[0];
        return sum * avg;
    } else {
#pragma unroll
        for (int k = r; k >= 1; --k) sum += c[-k];
#pragma unroll
        for (int k = 1; k <= r; ++k) sum += c[k];
#pragma unroll
        for (int k = r; k >= 1; --k) sum += c[-k * row];
#pragma unroll
        for (int k = 1; k <= r; ++k) sum += c[k * row];
        if constexpr (DIMS == 3) {
#pragma unroll
            for (int k = r; k >= 1; --k) sum += c[-k * plane];
#pragma unroll
            for (int k = 1; k <= r; ++k) sum += c[k * plane];
        }
        return sum * avg;
    }
}

constexpr int kBX = 64, kBY = 4;

template <typename T, int DIMS, int SHAPE, int ORDER, int R>
__global__ void __launch_bounds__(kBX * kBY)
    sweep_direct(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t begin, int64_t end,
                 int r, T avg) {
    const int64_t x = int64_t(blockIdx.x) * kBX + threadIdx.x;
    int64_t y, z;
    if constexpr (DIMS == 3) {
        y = int64_t(blockIdx.y) * kBY + threadIdx.y;
        z = begin + blockIdx.z;
        if (y >= g.ny) return;
    } else {
        y = begin + int64_t(blockIdx.y) * kBY + threadIdx.y;
        z = 0;
        if (y >= end) return;
    }
    if (x >= g.nx) return;
    const int64_t idx = g.origin + z * g.plane + y * g.row + x;
    out[idx] = cell<T, DIMS, SHAPE, ORDER, R>(in + idx, g.row, g.plane, r, avg);
}

template <typename T, int DIMS, int SHAPE, int ORDER, int R>
int launch_t(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
             hipStream_t s) {
    const Geom g = geom_of(l);
    const T avg = avg_weight<T>(l.prob);
    const int64_t n = end - begin;
    if (n <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    const unsigned gx = unsigned((g.nx + kBX - 1) / kBX);
    const dim3 block(kBX, kBY, 1);
    if constexpr (DIMS == 3) {
        const unsigned gy = unsigned((g.ny + kBY - 1) / kBY);
        for (int64_t z0 = begin; z0 < end; z0 += 65535) {
            const unsigned gz = unsigned(std::min<int64_t>(65535, end - z0));
            hipLaunchKernelGGL((sweep_direct<T, DIMS, SHAPE, ORDER, R>), dim3(gx, gy, gz), block, 0,
                               s, static_cast<const T*>(in), static_cast<T*>(out), g, z0, end,
                               l.prob.radius, avg);
            STENCIL_LAUNCH_CHECK();
        }
    } else {
        for (int64_t y0 = begin; y0 < end; y0 += int64_t(65535) * kBY) {
            const int64_t rows = std::min<int64_t>(int64_t(65535) * kBY, end - y0);
            const unsigned gy = unsigned((rows + kBY - 1) / kBY);
            hipLaunchKernelGGL((sweep_direct<T, DIMS, SHAPE, ORDER, R>), dim3(gx, gy, 1), block, 0,
                               s, static_cast<const T*>(in), static_cast<T*>(out), g, y0,
                               y0 + rows, l.prob.radius, avg);
            STENCIL_LAUNCH_CHECK();
        }
    }
    return STENCIL_OK;
}

template <typename T, int DIMS, int SHAPE, int ORDER>
int launch_r(const stencil_layout& l, const void* in, void* out, int64_t b, int64_t e,
             hipStream_t s) {
    switch (l.prob.radius) {
    case 1: return launch_t<T, DIMS, SHAPE, ORDER, 1>(l, in, out, b, e, s);
    case 2: return launch_t<T, DIMS, SHAPE, ORDER, 2>(l, in, out, b, e, s);
    case 3: return launch_t<T, DIMS, SHAPE, ORDER, 3>(l, in, out, b, e, s);
    case 4: return launch_t<T, DIMS, SHAPE, ORDER, 4>(l, in, out, b, e, s);
    default: return launch_t<T, DIMS, SHAPE, ORDER, 0>(l, in, out, b, e, s);
    }
}

template <typename T, int DIMS>
int launch_d(const stencil_layout& l, const void* in, void* out, int64_t b, int64_t e,
             hipStream_t s) {
    const stencil_problem& p = l.prob;
    if (p.shape == STENCIL_BOX) return launch_r<T, DIMS, STENCIL_BOX, STENCIL_ORDER_NAIVE>(l, in, out, b, e, s);
    if (p.order == STENCIL_ORDER_DMA) {
        if constexpr (DIMS == 2)
            return launch_r<T, DIMS, STENCIL_STAR, STENCIL_ORDER_DMA>(l, in, out, b, e, s);
        return set_error(STENCIL_EINVAL, "DMA sum order is defined for 2D star stencils only");
    }
    return launch_r<T, DIMS, STENCIL_STAR, STENCIL_ORDER_NAIVE>(l, in, out, b, e, s);
}

}  // namespace

int launch_direct(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                  hipStream_t s) {
    const stencil_problem& p = l.prob;
    if (p.dtype == STENCIL_F32)
        return p.dims == 3 ? launch_d<float, 3>(l, in, out, begin, end, s)
                           : launch_d<float, 2>(l, in, out, begin, end, s);
    return p.dims == 3 ? launch_d<double, 3>(l, in, out, begin, end, s)
                       : launch_d<double, 2>(l, in, out, begin, end, s);
}

}  // namespace stencil
