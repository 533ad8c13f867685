// kernels_tb2d.hip -- 2D star stencils, K sweeps per launch with the tile
// resident in LDS (temporal blocking): the MI355X counterpart of the
// reference's LDM-resident CPE blocks (src/stencil/slave/stencil_dma.cpp:
// 410-418 load once, 424-564 iterate in LDM).
//
// A workgroup loads a REGION (its output tile plus a ring of K*r cells) into
// two LDS buffers, runs K Jacobi sweeps between them -- step s updates the
// region shrunk by s*r on every side, cells outside the interior (Dirichlet
// ghosts) are never written and keep the values loaded into both buffers --
// and writes back the tile.  One launch replaces K launches and the halo is
// recomputed instead of exchanged, so no grid-wide barrier is needed.  At the
// reference's sizes (n <= 1024) a launch (~1.5 us) costs more than a sweep,
// so this is launch-latency bound, not HBM bound.
//
// Arithmetic: cell<...> is the same order-exact update as kernels_direct.hip
// (naive order = check_result, stencil.cpp:104-125; DMA order =
// stencil_dma.cpp:431-444 / 636-650), so K fused sweeps are bitwise equal to
// K single sweeps.
#include <cstdlib>

#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int ORDER, int R>
__device__ __forceinline__ T cell2d(const T* c, int row, T avg) {
    T sum = T(0);
    if constexpr (ORDER == STENCIL_ORDER_DMA) {
        if constexpr (R == 1) {
            return T(0.25) * (((c[-row] + c[-1]) + c[1]) + c[row]);
        } else {
#pragma unroll
            for (int k = -R; k <= R; ++k) sum += c[k];
#pragma unroll
            for (int k = -R; k <= R; ++k) sum += c[k * row];
            sum -= c[0] + c[0];
            return sum * avg;
        }
    } else {
#pragma unroll
        for (int k = R; k >= 1; --k) sum += c[-k];
#pragma unroll
        for (int k = 1; k <= R; ++k) sum += c[k];
#pragma unroll
        for (int k = R; k >= 1; --k) sum += c[-k * row];
#pragma unroll
        for (int k = 1; k <= R; ++k) sum += c[k * row];
        return sum * avg;
    }
}

constexpr int kThreads = 512;

// Region RX x RY cells (RX a multiple of 64), LDS row stride RX + 1 (odd
// stride spreads a column over banks).
template <typename T, int ORDER, int R, int RX, int RY>
__global__ void __launch_bounds__(kThreads)
    tb2d(const T* __restrict__ in, T* __restrict__ out, Geom g, int steps, int tiles_x, T avg) {
    constexpr int LXS = RX + 1;
    __shared__ T buf[2][RY][LXS];
    const int K = steps;
    const int ring = K * R;
    const int TX = RX - 2 * ring, TY = RY - 2 * ring;
    const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
    const int64_t x0 = int64_t(bx) * TX - ring, y0 = int64_t(by) * TY - ring;  // region origin (interior coords)
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;

    // load the region into both buffers (ghost cells and out-of-grid cells
    // are never written by the sweeps, so both buffers must hold them)
    for (int i = threadIdx.x; i < RX * RY; i += kThreads) {
        const int ry = i / RX, rx = i % RX;
        const int64_t y = y0 + ry, x = x0 + rx;
        T v = T(0);
        if (x >= -R && x < g.nx + R && y >= -R && y < g.ny + R) v = src[y * g.row + x];
        buf[0][ry][rx] = v;
        buf[1][ry][rx] = v;
    }
    __syncthreads();

    int cur = 0;
    for (int s = 1; s <= K; ++s) {
        const int lo = s * R;  // step s updates region cells [lo, R?-lo)
        const int wx = RX - 2 * lo, wy = RY - 2 * lo;
        const T* a = &buf[cur][0][0];
        T* b = &buf[cur ^ 1][0][0];
        for (int i = threadIdx.x; i < wx * wy; i += kThreads) {
            const int ry = lo + i / wx, rx = lo + i % wx;
            const int64_t y = y0 + ry, x = x0 + rx;
            if (x >= 0 && x < g.nx && y >= 0 && y < g.ny)
                b[ry * LXS + rx] = cell2d<T, ORDER, R>(a + ry * LXS + rx, LXS, avg);
        }
        cur ^= 1;
        __syncthreads();
    }

    for (int i = threadIdx.x; i < TX * TY; i += kThreads) {
        const int ty = i / TX, tx = i % TX;
        const int64_t y = y0 + ring + ty, x = x0 + ring + tx;
        if (x < g.nx && y < g.ny) dst[y * g.row + x] = buf[cur][ring + ty][ring + tx];
    }
}

template <typename T, int ORDER, int R>
int launch_tb(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    // 64 KB of LDS per buffer: fp64 128 x 64 cells, fp32 256 x 64 cells.
    constexpr int RX = sizeof(T) == 8 ? 128 : 256, RY = 63;
    const Geom g = geom_of(l);
    if (g.nx <= 0 || g.ny <= 0 || steps <= 0) return STENCIL_OK;
    const int ring = steps * R;
    const int TX = RX - 2 * ring, TY = RY - 2 * ring;
    if (TX < 8 || TY < 8) return set_error(STENCIL_EINVAL, "tb2d: %d steps of radius %d leave no tile", steps, R);
    const int64_t tx = (g.nx + TX - 1) / TX, ty = (g.ny + TY - 1) / TY;
    if (tx * ty > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "tb2d: grid too large");
    hipLaunchKernelGGL((tb2d<T, ORDER, R, RX, RY>), dim3(unsigned(tx * ty)), dim3(kThreads), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, steps, int(tx), avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

template <typename T, int ORDER>
int launch_r(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    switch (l.prob.radius) {
    case 1: return launch_tb<T, ORDER, 1>(l, in, out, steps, s);
    case 2: return launch_tb<T, ORDER, 2>(l, in, out, steps, s);
    case 3: return launch_tb<T, ORDER, 3>(l, in, out, steps, s);
    case 4: return launch_tb<T, ORDER, 4>(l, in, out, steps, s);
    default: return set_error(STENCIL_EUNSUPPORTED, "tb2d: radius > 4");
    }
}

}  // namespace

bool tb2d_supports(const stencil_problem& p) {
    return p.dims == 2 && p.shape == STENCIL_STAR && p.radius >= 1 && p.radius <= 4;
}

int tb2d_max_steps(const stencil_problem& p) {
    const char* e = std::getenv("STENCIL_TB2D_K");
    int k = e && *e ? std::atoi(e) : 8;
    // keep the output tile at least ~half the 63-row region
    const int cap = std::max(1, 16 / p.radius);
    return std::max(1, std::min(k, cap));
}

int launch_tb2d(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    if (!tb2d_supports(l.prob)) return set_error(STENCIL_EUNSUPPORTED, "tb2d: 2D star r<=4 only");
    const bool dma = l.prob.order == STENCIL_ORDER_DMA;
    if (l.prob.dtype == STENCIL_F32)
        return dma ? launch_r<float, STENCIL_ORDER_DMA>(l, in, out, steps, s)
                   : launch_r<float, STENCIL_ORDER_NAIVE>(l, in, out, steps, s);
    return dma ? launch_r<double, STENCIL_ORDER_DMA>(l, in, out, steps, s)
               : launch_r<double, STENCIL_ORDER_NAIVE>(l, in, out, steps, s);
}

}  // namespace stencil
