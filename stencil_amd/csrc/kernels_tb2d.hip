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
#include "strip2d.hpp"

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

constexpr int kRX = 64;  // region width: one column per lane
// region height kRY = NW * rows per wave; NW waves (template parameters)

// LDS image of the region with an R-cell pad on every side, so every
// neighbour read of every lane is in bounds: the sweep is computed for all
// rows unconditionally (all LDS reads of a step can be in flight together)
// and only the stores are predicated.
template <typename T, int ORDER, int R, int kWaves, int kRY>
__global__ void __launch_bounds__(64 * kWaves)
    tb2d(const T* __restrict__ in, T* __restrict__ out, Geom g, int steps, int tiles_x, T avg) {
    constexpr int LXS = kRX + 2 * R + 1;  // odd stride: a column spreads over banks
    constexpr int LYS = kRY + 2 * R;
    constexpr int RPW = kRY / kWaves;  // rows per wave
    __shared__ T buf[2][LYS * LXS];
    const int ring = steps * R;
    const int TX = kRX - 2 * ring, TY = kRY - 2 * ring;
    const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
    const int64_t x0 = int64_t(bx) * TX - ring, y0 = int64_t(by) * TY - ring;  // region origin
    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x = x0 + lane;
    const bool xin = x >= 0 && x < g.nx;
    const bool xld = x >= -R && x < g.nx + R;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;
    auto at = [&](int ry) { return (ry + R) * LXS + R + lane; };

    // Zero the pads (read only by discarded lanes), then load the region into
    // both buffers: ghost and out-of-grid cells are never written by a sweep.
    for (int i = threadIdx.y * 64 + lane; i < LYS * LXS; i += 64 * kWaves) {
        const int py = i / LXS, px = i % LXS;
        if (py < R || py >= R + kRY || px < R || px >= R + kRX) {
            buf[0][i] = T(0);
            buf[1][i] = T(0);
        }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int ry = w + kWaves * j;
        const int64_t y = y0 + ry;
        T v = T(0);
        if (xld && y >= -R && y < g.ny + R) v = src[y * g.row + x];
        buf[0][at(ry)] = v;
        buf[1][at(ry)] = v;
    }
    bool yin[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int64_t y = y0 + w + kWaves * j;
        yin[j] = y >= 0 && y < g.ny;
    }
    __syncthreads();

    int cur = 0;
    for (int s = 1; s <= steps; ++s) {
        const int lo = s * R;
        const bool cx = xin && lane >= lo && lane < kRX - lo;
        const T* a = buf[cur];
        T* b = buf[cur ^ 1];
        T v[RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) v[j] = cell2d<T, ORDER, R>(a + at(w + kWaves * j), LXS, avg);
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int ry = w + kWaves * j;
            if (cx && yin[j] && ry >= lo && ry < kRY - lo) b[at(ry)] = v[j];
        }
        cur ^= 1;
        __syncthreads();
    }

    const bool sx = lane >= ring && lane < ring + TX && x < g.nx;
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int ry = w + kWaves * j;
        const int64_t y = y0 + ry;
        if (sx && ry >= ring && ry < ring + TY && y < g.ny) dst[y * g.row + x] = buf[cur][at(ry)];
    }
}

template <typename T, int ORDER, int R, int kWaves, int kRY>
int launch_tb(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    static_assert(kRY % kWaves == 0, "rows per wave");
    static_assert(size_t(2) * (kRY + 2 * R) * (kRX + 2 * R + 1) * sizeof(T) <= 160 * 1024, "LDS budget");
    const Geom g = geom_of(l);
    if (g.nx <= 0 || g.ny <= 0 || steps <= 0) return STENCIL_OK;
    const int ring = steps * R;
    const int TX = kRX - 2 * ring, TY = kRY - 2 * ring;
    if (TX < 4 || TY < 4) return set_error(STENCIL_EINVAL, "tb2d: %d steps of radius %d leave no tile", steps, R);
    const int64_t tx = (g.nx + TX - 1) / TX, ty = (g.ny + TY - 1) / TY;
    if (tx * ty > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "tb2d: grid too large");
    hipLaunchKernelGGL((tb2d<T, ORDER, R, kWaves, kRY>), dim3(unsigned(tx * ty)), dim3(64, kWaves), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, steps, int(tx), avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

// The whole grid (ghost ring included) in ONE workgroup's LDS, two images:
// every sweep of the job in one launch, one workgroup barrier per sweep and
// no global traffic between the first load and the last store.  For the
// small grids the reference's own tests use (n = 32, 64): a K-step launch
// costs ~1.7 us of boundary per launch and its 8-wave strips ~1.5 us per
// sweep there.  Each thread owns up to k1MaxCells cells (offsets kept in
// registers).  Measured per sweep (tools/tb2d1_ab.sh): 32^2 0.5 vs 0.8-0.9
// us, 64^2 0.7 vs 0.8-1.0; at 96^2 (9 cells per thread) 1.1-1.2 vs 0.8-1.0,
// so only grids of <= 5 cells per thread take this path.
constexpr int k1Threads = 1024;
constexpr int k1MaxCells = 5;  // per thread: grids up to 5120 cells
template <typename T, int ORDER, int R>
__global__ void __launch_bounds__(k1Threads)
    tb2d1(const T* __restrict__ in, T* __restrict__ out, Geom g, int iterations, T avg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem1[];
    T* img0 = reinterpret_cast<T*>(smem1);
    const int nx = int(g.nx), ny = int(g.ny);
    const int S = nx + 2 * R;  // LDS row stride
    const int Hh = ny + 2 * R;
    T* img1 = img0 + S * Hh;
    const int tid = int(threadIdx.x);
    const T* __restrict__ src = in + g.origin;
    for (int i = tid; i < S * Hh; i += k1Threads) {
        const int y = i / S - R, x = i % S - R;
        const T v = src[int64_t(y) * g.row + x];
        img0[i] = v;
        img1[i] = v;
    }
    int off[k1MaxCells];  // LDS index of this thread's cells (interior only)
    int nc = 0;
#pragma unroll
    for (int c = 0; c < k1MaxCells; ++c) {
        const int i = tid + c * k1Threads;
        off[c] = i < nx * ny ? (i / nx + R) * S + i % nx + R : 0;
        nc += i < nx * ny ? 1 : 0;
    }
    __syncthreads();
    for (int it = 0; it < iterations; ++it) {
        const T* a = (it & 1) ? img1 : img0;
        T* b = (it & 1) ? img0 : img1;
#pragma unroll
        for (int c = 0; c < k1MaxCells; ++c)
            if (c < nc) b[off[c]] = cell2d<T, ORDER, R>(a + off[c], S, avg);
        __syncthreads();
    }
    const T* fin = (iterations & 1) ? img1 : img0;
    T* __restrict__ dst = out + g.origin;
#pragma unroll
    for (int c = 0; c < k1MaxCells; ++c) {
        if (c < nc) {
            const int i = tid + c * k1Threads;
            dst[int64_t(i / nx) * g.row + i % nx] = fin[off[c]];
        }
    }
}

template <typename T, int ORDER, int R>
int launch_tb1(const stencil_layout& l, const void* in, void* out, uint32_t iterations, hipStream_t s) {
    const Geom g = geom_of(l);
    const size_t lds = size_t(2) * size_t(g.nx + 2 * R) * size_t(g.ny + 2 * R) * sizeof(T);
    auto kern = tb2d1<T, ORDER, R>;
    // per device and cheap: set it on every launch (a process may drive several GPUs)
    STENCIL_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL(kern, dim3(1), dim3(k1Threads), lds, s, static_cast<const T*>(in), static_cast<T*>(out), g,
                       int(iterations), avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

template <typename T, int ORDER>
int launch_tb1_r(const stencil_layout& l, const void* in, void* out, uint32_t iterations, hipStream_t s) {
    switch (l.prob.radius) {
    case 1: return launch_tb1<T, ORDER, 1>(l, in, out, iterations, s);
    case 2: return launch_tb1<T, ORDER, 2>(l, in, out, iterations, s);
    case 3: return launch_tb1<T, ORDER, 3>(l, in, out, iterations, s);
    case 4: return launch_tb1<T, ORDER, 4>(l, in, out, iterations, s);
    default: return set_error(STENCIL_EUNSUPPORTED, "tb2d1: radius > 4");
    }
}

// Strip variant (R <= V): strip2d.hpp.
template <typename T, int ORDER, int R, int V, int RY, int NW, bool BF>
__global__ void __launch_bounds__(64 * NW)
    tb2ds(const T* __restrict__ in, T* __restrict__ out, Geom g, int steps, int tiles_x, T avg) {
    __shared__ __attribute__((aligned(16))) strip2d::Lds<T, R, V, NW> L;
    strip2d::region<T, ORDER, R, V, RY, NW, BF>(in, out, g, steps, steps * R, int(blockIdx.x) % tiles_x,
                                                int(blockIdx.x) / tiles_x, avg, L);
}

template <typename T, int ORDER, int R, int V, int RY, int NW, bool BF = false>
int launch_tbs(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    const Geom g = geom_of(l);
    if (g.nx <= 0 || g.ny <= 0 || steps <= 0) return STENCIL_OK;
    const int ring = steps * R;
    const int TX = 64 * V - 2 * ring, TY = NW * RY - 2 * ring;
    if (TX < 4 || TY < 4) return set_error(STENCIL_EINVAL, "tb2ds: %d steps of radius %d leave no tile", steps, R);
    const int64_t tx = (g.nx + TX - 1) / TX, ty = (g.ny + TY - 1) / TY;
    if (tx * ty > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "tb2ds: grid too large");
    hipLaunchKernelGGL((tb2ds<T, ORDER, R, V, RY, NW, BF>), dim3(unsigned(tx * ty)), dim3(64, NW), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, steps, int(tx), avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

int tenv_int(const char* name, int dflt) { return knob(name, dflt); }

// region shapes (STENCIL_TB2D_CFG = waves * 1000 + region height)
template <typename T, int ORDER, int R>
int launch_shape(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    const int cfg = tenv_int("STENCIL_TB2D_CFG", 0);
    if constexpr (R <= 2) {
        // strip variants: 9 V RY NW (V cells per lane, RY rows per wave, NW waves)
        switch (cfg) {
        case 92808: return launch_tbs<T, ORDER, R, 2, 8, 8>(l, in, out, steps, s);
        case 92816: return launch_tbs<T, ORDER, R, 2, 8, 16>(l, in, out, steps, s);
        case 92408: return launch_tbs<T, ORDER, R, 2, 4, 8>(l, in, out, steps, s);
        case 92416: return launch_tbs<T, ORDER, R, 2, 4, 16>(l, in, out, steps, s);
        case 92216: return launch_tbs<T, ORDER, R, 2, 2, 16>(l, in, out, steps, s);
        case 94808: return launch_tbs<T, ORDER, R, 4, 8, 8>(l, in, out, steps, s);
        case 92608: return launch_tbs<T, ORDER, R, 2, 6, 8>(l, in, out, steps, s);
        // the default shapes with branch-free ghost selects (strip2d::region BF; 9xxxx above branch per row)
        case 192416: return launch_tbs<T, ORDER, R, 2, 4, 16, true>(l, in, out, steps, s);
        case 192808: return launch_tbs<T, ORDER, R, 2, 8, 8, true>(l, in, out, steps, s);
        case 0:
            // default for r <= 2: 128 x 64 regions, 2 cells per lane (1024^2,
            // K = 8: fp64 559 vs 393 Gcell/s for the LDS kernel, fp32 709 vs
            // 520; tools/tb2d_ab.sh); fp64 as 16 waves x 4 rows (C1, K = 10: 694
            // vs 652 Gcell/s for 8 x 8 -- more waves hide the per-sweep
            // barrier), fp32 as 8 x 8.  Branch-free ghost selects (round 4,
            // tools/c1_ab.py, profiles/r04/r04d_c1_ab.txt): C1 fp64 762 vs 710,
            // DMA order 799 vs 724, fp32 972 vs 856 Gcell/s, bitwise equal.
            if constexpr (sizeof(T) == 8) return launch_tbs<T, ORDER, R, 2, 4, 16, true>(l, in, out, steps, s);
            return launch_tbs<T, ORDER, R, 2, 8, 8, true>(l, in, out, steps, s);
        default: break;
        }
    }
    // default 64 x 64 regions, 8 waves (1024^2, K = 8: fp64 400 vs 312
    // Gcell/s for 64 x 32 / 4 waves, fp32 520 vs 460; tools/tb2d_ab.sh)
    switch (cfg) {
    case 4032: return launch_tb<T, ORDER, R, 4, 32>(l, in, out, steps, s);
    case 8064: return launch_tb<T, ORDER, R, 8, 64>(l, in, out, steps, s);
    case 16128: return launch_tb<T, ORDER, R, 16, 128>(l, in, out, steps, s);
    case 12096: return launch_tb<T, ORDER, R, 12, 96>(l, in, out, steps, s);
    case 8128: return launch_tb<T, ORDER, R, 8, 128>(l, in, out, steps, s);
    default: return launch_tb<T, ORDER, R, 8, 64>(l, in, out, steps, s);
    }
}

template <typename T, int ORDER>
int launch_r(const stencil_layout& l, const void* in, void* out, int steps, hipStream_t s) {
    switch (l.prob.radius) {
    case 1: return launch_shape<T, ORDER, 1>(l, in, out, steps, s);
    case 2: return launch_shape<T, ORDER, 2>(l, in, out, steps, s);
    case 3: return launch_shape<T, ORDER, 3>(l, in, out, steps, s);
    case 4: return launch_shape<T, ORDER, 4>(l, in, out, steps, s);
    default: return set_error(STENCIL_EUNSUPPORTED, "tb2d: radius > 4");
    }
}

}  // namespace

bool tb2d_supports(const stencil_problem& p) {
    return p.dims == 2 && p.shape == STENCIL_STAR && p.radius >= 1 && p.radius <= 4;
}

int tb2d_max_steps(const stencil_problem& p) {
    const int kf = knob("STENCIL_TB2D_K", 0);
    const bool forced = kf != 0;
    const int k = forced ? kf : 8;
    // default: keep the output tile at least half of a 32-row region; an
    // explicit K may go up to a 16-cell-wide tile of the 64-wide region
    const int cap = std::max(1, (forced ? 24 : 8) / p.radius);
    return std::max(1, std::min(k, cap));
}

namespace {
// Workgroup slots for the round count: one per CU.  The occupancy API allows
// two strip workgroups per CU, but measured rounds behave as one per CU (C1
// fp64: 240 tiles 658 Gcell/s, 260 tiles 571), so the CU count it is.
int strip_slots() {
    int slots = 0;  // per device (resident_slots caches it); 0 when the query fails
    return resident_slots(reinterpret_cast<const void*>(&strip_slots), 0, true, &slots) == STENCIL_OK ? slots : 0;
}
}  // namespace

// Sweeps per launch in stencil_iterate: among K = 8/r .. 16/r whose tiles take
// no more rounds of one-per-CU workgroups than K = 8/r, the fewest launches
// for `iterations`, then the fewest tiles -- more sweeps per launch at no
// extra round (C1 1024^2 fp64: K = 10, 240 tiles on 256 CUs, 658 vs 610
// Gcell/s; K = 12 needs 260 tiles, a second round, 571; tools/tb2ds_ab.sh,
// tools/tb2d_kauto_ab.sh).  STENCIL_TB2D_K / _CFG and r > 2 keep
// tb2d_max_steps.
int tb2d_steps(const stencil_layout& l, uint32_t iterations) {
    const stencil_problem& p = l.prob;
    const int base = tb2d_max_steps(p);
    const int cfg = tenv_int("STENCIL_TB2D_CFG", 0);
    if (knob("STENCIL_TB2D_K", 0) != 0 || p.radius > 2 ||
        (cfg != 0 && cfg % 100000 != 92808 && cfg % 100000 != 92416))
        return base;  // 128 x 64 only
    const int slots = strip_slots();
    (void)hipGetLastError();
    if (slots <= 0) return base;
    auto tiles = [&](int k) -> int64_t {
        const int64_t h = int64_t(k) * p.radius, tx = 128 - 2 * h, ty = 64 - 2 * h;
        if (tx < 4 || ty < 4) return INT64_MAX / 2;
        return (p.nx + tx - 1) / tx * ((p.ny + ty - 1) / ty);
    };
    auto rounds = [&](int k) { return (tiles(k) + slots - 1) / slots; };
    auto launches = [&](int k) { return (int64_t(iterations) + k - 1) / k; };
    const int64_t r0 = rounds(base);
    int best = base;
    for (int k = base + 1; k <= 16 / p.radius; ++k) {
        if (rounds(k) > r0) continue;
        if (launches(k) < launches(best) || (launches(k) == launches(best) && tiles(k) < tiles(best))) best = k;
    }
    return best;
}

bool tb2d1_fits(const stencil_layout& l) {
    const stencil_problem& p = l.prob;
    if (!tb2d_supports(p) || p.nx <= 0 || p.ny <= 0) return false;
    if (knob("STENCIL_TB2D_SINGLE", 1) == 0) return false;
    const int64_t esz = p.dtype == STENCIL_F32 ? 4 : 8;
    const int64_t lds = 2 * (p.nx + 2 * p.radius) * (p.ny + 2 * p.radius) * esz;
    return p.nx * p.ny <= int64_t(k1Threads) * k1MaxCells && lds <= 160 * 1024;
}

// `iterations` sweeps of a grid that fits one workgroup (tb2d1_fits), from
// `in`; the result lands in `out`.
int launch_tb2d1(const stencil_layout& l, const void* in, void* out, uint32_t iterations, hipStream_t s) {
    if (!tb2d1_fits(l)) return set_error(STENCIL_EUNSUPPORTED, "tb2d1: grid does not fit one workgroup");
    const bool dma = l.prob.order == STENCIL_ORDER_DMA;
    if (l.prob.dtype == STENCIL_F32)
        return dma ? launch_tb1_r<float, STENCIL_ORDER_DMA>(l, in, out, iterations, s)
                   : launch_tb1_r<float, STENCIL_ORDER_NAIVE>(l, in, out, iterations, s);
    return dma ? launch_tb1_r<double, STENCIL_ORDER_DMA>(l, in, out, iterations, s)
               : launch_tb1_r<double, STENCIL_ORDER_NAIVE>(l, in, out, iterations, s);
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
