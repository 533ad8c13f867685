// kernels_zmarch.hip -- the 3D 7-point (star, r = 1, naive order) hot kernel.
//
// 2.5D z-marching: a workgroup owns a 64 x TY tile of the xy plane and a chunk
// of ZC planes.  It walks z once, so every input cell comes from HBM once
// (plus the tile halo, mostly L2 hits) and every output cell is written once:
// 2 * sizeof(T) bytes per cell-update, the algorithmic minimum.
//
//   * centre values of planes z-1, z, z+1, z+2 live in a 4-slot register ring
//     (plane z+3 is loaded right after plane z is computed, so every load has
//     two planes of compute to land);
//   * plane z (tile + 1-cell halo) is staged in LDS, double-buffered, one
//     barrier per plane; the x/y neighbours come from LDS, z neighbours from
//     registers;
//   * 64 lanes span x, so each wave's loads/stores are contiguous 512 B (fp64)
//     segments; rows are 128-byte aligned by the layout (stencil_layout_init).
//
// Sum order = the naive order of the reference generalised to 3D
// (x-, x+, y-, y+, z-, z+, from 0, then * avg), identical to
// kernels_direct.hip and oracle/oracle_impl.inc, so results are bitwise equal.
#include <cstdlib>

#include "common.hpp"

namespace stencil {
namespace {

constexpr int kTX = 64;  // tile width (x) = one wave
constexpr int kBY = 4;   // waves per workgroup (y)

template <typename T, int RY>
struct ZMarch7 {
    static constexpr int TY = kBY * RY;
    static constexpr int LX = kTX + 2;
    static constexpr int LY = TY + 2;

    const T* __restrict__ src;  // interior origin of input
    T* __restrict__ dst;        // interior origin of output
    int64_t plane;
    int64_t off[RY];  // in-plane offsets of this lane's centre cells
    bool ldok[RY];    // centre load in range (interior or ghost)
    bool cok[RY];     // cell is interior: compute + store
    int64_t hoff;     // in-plane offset of this lane's halo cell
    bool hok, hslot;  // halo load valid / lane owns a halo slot
    int hy, hx;       // halo LDS slot
    int64_t zlast;    // last plane that may be loaded (chunk end, a ghost or interior plane)
    T avg;

    T (*lds)[LY][LX];  // [2][LY][LX]
    T v[4][RY];
    T h[2];

    __device__ __forceinline__ void load_plane(T (&d)[RY], int64_t z) {
        if (z <= zlast) {
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = ldok[k] ? src[z * plane + off[k]] : T(0);
        }
    }
    __device__ __forceinline__ void load_halo(T& d, int64_t z) {
        if (z <= zlast) d = hok ? src[z * plane + hoff] : T(0);
    }

    template <int S>
    __device__ __forceinline__ void step(int64_t z) {
        constexpr int M = (S + 3) & 3, C = S, P = (S + 1) & 3;
        constexpr int B = S & 1;
        const int tx = threadIdx.x, ty = threadIdx.y;
#pragma unroll
        for (int k = 0; k < RY; ++k) lds[B][ty + kBY * k + 1][tx + 1] = v[C][k];
        if (hslot) lds[B][hy][hx] = h[B];
        load_halo(h[B], z + 2);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = ty + kBY * k + 1;
            T s = T(0);
            s += lds[B][yy][tx];
            s += lds[B][yy][tx + 2];
            s += lds[B][yy - 1][tx + 1];
            s += lds[B][yy + 1][tx + 1];
            s += v[M][k];
            s += v[P][k];
            if (cok[k]) dst[z * plane + off[k]] = s * avg;
        }
        load_plane(v[M], z + 3);
    }
};

template <typename T, int RY>
__global__ void __launch_bounds__(kTX * kBY)
    zmarch7(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
            int zchunk, T avg) {
    using K = ZMarch7<T, RY>;
    __shared__ T lds[2][K::LY][K::LX];
    const int tx = threadIdx.x, ty = threadIdx.y;
    const int64_t x0 = int64_t(blockIdx.x) * kTX, y0 = int64_t(blockIdx.y) * K::TY;
    const int64_t za = zbeg + int64_t(blockIdx.z) * zchunk;
    const int64_t zb = za + zchunk < zend ? za + zchunk : zend;
    const int64_t x = x0 + tx;

    K k;
    k.src = in + g.origin;
    k.dst = out + g.origin;
    k.plane = g.plane;
    k.avg = avg;
    k.lds = lds;
    k.zlast = zb;
#pragma unroll
    for (int i = 0; i < RY; ++i) {
        const int64_t y = y0 + ty + kBY * i;
        k.off[i] = y * g.row + x;
        k.ldok[i] = x <= g.nx && y <= g.ny;
        k.cok[i] = x < g.nx && y < g.ny;
    }
    // Halo roles: wave 0 row y0-1, wave 1 row y0+TY, wave 2 column x0-1,
    // wave 3 column x0+64 (lanes < TY).  Ghost cells (index -1 or n) are in
    // range; anything past them is only ever a neighbour of a non-computed cell.
    int64_t hy_g, hx_g;
    if (ty == 0) {
        hy_g = y0 - 1; hx_g = x; k.hy = 0; k.hx = tx + 1; k.hslot = true;
        k.hok = x <= g.nx;
    } else if (ty == 1) {
        hy_g = y0 + K::TY; hx_g = x; k.hy = K::TY + 1; k.hx = tx + 1; k.hslot = true;
        k.hok = x <= g.nx && hy_g <= g.ny;
    } else if (ty == 2) {
        hy_g = y0 + tx; hx_g = x0 - 1; k.hy = tx + 1; k.hx = 0; k.hslot = tx < K::TY;
        k.hok = k.hslot && hy_g <= g.ny;
    } else {
        hy_g = y0 + tx; hx_g = x0 + kTX; k.hy = tx + 1; k.hx = kTX + 1; k.hslot = tx < K::TY;
        k.hok = k.hslot && hy_g <= g.ny && hx_g <= g.nx;
    }
    k.hoff = hy_g * g.row + hx_g;

    k.load_plane(k.v[3], za - 1);
    k.load_plane(k.v[0], za);
    k.load_plane(k.v[1], za + 1);
    k.load_plane(k.v[2], za + 2);
    k.load_halo(k.h[0], za);
    k.load_halo(k.h[1], za + 1);

    for (int64_t z = za; z < zb; z += 4) {
        k.template step<0>(z);
        if (z + 1 < zb) k.template step<1>(z + 1);
        if (z + 2 < zb) k.template step<2>(z + 2);
        if (z + 3 < zb) k.template step<3>(z + 3);
    }
}

constexpr int kRY = 4;

int env_int(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return s && *s ? std::atoi(s) : dflt;
}

template <typename T>
int launch_zm(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
              hipStream_t s) {
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    constexpr int TY = ZMarch7<T, kRY>::TY;
    const int64_t gx = (g.nx + kTX - 1) / kTX, gy = (g.ny + TY - 1) / TY;
    // Aim for >= 2048 workgroups (8 per CU) while keeping chunks long enough
    // that the two re-read halo planes per chunk stay a few percent.
    int zc = env_int("STENCIL_ZCHUNK", 0);
    if (zc <= 0) {
        const int64_t tiles = gx * gy;
        int64_t want = (nz * tiles + 2047) / 2048;
        want = (want + 3) / 4 * 4;
        zc = int(std::max<int64_t>(8, std::min<int64_t>(want, 256)));
    }
    const int64_t gz = (nz + zc - 1) / zc;
    if (gz > 65535 || gy > 65535) return set_error(STENCIL_EINVAL, "grid too large for zmarch");
    hipLaunchKernelGGL((zmarch7<T, kRY>), dim3(unsigned(gx), unsigned(gy), unsigned(gz)),
                       dim3(kTX, kBY, 1), 0, s, static_cast<const T*>(in), static_cast<T*>(out),
                       g, begin, end, zc, avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

}  // namespace

bool zmarch_supports(const stencil_problem& p) {
    return p.dims == 3 && p.shape == STENCIL_STAR && p.radius == 1 &&
           p.order == STENCIL_ORDER_NAIVE;
}

int launch_zmarch(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                  hipStream_t s) {
    if (!zmarch_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "ZMARCH kernel supports 3D star r=1 only");
    return l.prob.dtype == STENCIL_F32 ? launch_zm<float>(l, in, out, begin, end, s)
                                       : launch_zm<double>(l, in, out, begin, end, s);
}

}  // namespace stencil
