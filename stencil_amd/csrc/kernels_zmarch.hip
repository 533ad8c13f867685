// kernels_zmarch.hip -- the 3D 7-point (star, r = 1, naive order) hot kernel.
//
// 2.5D z-marching: a workgroup owns a TX x TY tile of the xy plane and a chunk
// of planes.  It walks z once, so every input cell comes from HBM once (plus
// the tile halo) and every output cell is written once: 2 * sizeof(T) bytes
// per cell-update, the algorithmic minimum.
//
//   * each lane owns V consecutive x (V*sizeof(T) = 16 B: one dwordx4 load /
//     store per row), 64 lanes span TX = 64*V, 4 waves x RY rows span TY;
//   * centre values of planes z-1, z, z+1, z+2 live in a 4-slot register
//     ring (plane z+3 is loaded right after plane z is computed, so every
//     load has two planes of compute to land);
//   * plane z (tile + 1-cell halo) is staged in LDS, double-buffered, one
//     barrier per plane; x/y neighbours come from LDS (16-B aligned rows),
//     z neighbours from registers;
//   * XCD-aware tile order: workgroup b runs on XCD b % 8 (observed
//     round-robin dispatch; speed only, never correctness), so tiles are
//     numbered so that each XCD gets a contiguous block of the grid --
//     neighbouring tiles then share halo lines in the same 4 MB L2 instead of
//     fetching them again from HBM (rocprof r01: the first version read
//     1.56x the algorithmic bytes, mostly x-halo lines).
//
// Sum order = the naive order of the reference generalised to 3D
// (x-, x+, y-, y+, z-, z+, from 0, then * avg), identical to
// kernels_direct.hip and oracle/oracle_impl.inc, so results are bitwise equal.
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace stencil {
namespace {

constexpr int kBY = 4;  // waves per workgroup

// Native clang vectors: 16-B global/LDS accesses and usable with the
// nontemporal builtins.
template <typename T, int V>
struct Vec {
    typedef T type __attribute__((ext_vector_type(V)));
};

template <typename T, int V, int RY>
struct ZTile {
    static constexpr int TX = 64 * V;
    static constexpr int TY = kBY * RY;
    static constexpr int LX = TX + 2 * V;  // [V-1] left halo, [V, V+TX) tile, [V+TX] right halo
    static constexpr int LY = TY + 2;
};

template <typename T, int V, int RY>
__global__ void __launch_bounds__(64 * kBY)
    zmarch7(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
            int zchunk, int tiles_x, int tiles_y, int tiles_z, int remap, T avg) {
    using Tile = ZTile<T, V, RY>;
    using VT = typename Vec<T, V>::type;
    constexpr int TX = Tile::TX, TY = Tile::TY, LX = Tile::LX, LY = Tile::LY;
    __shared__ __attribute__((aligned(16))) T lds[2][LY][LX];

    // ---- XCD-aware tile order (speed only) ----
    const int nb = tiles_x * tiles_y * tiles_z;
    int t = blockIdx.x;
    if (remap && (nb & 7) == 0) t = (t & 7) * (nb >> 3) + (t >> 3);
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int bz = t / (tiles_x * tiles_y);

    const int lane = threadIdx.x, wy = threadIdx.y;
    const int64_t x0 = int64_t(bx) * TX, y0 = int64_t(by) * TY;
    const int64_t za = zbeg + int64_t(bz) * zchunk;
    const int64_t zb = za + zchunk < zend ? za + zchunk : zend;
    const int64_t x = x0 + int64_t(lane) * V;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;
    const int64_t plane = g.plane;

    int64_t off[RY];
    bool ldok[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int64_t y = y0 + wy + kBY * k;
        off[k] = y * g.row + x;
        ldok[k] = x <= g.nx && y <= g.ny;  // vector holds a needed cell (interior or ghost)
    }
    // Halo roles: wave 0 row y0-1, wave 1 row y0+TY (vector loads, like the
    // tile); wave 2 column x0-1, wave 3 column x0+TX (one element per lane,
    // lanes < TY).  Ghost cells (index -1 or n) are in range; anything past
    // them only neighbours cells that are not computed.
    int64_t hoff;
    bool hok, hvec, hslot;
    int hy, hx;
    if (wy < 2) {
        const int64_t yh = wy == 0 ? y0 - 1 : y0 + TY;
        hoff = yh * g.row + x;
        hvec = true;
        hslot = true;
        hok = x <= g.nx && yh <= g.ny;
        hy = wy == 0 ? 0 : TY + 1;
        hx = V + lane * V;
    } else {
        const int64_t yh = y0 + lane;
        const int64_t xh = wy == 2 ? x0 - 1 : x0 + TX;
        hoff = yh * g.row + xh;
        hvec = false;
        hslot = lane < TY;
        hok = hslot && yh <= g.ny && xh <= g.nx;
        hy = lane + 1;
        hx = wy == 2 ? V - 1 : V + TX;
    }

    VT v[4][RY];
    VT h[2];
    auto load_plane = [&](VT (&d)[RY], int64_t z) {
        if (z <= zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (ldok[k]) d[k] = *reinterpret_cast<const VT*>(src + z * plane + off[k]);
        }
    };
    auto load_halo = [&](VT& d, int64_t z) {
        if (z <= zb && hok) {
            if (hvec) d = *reinterpret_cast<const VT*>(src + z * plane + hoff);
            else d.x = src[z * plane + hoff];
        }
    };
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int k = 0; k < RY; ++k) v[s][k] = VT{};
    h[0] = VT{};
    h[1] = VT{};

    load_plane(v[3], za - 1);
    load_plane(v[0], za);
    load_plane(v[1], za + 1);
    load_plane(v[2], za + 2);
    load_halo(h[0], za);
    load_halo(h[1], za + 1);

    auto step = [&](auto S_, int64_t z) {
        constexpr int S = decltype(S_)::value;
        constexpr int M = (S + 3) & 3, C = S, P = (S + 1) & 3, B = S & 1;
#pragma unroll
        for (int k = 0; k < RY; ++k)
            *reinterpret_cast<VT*>(&lds[B][wy + kBY * k + 1][V + lane * V]) = v[C][k];
        if (hslot) {
            if (hvec) *reinterpret_cast<VT*>(&lds[B][hy][hx]) = h[B];
            else lds[B][hy][hx] = h[B].x;
        }
        load_halo(h[B], z + 2);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = wy + kBY * k + 1;
            const int xx = V + lane * V;
            const T* cr = &lds[B][yy][xx];
            const VT up = *reinterpret_cast<const VT*>(&lds[B][yy - 1][xx]);
            const VT dn = *reinterpret_cast<const VT*>(&lds[B][yy + 1][xx]);
            const T wl = cr[-1], er = cr[V];
            const T* c = reinterpret_cast<const T*>(&v[C][k]);
            const T* u = reinterpret_cast<const T*>(&up);
            const T* d = reinterpret_cast<const T*>(&dn);
            const T* zm = reinterpret_cast<const T*>(&v[M][k]);
            const T* zp = reinterpret_cast<const T*>(&v[P][k]);
            VT o;
            T* op = reinterpret_cast<T*>(&o);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                T s = T(0);
                s += j == 0 ? wl : c[j - 1];
                s += j == V - 1 ? er : c[j + 1];
                s += u[j];
                s += d[j];
                s += zm[j];
                s += zp[j];
                op[j] = s * avg;
            }
            const int64_t y = y0 + wy + kBY * k;
            if (y < g.ny) {
                T* p = dst + z * plane + off[k];
                if (x + V <= g.nx) {
                    __builtin_nontemporal_store(o, reinterpret_cast<VT*>(p));
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j)
                        if (x + j < g.nx) p[j] = op[j];
                }
            }
        }
        load_plane(v[M], z + 3);
    };

    for (int64_t z = za; z < zb; z += 4) {
        step(std::integral_constant<int, 0>{}, z);
        if (z + 1 < zb) step(std::integral_constant<int, 1>{}, z + 1);
        if (z + 2 < zb) step(std::integral_constant<int, 2>{}, z + 2);
        if (z + 3 < zb) step(std::integral_constant<int, 3>{}, z + 3);
    }
}

int env_int(const char* name, int dflt) { return knob(name, dflt); }

template <typename T, int V, int RY>
int launch_zm(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
              hipStream_t s) {
    using Tile = ZTile<T, V, RY>;
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    const int64_t gx = (g.nx + Tile::TX - 1) / Tile::TX, gy = (g.ny + Tile::TY - 1) / Tile::TY;
    // ~1024 workgroups (4 resident per CU x 256 CUs) of long z-chunks; the
    // chunk count is rounded to a multiple of 8 when possible so each XCD
    // owns whole chunks.
    int zc = env_int("STENCIL_ZCHUNK", 0);
    if (zc <= 0) {
        const int64_t tiles = gx * gy;
        int64_t chunks = std::max<int64_t>(1, (env_int("STENCIL_TARGET_WG", 1024) + tiles - 1) / tiles);
        if (chunks >= 8) chunks = (chunks + 7) / 8 * 8;
        chunks = std::min<int64_t>(chunks, nz);
        zc = int((nz + chunks - 1) / chunks);
        zc = std::max(zc, 4);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    const int64_t nb = gx * gy * gz;
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for zmarch");
    hipLaunchKernelGGL((zmarch7<T, V, RY>), dim3(unsigned(nb)), dim3(64, kBY, 1), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, begin, end, zc, int(gx),
                       int(gy), int(gz), env_int("STENCIL_ZM_REMAP", 0), avg_weight<T>(l.prob));
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
    const int ry = env_int("STENCIL_ZM_RY", 4);
    if (l.prob.dtype == STENCIL_F32)
        return ry == 2 ? launch_zm<float, 4, 2>(l, in, out, begin, end, s)
                       : launch_zm<float, 4, 4>(l, in, out, begin, end, s);
    return ry == 2 ? launch_zm<double, 2, 2>(l, in, out, begin, end, s)
                   : launch_zm<double, 2, 4>(l, in, out, begin, end, s);
}

}  // namespace stencil
