// kernels_temporal.hip -- two fused Jacobi sweeps per launch (temporal
// blocking) for the 3D 7-point star (r = 1, naive order).
//
// One launch reads grid t from HBM once and writes grid t+2 once; t+1 never
// leaves the chip.  Per launch: ~1.2 x 8 B read + 8 B written per cell for TWO
// updates, against 2 x 16 B for two plain sweeps.
//
// Geometry (a workgroup = NW waves; V = 16 B / sizeof(T) elements per lane):
//   * the workgroup's lanes cover an input REGION of 64*V x NW*RY cells of
//     each plane: the output tile (TX = 64V - 2V by TY = NW*RY - 4) plus a
//     2-cell ring (x: one V-vector per side, keeping 16-B alignment);
//   * it marches z over a chunk of output planes [za, zb).  Iteration p:
//        LDS_in  <- in(p-1)                       (double-buffered)
//        barrier
//        t1(p-1) =  S(in) on the region minus its outer ring, or in(p-1)
//                   where the cell is a ghost (Dirichlet: ghosts never change)
//        LDS_t1  <- t1(p-1)                       (double-buffered)
//        t2(p-2) =  S(t1) on the output tile, x/y neighbours of t1(p-2) from
//                   LDS (written last iteration), z neighbours t1(p-3),
//                   t1(p-1) from registers  -> store
//     one barrier per plane; in(p-2..p+1) and t1(p-3..p-1) live in 4-slot
//     register rings (plane p+2 is prefetched as soon as in(p-2) is dead).
//   * XCD-aware tile numbering as in kernels_zmarch.hip.
//
// Every cell of t1 and t2 is computed with exactly the single-sweep order
// (x-, x+, y-, y+, z-, z+, from 0, then * avg), so two fused steps are
// bitwise equal to two plain sweeps (tests/test_gpu_parity.py).
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int V>
struct Vec {
    typedef T type __attribute__((ext_vector_type(V)));
};

template <typename T, int V, int RY, int NW>
struct T2Tile;

__device__ __forceinline__ bool ld_ok_guard(bool b) { return b; }

template <typename T, int V, int RY, int NW>
struct T2Tile {
    static constexpr int RW = 64 * V;      // region width
    static constexpr int TX = RW - 2 * V;  // output tile width
    static constexpr int RH = NW * RY;     // region height
    static constexpr int TY = RH - 4;      // output tile height
    static constexpr int LX = RW + 2 * V;  // LDS row: pad V | region RW | pad V
    static constexpr int LY = RH + 2;      // LDS rows: pad | region RH | pad
};

template <typename T, int V, int RY, int NW, int R = 4>
__global__ void __launch_bounds__(64 * NW)
    temporal2_7pt(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
                  int zchunk, int tiles_x, int tiles_y, int tiles_z, int64_t t1_lo, int64_t t1_hi,
                  int64_t ld_lo, int64_t ld_hi, int remap, T avg) {
    using Tl = T2Tile<T, V, RY, NW>;
    using VT = typename Vec<T, V>::type;
    constexpr int TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LX = Tl::LX, LY = Tl::LY;
    __shared__ __attribute__((aligned(16))) T lin[2][LY][LX];
    __shared__ __attribute__((aligned(16))) T lt1[2][LY][LX];

    // ---- XCD-aware tile order (speed only) ----
    const int nb = tiles_x * tiles_y * tiles_z;
    int t = blockIdx.x;
    if (remap && (nb & 7) == 0) t = (t & 7) * (nb >> 3) + (t >> 3);
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int bz = t / (tiles_x * tiles_y);

    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x0 = int64_t(bx) * TX, y0 = int64_t(by) * TY;
    const int64_t x = x0 - V + int64_t(lane) * V;  // first element of this lane's vector
    const int64_t za = zbeg + int64_t(bz) * zchunk;
    const int64_t zb = za + zchunk < zend ? za + zchunk : zend;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;
    const int64_t plane = g.plane;

    // Zero the LDS pads once (they only ever feed discarded ring cells):
    // rows 0 and LY-1 whole, and V cells at both ends of every other row.
    {
        const int tid = threadIdx.y * 64 + threadIdx.x;
        constexpr int NPAD = 2 * LX + (LY - 2) * 2 * V;
        for (int i = tid; i < NPAD; i += 64 * NW) {
            int rr, cc;
            if (i < 2 * LX) {
                rr = i < LX ? 0 : LY - 1;
                cc = i % LX;
            } else {
                const int j = i - 2 * LX;
                rr = 1 + j / (2 * V);
                const int c = j % (2 * V);
                cc = c < V ? c : Tl::RW + c;
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                lin[b][rr][cc] = T(0);
                lt1[b][rr][cc] = T(0);
            }
        }
    }

    int64_t off[RY];
    bool ldok[RY], yin[RY], st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w + NW * k;  // region row
        const int64_t y = y0 - 2 + rr;
        off[k] = y * g.row + x;
        ldok[k] = y >= -1 && y <= g.ny && x <= g.nx;
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= 2 && rr < RH - 2 && y < g.ny && lane >= 1 && lane <= 62;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    // t1 is computed on planes [t1_lo, t1_hi) (interior, plus halo planes of
    // faces shared with a neighbouring slab) and copied elsewhere (Dirichlet
    // ghost planes); input planes [ld_lo, min(zb + 1, ld_hi)] are loaded.
    const int64_t zlast = zb + 1 < ld_hi ? zb + 1 : ld_hi;

    // Register rings of R slots (slot of plane q = (q - za) mod R): input
    // planes p-2 .. p+R-3 (plane p+R-2 is loaded as soon as p-2 is dead, so a
    // load has R-2 iterations to land) and t1 planes p-3 .. p-1.
    static_assert(R % 2 == 0 && R >= 4, "ring size must be even (LDS parity) and >= 4");
    VT vin[R][RY], vt1[R][RY];
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            vin[s][k] = VT{};
            vt1[s][k] = VT{};
        }

    auto load_plane = [&](VT (&d)[RY], int64_t z) {
        if (z >= ld_lo && z <= zlast) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (ldok[k]) d[k] = *reinterpret_cast<const VT*>(src + z * plane + off[k]);
        }
    };

#pragma unroll
    for (int i = -2; i <= R - 3; ++i) load_plane(vin[(i + R) % R], za + i);
    __syncthreads();  // LDS pads zeroed

    auto step = [&](auto S_, int64_t p) {
        constexpr int S = decltype(S_)::value;
        constexpr int I0 = S, I1 = (S + R - 1) % R, I2 = (S + R - 2) % R;  // in(p), in(p-1), in(p-2)
        constexpr int T1 = I1, T2 = I2, T3 = (S + R - 3) % R;             // t1(p-1), t1(p-2), t1(p-3)
        constexpr int B = S & 1, BP = B ^ 1;
        const int xx = V + lane * V;
        // 1. stage in(p-1)
#pragma unroll
        for (int k = 0; k < RY; ++k) *reinterpret_cast<VT*>(&lin[B][w + NW * k + 1][xx]) = vin[I1][k];
        __syncthreads();
        // 2. t1(p-1)
        const int64_t z1 = p - 1;
        const bool zin1 = z1 >= t1_lo && z1 < t1_hi;
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
            const T* cr = &lin[B][yy][xx];
            const VT up = *reinterpret_cast<const VT*>(&lin[B][yy - 1][xx]);
            const VT dn = *reinterpret_cast<const VT*>(&lin[B][yy + 1][xx]);
            const T wl = cr[-1], er = cr[V];
            const VT c = vin[I1][k], zm = vin[I2][k], zp = vin[I0][k];
            VT o;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                T s = T(0);
                s += j == 0 ? wl : c[j - 1];
                s += j == V - 1 ? er : c[j + 1];
                s += up[j];
                s += dn[j];
                s += zm[j];
                s += zp[j];
                o[j] = (zin1 && yin[k] && xin[j]) ? s * avg : c[j];
            }
            vt1[T1][k] = o;
            *reinterpret_cast<VT*>(&lt1[B][yy][xx]) = o;
        }
        // 3. t2(p-2): neighbours of t1(p-2) were staged last iteration.
        const int64_t z2 = p - 2;
        if (z2 >= za) {
#pragma unroll
            for (int k = 0; k < RY; ++k) {
                const int yy = w + NW * k + 1;
                const T* cr = &lt1[BP][yy][xx];
                const VT up = *reinterpret_cast<const VT*>(&lt1[BP][yy - 1][xx]);
                const VT dn = *reinterpret_cast<const VT*>(&lt1[BP][yy + 1][xx]);
                const T wl = cr[-1], er = cr[V];
                const VT c = vt1[T2][k], zm = vt1[T3][k], zp = vt1[T1][k];
                VT o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    T s = T(0);
                    s += j == 0 ? wl : c[j - 1];
                    s += j == V - 1 ? er : c[j + 1];
                    s += up[j];
                    s += dn[j];
                    s += zm[j];
                    s += zp[j];
                    o[j] = s * avg;
                }
                if (st[k]) {
                    T* q = dst + z2 * plane + off[k];
                    if (xst[V - 1]) {
                        __builtin_nontemporal_store(o, reinterpret_cast<VT*>(q));
                    } else {
#pragma unroll
                        for (int j = 0; j < V; ++j)
                            if (xst[j]) q[j] = o[j];
                    }
                }
            }
        }
        // 4. load in(p+R-2) into the slot of in(p-2), now dead
        load_plane(vin[I2], p + R - 2);
    };

    for (int64_t p = za; p <= zb + 1; p += R) {
        step(std::integral_constant<int, 0>{}, p);
        if (p + 1 <= zb + 1) step(std::integral_constant<int, 1>{}, p + 1);
        if (p + 2 <= zb + 1) step(std::integral_constant<int, 2>{}, p + 2);
        if (p + 3 <= zb + 1) step(std::integral_constant<int, 3>{}, p + 3);
        if constexpr (R > 4) {
            if (p + 4 <= zb + 1) step(std::integral_constant<int, 4 % R>{}, p + 4);
            if (p + 5 <= zb + 1) step(std::integral_constant<int, 5 % R>{}, p + 5);
        }
    }
}

// Variant: centre values come back from LDS instead of register rings.  A
// thread re-reads ITS OWN cells of in(p-2), in(p-1), t1(p-2) and t1(p-3) from
// the LDS buffers that still hold them (only the owner writes those words, so
// no extra barrier), which frees the t1 ring and most of the input ring; the
// freed VGPRs buy a deeper load lead: plane p+R-1 is requested at iteration p
// (R-1 iterations before first use) as soon as in(p-1) has been staged.
template <typename T, int V, int RY, int NW, int R>
__global__ void __launch_bounds__(64 * NW)
    temporal2_7pt_lc(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
                     int zchunk, int tiles_x, int tiles_y, int tiles_z, int64_t t1_lo, int64_t t1_hi,
                     int64_t ld_lo, int64_t ld_hi, int remap, T avg) {
    using Tl = T2Tile<T, V, RY, NW>;
    using VT = typename Vec<T, V>::type;
    constexpr int TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LX = Tl::LX, LY = Tl::LY;
    __shared__ __attribute__((aligned(16))) T lin[2][LY][LX];
    __shared__ __attribute__((aligned(16))) T lt1[2][LY][LX];
    static_assert(R % 2 == 0 && R >= 4, "ring size must be even and >= 4");

    const int nb = tiles_x * tiles_y * tiles_z;
    int t = blockIdx.x;
    if (remap && (nb & 7) == 0) t = (t & 7) * (nb >> 3) + (t >> 3);
    const int bx = t % tiles_x;
    const int by = (t / tiles_x) % tiles_y;
    const int bz = t / (tiles_x * tiles_y);

    const int lane = threadIdx.x, w = threadIdx.y;
    const int64_t x0 = int64_t(bx) * TX, y0 = int64_t(by) * TY;
    const int64_t x = x0 - V + int64_t(lane) * V;
    const int64_t za = zbeg + int64_t(bz) * zchunk;
    const int64_t zb = za + zchunk < zend ? za + zchunk : zend;
    const T* __restrict__ src = in + g.origin;
    T* __restrict__ dst = out + g.origin;
    const int64_t plane = g.plane;

    {
        const int tid = threadIdx.y * 64 + threadIdx.x;
        constexpr int NPAD = 2 * LX + (LY - 2) * 2 * V;
        for (int i = tid; i < NPAD; i += 64 * NW) {
            int rr, cc;
            if (i < 2 * LX) {
                rr = i < LX ? 0 : LY - 1;
                cc = i % LX;
            } else {
                const int j = i - 2 * LX;
                rr = 1 + j / (2 * V);
                const int c = j % (2 * V);
                cc = c < V ? c : Tl::RW + c;
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                lin[b][rr][cc] = T(0);
                lt1[b][rr][cc] = T(0);
            }
        }
    }

    int64_t off[RY];
    bool ldok[RY], yin[RY], st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w + NW * k;
        const int64_t y = y0 - 2 + rr;
        off[k] = y * g.row + x;
        ldok[k] = y >= -1 && y <= g.ny && x <= g.nx;
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= 2 && rr < RH - 2 && y < g.ny && lane >= 1 && lane <= 62;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }
    const int64_t zlast = zb + 1 < ld_hi ? zb + 1 : ld_hi;

    // slot of plane q = (q - za + 1) mod R: slot 0 holds in(za-1); plane
    // p-1+R is requested at iteration p and first used at iteration p+R-1
    VT vin[R][RY];
#pragma unroll
    for (int s2 = 0; s2 < R; ++s2)
#pragma unroll
        for (int k = 0; k < RY; ++k) vin[s2][k] = VT{};

    auto load_plane = [&](VT (&d)[RY], int64_t z) {
        if (z >= ld_lo && z <= zlast) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (ld_ok_guard(ldok[k])) d[k] = *reinterpret_cast<const VT*>(src + z * plane + off[k]);
        }
    };

    // in(za-2) goes straight to LDS buffer 1 (it is read at iteration za as in(p-2))
    {
        VT tmp[RY];
#pragma unroll
        for (int k = 0; k < RY; ++k) tmp[k] = VT{};
        load_plane(tmp, za - 2);
#pragma unroll
        for (int k = 0; k < RY; ++k)
            *reinterpret_cast<VT*>(&lin[1][w + NW * k + 1][V + lane * V]) = tmp[k];
    }
#pragma unroll
    for (int i = 0; i < R; ++i) load_plane(vin[i], za - 1 + i);
    __syncthreads();

    auto step = [&](auto S_, int64_t p) {
        constexpr int S = decltype(S_)::value;
        constexpr int IM1 = S, I0 = (S + 1) % R;  // slots of in(p-1), in(p)
        constexpr int B = S & 1, BP = B ^ 1;
        const int xx = V + lane * V;
        // 1. stage in(p-1); its register slot is free again: request plane p-1+R
#pragma unroll
        for (int k = 0; k < RY; ++k) *reinterpret_cast<VT*>(&lin[B][w + NW * k + 1][xx]) = vin[IM1][k];
        load_plane(vin[IM1], p - 1 + R);
        __syncthreads();
        const int64_t z1 = p - 1;
        const bool zin1 = z1 >= t1_lo && z1 < t1_hi;
        const bool do2 = p - 2 >= za;
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
            // own centres still in LDS
            const VT c = *reinterpret_cast<const VT*>(&lin[B][yy][xx]);    // in(p-1)
            const VT zm = *reinterpret_cast<const VT*>(&lin[BP][yy][xx]);  // in(p-2)
            const VT t3 = *reinterpret_cast<const VT*>(&lt1[B][yy][xx]);   // t1(p-3)
            const VT up = *reinterpret_cast<const VT*>(&lin[B][yy - 1][xx]);
            const VT dn = *reinterpret_cast<const VT*>(&lin[B][yy + 1][xx]);
            const T wl = lin[B][yy][xx - 1], er = lin[B][yy][xx + V];
            const VT zp = vin[I0][k];
            VT o;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                T s = T(0);
                s += j == 0 ? wl : c[j - 1];
                s += j == V - 1 ? er : c[j + 1];
                s += up[j];
                s += dn[j];
                s += zm[j];
                s += zp[j];
                o[j] = (zin1 && yin[k] && xin[j]) ? s * avg : c[j];
            }
            *reinterpret_cast<VT*>(&lt1[B][yy][xx]) = o;  // t1(p-1) replaces t1(p-3)
            if (do2) {
                const T* cr = &lt1[BP][yy][xx];
                const VT c2 = *reinterpret_cast<const VT*>(cr);  // t1(p-2)
                const VT up2 = *reinterpret_cast<const VT*>(&lt1[BP][yy - 1][xx]);
                const VT dn2 = *reinterpret_cast<const VT*>(&lt1[BP][yy + 1][xx]);
                const T wl2 = cr[-1], er2 = cr[V];
                VT o2;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    T s = T(0);
                    s += j == 0 ? wl2 : c2[j - 1];
                    s += j == V - 1 ? er2 : c2[j + 1];
                    s += up2[j];
                    s += dn2[j];
                    s += t3[j];
                    s += o[j];
                    o2[j] = s * avg;
                }
                if (st[k]) {
                    T* q = dst + (p - 2) * plane + off[k];
                    if (xst[V - 1]) {
                        __builtin_nontemporal_store(o2, reinterpret_cast<VT*>(q));
                    } else {
#pragma unroll
                        for (int j = 0; j < V; ++j)
                            if (xst[j]) q[j] = o2[j];
                    }
                }
            }
        }
    };

    for (int64_t p = za; p <= zb + 1; p += R) {
        step(std::integral_constant<int, 0>{}, p);
        if (p + 1 <= zb + 1) step(std::integral_constant<int, 1>{}, p + 1);
        if (p + 2 <= zb + 1) step(std::integral_constant<int, 2>{}, p + 2);
        if (p + 3 <= zb + 1) step(std::integral_constant<int, 3>{}, p + 3);
        if constexpr (R > 4) {
            if (p + 4 <= zb + 1) step(std::integral_constant<int, 4 % R>{}, p + 4);
            if (p + 5 <= zb + 1) step(std::integral_constant<int, 5 % R>{}, p + 5);
        }
        if constexpr (R > 6) {
            if (p + 6 <= zb + 1) step(std::integral_constant<int, 6 % R>{}, p + 6);
            if (p + 7 <= zb + 1) step(std::integral_constant<int, 7 % R>{}, p + 7);
        }
    }
}

int env_int(const char* name, int dflt) { return knob(name, dflt); }

template <typename T, int V, int RY, int NW, int R = 4, bool LC = false>
int launch_t2(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
              hipStream_t s) {
    using Tl = T2Tile<T, V, RY, NW>;
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    // XCD-aware tile numbering is OFF by default here: with it each XCD marches
    // its own z-region and the fused kernel measured 4 % slower (585 vs 607
    // Gcell/s, same box, 512^3 fp64); neighbouring tiles' halo re-reads are
    // absorbed by the die-level Infinity Cache either way.
    const int remap = env_int("STENCIL_T2_REMAP", 0);
    int zc = env_int("STENCIL_T2_ZCHUNK", 0);
    if (zc <= 0) {
        // ~1900 workgroups (7-8 per CU, one resident at a time): 512^3 ->
        // 20 chunks of 26 planes, the fastest chunk length measured.
        const int64_t tiles = gx * gy;
        int64_t chunks = std::max<int64_t>(1, (env_int("STENCIL_T2_WG", 1900) + tiles - 1) / tiles);
        if (remap && chunks >= 8) chunks = (chunks + 7) / 8 * 8;
        chunks = std::min<int64_t>(chunks, nz);
        zc = int((nz + chunks - 1) / chunks);
        zc = std::max(zc, 8);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    const int64_t nb = gx * gy * gz;
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for temporal2");
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if ((lo || hi) && l.zghost < 2)
        return set_error(STENCIL_EINVAL, "fused steps across a slab halo need halo >= 2 (got %lld)", (long long)l.zghost);
    const int64_t t1_lo = lo ? -1 : 0, t1_hi = hi ? g.nz + 1 : g.nz;
    const int64_t ld_lo = lo ? -2 : -1, ld_hi = hi ? g.nz + 1 : g.nz;
    if constexpr (LC)
        hipLaunchKernelGGL((temporal2_7pt_lc<T, V, RY, NW, R>), dim3(unsigned(nb)), dim3(64, NW, 1), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(out), g, begin, end, zc, int(gx),
                           int(gy), int(gz), t1_lo, t1_hi, ld_lo, ld_hi, remap, avg_weight<T>(l.prob));
    else
        hipLaunchKernelGGL((temporal2_7pt<T, V, RY, NW, R>), dim3(unsigned(nb)), dim3(64, NW, 1), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(out), g, begin, end, zc, int(gx),
                           int(gy), int(gz), t1_lo, t1_hi, ld_lo, ld_hi, remap, avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

}  // namespace

bool temporal2_supports(const stencil_problem& p) {
    return p.dims == 3 && p.shape == STENCIL_STAR && p.radius == 1 &&
           p.order == STENCIL_ORDER_NAIVE;
}

int launch_temporal2(const stencil_layout& l, const void* in, void* out, int64_t begin,
                     int64_t end, hipStream_t s) {
    if (!temporal2_supports(l.prob))
        return set_error(STENCIL_EUNSUPPORTED, "TEMPORAL2 supports 3D star r=1 naive order only");
    // Workgroup shape RY rows per wave x NW waves (region 64V x RY*NW).
    // Default: the LDS-centre kernel (temporal2_7pt_lc), 2 rows x 16 waves,
    // 4-slot input ring: +5.5 % (fp64) / +5.8 % (fp32) over temporal2_7pt
    // measured in one process on one MI355X.
    const int cfg = env_int("STENCIL_T2_CFG", 1004);
    if (l.prob.dtype == STENCIL_F32) {
        switch (cfg) {
        case 48: return launch_t2<float, 4, 4, 8>(l, in, out, begin, end, s);
        case 28: return launch_t2<float, 4, 2, 8>(l, in, out, begin, end, s);
        case 216: return launch_t2<float, 4, 2, 16>(l, in, out, begin, end, s);
        default: return launch_t2<float, 4, 2, 16, 4, true>(l, in, out, begin, end, s);
        }
    }
    switch (cfg) {
    case 48: return launch_t2<double, 2, 4, 8>(l, in, out, begin, end, s);
    case 28: return launch_t2<double, 2, 2, 8>(l, in, out, begin, end, s);
    case 84: return launch_t2<double, 2, 8, 4>(l, in, out, begin, end, s);
    case 216: return launch_t2<double, 2, 2, 16>(l, in, out, begin, end, s);
    case 1044: return launch_t2<double, 2, 4, 8, 4, true>(l, in, out, begin, end, s);
    case 1312: return launch_t2<double, 2, 3, 12, 4, true>(l, in, out, begin, end, s);
    default: return launch_t2<double, 2, 2, 16, 4, true>(l, in, out, begin, end, s);
    }
}

}  // namespace stencil
