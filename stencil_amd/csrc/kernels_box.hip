// kernels_box.hip -- 3D 27-point box stencil (r = 1), one sweep or two fused
// sweeps per launch, z-marching with incremental partial sums.
//
// The box order is lexicographic (dz, dy, dx) with the centre skipped
// (oracle/oracle_impl.inc): the 9 terms of plane z-1 come
// first, then the 8 of plane z, then the 9 of plane z+1.  So when input plane
// q is staged in LDS, every lane can
//     start    the sum of output plane q+1   (0 + its 9 dz=-1 terms),
//     continue the sum of output plane q     (+ its 8 dz=0 terms),
//     finish   the sum of output plane q-1   (+ its 9 dz=+1 terms) -> * avg,
// which performs every cell's 26 additions in exactly the reference order
// while only ONE plane of the input lives in LDS at a time and two running
// sums per cell live in registers.
//
// STEPS = 2 chains a second such pipeline on the t+1 planes: t1(q-1) is
// finished at iteration q, staged in LDS, and consumed one iteration later
// (start t2(q-1), continue t2(q-2), finish t2(q-3) -> store).  Ghost cells
// of t1 are Dirichlet copies of the input; slab-halo planes (HALO_LO/HI) are
// advanced like interior ones.  Geometry and XCD-aware tile order follow
// kernels_temporal.hip: lanes cover the tile plus a ring of STEPS cells in y
// and one 16-B vector in x.
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace stencil {
namespace {

template <typename T, int V>
struct BVec {
    typedef T type __attribute__((ext_vector_type(V)));
};

template <typename T, int V, int RY, int NW, int STEPS>
struct BoxTile {
    static constexpr int RW = 64 * V;
    static constexpr int TX = RW - 2 * V;
    static constexpr int RH = NW * RY;
    static constexpr int TY = RH - 2 * STEPS;
    static constexpr int LX = RW + 2 * V;
    static constexpr int LY = RH + 2;
};

template <typename T, int V, int RY, int NW, int STEPS>
__global__ void __launch_bounds__(64 * NW)
    box27_zmarch(const T* __restrict__ in, T* __restrict__ out, Geom g, int64_t zbeg, int64_t zend,
                 int zchunk, int tiles_x, int tiles_y, int tiles_z, int64_t t1_lo, int64_t t1_hi,
                 int64_t ld_lo, int64_t ld_hi, int remap, T avg) {
    using Tl = BoxTile<T, V, RY, NW, STEPS>;
    using VT = typename BVec<T, V>::type;
    constexpr int TX = Tl::TX, TY = Tl::TY, RH = Tl::RH, LX = Tl::LX, LY = Tl::LY, RW = Tl::RW;
    // Input planes rotate through 4 LDS buffers (slot = plane mod 4): a plane
    // is read at its own iteration and at the next one, so its buffer must
    // not be rewritten before two barriers have passed.  t1 planes (STEPS=2)
    // are read only one iteration after being written: 2 buffers.
    __shared__ __attribute__((aligned(16))) T lin[4][LY][LX];
    __shared__ __attribute__((aligned(16))) T lt1[STEPS == 2 ? 2 : 1][LY][LX];

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

    {  // zero the LDS pads once
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
                cc = c < V ? c : RW + c;
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) lin[b][rr][cc] = T(0);
            if constexpr (STEPS == 2) {
                lt1[0][rr][cc] = T(0);
                lt1[1][rr][cc] = T(0);
            }
        }
    }

    int64_t off[RY];
    bool ldok[RY], yin[RY], st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const int rr = w + NW * k;
        const int64_t y = y0 - STEPS + rr;
        off[k] = y * g.row + x;
        ldok[k] = y >= -1 && y <= g.ny && x <= g.nx;
        yin[k] = y >= 0 && y < g.ny;
        st[k] = rr >= STEPS && rr < RH - STEPS && y < g.ny && lane >= 1 && lane <= 62;
    }
    bool xin[V], xst[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        xin[j] = x + j >= 0 && x + j < g.nx;
        xst[j] = x + j < g.nx;
    }

    // Iterations q0..q1 over input planes; slot(m) = (m - q0) & 3.
    const int64_t q0 = za - STEPS;
    const int64_t q1 = STEPS == 2 ? zb + 2 : zb;
    const int64_t in_last = STEPS == 2 ? zb + 1 : zb;  // last input plane any output needs
    const int64_t zlast = in_last < ld_hi ? in_last : ld_hi;
    // planes whose stage-1 result is needed
    const int64_t s1_lo = STEPS == 2 ? za - 1 : za, s1_hi = STEPS == 2 ? zb + 1 : zb;

    VT vin[4][RY], p1[1][RY], p2[4][RY];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            vin[s][k] = VT{};
            p2[s][k] = VT{};
        }
#pragma unroll
    for (int k = 0; k < RY; ++k) p1[0][k] = VT{};

    auto load_plane = [&](VT (&d)[RY], int64_t z) {
        if (z >= ld_lo && z <= zlast) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (ldok[k]) d[k] = *reinterpret_cast<const VT*>(src + z * plane + off[k]);
        }
    };

    load_plane(vin[0], q0);
    load_plane(vin[1], q0 + 1);
    load_plane(vin[2], q0 + 2);
    __syncthreads();  // pads zeroed

    // 3x(V+2) neighbourhood of this lane's vector, row yy of LDS plane b.
    auto hood = [&](const T (&pl)[LY][LX], int yy, T (&nv)[3][V + 2]) {
        const int xx = V + lane * V;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const T* row = &pl[yy - 1 + r][xx];
            const VT c = *reinterpret_cast<const VT*>(row);
            nv[r][0] = row[-1];
#pragma unroll
            for (int j = 0; j < V; ++j) nv[r][j + 1] = c[j];
            nv[r][V + 1] = row[V];
        }
    };
    // dz = -1 or +1 role: 9 terms, (dy, dx) lexicographic.
    auto add9 = [&](T s, const T (&nv)[3][V + 2], int j) {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) s += nv[r][j + dx];
        return s;
    };
    // dz = 0 role: 8 terms, centre skipped.
    auto add8 = [&](T s, const T (&nv)[3][V + 2], int j) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) s += nv[0][j + dx];
        s += nv[1][j];
        s += nv[1][j + 2];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) s += nv[2][j + dx];
        return s;
    };

    auto store_out = [&](const VT& o, int64_t z, int k) {
        T* p = dst + z * plane + off[k];
        if (xst[V - 1]) {
            __builtin_nontemporal_store(o, reinterpret_cast<VT*>(p));
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j)
                if (xst[j]) p[j] = o[j];
        }
    };

    // Iteration q: LDS_in[q] <- in(q) (LDS_in[q-1] still holds in(q-1)).
    //  stage 1: finish plane q-1 (+9 terms of plane q) and build plane q from
    //           scratch (9 terms of plane q-1, then 8 of plane q): one running
    //           sum per cell is carried to the next iteration.
    //  stage 2: on t1(q-2) (LDS_t1[B^1], staged last iteration): finish
    //           t2(q-3), continue t2(q-2), start t2(q-1) -- two carried sums.
    auto step = [&](auto S_, int64_t q) {
        constexpr int S = decltype(S_)::value;
        constexpr int CQ = S, CP = (S + 3) & 3;  // slots of planes q, q-1 (= q+3)
        constexpr int B = S & 1, BP = B ^ 1;
        const int xx = V + lane * V;
#pragma unroll
        for (int k = 0; k < RY; ++k) *reinterpret_cast<VT*>(&lin[CQ][w + NW * k + 1][xx]) = vin[CQ][k];
        load_plane(vin[CP], q + 3);  // slot of q-1: in(q-1) now lives in LDS_in[BP]
        __syncthreads();
        const bool st_fin = q - 1 >= s1_lo && q - 1 < s1_hi;
        const bool st_new = q >= s1_lo && q < s1_hi;
        const bool zin1 = q - 1 >= t1_lo && q - 1 < t1_hi;
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            const int yy = w + NW * k + 1;
            VT nw;
            if (st_new) {  // 9 terms of plane q-1 first (one neighbourhood live at a time)
                T np[3][V + 2];
                hood(lin[CP], yy, np);
#pragma unroll
                for (int j = 0; j < V; ++j) nw[j] = add9(T(0), np, j);
            }
            T nq[3][V + 2];
            hood(lin[CQ], yy, nq);
            if (st_fin) {
                VT fin, o;
#pragma unroll
                for (int j = 0; j < V; ++j) fin[j] = add9(p1[0][k][j], nq, j);
                if constexpr (STEPS == 1) {
#pragma unroll
                    for (int j = 0; j < V; ++j) o[j] = fin[j] * avg;
                    if (st[k]) store_out(o, q - 1, k);
                } else {
                    const VT c = *reinterpret_cast<const VT*>(&lin[CP][yy][xx]);  // in(q-1)
#pragma unroll
                    for (int j = 0; j < V; ++j) o[j] = (zin1 && yin[k] && xin[j]) ? fin[j] * avg : c[j];
                    *reinterpret_cast<VT*>(&lt1[B][yy][xx]) = o;
                }
            }
            if (st_new) {
#pragma unroll
                for (int j = 0; j < V; ++j) nw[j] = add8(nw[j], nq, j);
                p1[0][k] = nw;
            }
        }
        if constexpr (STEPS == 2) {
            const int64_t m = q - 2;  // t1 plane staged last iteration
            if (m >= s1_lo && m < s1_hi) {
                const bool t_start = m + 1 >= za && m + 1 < zb;
                const bool t_mid = m >= za && m < zb;
                const bool t_fin = m - 1 >= za && m - 1 < zb;
                constexpr int MN = (S + 3) & 3, MQ = (S + 2) & 3, MP = (S + 1) & 3;  // t2 slots m+1, m, m-1
#pragma unroll
                for (int k = 0; k < RY; ++k) {
                    T nv[3][V + 2];
                    hood(lt1[BP], w + NW * k + 1, nv);
                    VT o;
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        if (t_fin) o[j] = add9(p2[MP][k][j], nv, j) * avg;
                        if (t_mid) p2[MQ][k][j] = add8(p2[MQ][k][j], nv, j);
                        if (t_start) p2[MN][k][j] = add9(T(0), nv, j);
                    }
                    if (t_fin && st[k]) store_out(o, m - 1, k);
                }
            }
        }
    };

    for (int64_t q = q0; q <= q1; q += 4) {
        step(std::integral_constant<int, 0>{}, q);
        if (q + 1 <= q1) step(std::integral_constant<int, 1>{}, q + 1);
        if (q + 2 <= q1) step(std::integral_constant<int, 2>{}, q + 2);
        if (q + 3 <= q1) step(std::integral_constant<int, 3>{}, q + 3);
    }
}

int env_int(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return s && *s ? std::atoi(s) : dflt;
}

template <typename T, int V, int RY, int NW, int STEPS>
int launch_box(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
               hipStream_t s) {
    using Tl = BoxTile<T, V, RY, NW, STEPS>;
    const Geom g = geom_of(l);
    const int64_t nz = end - begin;
    if (nz <= 0 || g.nx <= 0 || g.ny <= 0) return STENCIL_OK;
    const int64_t gx = (g.nx + Tl::TX - 1) / Tl::TX, gy = (g.ny + Tl::TY - 1) / Tl::TY;
    int zc = env_int("STENCIL_BOX_ZCHUNK", 0);
    if (zc <= 0) {
        const int64_t tiles = gx * gy;
        int64_t chunks = std::max<int64_t>(1, (env_int("STENCIL_BOX_WG", 768) + tiles - 1) / tiles);
        if (chunks >= 8) chunks = (chunks + 7) / 8 * 8;
        chunks = std::min<int64_t>(chunks, nz);
        zc = int((nz + chunks - 1) / chunks);
        zc = std::max(zc, 8);
    }
    const int64_t gz = (nz + zc - 1) / zc;
    const int64_t nb = gx * gy * gz;
    if (nb > (int64_t(1) << 31) - 1) return set_error(STENCIL_EINVAL, "grid too large for box27");
    const bool lo = l.prob.flags & STENCIL_HALO_LO, hi = l.prob.flags & STENCIL_HALO_HI;
    if (STEPS == 2 && (lo || hi) && l.zghost < 2)
        return set_error(STENCIL_EINVAL, "fused steps across a slab halo need halo >= 2");
    const int64_t t1_lo = (STEPS == 2 && lo) ? -1 : 0, t1_hi = (STEPS == 2 && hi) ? g.nz + 1 : g.nz;
    int64_t ld_lo = (STEPS == 2 && lo) ? -2 : -1, ld_hi = (STEPS == 2 && hi) ? g.nz + 1 : g.nz;
    if (STEPS == 1) {  // single sweeps may cover slab-halo planes (stencil_sweep): load what they read
        ld_lo = std::min<int64_t>(ld_lo, begin - 1);
        ld_hi = std::max<int64_t>(ld_hi, end);
    }
    hipLaunchKernelGGL((box27_zmarch<T, V, RY, NW, STEPS>), dim3(unsigned(nb)), dim3(64, NW, 1), 0, s,
                       static_cast<const T*>(in), static_cast<T*>(out), g, begin, end, zc, int(gx),
                       int(gy), int(gz), t1_lo, t1_hi, ld_lo, ld_hi, env_int("STENCIL_BOX_REMAP", 0),
                       avg_weight<T>(l.prob));
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

}  // namespace

bool box27_supports(const stencil_problem& p) {
    return p.dims == 3 && p.shape == STENCIL_BOX && p.radius == 1 && p.order == STENCIL_ORDER_NAIVE;
}

int launch_box27(const stencil_layout& l, const void* in, void* out, int64_t begin, int64_t end,
                 int steps, hipStream_t s) {
    if (!box27_supports(l.prob)) return set_error(STENCIL_EUNSUPPORTED, "box27 kernel: 3D box r=1 only");
    // Workgroup shapes (rows per wave x waves): single sweeps 2x16, fused
    // pairs 1x16 (both 16 waves in <= 128 VGPRs without spills; a 2-row
    // fused shape spills at every wave count tried).
    const int cfg = env_int("STENCIL_BOX_CFG", 0);
    if (l.prob.dtype == STENCIL_F32) {
        if (steps == 2) return launch_box<float, 4, 1, 16, 2>(l, in, out, begin, end, s);
        return launch_box<float, 4, 2, 16, 1>(l, in, out, begin, end, s);
    }
    if (steps == 2) {
        switch (cfg) {
        default: return launch_box<double, 2, 1, 16, 2>(l, in, out, begin, end, s);
        }
    }
    return cfg == 48 ? launch_box<double, 2, 4, 8, 1>(l, in, out, begin, end, s)
                     : launch_box<double, 2, 2, 16, 1>(l, in, out, begin, end, s);
}

}  // namespace stencil
