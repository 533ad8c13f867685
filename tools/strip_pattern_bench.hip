// strip_pattern_bench.hip -- diagnostic (not part of the product): what does
// C3's fp32 strip kernel's MEMORY PATTERN cost without its arithmetic, LDS
// hand-offs and selects?  (zmarch_pattern_bench.hip asked the same of C2.)
//
// 4096^2 x 256 fp32 in the engine's layout (row 4160 floats, 4098 rows, 258
// planes).  Every variant is a pure copy in -> out of the interior with the
// kernel's z-march: per plane step each wave loads its RY rows two planes
// ahead into a 4-plane register ring and stores (nontemporal) the plane the
// K-step pipeline would store K steps later, one workgroup barrier per step.
// One workgroup per (tile, whole z range), as AUTO launches this grid
// (4932 workgroups, about 20 rounds on 256 CUs), in the XCD-patch order of the
// kernel (16 tiles wide) or tile-major.
//   flat      one coalesced 16-B-per-lane copy of the padded grids
//   ring      tkstrip_7pt<float,2,5,8,5>'s geometry: 128 x 40 regions at
//             x = 116 bx - 6, y = 30 by - 5 read, the inner 116 x 30 written
//   tile      128 x 40 regions tiling the interior exactly (no over-fetch)
//   wide      256 x 40 regions (4 cells per lane), 240 x 30 written
//   tall      128 x 80 regions (16 waves x 5 rows), 116 x 70 written
// usage: tools/strip_pattern_bench [reps]  (ms per pass, GB/s of compulsory bytes)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

constexpr int NX = 4096, NY = 4096, NZ = 256, ROW = 4160, ROWS = NY + 2, PLANES = NZ + 2, OX = 32;
constexpr long PLANE = long(ROW) * ROWS;
constexpr long ORIGIN = PLANE + ROW + OX;  // interior (0,0,0)

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void flat_copy(const f4* __restrict__ a, f4* __restrict__ b, long n) {
    for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(a[i], &b[i]);
}

// V cells per lane, RY rows per wave, NW waves, DELAY = K; output tile tx x ty,
// region origin (bx * tx - ring_x, by * ty - ring_y); xcd_pw > 0: the kernel's
// XCD-patch work order (one whole-z chunk per tile)
template <int V, int RY, int NW, int DELAY>
__global__ void __launch_bounds__(64 * NW)
    march(const float* __restrict__ in, float* __restrict__ out, int tx, int ty, int tiles_x, int tiles_y, int ring_x,
          int ring_y, int xcd_pw) {
    typedef float VT __attribute__((ext_vector_type(V)));
    const long tiles = long(tiles_x) * tiles_y;
    long t = blockIdx.x;
    if (xcd_pw > 0) {
        const long per = (tiles + 7) / 8;
        const long u = long(blockIdx.x % 8) * per + blockIdx.x / 8;
        if (u >= tiles) return;
        const long strip = u / (long(xcd_pw) * tiles_y), rem = u - strip * xcd_pw * tiles_y;
        const long sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
        t = rem / sw * tiles_x + strip * xcd_pw + rem % sw;
    }
    if (t >= tiles) return;
    const int bx = int(t % tiles_x), by = int(t / tiles_x);
    const int lane = threadIdx.x, w = threadIdx.y;
    const long x = long(bx) * tx - ring_x + lane * V;
    long off[RY];
    bool st[RY];
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * ty - ring_y + w * RY + k;
        const int rr = w * RY + k;
        const long yc = y < -1 ? -1 : (y > NY ? NY : y);
        const long xc = x < -V ? -V : (x > NX ? NX : x);
        off[k] = ORIGIN + yc * ROW + xc;
        st[k] = rr >= ring_y && rr < NW * RY - ring_y && y < NY && y >= 0 && lane * V >= ring_x &&
                lane * V < 64 * V - ring_x && x < NX && x >= 0;
    }
    __shared__ float sink[64 * NW];
    VT ring[4][RY];
    auto load = [&](VT(&d)[RY], int z) {
        const int zz = z < -1 ? -1 : (z > NZ ? NZ : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) {
            if constexpr (V == 3) __builtin_memcpy(&d[k], in + zz * PLANE + off[k], 12);  // 4-B aligned
            else d[k] = *reinterpret_cast<const VT*>(in + zz * PLANE + off[k]);
        }
    };
    const int za = 0, zb = NZ;
    load(ring[0], za - DELAY);
    load(ring[1], za - DELAY + 1);
    float acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __syncthreads();
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (st[k]) {
                    if constexpr (V == 3) {
#pragma unroll
                        for (int j = 0; j < 3; ++j) __builtin_nontemporal_store(ring[(S + 2) % 4][k][j], out + zo * PLANE + off[k] + j);
                    } else {
                        __builtin_nontemporal_store(ring[(S + 2) % 4][k], reinterpret_cast<VT*>(out + zo * PLANE + off[k]));
                    }
                }
        }
        acc += ring[S][0][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    int p = za - DELAY;
    for (; p + 3 <= zb + DELAY; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[w * 64 + lane] = acc;  // keep the loads alive
}

// PAIRED rows: a 128-wide region loaded with 16-B lane vectors -- lanes
// 0..31 hold 4 cells of row 2m, lanes 32..63 the same x of row 2m+1 (RP
// register rows = 2 RP region rows per wave): the same region as `ring` with
// half the load / store instructions
template <int RP, int NW, int DELAY>
__global__ void __launch_bounds__(64 * NW)
    march_pair(const float* __restrict__ in, float* __restrict__ out, int tx, int ty, int tiles_x, int tiles_y,
               int ring_x, int ring_y, int xcd_pw) {
    typedef float VT __attribute__((ext_vector_type(4)));
    const long tiles = long(tiles_x) * tiles_y;
    long t = blockIdx.x;
    if (xcd_pw > 0) {
        const long per = (tiles + 7) / 8;
        const long u = long(blockIdx.x % 8) * per + blockIdx.x / 8;
        if (u >= tiles) return;
        const long strip = u / (long(xcd_pw) * tiles_y), rem = u - strip * xcd_pw * tiles_y;
        const long sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
        t = rem / sw * tiles_x + strip * xcd_pw + rem % sw;
    }
    if (t >= tiles) return;
    const int bx = int(t % tiles_x), by = int(t / tiles_x);
    const int lane = threadIdx.x, w = threadIdx.y, half = lane >> 5, hl = lane & 31;
    const long x = long(bx) * tx - ring_x + hl * 4;
    long off[RP];
    bool st[RP];
    for (int k = 0; k < RP; ++k) {
        const int rr = w * RP * 2 + 2 * k + half;
        const long y = long(by) * ty - ring_y + rr;
        const long yc = y < -1 ? -1 : (y > NY ? NY : y);
        const long xc = x < -4 ? -4 : (x > NX ? NX : x);
        off[k] = ORIGIN + yc * ROW + xc;
        st[k] = rr >= ring_y && rr < NW * RP * 2 - ring_y && y < NY && y >= 0 && hl * 4 >= ring_x &&
                hl * 4 < 128 - ring_x && x < NX && x >= 0;
    }
    __shared__ float sink[64 * NW];
    VT ring[4][RP];
    auto load = [&](VT(&d)[RP], int z) {
        const int zz = z < -1 ? -1 : (z > NZ ? NZ : z);
#pragma unroll
        for (int k = 0; k < RP; ++k) d[k] = *reinterpret_cast<const VT*>(in + zz * PLANE + off[k]);
    };
    const int za = 0, zb = NZ;
    load(ring[0], za - DELAY);
    load(ring[1], za - DELAY + 1);
    float acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __syncthreads();
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RP; ++k)
                if (st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], reinterpret_cast<VT*>(out + zo * PLANE + off[k]));
        }
        acc += ring[S][0][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    int p = za - DELAY;
    for (; p + 3 <= zb + DELAY; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[w * 64 + lane] = acc;  // keep the loads alive
}

// GLDS: the ring geometry (128 x 40 -> 116 x 30, V = 2 register layout)
// with the input planes fetched by inline-asm global_load_lds_dwordx4 (lane
// l: 16 B = cells 4(l%32) .. +3 of row 2i + l/32 of the wave's strip) into
// an LDS ring D planes ahead, then ds_read_b64 into the registers; the
// stores stay 8-B lane vectors.  Raw s_barrier and a counted vmcnt (the
// compiler sees no LDS-DMA, so it does not drain it); the count assumes no
// store after the DMA (waves 0 and 7 store nothing), so it is conservative.
template <int D>
__global__ void __launch_bounds__(512) march_glds(const float* __restrict__ in, float* __restrict__ out, int tiles_x,
                                                  int tiles_y, int xcd_pw) {
    constexpr int RY = 5, NW = 8, DELAY = 5, TX = 116, TY = 30, RX = 6, RYR = 5, NL = D + 1, NI = (RY + 1) / 2;
    typedef float VT __attribute__((ext_vector_type(2)));
    const long tiles = long(tiles_x) * tiles_y;
    long t = blockIdx.x;
    if (xcd_pw > 0) {
        const long per = (tiles + 7) / 8;
        const long u = long(blockIdx.x % 8) * per + blockIdx.x / 8;
        if (u >= tiles) return;
        const long strip = u / (long(xcd_pw) * tiles_y), rem = u - strip * xcd_pw * tiles_y;
        const long sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
        t = rem / sw * tiles_x + strip * xcd_pw + rem % sw;
    }
    if (t >= tiles) return;
    const int bx = int(t % tiles_x), by = int(t / tiles_x);
    const int lane = threadIdx.x, w = threadIdx.y;
    __shared__ __attribute__((aligned(16))) float lds[NL][NW * RY][128];
    const long x = long(bx) * TX - RX + 2 * lane;
    const long xg = long(bx) * TX - RX + 4 * (lane % 32);
    long goff[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = 2 * i + lane / 32;
        const long y = long(by) * TY - RYR + w * RY + (k < RY ? k : RY - 1);
        const long yc = y < -1 ? -1 : (y > NY ? NY : y);
        const long xc = xg < -4 ? -4 : (xg > NX ? NX : xg);
        goff[i] = ORIGIN + yc * ROW + xc;
    }
    long off[RY];
    bool st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * TY - RYR + w * RY + k;
        const int rr = w * RY + k;
        const long yc = y < -1 ? -1 : (y > NY ? NY : y);
        const long xc = x < -2 ? -2 : (x > NX ? NX : x);
        off[k] = ORIGIN + yc * ROW + xc;
        st[k] = rr >= RYR && rr < NW * RY - RYR && y < NY && y >= 0 && lane * 2 >= RX && lane * 2 < 128 - RX &&
                x < NX && x >= 0;
    }
    __shared__ float sink[64 * NW];
    VT ring[4][RY];
    const int za = 0, zb = NZ;
    auto slot_of = [&](int z) { return (z - za + 2 * NL * 1024) % NL; };
    auto issue = [&](int z) {
        const int zz = z < -1 ? -1 : (z > NZ ? NZ : z);
        const int slot = slot_of(z);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (2 * i + 1 < RY || lane < 32) {
                const unsigned la = __builtin_amdgcn_readfirstlane(
                    unsigned(reinterpret_cast<uintptr_t>(&lds[slot][w * RY + 2 * i][0])));
                const float* gp = in + zz * PLANE + goff[i];
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gp), "s"(la)
                             : "memory", "m0");
            }
        }
    };
    auto fetch = [&](VT(&d)[RY], int z) {
        const int slot = slot_of(z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(&lds[slot][w * RY + k][2 * lane]);
    };
    const int p0 = za - DELAY;
    for (int i = 0; i < D; ++i) issue(p0 + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fetch(ring[0], p0);
    float acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * NI) : "memory");
        fetch(ring[(S + 1) % 4], p + 1);
        issue(p + D);
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], reinterpret_cast<VT*>(out + zo * PLANE + off[k]));
        }
        acc += ring[S][0][0];
    };
    int p = p0;
    for (; p + 3 <= zb + DELAY; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sink[w * 64 + lane] = acc;  // keep the loads alive
}

// STAGED STORES: the V = 2 register layout (8-B loads straight to registers,
// as `ring`), but each output plane goes to an LDS image of the wave's own
// rows (ds_write_b64) and leaves as 16-B lane vectors (ds_read_b128: lanes
// 0..31 row 2i, 32..63 row 2i+1) -- no barrier (a wave reads back only its own
// rows).  x ring 8 cells (TX = 112), so every stored lane vector is whole.
template <int RY>
__global__ void __launch_bounds__(512) march_sst(const float* __restrict__ in, float* __restrict__ out, int tiles_x,
                                                 int tiles_y, int xcd_pw) {
    constexpr int NW = 8, DELAY = 5, TX = 112, RX = 8, RYR = 5, TY = NW * RY - 2 * RYR, NI = (RY + 1) / 2;
    typedef float VT __attribute__((ext_vector_type(2)));
    typedef float V4 __attribute__((ext_vector_type(4)));
    const long tiles = long(tiles_x) * tiles_y;
    long t = blockIdx.x;
    if (xcd_pw > 0) {
        const long per = (tiles + 7) / 8;
        const long u = long(blockIdx.x % 8) * per + blockIdx.x / 8;
        if (u >= tiles) return;
        const long strip = u / (long(xcd_pw) * tiles_y), rem = u - strip * xcd_pw * tiles_y;
        const long sw = tiles_x - strip * xcd_pw < xcd_pw ? tiles_x - strip * xcd_pw : xcd_pw;
        t = rem / sw * tiles_x + strip * xcd_pw + rem % sw;
    }
    if (t >= tiles) return;
    const int bx = int(t % tiles_x), by = int(t / tiles_x);
    const int lane = threadIdx.x, w = threadIdx.y;
    __shared__ __attribute__((aligned(16))) float img[NW * RY][128];
    const long x = long(bx) * TX - RX + 2 * lane;
    long off[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * TY - RYR + w * RY + k;
        const long yc = y < -1 ? -1 : (y > NY ? NY : y);
        const long xc = x < -2 ? -2 : (x > NX ? NX : x);
        off[k] = ORIGIN + yc * ROW + xc;
    }
    // 16-B store lanes: cells 4(l%32) .. +3 of row 2i + l/32
    const long xs = long(bx) * TX - RX + 4 * (lane % 32);
    long soff[NI];
    bool sst[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = 2 * i + lane / 32;
        const int rr = w * RY + k;
        const long y = long(by) * TY - RYR + rr;
        sst[i] = k < RY && rr >= RYR && rr < NW * RY - RYR && y >= 0 && y < NY && 4 * (lane % 32) >= RX &&
                 4 * (lane % 32) < 128 - RX && xs >= 0 && xs + 3 < NX;
        soff[i] = ORIGIN + (y < 0 ? 0 : y) * ROW + (xs < 0 ? 0 : xs);
    }
    __shared__ float sink[64 * NW];
    VT ring[4][RY];
    auto load = [&](VT(&d)[RY], int z) {
        const int zz = z < -1 ? -1 : (z > NZ ? NZ : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(in + zz * PLANE + off[k]);
    };
    const int za = 0, zb = NZ;
    load(ring[0], za - DELAY);
    load(ring[1], za - DELAY + 1);
    float acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __syncthreads();
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k) *reinterpret_cast<VT*>(&img[w * RY + k][2 * lane]) = ring[(S + 2) % 4][k];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const V4 v = *reinterpret_cast<const V4*>(&img[w * RY + (2 * i + lane / 32 < RY ? 2 * i + lane / 32 : 0)][4 * (lane % 32)]);
                if (sst[i]) __builtin_nontemporal_store(v, reinterpret_cast<V4*>(out + zo * PLANE + soff[i]));
            }
        }
        acc += ring[S][0][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    int p = za - DELAY;
    for (; p + 3 <= zb + DELAY; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[w * 64 + lane] = acc;  // keep the loads alive
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const long elems = PLANE * PLANES + 256;
    float *a, *b;
    CK(hipMalloc(&a, elems * 4));
    CK(hipMalloc(&b, elems * 4));
    CK(hipMemset(a, 0, elems * 4));
    CK(hipMemset(b, 0, elems * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < reps; ++rep) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < 3; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms / 3);
        }
        std::printf("%-40s %8.4f ms  %7.0f GB/s compulsory (%.2f GB)\n", name, best, bytes / (best * 1e-3) / 1e9,
                    bytes / 1e9);
        std::fflush(stdout);
    };
    const double comp = 2.0 * 4.0 * double(NX) * NY * NZ;
    timeit("flat copy (padded grid)", 2.0 * elems * 4, [&] {
        hipLaunchKernelGGL(flat_copy, dim3(8192), dim3(256), 0, 0, (const f4*)a, (f4*)b, elems / 4);
    });
    auto geo = [&](const char* name, auto kern, int nw, int tx, int ty, int rx, int ry, int pw) {
        const int gx = (NX + tx - 1) / tx, gy = (NY + ty - 1) / ty;
        const long n = pw > 0 ? (long(gx) * gy + 7) / 8 * 8 : long(gx) * gy;
        char full[96];
        std::snprintf(full, sizeof full, "%s (%dx%d tiles, %s)", name, gx, gy, pw > 0 ? "XCD patch" : "tile-major");
        timeit(full, comp, [&] {
            hipLaunchKernelGGL(kern, dim3(unsigned(n)), dim3(64, nw), 0, 0, a, b, tx, ty, gx, gy, rx, ry, pw);
        });
    };
    const int mode = argc > 2 ? std::atoi(argv[2]) : 0;
    if (mode == 0) {
        for (int pw : {16, 0}) {
            geo("ring 128x40 -> 116x30, K=5", march<2, 5, 8, 5>, 8, 116, 30, 6, 5, pw);
            geo("tile 128x40 (no over-fetch)", march<2, 5, 8, 5>, 8, 128, 40, 0, 0, pw);
            geo("wide 256x40 -> 240x30", march<4, 5, 8, 5>, 8, 240, 30, 8, 5, pw);
            geo("tall 128x80 -> 116x70 (16 waves)", march<2, 5, 16, 5>, 16, 116, 70, 6, 5, pw);
        }
    } else if (mode == 4) {
        // the V = 2 register layout with 16-B stores staged through LDS (x ring 8: TX = 112)
        for (int pw : {16, 0}) {
            geo("ring 128x40 -> 116x30, K=5", march<2, 5, 8, 5>, 8, 116, 30, 6, 5, pw);
            geo("ring8 128x40 -> 112x30 (x ring 8)", march<2, 5, 8, 5>, 8, 112, 30, 8, 5, pw);
            const int gx = (NX + 111) / 112, gy = (NY + 29) / 30;
            const long n = pw > 0 ? (long(gx) * gy + 7) / 8 * 8 : long(gx) * gy;
            timeit(pw ? "sst RY5 16-B stores via LDS (XCD patch)" : "sst RY5 16-B stores via LDS (tile-major)", comp, [&] {
                hipLaunchKernelGGL(march_sst<5>, dim3(unsigned(n)), dim3(64, 8), 0, 0, a, b, gx, gy, pw);
            });
            geo("pair 128x48 -> 112x38, 16-B loads", march_pair<3, 8, 5>, 8, 112, 38, 8, 5, pw);
        }
    } else if (mode == 3) {
        // the ring geometry with LDS-DMA 16-B input loads (register layout kept)
        for (int pw : {16, 0}) {
            geo("ring 128x40 -> 116x30, K=5", march<2, 5, 8, 5>, 8, 116, 30, 6, 5, pw);
            const int gx = (NX + 115) / 116, gy = (NY + 29) / 30;
            const long n = pw > 0 ? (long(gx) * gy + 7) / 8 * 8 : long(gx) * gy;
            timeit(pw ? "glds D=3 (XCD patch)" : "glds D=3 (tile-major)", comp, [&] {
                hipLaunchKernelGGL(march_glds<3>, dim3(unsigned(n)), dim3(64, 8), 0, 0, a, b, gx, gy, pw);
            });
            timeit(pw ? "glds D=2 (XCD patch)" : "glds D=2 (tile-major)", comp, [&] {
                hipLaunchKernelGGL(march_glds<2>, dim3(unsigned(n)), dim3(64, 8), 0, 0, a, b, gx, gy, pw);
            });
            geo("pair 128x48 -> 112x38, 16-B loads", march_pair<3, 8, 5>, 8, 112, 38, 8, 5, pw);
        }
    } else if (mode == 2) {
        // the same 128-wide regions with 16-B lane loads (paired rows) against 8-B ones
        for (int pw : {16, 0}) {
            geo("ring 128x40 -> 116x30, K=5", march<2, 5, 8, 5>, 8, 116, 30, 6, 5, pw);
            geo("v2 128x48 -> 116x38, K=5 (RY 6)", march<2, 6, 8, 5>, 8, 116, 38, 6, 5, pw);
            geo("pair 128x48 -> 112x38, 16-B loads", march_pair<3, 8, 5>, 8, 112, 38, 8, 5, pw);
            geo("pair 128x32 -> 112x22, 16-B loads", march_pair<2, 8, 5>, 8, 112, 22, 8, 5, pw);
            geo("v4 256x32 -> 240x22, K=5 (RY 4)", march<4, 4, 8, 5>, 8, 240, 22, 8, 5, pw);
        }
    } else {
        // candidate shapes that fit the strip kernel's VGPR / LDS budget (per sweep: ms / K)
        for (int pw : {16, 0}) {
            geo("ring 128x40 -> 116x30, K=5", march<2, 5, 8, 5>, 8, 116, 30, 6, 5, pw);
            geo("v3 192x40 -> 180x30, K=5", march<3, 5, 8, 5>, 8, 180, 30, 6, 5, pw);
            geo("v4 256x32 -> 240x22, K=5 (RY 4)", march<4, 4, 8, 5>, 8, 240, 22, 8, 5, pw);
            geo("v4 256x40 -> 248x32, K=4", march<4, 5, 8, 4>, 8, 248, 32, 4, 4, pw);
            geo("v3 192x48 -> 180x38, K=5 (RY 6)", march<3, 6, 8, 5>, 8, 180, 38, 6, 5, pw);
            geo("v2 128x48 -> 116x38, K=5 (RY 6)", march<2, 6, 8, 5>, 8, 116, 38, 6, 5, pw);
        }
    }
    return 0;
}
