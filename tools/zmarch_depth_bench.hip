// zmarch_depth_bench.hip -- diagnostic (not part of the product): does the
// 7-point K-step kernel's z-march move more bytes per second with more input
// planes in flight per CU?
//
// The pattern of tkstrip_7pt at 512^3 fp64 (tools/zmarch_pattern_bench.hip's
// "ring"): 64 x 56 regions at x = 56 bx - 4, y = 48 by - 4 read, the inner
// 56 x 48 written 4 steps later, one barrier per plane step, 8 waves x 7 rows,
// z-chunks of 171 planes (330 workgroups: the packed schedule's count).
// Variants, by how the next planes travel:
//   reg D    register ring, loads issued D planes ahead (tkstrip: D = 2)
//   glds D   global_load_lds of the wave's own rows into an LDS ring of D + 1
//            plane slots, D planes ahead; each step reads plane p+1 from its
//            slot into a 3-plane register ring (one VGPR plane fewer than
//            reg 2, D planes of HBM latency hidden without registers)
// usage: tools/zmarch_depth_bench  (prints ms per pass and GB/s)
#include <hip/hip_runtime.h>

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

constexpr int N = 512, ROW = 528, ROWS = 514, PLANES = 514, OX = 16;
constexpr long PLANE = long(ROW) * ROWS;
constexpr long ORIGIN = PLANE + ROW + OX;  // interior (0,0,0)
constexpr int RY = 7, NW = 8, DELAY = 4, RING = 4;
constexpr int TX = 56, TY = 48;

struct Work {
    int tiles_x, tiles_y, zchunk;
};

__device__ __forceinline__ void region(const Work& wk, int& bx, int& by, int& za, int& zb) {
    const int tiles = wk.tiles_x * wk.tiles_y;
    const int t = blockIdx.x % tiles, c = blockIdx.x / tiles;
    bx = t % wk.tiles_x;
    by = t / wk.tiles_x;
    za = c * wk.zchunk;
    zb = za + wk.zchunk < N ? za + wk.zchunk : N;
}

// register ring, loads D planes ahead
template <int D>
__global__ void __launch_bounds__(64 * NW) march_reg(const double* __restrict__ in, double* __restrict__ out, Work wk) {
    int bx, by, za, zb;
    region(wk, bx, by, za, zb);
    const int lane = threadIdx.x, w = threadIdx.y;
    const long x = long(bx) * TX - RING + lane;
    long off[RY];
    bool st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * TY - RING + w * RY + k;
        const int rr = w * RY + k;
        const long yc = y < -1 ? -1 : (y > N ? N : y);
        const long xc = x < -1 ? -1 : (x > N ? N : x);
        off[k] = ORIGIN + yc * ROW + xc;
        st[k] = rr >= RING && rr < NW * RY - RING && y < N && y >= 0 && lane >= RING && lane < 64 - RING && x < N;
    }
    __shared__ double sink[64 * NW];
    constexpr int NS = D + 2 + DELAY;  // planes p-DELAY .. p+D live
    double ring[NS][RY];
    auto load = [&](double (&d)[RY], int z) {
        const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = in[zz * PLANE + off[k]];
    };
    const int p0 = za - DELAY;
#pragma unroll
    for (int i = 0; i < D; ++i) load(ring[i], p0 + i);
    double acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;  // (p - p0) % NS
        __syncthreads();
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (st[k]) __builtin_nontemporal_store(ring[(S + NS - DELAY) % NS][k], out + zo * PLANE + off[k]);
        }
        acc += ring[S][0];
        load(ring[(S + D) % NS], p + D);
    };
    int p = p0;
    // whole groups of NS steps: up to NS - 1 extra steps past the chunk
    // (clamped loads of the last plane, no stores)
    for (; p <= zb; p += NS) {
        [&]<int... I>(std::integer_sequence<int, I...>) { (step(std::integral_constant<int, I>{}, p + I), ...); }
        (std::make_integer_sequence<int, NS>{});
    }
    sink[w * 64 + lane] = acc;
}

// LDS ring filled by global_load_lds, D planes ahead
template <int D>
__global__ void __launch_bounds__(64 * NW) march_glds(const double* __restrict__ in, double* __restrict__ out, Work wk) {
    int bx, by, za, zb;
    region(wk, bx, by, za, zb);
    const int lane = threadIdx.x, w = threadIdx.y;
    constexpr int NL = D + 1;
    __shared__ __attribute__((aligned(16))) double lds[NL][NW * RY][64];
    const long x = long(bx) * TX - RING + lane;
    // glds: lane l loads 16 B = cells 2(l%32), 2(l%32)+1 of row 2i + l/32
    const long xg = long(bx) * TX - RING + 2 * (lane % 32);
    long goff[(RY + 1) / 2];
#pragma unroll
    for (int i = 0; i < (RY + 1) / 2; ++i) {
        const int k = 2 * i + lane / 32;
        const long y = long(by) * TY - RING + w * RY + (k < RY ? k : RY - 1);
        const long yc = y < -1 ? -1 : (y > N ? N : y);
        const long xc = xg < -2 ? -2 : (xg > N - 2 ? N - 2 : xg);
        goff[i] = ORIGIN + yc * ROW + xc;
    }
    long off[RY];
    bool st[RY];
#pragma unroll
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * TY - RING + w * RY + k;
        const int rr = w * RY + k;
        off[k] = ORIGIN + y * ROW + x;
        st[k] = rr >= RING && rr < NW * RY - RING && y < N && y >= 0 && lane >= RING && lane < 64 - RING && x < N;
    }
    __shared__ double sink[64 * NW];
    constexpr int NS = 3 + DELAY;
    double ring[NS][RY];
    auto issue = [&](int z) {
        const int zz = z < -1 ? -1 : (z > N ? N : z);
        const int slot = (z - za + 2 * NL * 1024) % NL;
#pragma unroll
        for (int i = 0; i < (RY + 1) / 2; ++i) {
            // inline asm: the compiler then sees no LDS-DMA, so it neither
            // drains it (vmcnt(0)) at the barrier nor before the slot reads;
            // the counted wait below orders them
            if (2 * i + 1 < RY || lane < 32) {
                const unsigned la = __builtin_amdgcn_readfirstlane(
                    unsigned(reinterpret_cast<uintptr_t>(&lds[slot][w * RY + 2 * i][0])));
                const double* gp = in + zz * PLANE + goff[i];
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gp), "s"(la)
                             : "memory", "m0");
            }
        }
    };
    auto fetch = [&](double (&d)[RY], int z) {
        const int slot = (z - za + 2 * NL * 1024) % NL;
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = lds[slot][w * RY + k][lane];
    };
    const int p0 = za - DELAY;
    for (int i = 0; i < D; ++i) issue(p0 + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fetch(ring[0], p0);
    double acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;  // (p - p0) % NS
        // raw barrier: __syncthreads() would wait vmcnt(0) for the LDS-DMA in flight
        __builtin_amdgcn_s_barrier();
        // plane p+1's glds (issued at step p+1-D) has landed once at most the
        // ops issued after it are outstanding: per step 4 glds and the wave's
        // stores (>= 3 rows for every wave in the steady state; this pattern
        // bench does not care about the first steps' data)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 4 + (D - 1) * 3) : "memory");
        const int zo = p - DELAY;
        fetch(ring[(S + 1) % NS], p + 1);
        issue(p + D);
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (st[k]) __builtin_nontemporal_store(ring[(S + NS - DELAY) % NS][k], out + zo * PLANE + off[k]);
        }
        acc += ring[S][0];
    };
    int p = p0;
    for (; p <= zb; p += NS) {
        [&]<int... I>(std::integer_sequence<int, I...>) { (step(std::integral_constant<int, I>{}, p + I), ...); }
        (std::make_integer_sequence<int, NS>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sink[w * 64 + lane] = acc;
}

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ void flat_copy(const dv2* __restrict__ a, dv2* __restrict__ b, long n) {
    for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(a[i], &b[i]);
}

int main() {
    const long elems = PLANE * PLANES + 64;
    double *a, *b;
    CK(hipMalloc(&a, elems * 8));
    CK(hipMalloc(&b, elems * 8));
    CK(hipMemset(a, 0, elems * 8));
    CK(hipMemset(b, 0, elems * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < 7; ++rep) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms / 10);
        }
        std::printf("%-28s %8.4f ms  %7.0f GB/s compulsory (%.2f GB)\n", name, best, bytes / (best * 1e-3) / 1e9,
                    bytes / 1e9);
        std::fflush(stdout);
    };
    const double comp = 2.0 * 8.0 * double(N) * N * N;
    timeit("flat copy (padded grid)", 2.0 * elems * 8, [&] {
        hipLaunchKernelGGL(flat_copy, dim3(4096), dim3(256), 0, 0, (const dv2*)a, (dv2*)b, elems / 2);
    });
    for (int chunks : {2, 3, 4}) {
        Work wk{(N + TX - 1) / TX, (N + TY - 1) / TY, (N + chunks - 1) / chunks};
        const dim3 grid(wk.tiles_x * wk.tiles_y * chunks), block(64, NW);
        char name[64];
#define REG(D)                                                                                   \
    std::snprintf(name, sizeof name, "reg %d, %d chunks", D, chunks);                           \
    timeit(name, comp, [&] { hipLaunchKernelGGL(march_reg<D>, grid, block, 0, 0, a, b, wk); });
#define GLDS(D)                                                                                  \
    std::snprintf(name, sizeof name, "glds %d, %d chunks", D, chunks);                          \
    timeit(name, comp, [&] { hipLaunchKernelGGL(march_glds<D>, grid, block, 0, 0, a, b, wk); });
        REG(2) REG(3) REG(4) REG(6)
        GLDS(2) GLDS(3) GLDS(4)
    }
    return 0;
}
