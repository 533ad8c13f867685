// zmarch_pattern_bench.hip -- diagnostic (not part of the product): what does
// the 7-point K-step kernel's MEMORY PATTERN cost without its arithmetic?
//
// 512^3 fp64 in the engine's padded layout (row 528, 514 rows, 514 planes).
// Every variant is a pure copy in->out of the interior with a z-march:
//   flat     one coalesced 16-B-per-lane copy of the padded grids (the
//            bench's copy-kernel calibration)
//   tile     z-march over 64 x 56 regions that tile the interior exactly
//            (no overlap): each cell read once, written once
//   ring     tkstrip's pattern: 64 x 56 regions at x = 56 bx - 4,
//            y = 48 by - 4 (K = 4 ring) read, the inner 56 x 48 written
//            (x over-fetch 1.43 in 128-B lines, y 1.17)
//   ring2    the same with regions twice as wide (128 x 56, 120 x 48 written):
//            what halving the x over-fetch would buy
// Each workgroup marches whole z-chunks (2 chunks of 256 planes, as tkstrip's
// packed schedule roughly does): per plane step each wave loads its RY rows
// two planes ahead into a register ring and stores the plane loaded four
// steps earlier (the K-step pipeline's delay), one barrier per step.
// usage: tools/zmarch_pattern_bench  (prints ms per pass and GB/s)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

typedef double d2 __attribute__((ext_vector_type(2)));
__global__ void flat_copy(const d2* __restrict__ a, d2* __restrict__ b, long n) {
    for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(a[i], &b[i]);
}

// RY rows per wave, NW waves; V cells per lane; region origin (x0, y0); rows
// [ylo, yhi) and lanes [llo, lhi) of the region are written.
template <int V, int RY, int NW, int DELAY>
__global__ void __launch_bounds__(64 * NW)
    march(const double* __restrict__ in, double* __restrict__ out, int tx, int ty, int tiles_x, int tiles_y,
          int ring_x, int ring_y, int zchunk) {
    typedef double VT __attribute__((ext_vector_type(V)));
    const int t = blockIdx.x % (tiles_x * tiles_y), c = blockIdx.x / (tiles_x * tiles_y);
    const int bx = t % tiles_x, by = t / tiles_x;
    const int lane = threadIdx.x, w = threadIdx.y;
    const long x = long(bx) * tx - ring_x + lane * V;
    const int za = c * zchunk, zb = za + zchunk < N ? za + zchunk : N;
    long off[RY];
    bool st[RY];
    for (int k = 0; k < RY; ++k) {
        long y = long(by) * ty - ring_y + w * RY + k;
        const int rr = w * RY + k;
        const long yc = y < -1 ? -1 : (y > N ? N : y);
        const long xc = x < -V ? -V : (x > N ? N : x);
        off[k] = ORIGIN + yc * ROW + xc;
        st[k] = rr >= ring_y && rr < NW * RY - ring_y && y < N && y >= 0 && lane * V >= ring_x &&
                lane * V < 64 * V - ring_x && x < N && x >= 0;
    }
    __shared__ double sink[64 * NW];
    VT ring[4][RY];
    auto load = [&](VT(&d)[RY], int z) {
        const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = *reinterpret_cast<const VT*>(in + zz * PLANE + off[k]);
    };
    load(ring[0], za - 4);
    load(ring[1], za - 3);
    double acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __syncthreads();
        const int zo = p - DELAY;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], reinterpret_cast<VT*>(out + zo * PLANE + off[k]));
        }
        acc += ring[S][0][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    int p = za - 4;
    for (; p + 3 <= zb + DELAY; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[w * 64 + lane] = acc;  // keep the loads alive
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
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms / 10);
        }
        std::printf("%-34s %8.4f ms  %7.0f GB/s compulsory (%.2f GB)\n", name, best, bytes / (best * 1e-3) / 1e9,
                    bytes / 1e9);
    };
    const double comp = 2.0 * 8.0 * double(N) * N * N;
    timeit("flat copy (padded grid)", 2.0 * elems * 8, [&] {
        hipLaunchKernelGGL(flat_copy, dim3(4096), dim3(256), 0, 0, (const d2*)a, (d2*)b, elems / 2);
    });
    for (int chunks : {2, 3}) {
        const int zc = (N + chunks - 1) / chunks;
        char name[64];
        // tile: 64 x 56 regions tiling the interior, everything written
        {
            const int tx = 64, ty = 56, gx = N / tx, gy = (N + ty - 1) / ty;
            std::snprintf(name, sizeof name, "tile 64x56, %d z-chunks", chunks);
            timeit(name, comp, [&] {
                hipLaunchKernelGGL((march<1, 7, 8, 2>), dim3(gx * gy * chunks), dim3(64, 8), 0, 0, a, b, tx, ty, gx, gy,
                                   0, 0, zc);
            });
        }
        {
            const int tx = 56, ty = 48, gx = (N + tx - 1) / tx, gy = (N + ty - 1) / ty;
            std::snprintf(name, sizeof name, "ring 64x56 -> 56x48, %d z-chunks", chunks);
            timeit(name, comp, [&] {
                hipLaunchKernelGGL((march<1, 7, 8, 2>), dim3(gx * gy * chunks), dim3(64, 8), 0, 0, a, b, tx, ty, gx, gy,
                                   4, 4, zc);
            });
        }
        {
            const int tx = 120, ty = 48, gx = (N + tx - 1) / tx, gy = (N + ty - 1) / ty;
            std::snprintf(name, sizeof name, "ring2 128x56 -> 120x48, %d z-ch", chunks);
            timeit(name, comp, [&] {
                hipLaunchKernelGGL((march<2, 7, 8, 2>), dim3(gx * gy * chunks), dim3(64, 8), 0, 0, a, b, tx, ty, gx, gy,
                                   4, 4, zc);
            });
        }
        {
            const int tx = 128, ty = 56, gx = N / tx, gy = (N + ty - 1) / ty;
            std::snprintf(name, sizeof name, "tile2 128x56, %d z-chunks", chunks);
            timeit(name, comp, [&] {
                hipLaunchKernelGGL((march<2, 7, 8, 2>), dim3(gx * gy * chunks), dim3(64, 8), 0, 0, a, b, tx, ty, gx, gy,
                                   0, 0, zc);
            });
        }
    }
    return 0;
}
