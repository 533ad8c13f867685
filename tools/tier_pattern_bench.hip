// tier_pattern_bench.hip -- diagnostic (not part of the product): the C2
// decision gate of VERDICT r03 item 1.  Before building either of two
// byte-reducing designs of the K = 4 strip kernel, measure what its MEMORY
// PATTERN costs (no arithmetic), as tools/zmarch_pattern_bench.hip did for
// the kernel as built (0.433 ms per pass of 4 sweeps at 512^3 fp64).  The
// gate: build a design only if its pattern beats 0.40 ms per 4 sweeps.
//
// 512^3 fp64 in the engine's padded layout (row 528, 514 rows, 514 planes).
//
//   ring    the kernel as built: 64 x 56 regions (K = 4 ring) read, the inner
//           56 x 48 written four plane steps later, 2 z-chunks, 220
//           workgroups, one barrier per plane step.  One pass = 4 sweeps.
//
//   tier    (a) a second temporal tier through the Infinity Cache: 110
//           PRODUCER workgroups march the ring pattern over the whole z range
//           and store their 56 x 48 output (the grid after 4 sweeps) into a
//           ring of R plane slots; 110 CONSUMER workgroups march behind them,
//           read 64 x 56 regions of those slots (their neighbours' outputs
//           give the ring) and write the grid after 8 sweeps.  Only A and C
//           touch HBM: the R-slot ring (R x 2.2 MB) stays in the Infinity
//           Cache.  Hand-off (MI355X_MICROARCH.md, hand-off table row 1):
//           slot stores and loads `sc1`; per plane each producer publishes
//           "planes stored" after every wave's counted vmcnt wait and a
//           barrier; each consumer publishes "planes read" once every wave
//           has its loads; a consumer polls its <= 9 producers before loading
//           a plane, a producer polls its <= 9 consumers before reusing a
//           slot.  Every slot cell carries its plane number as a tag and the
//           consumers count the cells whose tag is wrong (stale hand-offs).
//           One pass = 8 sweeps.  220 workgroups, one per CU, all resident.
//
//   yshare  (b) no redundant ring in y: 64 x 56 regions with the x ring only
//           (56 x 56 written), neighbouring tiles in y exchange 4 boundary
//           rows per side and plane step through sc1 stores + step flags
//           (one hand-off per plane step: a lower bound on the design, which
//           needs one per stage).  2 z-chunks, 200 workgroups.  One pass = 4
//           sweeps.
//
// usage: tools/tier_pattern_bench [R]   (prints ms per pass, ms per 4 sweeps)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
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
constexpr long ORIGIN = PLANE + ROW + OX;  // interior (0,0,0) of a grid
constexpr long PORIGIN = ROW + OX;         // interior (0,0) of a plane slot
constexpr int RY = 7, NW = 8, TX = 56, TY = 48, RING = 4, K = 4;
constexpr int GX = (N + TX - 1) / TX, GY = (N + TY - 1) / TY, TILES = GX * GY;  // 10 x 11 = 110
constexpr int FLAG_STRIDE = 32;  // one 128-B line per flag

__device__ __forceinline__ uint32_t poll_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Spin until *p >= need, with a budget (~0.1 s): a wait that gives up bumps
// *fail and returns, so every wave of the grid reaches its end whatever
// happens (a lost workgroup then shows as wrong tags, never as a hang).
__device__ __forceinline__ void wait_ge(const uint32_t* p, uint32_t need, unsigned* fail) {
    for (int it = 0; poll_ld(p) < need; ++it) {
        if (it > (1 << 22) || (it % 1024 == 0 && poll_ld(fail) != 0)) {  // after one timeout every wait bails
            atomicAdd(fail, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ double sc1_ld(const double* p) {
    const uint64_t u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_bit_cast(double, u);
}
__device__ __forceinline__ void sc1_st(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Region geometry of tile t: per row k of wave w the clamped offset (within a
// plane) and whether the cell is an output cell.
struct Rows {
    long off[RY];
    bool st[RY];
    bool in[RY];  // a grid interior cell (tag-checked)
};
__device__ __forceinline__ void region(int t, int ring_y, int ty, int gx, Rows& r) {
    const int bx = t % gx, by = t / gx;
    const int lane = threadIdx.x, w = threadIdx.y;
    const long x = long(bx) * TX - RING + lane;
    for (int k = 0; k < RY; ++k) {
        const long y = long(by) * ty - ring_y + w * RY + k;
        const int rr = w * RY + k;
        const long yc = y < -1 ? -1 : (y > N ? N : y);
        const long xc = x < -1 ? -1 : (x > N ? N : x);
        r.off[k] = yc * ROW + xc;
        r.in[k] = y >= 0 && y < N && x >= 0 && x < N;
        r.st[k] = rr >= ring_y && rr < NW * RY - ring_y && lane >= RING && lane < 64 - RING && r.in[k];
    }
}

// ------------------------------------------------------------------ ring
__global__ void __launch_bounds__(64 * NW) ring_march(const double* __restrict__ in, double* __restrict__ out, int zchunk) {
    const int t = blockIdx.x % TILES, c = blockIdx.x / TILES;
    Rows r;
    region(t, RING, TY, GX, r);
    const int za = c * zchunk, zb = za + zchunk < N ? za + zchunk : N;
    __shared__ double sink[64 * NW];
    double ring[4][RY];
    auto load = [&](double(&d)[RY], int z) {
        const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = in[ORIGIN + zz * PLANE + r.off[k]];
    };
    load(ring[0], za - 4);
    load(ring[1], za - 3);
    double acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        __syncthreads();
        const int zo = p - K;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (r.st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], out + ORIGIN + zo * PLANE + r.off[k]);
        }
        acc += ring[S][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    for (int p = za - 4; p + 3 <= zb + K; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[threadIdx.y * 64 + threadIdx.x] = acc;
}

// ------------------------------------------------------------------ tier
// blockIdx: b < 112 producers (tile b), 112 <= b < 224 consumers (tile b - 112)
// prod[t] = planes of tile t stored in the slots so far (planes [0, prod) ready)
// cons[t] = planes consumer t has loaded so far
__global__ void __launch_bounds__(64 * (NW + 1))
    tier_march(const double* __restrict__ A, double* __restrict__ B, double* __restrict__ C, uint32_t* prod,
               uint32_t* cons, unsigned* bad, unsigned* fail, int R, uint32_t epoch) {
    const bool producer = blockIdx.x < 112;
    const int t = producer ? blockIdx.x : blockIdx.x - 112;
    if (t >= TILES) return;
    const int lane = threadIdx.x, w = threadIdx.y;
    // waves 0..NW-1 move the data; wave NW (no memory traffic of its own, so
    // its polls never wait behind the data waves' loads) polls and publishes
    const bool syncw = w == NW;
    Rows r;
    region(t, RING, TY, GX, r);
    const int bx = t % GX, by = t / GX;
    // the <= 9 tiles whose outputs this tile's region covers (and, by symmetry,
    // whose regions cover this tile's output): polled by lanes 0..8 of the sync wave
    int nb = -1;
    if (syncw && lane < 9) {
        const int nx = bx + lane % 3 - 1, ny = by + lane / 3 - 1;
        if (nx >= 0 && nx < GX && ny >= 0 && ny < GY) nb = ny * GX + nx;
    }
    const uint32_t base = epoch * uint32_t(N);  // flags count on across launches
    __shared__ double sink[64 * (NW + 1)];
    double ring[4][RY];
    unsigned badc = 0;
    if (producer) {
        auto load = [&](double(&d)[RY], int z) {
            if (syncw) return;
            const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = A[ORIGIN + zz * PLANE + r.off[k]];
        };
        load(ring[0], -4);
        load(ring[1], -3);
        double acc = 0;
        auto step = [&](auto S_, int p) {
            constexpr int S = decltype(S_)::value;
            const int zo = p - K;
            if (!syncw) {
                // loads of plane p and the stores of step p-1 done (plane
                // p+1's RY loads, issued after them, may still be in flight)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
            } else if (nb >= 0 && zo >= R) {  // slot of plane zo free: its consumers have read plane zo - R
                wait_ge(cons + nb * FLAG_STRIDE, base + uint32_t(zo - R + 1), fail);
            }
            __syncthreads();
            if (syncw) {
                if (lane == 0 && zo - 1 >= 0 && zo - 1 < N) flag_st(prod + t * FLAG_STRIDE, base + uint32_t(zo));
                return;
            }
            if (zo >= 0 && zo < N) {
                double* slot = B + long(zo % R) * PLANE + PORIGIN;
#pragma unroll
                for (int k = 0; k < RY; ++k)
                    if (r.st[k]) sc1_st(slot + r.off[k], double(zo) + 0.0 * ring[(S + 2) % 4][k]);
            }
            acc += ring[S][0];
            load(ring[(S + 2) % 4], p + 2);
        };
        int p = -4;
        for (; p + 3 <= N + K; p += 4) {
            step(std::integral_constant<int, 0>{}, p);
            step(std::integral_constant<int, 1>{}, p + 1);
            step(std::integral_constant<int, 2>{}, p + 2);
            step(std::integral_constant<int, 3>{}, p + 3);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (syncw && lane == 0) flag_st(prod + t * FLAG_STRIDE, base + uint32_t(N));
        sink[w * 64 + lane] = acc;
        return;
    }
    // consumer: reads slot planes (its own + neighbours' outputs), writes C
    auto load = [&](double(&d)[RY], int z) {
        if (syncw) return;
        if (z < 0 || z >= N) {  // the grid's z-ghost planes: fixed, from A
            const int zz = z < 0 ? -1 : N;
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = A[ORIGIN + zz * PLANE + r.off[k]];
        } else {
            const double* slot = B + long(z % R) * PLANE + PORIGIN;
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = sc1_ld(slot + r.off[k]);
        }
    };
    load(ring[0], -4);
    load(ring[1], -3);
    double acc = 0;
    auto check = [&](const double(&d)[RY], int z) {
        if (z < 0 || z >= N) return;
#pragma unroll
        for (int k = 0; k < RY; ++k) badc += (r.in[k] && d[k] != double(z)) ? 1u : 0u;
    };
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        const int zo = p - K;
        if (!syncw) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
            check(ring[S], p);
        } else if (nb >= 0 && p + 2 >= 0 && p + 2 < N) {  // plane p+2 stored by every producer in reach
            wait_ge(prod + nb * FLAG_STRIDE, base + uint32_t(p + 3), fail);
        }
        __syncthreads();
        if (syncw) {
            // every data wave has plane p in registers: its slot may be reused
            if (lane == 0 && p >= 0 && p < N) flag_st(cons + t * FLAG_STRIDE, base + uint32_t(p + 1));
            return;
        }
        if (zo >= 0 && zo < N) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (r.st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], C + ORIGIN + zo * PLANE + r.off[k]);
        }
        acc += ring[S][0];
        load(ring[(S + 2) % 4], p + 2);
    };
    int p = -4;
    for (; p + 3 <= N + K; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (syncw && lane == 0) flag_st(cons + t * FLAG_STRIDE, base + uint32_t(N));
    sink[w * 64 + lane] = acc;
    if (badc) atomicAdd(bad, badc);
}

// The same pipeline WITHOUT a dedicated sync wave (the real K = 4 kernel's
// 8 waves already hold 253 VGPRs each: no room for a ninth): wave 0 polls,
// and to keep its loads pipelined it PREFETCHES the flags -- the poll load is
// issued at step p before the step's ring loads, and read at step p + 1
// behind the counted vmcnt(RY) the step waits for anyway; only a flag still
// short then spins (draining wave 0's loads).
__global__ void __launch_bounds__(64 * NW)
    tier_w0_march(const double* __restrict__ A, double* __restrict__ B, double* __restrict__ C, uint32_t* prod,
                  uint32_t* cons, unsigned* bad, unsigned* fail, unsigned* spins, int R, uint32_t epoch) {
    const bool producer = blockIdx.x < 112;
    const int t = producer ? blockIdx.x : blockIdx.x - 112;
    if (t >= TILES) return;
    const int lane = threadIdx.x, w = threadIdx.y;
    Rows r;
    region(t, RING, TY, GX, r);
    const int bx = t % GX, by = t / GX;
    // every lane of wave 0 polls a flag (branch-free, so the compiler's
    // vmcnt bookkeeping stays exact): lanes 0..8 their neighbour's, the rest
    // (and neighbours off the grid) a flag that is always ahead (index 127)
    int nb = 127;
    if (w == 0 && lane < 9) {
        const int nx = bx + lane % 3 - 1, ny = by + lane / 3 - 1;
        if (nx >= 0 && nx < GX && ny >= 0 && ny < GY) nb = ny * GX + nx;
    }
    const uint32_t base = epoch * uint32_t(N);
    __shared__ double sink[64 * NW];
    double ring[4][RY];
    unsigned badc = 0, spin = 0;
    uint32_t pv = 0;  // the prefetched flag of this lane's neighbour
    uint32_t* const watched = producer ? cons : prod;
    auto check_flag = [&](uint32_t need) {  // wave 0: the prefetched value, else spin on fresh polls
        if (pv < need) {
            ++spin;
            wait_ge(watched + nb * FLAG_STRIDE, need, fail);
        }
    };
    auto prefetch_flag = [&] { pv = poll_ld(watched + nb * FLAG_STRIDE); };
    if (producer) {
        auto load = [&](double(&d)[RY], int z) {
            const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
            for (int k = 0; k < RY; ++k) d[k] = A[ORIGIN + zz * PLANE + r.off[k]];
        };
        load(ring[0], -4);
        load(ring[1], -3);
        double acc = 0;
        auto step = [&](auto S_, int p) {
            constexpr int S = decltype(S_)::value;
            const int zo = p - K;
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
            if (w == 0) check_flag(base + uint32_t(zo >= R ? zo - R + 1 : 0));
            __syncthreads();
            if (w == 0 && lane == 0 && zo - 1 >= 0 && zo - 1 < N) flag_st(prod + t * FLAG_STRIDE, base + uint32_t(zo));
            if (zo >= 0 && zo < N) {
                double* slot = B + long(zo % R) * PLANE + PORIGIN;
#pragma unroll
                for (int k = 0; k < RY; ++k)
                    if (r.st[k]) sc1_st(slot + r.off[k], double(zo) + 0.0 * ring[(S + 2) % 4][k]);
            }
            acc += ring[S][0];
            if (w == 0) prefetch_flag();
            load(ring[(S + 2) % 4], p + 2);
        };
        for (int p = -4; p + 3 <= N + K; p += 4) {
            step(std::integral_constant<int, 0>{}, p);
            step(std::integral_constant<int, 1>{}, p + 1);
            step(std::integral_constant<int, 2>{}, p + 2);
            step(std::integral_constant<int, 3>{}, p + 3);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0 && lane == 0) flag_st(prod + t * FLAG_STRIDE, base + uint32_t(N));
        sink[w * 64 + lane] = acc;
        if (spin && lane == 0 && w == 0) atomicAdd(spins, spin);
        return;
    }
    auto load = [&](double(&d)[RY], int z) {  // branch-free: the slot, or the grid's fixed z-ghost plane
        const bool ghost = z < 0 || z >= N;
        const double* src = ghost ? A + ORIGIN + long(z < 0 ? -1 : N) * PLANE : B + long((z < 0 ? 0 : z) % R) * PLANE + PORIGIN;
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = sc1_ld(src + r.off[k]);
    };
    load(ring[0], -4);
    load(ring[1], -3);
    double acc = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        const int zo = p - K;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
#pragma unroll
        for (int k = 0; k < RY; ++k) badc += (p >= 0 && p < N && r.in[k] && ring[S][k] != double(p)) ? 1u : 0u;
        if (w == 0) check_flag(base + uint32_t(p + 3 < 1 ? 0 : (p + 3 > N ? N : p + 3)));
        __syncthreads();
        if (w == 0 && lane == 0 && p >= 0 && p < N) flag_st(cons + t * FLAG_STRIDE, base + uint32_t(p + 1));
        if (zo >= 0 && zo < N) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (r.st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], C + ORIGIN + zo * PLANE + r.off[k]);
        }
        acc += ring[S][0];
        if (w == 0) prefetch_flag();
        load(ring[(S + 2) % 4], p + 2);
    };
    for (int p = -4; p + 3 <= N + K; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w == 0 && lane == 0) flag_st(cons + t * FLAG_STRIDE, base + uint32_t(N));
    sink[w * 64 + lane] = acc;
    if (badc) atomicAdd(bad, badc);
    if (spin && lane == 0 && w == 0) atomicAdd(spins, spin);
}

// ------------------------------------------------------------------ yshare
// 64 x 56 regions, x ring 4 (56 written), no y ring (56 rows written); per
// plane step each workgroup stores its 4 top and 4 bottom rows into an
// exchange buffer (sc1), publishes the step, waits for its y-neighbours'
// step flags and loads their rows (sc1).
constexpr int YTY = RY * NW;                           // 56
constexpr int YGY = (N + YTY - 1) / YTY;               // 10
constexpr int YTILES = GX * YGY;                        // 100
__global__ void __launch_bounds__(64 * (NW + 1))
    yshare_march(const double* __restrict__ in, double* __restrict__ out, double* __restrict__ xb, uint32_t* stepf,
                 int zchunk, uint32_t epoch, unsigned* fail) {
    const int t = blockIdx.x % YTILES, c = blockIdx.x / YTILES;
    const int lane = threadIdx.x, w = threadIdx.y;
    const bool syncw = w == NW;  // the polling / publishing wave
    Rows r;
    region(t, 0, YTY, GX, r);
    const int bx = t % GX, by = t / GX;
    const int za = c * zchunk, zb = za + zchunk < N ? za + zchunk : N;
    const int self = blockIdx.x;
    int nb = -1;  // lanes 0 / 1 of the sync wave: the tile below / above, same chunk
    if (syncw && lane < 2) {
        const int ny = by + (lane == 0 ? -1 : 1);
        if (ny >= 0 && ny < YGY) nb = c * YTILES + ny * GX + bx;
    }
    // exchange rows: workgroup b, parity q, side s (0 bottom, 1 top), row j < 4, lane
    auto xrow = [&](int b, int q, int s, int j) { return xb + ((((long(b) * 2 + q) * 2 + s) * 4 + j) * 64); };
    const uint32_t base = epoch * 1024u;
    __shared__ double sink[64 * (NW + 1)];
    double ring[4][RY];
    auto load = [&](double(&d)[RY], int z) {
        if (syncw) return;
        const int zz = z < -1 ? -1 : (z > N ? N : z);
#pragma unroll
        for (int k = 0; k < RY; ++k) d[k] = in[ORIGIN + zz * PLANE + r.off[k]];
    };
    load(ring[0], za - 4);
    load(ring[1], za - 3);
    double acc = 0;
    int step_no = 0;
    auto step = [&](auto S_, int p) {
        constexpr int S = decltype(S_)::value;
        const int q = step_no & 1;
        // this step's boundary rows out: rows 0..3 live in wave 0, rows 52..55 in wave NW-1
        if (w == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j) sc1_st(xrow(self, q, 0, j) + lane, ring[S][j]);
        if (w == NW - 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) sc1_st(xrow(self, q, 1, j) + lane, ring[S][RY - 4 + j]);
        if (!syncw) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RY) : "memory");
        __syncthreads();
        if (syncw) {
            if (lane == 0) flag_st(stepf + self * FLAG_STRIDE, base + uint32_t(step_no + 1));
            if (nb >= 0) wait_ge(stepf + nb * FLAG_STRIDE, base + uint32_t(step_no + 1), fail);
        }
        __syncthreads();
        ++step_no;
        if (syncw) return;
        double hal = 0;
        if (w == 0 && by > 0)
#pragma unroll
            for (int j = 0; j < 4; ++j) hal += sc1_ld(xrow(self - GX, q, 1, j) + lane);
        if (w == NW - 1 && by < YGY - 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) hal += sc1_ld(xrow(self + GX, q, 0, j) + lane);
        const int zo = p - K;
        if (zo >= za && zo < zb) {
#pragma unroll
            for (int k = 0; k < RY; ++k)
                if (r.st[k]) __builtin_nontemporal_store(ring[(S + 2) % 4][k], out + ORIGIN + zo * PLANE + r.off[k]);
        }
        acc += ring[S][0] + hal;
        load(ring[(S + 2) % 4], p + 2);
    };
    for (int p = za - 4; p + 3 <= zb + K; p += 4) {
        step(std::integral_constant<int, 0>{}, p);
        step(std::integral_constant<int, 1>{}, p + 1);
        step(std::integral_constant<int, 2>{}, p + 2);
        step(std::integral_constant<int, 3>{}, p + 3);
    }
    sink[w * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 16;
    if (R < 8 || R > 64) {
        std::fprintf(stderr, "R must be 8..64\n");
        return 2;
    }
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (cus < 224) {
        std::fprintf(stderr, "needs >= 224 CUs for the resident producer/consumer grid (have %d)\n", cus);
        return 2;
    }
    const long elems = PLANE * PLANES + 64;
    double *a, *b, *c, *slots, *xb;
    uint32_t *prod, *cons, *stepf;
    unsigned* bad;
    CK(hipMalloc(&a, elems * 8));
    CK(hipMalloc(&c, elems * 8));
    CK(hipMalloc(&b, elems * 8));
    CK(hipMalloc(&slots, long(R) * PLANE * 8 + 64 * 8));
    CK(hipMalloc(&xb, 2L * YTILES * 2 * 2 * 4 * 64 * 8));
    CK(hipMalloc(&prod, 128 * FLAG_STRIDE * 4));
    CK(hipMalloc(&cons, 128 * FLAG_STRIDE * 4));
    CK(hipMalloc(&stepf, 2 * YTILES * FLAG_STRIDE * 4));
    CK(hipMalloc(&bad, 16));
    CK(hipMemset(a, 0, elems * 8));
    CK(hipMemset(b, 0, elems * 8));
    CK(hipMemset(c, 0, elems * 8));
    CK(hipMemset(slots, 0xff, long(R) * PLANE * 8 + 64 * 8));  // NaN tags: a read before its store is caught
    CK(hipMemset(prod, 0, 128 * FLAG_STRIDE * 4));
    CK(hipMemset(cons, 0, 128 * FLAG_STRIDE * 4));
    CK(hipMemset(stepf, 0, 2 * YTILES * FLAG_STRIDE * 4));
    CK(hipMemset(bad, 0, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, int sweeps, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.f;
        constexpr int reps = 7, per = 10;
        for (int rep = 0; rep < reps; ++rep) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < per; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms / per);
            sum += ms / per;
        }
        std::printf("%-44s best %8.4f ms per pass (%d sweeps) = %7.4f ms per 4 sweeps; mean %7.4f\n", name, best, sweeps,
                    best * 4.0 / sweeps, sum / reps * 4.0 / sweeps);
        std::fflush(stdout);
    };
    timeit("ring 64x56 -> 56x48, 2 z-chunks (as built)", 4, [&] {
        hipLaunchKernelGGL(ring_march, dim3(TILES * 2), dim3(64, NW), 0, 0, a, b, N / 2);
    });
    uint32_t epoch = 0;
    char name[96];
    std::snprintf(name, sizeof name, "tier: 110 producers + 110 consumers, R=%d", R);
    timeit(name, 8, [&] {
        hipLaunchKernelGGL(tier_march, dim3(224), dim3(64, NW + 1), 0, 0, a, slots, c, prod, cons, bad, bad + 1, R, epoch);
        ++epoch;
    });
    unsigned badh[4] = {};
    CK(hipMemcpy(badh, bad, 16, hipMemcpyDeviceToHost));
    std::printf("tier hand-off check: %u stale cells over %u launches (%.3g cells read per launch), %u waits gave up\n",
                badh[0], epoch, double(TILES) * 64 * RY * NW * (N + 8), badh[1]);
    std::fflush(stdout);
    // the wave-0 variant on fresh flags / slots
    CK(hipMemset(prod, 0, 128 * FLAG_STRIDE * 4));
    CK(hipMemset(cons, 0, 128 * FLAG_STRIDE * 4));
    CK(hipMemset(slots, 0xff, long(R) * PLANE * 8 + 64 * 8));
    CK(hipMemset(bad, 0, 16));
    {  // flag 127 (lanes without a neighbour poll it): always far ahead
        std::vector<uint32_t> hi(FLAG_STRIDE, 0xF0000000u);
        CK(hipMemcpy(prod + 127 * FLAG_STRIDE, hi.data(), FLAG_STRIDE * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(cons + 127 * FLAG_STRIDE, hi.data(), FLAG_STRIDE * 4, hipMemcpyHostToDevice));
    }
    uint32_t epoch0 = 0;
    std::snprintf(name, sizeof name, "tier, wave-0 prefetched polls, R=%d", R);
    timeit(name, 8, [&] {
        hipLaunchKernelGGL(tier_w0_march, dim3(224), dim3(64, NW), 0, 0, a, slots, c, prod, cons, bad, bad + 1, bad + 3,
                           R, epoch0);
        ++epoch0;
    });
    CK(hipMemcpy(badh, bad, 16, hipMemcpyDeviceToHost));
    std::printf("tier wave-0: %u stale cells over %u launches, %u waits gave up, %u spins (flag short when read)\n",
                badh[0], epoch0, badh[1], badh[3]);
    std::fflush(stdout);
    CK(hipMemset(bad, 0, 16));
    uint32_t yepoch = 0;
    timeit("yshare: 64x56 -> 56x56, y rows by hand-off, 2 z-ch", 4, [&] {
        hipLaunchKernelGGL(yshare_march, dim3(YTILES * 2), dim3(64, NW + 1), 0, 0, a, b, xb, stepf, N / 2, yepoch, bad + 2);
        ++yepoch;
    });
    CK(hipMemcpy(badh, bad, 16, hipMemcpyDeviceToHost));
    std::printf("yshare: %u waits gave up\n", badh[2]);
    timeit("ring again", 4, [&] {
        hipLaunchKernelGGL(ring_march, dim3(TILES * 2), dim3(64, NW), 0, 0, a, b, N / 2);
    });
    return 0;
}
