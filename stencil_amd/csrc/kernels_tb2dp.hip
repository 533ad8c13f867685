// kernels_tb2dp.hip -- the whole 2D job in ONE launch: persistent
// workgroups, one per tile, that keep iterating and synchronise only with
// their eight neighbour tiles.
//
// This is the GPU counterpart of the reference's LDM-resident design
// (src/stencil/slave/stencil_dma.cpp:410-418 load the block once, 424-564
// iterate, exchanging halos with the neighbour CPEs) and of its RMA variant's
// neighbour-only synchronisation (stencil_rma.cpp:198-255, 360: reply
// counters instead of a whole-array barrier).  Where the CPE exchanges a
// 1-cell halo every sweep, a workgroup here exchanges a K*r-cell ring every K
// sweeps (temporal blocking, as tb2ds does per launch): each block of K sweeps
// is strip2d::region -- load tile + ring from the grid written by the previous
// block, K sweeps in registers, store the tile -- and between blocks a tile
// waits only for the neighbours whose cells its ring reads.
//
// Protocol (flags[t] = number of blocks tile t has stored, zeroed before the
// launch):
//   block b reads grid b&1 and writes grid (b+1)&1;
//   before block b (b > 0) a tile waits until flags[n] >= b for its <= 8
//   neighbours n (their block b-1 output, which its ring reads);
//   after storing, every wave drains its stores (s_waitcnt vmcnt(0)), the
//   workgroup meets at a barrier, and one lane releases at agent scope and
//   publishes flags[t] = b+1 (the sequence of the face-signalled 3D kernel,
//   MI355X_MICROARCH.md visibility rules).
// Write-after-read: block b+1 of tile t overwrites grid b&1, which its
// neighbours read in block b; it starts only after they published b, i.e.
// after their block-b loads.  The workgroups must all be resident at once:
// the launch is cooperative (hipLaunchCooperativeKernel refuses a grid that
// does not fit), and a wait that exceeds ~2 s (s_memrealtime, 100 MHz) makes
// the tile store NaN over its cells, raise the abort word (flags[tiles]) that
// every other waiting tile also watches, and leave: a broken launch cannot
// hang, and its result is visibly wrong.
#include <cstdlib>

#include "common.hpp"
#include "strip2d.hpp"

namespace stencil {
namespace {

constexpr uint64_t kWaitTicks = 200ull * 1000 * 1000;  // 2 s of s_memrealtime

// DIAG (timing experiments only, results wrong): 1 = no acquire / release
// fences, 2 = no neighbour waits either
template <typename T, int ORDER, int R, int V, int RY, int NW, int DIAG = 0>
__global__ void __launch_bounds__(64 * NW)
    tb2dp(T* __restrict__ a, T* __restrict__ b, Geom g, int iterations, int K, int tiles_x, int tiles_y, T avg,
          unsigned* __restrict__ flags) {
    __shared__ __attribute__((aligned(16))) strip2d::Lds<T, R, V, NW> L;
    __shared__ int bail;
    const int tile = int(blockIdx.x);
    if (tile >= tiles_x * tiles_y) return;  // never waited on
    const int bx = tile % tiles_x, by = tile / tiles_x;
    const int H = K * R;
    const int nblk = (iterations + K - 1) / K;
    // lane l < 9 of wave 0 watches neighbour (l % 3 - 1, l / 3 - 1)
    const int l = int(threadIdx.x);
    const int nx_ = bx + l % 3 - 1, ny_ = by + l / 3 - 1;
    const bool watch = threadIdx.y == 0 && l < 9 && l != 4 && nx_ >= 0 && nx_ < tiles_x && ny_ >= 0 && ny_ < tiles_y;
    const unsigned* nflag = flags + (watch ? ny_ * tiles_x + nx_ : tile);

    for (int blk = 0; blk < nblk; ++blk) {
        const T* src = (blk & 1) ? b : a;
        T* dst = (blk & 1) ? a : b;
        if (blk > 0 && DIAG < 2) {
            if (threadIdx.y == 0) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                bool late = false;
                unsigned* abort_word = flags + tiles_x * tiles_y;
                for (;;) {
                    const bool ready =
                        !watch || __hip_atomic_load(nflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= unsigned(blk);
                    if (__builtin_amdgcn_ballot_w64(!ready) == 0) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks ||
                        __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                        late = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (l == 0) {
                    bail = late;
                    if (late) __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __syncthreads();
            // every wave: no stale L1 / L2 lines of the neighbours' cells
            if constexpr (DIAG == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (bail) {
                strip2d::poison<T, R, V, RY, NW>(dst, g, H, bx, by);
                return;
            }
        }
        strip2d::region<T, ORDER, R, V, RY, NW>(src, dst, g, iterations - blk * K < K ? iterations - blk * K : K, H,
                                                bx, by, avg, L);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && threadIdx.y == 0) {
            if constexpr (DIAG == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_store(&flags[tile], unsigned(blk + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename T, int ORDER, int R, int V, int RY, int NW>
int launch_tbp(const stencil_layout& l, void* a, void* b, uint32_t iterations, int K, hipStream_t s,
               int* final_in_b, bool dry) {
    const Geom g = geom_of(l);
    const int H = K * R;
    const int TX = 64 * V - 2 * H, TY = NW * RY - 2 * H;
    if (TX < 4 || TY < 4 || TX < H || TY < H)
        return set_error(STENCIL_EUNSUPPORTED, "tb2dp: %d steps of radius %d leave no tile", K, R);
    const int64_t tx = (g.nx + TX - 1) / TX, ty = (g.ny + TY - 1) / TY;
#ifdef STENCIL_DIAG
    // timing experiments only (results wrong on purpose): never in the product build
    static const int diag = knob("STENCIL_TB2DP_DIAG", 0);
    auto kern = diag == 1 ? tb2dp<T, ORDER, R, V, RY, NW, 1> : diag == 2 ? tb2dp<T, ORDER, R, V, RY, NW, 2>
                                                                         : tb2dp<T, ORDER, R, V, RY, NW, 0>;
#else
    auto kern = tb2dp<T, ORDER, R, V, RY, NW, 0>;
#endif
    int dev = 0, cus = 0, per_cu = 0, coop = 0;
    STENCIL_HIP_CHECK(hipGetDevice(&dev));
    STENCIL_HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    STENCIL_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    STENCIL_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, 0));
    if (!coop || tx * ty > int64_t(cus) * per_cu)
        return set_error(STENCIL_EUNSUPPORTED, "tb2dp: %lld tiles do not fit the %d x %d resident workgroups",
                         (long long)(tx * ty), cus, per_cu);
    if (dry) return STENCIL_OK;
    if (final_in_b) *final_in_b = int(((iterations + K - 1) / K) % 2);
    if (iterations == 0 || g.nx <= 0 || g.ny <= 0) {
        if (final_in_b) *final_in_b = 0;
        return STENCIL_OK;
    }
    unsigned* flags = nullptr;
    const size_t fbytes = size_t(tx * ty + 1) * sizeof(unsigned);  // + the abort word
    STENCIL_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&flags), fbytes, s));
    STENCIL_HIP_CHECK(hipMemsetAsync(flags, 0, fbytes, s));
    T* pa = static_cast<T*>(a);
    T* pb = static_cast<T*>(b);
    int it = int(iterations), k = K, ntx = int(tx), nty = int(ty);
    T avg = avg_weight<T>(l.prob);
    void* args[] = {&pa, &pb, const_cast<Geom*>(&g), &it, &k, &ntx, &nty, &avg, &flags};
    const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kern), dim3(unsigned(tx * ty)),
                                                    dim3(64, NW), args, 0, s);
    (void)hipFreeAsync(flags, s);
    if (e != hipSuccess) return set_error(STENCIL_EHIP, "tb2dp launch: %s", hipGetErrorString(e));
    return STENCIL_OK;
}

template <typename T, int ORDER>
int launch_order(const stencil_layout& l, void* a, void* b, uint32_t iterations, int K, hipStream_t s, int* fin,
                 bool dry) {
    switch (l.prob.radius) {
    case 1: return launch_tbp<T, ORDER, 1, 2, 8, 8>(l, a, b, iterations, K, s, fin, dry);
    case 2: return launch_tbp<T, ORDER, 2, 2, 8, 8>(l, a, b, iterations, K, s, fin, dry);
    default: return set_error(STENCIL_EUNSUPPORTED, "tb2dp: radius <= 2 only");
    }
}

}  // namespace

bool tb2dp_supports(const stencil_problem& p) {
    return p.dims == 2 && p.shape == STENCIL_STAR && p.radius >= 1 && p.radius <= 2;
}

int tb2dp_steps(const stencil_problem& p) {
    const int k = knob("STENCIL_TB2DP_K", 8 / p.radius);
    return std::max(1, std::min(k, 24 / p.radius));
}

namespace {
int dispatch(const stencil_layout& l, void* a, void* b, uint32_t iterations, hipStream_t s, int* final_in_b,
             bool dry) {
    if (!tb2dp_supports(l.prob)) return set_error(STENCIL_EUNSUPPORTED, "tb2dp: 2D star r <= 2 only");
    const int K = tb2dp_steps(l.prob);
    const bool dma = l.prob.order == STENCIL_ORDER_DMA;
    if (l.prob.dtype == STENCIL_F32)
        return dma ? launch_order<float, STENCIL_ORDER_DMA>(l, a, b, iterations, K, s, final_in_b, dry)
                   : launch_order<float, STENCIL_ORDER_NAIVE>(l, a, b, iterations, K, s, final_in_b, dry);
    return dma ? launch_order<double, STENCIL_ORDER_DMA>(l, a, b, iterations, K, s, final_in_b, dry)
               : launch_order<double, STENCIL_ORDER_NAIVE>(l, a, b, iterations, K, s, final_in_b, dry);
}
}  // namespace

int launch_tb2dp(const stencil_layout& l, void* a, void* b, uint32_t iterations, hipStream_t s, int* final_in_b) {
    return dispatch(l, a, b, iterations, s, final_in_b, false);
}

bool tb2dp_fits(const stencil_layout& l) {
    const bool ok = dispatch(l, nullptr, nullptr, 0, nullptr, nullptr, true) == STENCIL_OK;
    clear_error();
    return ok;
}

}  // namespace stencil
