// api.hip -- the C-ABI of libstencil_hip.so (declared in include/stencil_hip.h).
//
// Host-side orchestration: layout, allocation, initial condition, transfers,
// kernel-family dispatch, the ping-pong iteration loop, and the
// reference-compatible entry points stencil_iterate_{dma, dma_static_unroll,
// dma_slave_pack, rma} that replace the Sunway CPE kernels
// (src/stencil/slave/stencil_slave.hpp:26-46).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.hpp"

namespace stencil {

namespace {
thread_local int g_last_code = STENCIL_OK;
thread_local char g_last_msg[512] = "";
}  // namespace

thread_local LaunchInfo* tl_dry_launch = nullptr;
thread_local bool tl_sustained = false;

int set_error(int code, const char* fmt, ...) {
    g_last_code = code;
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_last_msg, sizeof g_last_msg, fmt, ap);
    va_end(ap);
    return code;
}

void clear_error() {
    g_last_code = STENCIL_OK;
    g_last_msg[0] = '\0';
}

int resident_slots(const void* kern, int threads, bool one_per_cu, int* slots) {
    int dev = 0;
    STENCIL_HIP_CHECK(hipGetDevice(&dev));
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, int, bool>, int> cache;
    const auto key = std::make_tuple(dev, kern, threads, one_per_cu);
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(key);
        if (it != cache.end()) {
            *slots = it->second;
            return STENCIL_OK;
        }
    }
    int cus = 0, per_cu = 1;
    STENCIL_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (!one_per_cu) STENCIL_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0));
    const int n = std::max(1, cus * std::max(1, per_cu));
    std::lock_guard<std::mutex> lock(mu);
    cache[key] = n;
    *slots = n;
    return STENCIL_OK;
}

namespace {

inline size_t elem_size(const stencil_problem& p) { return p.dtype == STENCIL_F32 ? 4 : 8; }

int check_problem(const stencil_problem* p) {
    if (!p) return set_error(STENCIL_EINVAL, "null problem");
    if (p->dims != 2 && p->dims != 3) return set_error(STENCIL_EINVAL, "dims must be 2 or 3 (got %d)", p->dims);
    if (p->dtype != STENCIL_F32 && p->dtype != STENCIL_F64) return set_error(STENCIL_EINVAL, "bad dtype %d", p->dtype);
    if (p->shape != STENCIL_STAR && p->shape != STENCIL_BOX) return set_error(STENCIL_EINVAL, "bad shape %d", p->shape);
    if (p->radius < 1 || p->radius > 64) return set_error(STENCIL_EINVAL, "radius must be in [1, 64] (got %d)", p->radius);
    if (p->order != STENCIL_ORDER_NAIVE && p->order != STENCIL_ORDER_DMA) return set_error(STENCIL_EINVAL, "bad order %d", p->order);
    if (p->order == STENCIL_ORDER_DMA && (p->dims != 2 || p->shape != STENCIL_STAR))
        return set_error(STENCIL_EINVAL, "DMA sum order is defined for 2D star stencils only");
    if (p->kernel < STENCIL_KERNEL_AUTO || p->kernel > STENCIL_KERNEL_PERSISTENT) return set_error(STENCIL_EINVAL, "bad kernel %d", p->kernel);
    if (p->nx < 0 || p->ny < 0 || p->nz < 0) return set_error(STENCIL_EINVAL, "negative extent");
    if (p->dims == 2 && p->nz != 1) return set_error(STENCIL_EINVAL, "2D problems need nz = 1");
    if (p->halo < 0 || (p->halo > 0 && p->halo < p->radius) || p->halo > 64)
        return set_error(STENCIL_EINVAL, "halo must be 0 or in [radius, 64] (got %d)", p->halo);
    if (p->dims == 2 && p->halo > p->radius) return set_error(STENCIL_EINVAL, "2D grids have radius-deep ghosts only");
    if (p->flags & ~(STENCIL_HALO_LO | STENCIL_HALO_HI)) return set_error(STENCIL_EINVAL, "bad flags %d", p->flags);
    if (p->kernel == STENCIL_KERNEL_ZMARCH && !march_supported(*p))
        return set_error(STENCIL_EUNSUPPORTED, "ZMARCH kernels cover 3D r=1 naive star (7-pt) and box (27-pt) only");
    if (p->kernel == STENCIL_KERNEL_TEMPORAL2 && !fused_supported(*p) && !tb2d_supports(*p))
        return set_error(STENCIL_EUNSUPPORTED,
                         "TEMPORAL2 kernels cover 3D r=1 naive star/box and 2D star r<=4 only");
    if (p->kernel == STENCIL_KERNEL_TEMPORALK && !temporal2_supports(*p))
        return set_error(STENCIL_EUNSUPPORTED, "TEMPORALK kernels cover the 3D r=1 naive 7-point star only");
    if (p->kernel == STENCIL_KERNEL_PERSISTENT && !tb2dp_supports(*p))
        return set_error(STENCIL_EUNSUPPORTED, "the PERSISTENT kernel covers 2D star stencils with r <= 2 only");
    return STENCIL_OK;
}

int check_layout(const stencil_layout* l) {
    if (!l) return set_error(STENCIL_EINVAL, "null layout");
    return check_problem(&l->prob);
}

// Resolve AUTO to a concrete single-sweep kernel family.
int sweep_family(const stencil_problem& p) {
    if (p.kernel == STENCIL_KERNEL_DIRECT) return STENCIL_KERNEL_DIRECT;
    if (march_supported(p)) return STENCIL_KERNEL_ZMARCH;
    return STENCIL_KERNEL_DIRECT;
}

// Does stencil_iterate fuse pairs of sweeps?  Explicit TEMPORAL2, or AUTO on
// a problem a fused kernel supports (STENCIL_NO_T2=1 disables the latter).
bool iterate_fused(const stencil_problem& p) {
    if (p.kernel == STENCIL_KERNEL_TEMPORAL2 || p.kernel == STENCIL_KERNEL_TEMPORALK) return true;
    // AUTO fuses the 7-point star (TEMPORALK, K = 4) and the 27-point box
    // (the 2-step BOXK kernel: +50-90 % fp64, +9-37 % fp32 over the single
    // sweep on MI355X).
    if (p.kernel != STENCIL_KERNEL_AUTO || !fused_supported(p)) return false;
    return knob("STENCIL_NO_T2", 0) == 0;
}

// Steps per launch of the deep temporal-blocking family (kernels_strip.hip,
// kernels_temporalk.hip) in stencil_iterate, for explicit TEMPORALK and for
// AUTO on the 7-point star (STENCIL_NO_TK=1 or STENCIL_NO_T2=1 turn the
// latter off); 0 = not used.  K = STENCIL_TK_STEPS (3, 4 or 5), else the
// measured best (MI355X, tools/strip_ab.sh): 4 for fp64 (5: -3 % at 512^3,
// -5 % at 2048^2 x 512) and for small fp32 planes, 5 for fp32 planes of
// >= 1024^2 cells (+24 % at 2048^2 x 512, -9 % at 512^3).
int iterate_tk_steps(const stencil_problem& p) {
    if (!temporal2_supports(p)) return 0;
    if (p.kernel == STENCIL_KERNEL_AUTO) {
        if (!iterate_fused(p)) return 0;
        if (knob("STENCIL_NO_TK", 0) != 0) return 0;
    } else if (p.kernel != STENCIL_KERNEL_TEMPORALK) {
        return 0;
    }
    const int steps = api_knob("STENCIL_TK_STEPS", p.dtype == STENCIL_F32 && p.nx * p.ny >= (int64_t(1) << 20) ? 5 : 4);
    return steps >= 3 && steps <= 5 ? steps : 0;
}

// Sweeps per launch of the 27-point box in stencil_iterate (AUTO, or explicit
// TEMPORALK): K-step launches of kernels_boxk.hip, remainder as a pair / single
// (STENCIL_BOX_STEPS=3|4 forces K, 2: pairs only).  K = 3 beat pairs
// (profiles/r02e_ab_box_k3.log: 2048^2 x 256 fp64 717 vs 651 Gcell/s, fp32
// 1242 vs 1182).  K = 4: since round 3's box order the strip kernel runs it
// in 5 x 8 rows without spilling: 2048^2 x 256 fp64 1108 vs 743 (K = 3),
// fp32 1997 vs 1538, 512^3 fp64 1096 vs 870 (profiles/r03/r03k_ab_box*.txt);
// planes below 384^2 keep K = 3 (fewer, narrower tiles).  0 = not used.
int iterate_box_steps(const stencil_problem& p) {
    if (!box27_supports(p)) return 0;
    if (!(p.kernel == STENCIL_KERNEL_TEMPORALK || (p.kernel == STENCIL_KERNEL_AUTO && iterate_fused(p)))) return 0;
    const int steps = api_knob("STENCIL_BOX_STEPS", p.nx * p.ny >= int64_t(384) * 384 ? 4 : 3);
    return steps == 3 || steps == 4 ? steps : 0;
}

// The two-tier 7-point launch (8 sweeps, kernels_strip.hip TIER; DESIGN.md
// §9.1f) where the grid's tiles fit twice on the device: STENCIL_TK_TIER=1
// (experiment, debug library) until measured faster.
bool iterate_tier(const stencil_layout& l) {
    if (iterate_tk_steps(l.prob) != 4 || l.prob.dtype != STENCIL_F64) return false;
    if (knob("STENCIL_TK_TIER", 0) != 1) return false;
    return tier_eligible(l);
}

// 2D problems iterate K sweeps per launch with the tile resident in LDS
// (kernels_tb2d.hip) unless a single-sweep family is forced.
bool iterate_tb2d(const stencil_problem& p) {
    if (!tb2d_supports(p)) return false;
    if (p.kernel == STENCIL_KERNEL_TEMPORAL2 || p.kernel == STENCIL_KERNEL_PERSISTENT) return true;
    return p.kernel == STENCIL_KERNEL_AUTO && knob("STENCIL_NO_T2", 0) == 0;
}

// The whole 2D job as one persistent launch (kernels_tb2dp.hip): explicit
// PERSISTENT, or AUTO when STENCIL_TB2DP=1.  Falls back to the K-step launches
// when the tiles do not all fit on the GPU at once.
bool iterate_persistent(const stencil_problem& p) {
    if (!tb2dp_supports(p)) return false;
    if (p.kernel == STENCIL_KERNEL_PERSISTENT) return true;
    return p.kernel == STENCIL_KERNEL_AUTO && iterate_tb2d(p) && knob("STENCIL_TB2DP", 0) == 1;
}

int launch_single(const stencil_layout& l, const void* in, void* out, int64_t b, int64_t e, hipStream_t s) {
    if (sweep_family(l.prob) == STENCIL_KERNEL_ZMARCH)
        return zmarch_supports(l.prob) ? launch_zmarch(l, in, out, b, e, s) : launch_box27(l, in, out, b, e, 1, s);
    return launch_direct(l, in, out, b, e, s);
}

// Two fused sweeps.  27-point box: the separable-sum z-march
// (kernels_boxk.hip), K = 2.
int launch_fused(const stencil_layout& l, const void* in, void* out, int64_t b, int64_t e, hipStream_t s) {
    if (temporal2_supports(l.prob)) return launch_temporal2(l, in, out, b, e, s);
    return launch_boxk(l, in, out, b, e, 2, s);
}

inline hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

// ---- initial condition ----------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ void u01(uint64_t u, float& f) { f = float(u >> 40) * 0x1.0p-24f; }
__device__ __forceinline__ void u01(uint64_t u, double& d) { d = double(u >> 11) * 0x1.0p-53; }

// Every allocated element, grid-stride: a dispatch holds at most 2^32 - 1
// work-items per dimension (the AQL packet's grid size is 32-bit), and a
// 4096^3 fp32 grid has 17.5e9 elements -- a one-thread-per-element grid
// would be truncated modulo 2^32 and leave most planes unfilled.  Padding
// columns (outside the ghost ring) get 0; ghost cells follow
// stencil.cpp:190-207 generalised to 3D.
template <typename T>
__global__ void fill_initial_kernel(T* __restrict__ buf, Geom g, int64_t elems, int64_t row,
                                    int64_t rows, int64_t origin_x, int r, int zg, int dims, int kind,
                                    uint64_t seed) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < elems;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t pz = i / (row * rows);
        const int64_t rem = i - pz * row * rows;
        const int64_t py = rem / row;
        const int64_t px = rem - py * row;
        const int64_t x = px - origin_x, y = py - r, z = dims == 3 ? pz - zg : 0;
        T v = T(0);
        const bool in_x = x >= -r && x < g.nx + r;
        if (in_x) {
            const bool xghost = x < 0 || x >= g.nx;
            const bool interior = !xghost && y >= 0 && y < g.ny && z >= 0 && z < g.nz;
            if (xghost) {
                v = T(1);
            } else if (interior && kind == STENCIL_INIT_RANDOM) {
                const uint64_t lin = (uint64_t(z) * uint64_t(g.ny) + uint64_t(y)) * uint64_t(g.nx) + uint64_t(x);
                u01(splitmix64(seed + lin), v);
            }
        }
        buf[i] = v;
    }
}

// Deterministic per-plane sums: one workgroup per slow-axis index, fixed
// lane -> element mapping and a fixed tree, so equal grids give equal bits.
template <typename T>
__global__ void __launch_bounds__(256) plane_sums_kernel(const T* __restrict__ buf, Geom g, int dims,
                                                         double* __restrict__ out) {
    __shared__ double red[256];
    const int64_t s = blockIdx.x;
    const int64_t ny = dims == 3 ? g.ny : 1;
    const int64_t base = g.origin + (dims == 3 ? s * g.plane : s * g.row);
    double acc = 0.0;
    for (int64_t y = 0; y < ny; ++y)
        for (int64_t x = threadIdx.x; x < g.nx; x += 256) acc += double(buf[base + y * g.row + x]);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (int(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[s] = red[0];
}

// One lane polls two face counters (agent-scope relaxed loads: they bypass
// L1, MI355X_MICROARCH.md §visibility) until both reach their targets, so the
// kernels queued behind it on its stream (the RCCL send of the faces) start
// only then; the producers released before adding.  Gives up after 10 s of
// s_memrealtime (100 MHz) and sets *timeout instead of holding the queue.
// The flag is sticky: once a wait has given up, later waits on the same flag
// return at once, so a lost peer costs one timeout, not one per round (the
// job's run() then reports the failure).
__global__ void __launch_bounds__(64) wait_counters_kernel(const uint32_t* __restrict__ c, uint32_t tlo, uint32_t thi,
                                                           uint32_t* __restrict__ timeout) {
    if (threadIdx.x != 0) return;
    if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t a = __hip_atomic_load(&c[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t b = __hip_atomic_load(&c[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a >= tlo && b >= thi) return;
        // the host sets the flag to release a wait (a slab job that failed)
        if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > uint64_t(1000) * 1000 * 1000) {
            __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// The exchange-completion word of a slab (stencil_exchange_done): one lane's
// relaxed agent-scope vector store, queued behind the exchange's transfers on
// their stream (kernel boundaries order it after them); the gated launches
// poll it (kernels_strip.hip gate_wait).
__global__ void __launch_bounds__(64) exchange_done_kernel(uint32_t* __restrict__ word, uint32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Streaming copy used to calibrate attainable HBM bandwidth: 4 independent
// 16-B loads in flight per lane, one pass, no grid-stride loop.
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) copy_kernel(f32x4* __restrict__ dst, const f32x4* __restrict__ src,
                                                   int64_t n) {
    const int64_t base = int64_t(blockIdx.x) * 1024 + threadIdx.x;
    f32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k * 256 < n) v[k] = __builtin_nontemporal_load(src + base + k * 256);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k * 256 < n) __builtin_nontemporal_store(v[k], dst + base + k * 256);
}


}  // namespace
}  // namespace stencil

using namespace stencil;

namespace stencil {
int signal_launch_geometry(const stencil_layout& l, int64_t begin, int64_t end, int steps, int64_t* tiles,
                           int64_t* workgroups, int* slots) {
    LaunchInfo info;
    tl_dry_launch = &info;
    int nsig = 0;
    void* fake_out = reinterpret_cast<void*>(uintptr_t(1));  // never touched in a dry launch
    const int rc = box27_supports(l.prob)
                       ? launch_boxk_signal(l, nullptr, fake_out, begin, end, steps, nullptr, nullptr, &nsig, nullptr)
                       : launch_tkstrip_signal(l, nullptr, fake_out, begin, end, steps, nullptr, nullptr, &nsig, nullptr);
    tl_dry_launch = nullptr;
    if (rc != STENCIL_OK) return rc;
    if (info.steps == 0) return set_error(STENCIL_EUNSUPPORTED, "no face-signalled launch was described");
    *tiles = nsig;  // one face signal per tile and face
    *workgroups = info.workgroups;
    *slots = info.slots;
    return STENCIL_OK;
}
}  // namespace stencil

extern "C" {

const char* stencil_strerror(int code) {
    switch (code) {
    case STENCIL_OK: return "success";
    case STENCIL_EINVAL: return "invalid argument";
    case STENCIL_EHIP: return "HIP runtime error";
    case STENCIL_ENOMEM: return "out of device memory";
    case STENCIL_ENODEV: return "no usable GPU";
    case STENCIL_EUNSUPPORTED: return "unsupported combination";
    case STENCIL_ETIMEOUT: return "a device wait passed its deadline";
    default: return "unknown error";
    }
}

const char* stencil_last_error_message(void) { return g_last_msg; }
int stencil_last_error(void) { return g_last_code; }

constexpr int64_t kPitchPeriod = 32768;  // bytes (stencil_layout_init's pitch rule)

// The row-pitch rule (round 5): pitches of 32 KiB or more
// whose residue r modulo 32 KiB lies in [-512, +256] B run the K-step kernels
// 3-30 % slower; such a row is padded to residue 384 (r in [-256, 256]) or by
// 128 B (r in [-512, -257]: -512 measured fast at +128).  Residues -256 and
// -128 go to 384 too: 128 B more would land them on -128 / 0, inside the slow
// window.  Returns the bytes to add.
int64_t pitch_pad_bytes(int64_t pitch) {
    if (pitch < kPitchPeriod - 512) return 0;
    const int64_t r = pitch % kPitchPeriod;
    if (pitch >= kPitchPeriod && r <= 256) return 384 - r;
    if (r >= kPitchPeriod - 256) return kPitchPeriod - r + 384;
    if (r >= kPitchPeriod - 512) return 128;
    return 0;
}

int stencil_layout_init(const stencil_problem* prob, stencil_layout* out) {
    if (int rc = check_problem(prob)) return rc;
    if (!out) return set_error(STENCIL_EINVAL, "null layout");
    const stencil_problem& p = *prob;
    const int64_t r = p.radius;
    const int64_t align = 128 / int64_t(elem_size(p));  // elements per 128 B
    const int64_t origin_x = (r + align - 1) / align * align;
    stencil_layout l{};
    l.prob = p;
    l.row = (origin_x + p.nx + r + align - 1) / align * align;
    // Row pitches just below or above a multiple of 32 KiB run the K-step
    // kernels slower (4096-wide fp64, 33024 B: 1196-1238 Gcell/s against
    // 1246-1311 at 33152; 8160-wide fp64, 65536 B: 1063-1087 against
    // 1171-1262 with 128 B more; 8192-wide fp32, 33024 B: 2226 against 2531 at
    // 33152; 4000-wide fp64, 32256 B: -3 %): pitch_pad_bytes() moves such rows
    // to a residue measured fast.  Scans of 20 widths x 2 plane heights,
    // DESIGN.md §9.1i, profiles/r05/r05h_pitchscan_*, r05i_pitchscan_*.
    {
        const int64_t pitch = l.row * int64_t(elem_size(p));
        // STENCIL_ROW_RULE=0 (debug library, the pitch scans): the raw pitch
        if (knob("STENCIL_ROW_RULE", 1)) l.row += pitch_pad_bytes(pitch) / int64_t(elem_size(p));
    }
    // STENCIL_ROW_PAD (debug library, experiments): extra elements per row, in
    // whole 128-B units (the row-pitch scans)
    l.row += (std::max(0, knob("STENCIL_ROW_PAD", 0)) + align - 1) / align * align;
    l.rows = p.ny + 2 * r;
    l.plane = l.row * l.rows;
    l.zghost = p.dims == 3 ? std::max<int64_t>(r, p.halo) : 0;
    l.planes = p.dims == 3 ? p.nz + 2 * l.zghost : 1;
    l.origin = l.zghost * l.plane + r * l.row + origin_x;
    l.elems = l.plane * l.planes;
    l.bytes = l.elems * int64_t(elem_size(p));
    *out = l;
    clear_error();
    return STENCIL_OK;
}

int64_t stencil_slow_extent(const stencil_layout* l) {
    return l->prob.dims == 3 ? l->prob.nz : l->prob.ny;
}

int stencil_device_count(int* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (count) *count = n;
    if (n == 0) return set_error(STENCIL_ENODEV, "no HIP device visible");
    return STENCIL_OK;
}

int stencil_set_device(int device) {
    STENCIL_HIP_CHECK(hipSetDevice(device));
    return STENCIL_OK;
}

int stencil_synchronize(void* stream) {
    STENCIL_HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
    return STENCIL_OK;
}

int stencil_alloc(const stencil_layout* l, void** dev) {
    if (int rc = check_layout(l)) return rc;
    if (!dev) return set_error(STENCIL_EINVAL, "null out pointer");
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, size_t(l->bytes) + 256);  // tail pad for vector over-reads
    if (e != hipSuccess) return set_error(STENCIL_ENOMEM, "hipMalloc(%lld) failed: %s", (long long)l->bytes, hipGetErrorString(e));
    *dev = p;
    return STENCIL_OK;
}

int stencil_free(void* dev) {
    STENCIL_HIP_CHECK(hipFree(dev));
    return STENCIL_OK;
}

int stencil_fill_initial(const stencil_layout* l, void* dev, int init_kind, uint64_t seed, void* stream) {
    if (int rc = check_layout(l)) return rc;
    if (init_kind != STENCIL_INIT_REFERENCE && init_kind != STENCIL_INIT_RANDOM)
        return set_error(STENCIL_EINVAL, "bad init kind %d", init_kind);
    const Geom g = geom_of(*l);
    const int64_t r = l->prob.radius;
    const int64_t origin_x = l->origin - r * l->row - l->zghost * l->plane;
    const int64_t blocks = std::min<int64_t>((l->elems + 255) / 256, int64_t(1) << 22);  // <= 2^30 work-items
    if (l->prob.dtype == STENCIL_F32)
        hipLaunchKernelGGL(fill_initial_kernel<float>, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream),
                           static_cast<float*>(dev), g, l->elems, l->row, l->rows, origin_x, int(r),
                           int(l->zghost), l->prob.dims, init_kind, seed);
    else
        hipLaunchKernelGGL(fill_initial_kernel<double>, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream),
                           static_cast<double*>(dev), g, l->elems, l->row, l->rows, origin_x, int(r),
                           int(l->zghost), l->prob.dims, init_kind, seed);
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

static int copy_grid(const stencil_layout* l, void* dev, const void* host_src, void* host_dst,
                     int64_t host_row, int64_t host_rows, void* stream) {
    if (int rc = check_layout(l)) return rc;
    const stencil_problem& p = l->prob;
    const int64_t r = p.radius;
    const size_t es = elem_size(p);
    const int64_t width = p.nx + 2 * r, height = p.ny + 2 * r;
    if (host_row < width || host_rows < height) return set_error(STENCIL_EINVAL, "host array too small");
    // Host planes cover z = -r .. nz+r-1 (3D) or the single 2D plane; device
    // planes beyond the host's ghosts (zghost > r) are left untouched.
    const int64_t hplanes = p.dims == 3 ? p.nz + 2 * r : 1;
    for (int64_t hz = 0; hz < hplanes; ++hz) {
        const int64_t z = p.dims == 3 ? hz - r : 0;
        char* d = static_cast<char*>(dev) + size_t(l->origin + z * l->plane - r * l->row - r) * es;
        if (host_src) {
            const char* h = static_cast<const char*>(host_src) + size_t(hz * host_row * host_rows) * es;
            STENCIL_HIP_CHECK(hipMemcpy2DAsync(d, size_t(l->row) * es, h, size_t(host_row) * es, size_t(width) * es,
                                               size_t(height), hipMemcpyHostToDevice, as_stream(stream)));
        } else {
            char* h = static_cast<char*>(host_dst) + size_t(hz * host_row * host_rows) * es;
            STENCIL_HIP_CHECK(hipMemcpy2DAsync(h, size_t(host_row) * es, d, size_t(l->row) * es, size_t(width) * es,
                                               size_t(height), hipMemcpyDeviceToHost, as_stream(stream)));
        }
    }
    return STENCIL_OK;
}

int stencil_upload(const stencil_layout* l, void* dev, const void* host, int64_t host_row, int64_t host_rows,
                   void* stream) {
    return copy_grid(l, dev, host, nullptr, host_row, host_rows, stream);
}

int stencil_download(const stencil_layout* l, const void* dev, void* host, int64_t host_row, int64_t host_rows,
                     void* stream) {
    return copy_grid(l, const_cast<void*>(dev), nullptr, host, host_row, host_rows, stream);
}

int stencil_copy_planes(const stencil_layout* l, const void* src, int64_t src_first, void* dst, int64_t dst_first,
                        int64_t count, void* stream) {
    if (int rc = check_layout(l)) return rc;
    const int64_t r = l->prob.dims == 3 ? l->zghost : l->prob.radius;
    const int64_t n = stencil_slow_extent(l);
    if (count < 0 || src_first < -r || dst_first < -r || src_first + count > n + r || dst_first + count > n + r)
        return set_error(STENCIL_EINVAL, "plane range out of bounds");
    const size_t es = elem_size(l->prob);
    const int64_t unit = l->prob.dims == 3 ? l->plane : l->row;
    // First allocated element of slow-axis index k: for 3D the whole plane,
    // for 2D the whole padded row.
    const int64_t base = l->prob.dims == 3 ? l->zghost * l->plane : (l->origin - (l->origin % l->row));
    const char* s = static_cast<const char*>(src) + size_t(base + src_first * unit) * es;
    char* d = static_cast<char*>(dst) + size_t(base + dst_first * unit) * es;
    if (count == 0) return STENCIL_OK;
    STENCIL_HIP_CHECK(hipMemcpyAsync(d, s, size_t(count * unit) * es, hipMemcpyDeviceToDevice, as_stream(stream)));
    return STENCIL_OK;
}

int stencil_sweep(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end, void* stream) {
    if (int rc = check_layout(l)) return rc;
    // A 3D slab may also advance the halo planes of a face shared with a
    // neighbour (HALO_LO/HI) as deep as its ghost layers allow beyond the
    // stencil radius: two sweeps per 2-plane exchange (communication-avoiding
    // temporal blocking across slabs).
    const int64_t ext = l->prob.dims == 3 ? l->zghost - l->prob.radius : 0;
    const int64_t lo = (l->prob.flags & STENCIL_HALO_LO) ? -ext : 0;
    const int64_t hi = stencil_slow_extent(l) + ((l->prob.flags & STENCIL_HALO_HI) ? ext : 0);
    if (begin < lo || end > hi || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range [%lld, %lld) out of bounds [%lld, %lld)", (long long)begin,
                         (long long)end, (long long)lo, (long long)hi);
    if (in == out) return set_error(STENCIL_EINVAL, "in-place sweeps are not supported (Jacobi ping-pong)");
    const int rc = launch_single(*l, in, out, begin, end, as_stream(stream));
    if (rc == STENCIL_OK) clear_error();
    return rc;
}

int stencil_sweep2(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end, void* stream) {
    if (int rc = check_layout(l)) return rc;
    if (!fused_supported(l->prob)) return set_error(STENCIL_EUNSUPPORTED, "no fused two-step kernel for this problem");
    if (begin < 0 || end > stencil_slow_extent(l) || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range out of bounds");
    if (in == out) return set_error(STENCIL_EINVAL, "in-place sweeps are not supported");
    const int rc = launch_fused(*l, in, out, begin, end, as_stream(stream));
    if (rc == STENCIL_OK) clear_error();
    return rc;
}

int stencil_sweepk(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end, int32_t steps,
                   void* stream) {
    if (steps == 1) return stencil_sweep(l, in, out, begin, end, stream);
    if (steps == 2) return stencil_sweep2(l, in, out, begin, end, stream);
    if (int rc = check_layout(l)) return rc;
    if (steps < 3 || steps > 5) return set_error(STENCIL_EINVAL, "steps must be 1..5 (got %d)", steps);
    const bool box = box27_supports(l->prob);
    // the box's K = 5 strip shapes are debug configurations only (DESIGN.md
    // §9.2e: they lose to K = 4); the product library has no K = 5 box launch
    const int box_max = stencil_debug_knobs() ? 5 : 4;
    if (!temporal2_supports(l->prob) && !(box && steps <= box_max))
        return set_error(STENCIL_EUNSUPPORTED,
                         "3- to 5-step fused sweeps cover the 3D r=1 naive 7-point star (3..5) and box (3..%d) only",
                         box_max);
    if (begin < 0 || end > stencil_slow_extent(l) || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range out of bounds");
    if (in == out) return set_error(STENCIL_EINVAL, "in-place sweeps are not supported");
    const int rc = box ? launch_boxk(*l, in, out, begin, end, steps, as_stream(stream))
                       : launch_temporalk(*l, in, out, begin, end, steps, as_stream(stream));
    if (rc == STENCIL_OK) clear_error();
    return rc;
}

int stencil_sweepk_geometry(const stencil_layout* l, int64_t begin, int64_t end, int32_t steps, int64_t* workgroups,
                            int32_t* zchunk, int32_t* packed) {
    if (int rc = check_layout(l)) return rc;
    if (!temporal2_supports(l->prob) || steps < 3 || steps > 5)
        return set_error(STENCIL_EUNSUPPORTED, "geometry: the K-step kernel of the 3D r=1 7-point star, steps 3..5");
    if (begin < 0 || end > stencil_slow_extent(l) || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range out of bounds");
    if (knob("STENCIL_TK_STRIP", 1) == 0)  // the interleaved-row kernel has no dry mode
        return set_error(STENCIL_EUNSUPPORTED, "geometry: not the strip kernel (STENCIL_TK_STRIP=0)");
    LaunchInfo info;
    tl_dry_launch = &info;
    // in/out are never touched in a dry launch
    const int rc = launch_temporalk(*l, nullptr, reinterpret_cast<void*>(uintptr_t(1)), begin, end, steps, nullptr);
    tl_dry_launch = nullptr;
    if (rc != STENCIL_OK) return rc;
    if (info.steps == 0) return set_error(STENCIL_EUNSUPPORTED, "geometry: no strip launch was described");
    if (workgroups) *workgroups = info.workgroups;
    if (zchunk) *zchunk = info.zchunk;
    if (packed) *packed = info.packed;
    clear_error();
    return STENCIL_OK;
}


int stencil_sweepk_signal(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                          int32_t steps, uint32_t* counters, uint64_t* face_signal, int32_t* signals_per_face,
                          void* stream) {
    if (int rc = check_layout(l)) return rc;
    if (!counters) return set_error(STENCIL_EINVAL, "null counters");
    if (begin < 0 || end > stencil_slow_extent(l) || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range out of bounds");
    if (in == out) return set_error(STENCIL_EINVAL, "in-place sweeps are not supported");
    int nsig = 0;
    auto* fsig = reinterpret_cast<unsigned long long*>(face_signal);
    const int rc = box27_supports(l->prob)
                       ? launch_boxk_signal(*l, in, out, begin, end, steps, counters, fsig, &nsig, as_stream(stream))
                       : launch_tkstrip_signal(*l, in, out, begin, end, steps, counters, fsig, &nsig,
                                               as_stream(stream));
    if (rc == STENCIL_OK) {
        if (signals_per_face) *signals_per_face = nsig;
        clear_error();
    }
    return rc;
}

int stencil_sweepk_signal_gated(const stencil_layout* l, const void* in, void* out, int64_t begin, int64_t end,
                                int32_t steps, uint32_t* counters, uint64_t* face_signal, uint32_t gate_need,
                                uint32_t* release_flag, int32_t* signals_per_face, void* stream) {
    if (int rc = check_layout(l)) return rc;
    if (!counters) return set_error(STENCIL_EINVAL, "null counters");
    if (begin < 0 || end > stencil_slow_extent(l) || begin > end)
        return set_error(STENCIL_EINVAL, "sweep range out of bounds");
    if (in == out) return set_error(STENCIL_EINVAL, "in-place sweeps are not supported");
    if (box27_supports(l->prob)) return set_error(STENCIL_EUNSUPPORTED, "the halo-gated launch is the 7-point star's");
    int nsig = 0;
    StripGate gate;
    gate.word = counters + 3;
    gate.release = release_flag;
    gate.need = gate_need;
    const int rc = launch_tkstrip_signal(*l, in, out, begin, end, steps, counters,
                                         reinterpret_cast<unsigned long long*>(face_signal), &nsig,
                                         as_stream(stream), gate);
    if (rc == STENCIL_OK) {
        if (signals_per_face) *signals_per_face = nsig;
        clear_error();
    }
    return rc;
}

int stencil_exchange_done(uint32_t* counters, uint32_t value, void* stream) {
    clear_error();
    if (!counters) return set_error(STENCIL_EINVAL, "null counters");
    hipLaunchKernelGGL(exchange_done_kernel, dim3(1), dim3(64), 0, as_stream(stream), counters + 3, value);
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

int stencil_wait_counters(const uint32_t* counters, uint32_t target_lo, uint32_t target_hi, uint32_t* timeout_flag,
                          void* stream) {
    clear_error();
    if (!counters || !timeout_flag) return set_error(STENCIL_EINVAL, "null counters / flag");
    hipLaunchKernelGGL(wait_counters_kernel, dim3(1), dim3(64), 0, as_stream(stream), counters, target_lo, target_hi,
                       timeout_flag);
    STENCIL_LAUNCH_CHECK();
    return STENCIL_OK;
}

int stencil_face_signal_create(uint64_t** face_signal) {
    clear_error();
    if (!face_signal) return set_error(STENCIL_EINVAL, "null face_signal");
    *face_signal = nullptr;
    int dev = 0, ok = 0;
    STENCIL_HIP_CHECK(hipGetDevice(&dev));
    STENCIL_HIP_CHECK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, dev));
    if (!ok) return set_error(STENCIL_EUNSUPPORTED, "device cannot wait on stream values");
    void* p = nullptr;
    STENCIL_HIP_CHECK(hipExtMallocWithFlags(&p, sizeof(uint64_t), hipMallocSignalMemory));
    *face_signal = static_cast<uint64_t*>(p);
    return STENCIL_OK;
}

int stencil_face_signal_destroy(uint64_t* face_signal) {
    clear_error();
    if (face_signal) STENCIL_HIP_CHECK(hipFree(face_signal));
    return STENCIL_OK;
}

int stencil_face_signal_reset(uint64_t* face_signal, void* stream) {
    clear_error();
    if (!face_signal) return set_error(STENCIL_EINVAL, "null face_signal");
    STENCIL_HIP_CHECK(hipStreamWriteValue64(as_stream(stream), face_signal, 0, 0));
    return STENCIL_OK;
}

int stencil_face_signal_read(const uint64_t* face_signal, uint64_t* value) {
    clear_error();
    if (!face_signal || !value) return set_error(STENCIL_EINVAL, "null face_signal / value");
    STENCIL_HIP_CHECK(hipMemcpy(value, face_signal, sizeof(uint64_t), hipMemcpyDefault));
    return STENCIL_OK;
}

int stencil_wait_face_signal(const uint64_t* face_signal, uint64_t target, void* stream) {
    clear_error();
    if (!face_signal) return set_error(STENCIL_EINVAL, "null face_signal");
    STENCIL_HIP_CHECK(hipStreamWaitValue64(as_stream(stream), const_cast<uint64_t*>(face_signal), target,
                                           hipStreamWaitValueGte, ~uint64_t(0)));
    return STENCIL_OK;
}

int stencil_plan(const stencil_layout* l, uint32_t iterations, int64_t* launches, int32_t* kernel) {
    if (int rc = check_layout(l)) return rc;
    if (iterate_persistent(l->prob) && tb2dp_fits(*l)) {
        if (launches) *launches = iterations ? 1 : 0;
        if (kernel) *kernel = STENCIL_KERNEL_PERSISTENT;
        return STENCIL_OK;
    }
    if (iterate_tb2d(l->prob) && tb2d1_fits(*l)) {
        if (launches) *launches = iterations ? 1 : 0;
        if (kernel) *kernel = STENCIL_KERNEL_TEMPORAL2;
        return STENCIL_OK;
    }
    if (iterate_tb2d(l->prob)) {
        const int64_t k = tb2d_steps(*l, iterations);
        if (launches) *launches = (int64_t(iterations) + k - 1) / k;
        if (kernel) *kernel = STENCIL_KERNEL_TEMPORAL2;
        return STENCIL_OK;
    }
    const bool t2 = !iterate_tb2d(l->prob) && iterate_fused(l->prob);
    const int64_t kb = iterate_box_steps(l->prob);
    const int64_t k = kb ? kb : iterate_tk_steps(l->prob);
    int64_t n = iterations;
    int64_t tier = 0;  // two-tier launches of 8 sweeps
    if (iterate_tier(*l)) {
        tier = n / 8;
        n %= 8;
    }
    if (k) {
        const int64_t r = n % k;
        n = n / k + r / 2 + r % 2;
    } else if (t2) {
        n = n / 2 + n % 2;
    }
    if (launches) *launches = n + tier;
    if (kernel) *kernel = (k && !kb) ? STENCIL_KERNEL_TEMPORALK : t2 || kb ? STENCIL_KERNEL_TEMPORAL2 : sweep_family(l->prob);
    return STENCIL_OK;
}

// The device's clock settles over the first ~15 ms of a heavy stream of
// launches after the GPU has idled: launches run fast for a few, then up to
// 1.45x slower, then recover over ~30 launches (512^3 fp64 K = 4, 440-460 us
// steady; tools/ramp_probe.py, profiles/r04/r04a_ramp.txt -- not the data,
// not first touch: a fresh grid straight after streaming work runs steady
// from its first launch).  prepare() therefore runs the job's own launch
// (a -> b, `a` unchanged) for about this much device time after the shape's
// one-time choices; the caller's timed region then measures the settled state.
constexpr float kSettleMs = 25.f;
constexpr float kSettleMaxLaunches = 2048.f;  // a 14-us C1 launch needs ~1800 for 25 ms

int stencil_prepare(const stencil_layout* l, const void* a, void* b, void* stream) {
    return stencil_prepare2(l, a, b, stream, nullptr, nullptr);
}

int stencil_prepare2(const stencil_layout* l, const void* a, void* b, void* stream, int64_t* settle_launches,
                     float* settle_ms) {
    if (settle_launches) *settle_launches = 0;
    if (settle_ms) *settle_ms = 0.f;
    if (int rc = check_layout(l)) return rc;
    if (!a || !b || a == b) return set_error(STENCIL_EINVAL, "need two distinct grids");
    hipStream_t s = as_stream(stream);
    const int64_t n = stencil_slow_extent(l);
    // 2D K-step launches have no per-shape choice, but settle the clock the same way
    // (C1: a 100-sweep job is 10 launches of ~14 us, all inside the ramp otherwise)
    const bool t2 = !iterate_persistent(l->prob) && iterate_tb2d(l->prob) && !tb2d1_fits(*l);
    auto launch = [&]() -> int {
        if (t2) return launch_tb2d(*l, a, b, tb2d_steps(*l, 1000), s);
        if (const int k = iterate_tk_steps(l->prob)) return launch_temporalk(*l, a, b, 0, n, k, s);
        if (const int k = iterate_box_steps(l->prob)) return launch_boxk(*l, a, b, 0, n, k, s);
        return STENCIL_OK;
    };
    if (!t2 && (iterate_persistent(l->prob) || iterate_tb2d(l->prob))) return STENCIL_OK;
    if (!t2 && !iterate_tk_steps(l->prob) && !iterate_box_steps(l->prob)) return STENCIL_OK;
    int rc = launch();  // the shape's one-time choices (the z-chunk schedule trial)
    if (rc != STENCIL_OK) return rc;
    {
        // and those of the long-job plan (the XCD-patch tables' own trial), so
        // that neither trial runs inside the caller's timed job
        const SustainedScope sustained(true);
        if ((rc = launch()) != STENCIL_OK) return rc;
    }
    // settle: one timed launch, then as many as make kSettleMs of device time
    hipEvent_t e0 = nullptr, e1 = nullptr;
    STENCIL_HIP_CHECK(hipEventCreate(&e0));
    STENCIL_HIP_CHECK(hipEventCreate(&e1));
    float ms = 0.f;
    hipError_t e = hipEventRecord(e0, s);
    if (e == hipSuccess && (rc = launch()) == STENCIL_OK) {
        e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != STENCIL_OK) return rc;
    if (e != hipSuccess) return set_error(STENCIL_EHIP, "prepare: %s", hipGetErrorString(e));
    const int more = ms > 0.f ? int(std::min(kSettleMaxLaunches, kSettleMs / ms)) : 0;
    for (int i = 0; i < more && rc == STENCIL_OK; ++i) rc = launch();
    // what ran before the caller's timed region: the trial launch, the timed
    // one and `more` (their device time estimated from the timed one)
    if (settle_launches) *settle_launches = 3 + more;
    if (settle_ms) *settle_ms = ms * float(3 + more);
    if (rc == STENCIL_OK) clear_error();
    return rc;
}

int stencil_iterate(const stencil_layout* l, void* a, void* b, uint32_t iterations, void* stream, int* final_in_b,
                    float* elapsed_ms) {
    if (int rc = check_layout(l)) return rc;
    if (!a || !b || a == b) return set_error(STENCIL_EINVAL, "need two distinct grids");
    hipStream_t s = as_stream(stream);
    const SustainedScope sustained(iterations >= kSustainedSweeps);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (elapsed_ms) {
        STENCIL_HIP_CHECK(hipEventCreate(&e0));
        STENCIL_HIP_CHECK(hipEventCreate(&e1));
        STENCIL_HIP_CHECK(hipEventRecord(e0, s));
    }
    const int64_t n = stencil_slow_extent(l);
    const bool t2 = iterate_fused(l->prob);
    void* in = a;
    void* out = b;
    uint32_t i = 0;
    int rc = STENCIL_OK;
    if (iterate_persistent(l->prob)) {
        int fin = 0;
        rc = launch_tb2dp(*l, a, b, iterations, s, &fin);
        if (rc == STENCIL_OK) {
            i = iterations;
            if (fin) std::swap(in, out);  // `in` names the grid holding the result
        } else if (rc == STENCIL_EUNSUPPORTED) {
            rc = STENCIL_OK;  // tiles do not fit at once: K-step launches below
            clear_error();
        }
    }
    if (iterate_tb2d(l->prob) && rc == STENCIL_OK && i < iterations && tb2d1_fits(*l)) {
        // the whole grid in one workgroup's LDS: every sweep in one launch,
        // the result where the per-sweep ping-pong would leave it
        rc = launch_tb2d1(*l, in, (iterations - i) % 2 ? out : in, iterations - i, s);
        if (rc == STENCIL_OK) {
            if ((iterations - i) % 2) std::swap(in, out);
            i = iterations;
        }
    }
    if (iterate_tb2d(l->prob) && rc == STENCIL_OK) {
        const uint32_t k = uint32_t(tb2d_steps(*l, iterations));
        for (; i < iterations && rc == STENCIL_OK;) {
            const uint32_t n2 = std::min(k, iterations - i);
            rc = launch_tb2d(*l, in, out, int(n2), s);
            std::swap(in, out);
            i += n2;
        }
    }
    if (rc == STENCIL_OK && iterations - i >= 8 && iterate_tier(*l)) {
        TierJob tj;
        rc = tier_begin(*l, s, &tj);
        if (rc == STENCIL_EUNSUPPORTED) {  // the device's buffer is in use: K = 4 launches below
            rc = STENCIL_OK;
            clear_error();
        } else {
            for (; i + 8 <= iterations && rc == STENCIL_OK; i += 8) {
                rc = tier_launch(*l, in, out, &tj, s);
                std::swap(in, out);
            }
            bool failed = false;
            const int rc2 = tier_end(&tj, s, &failed);
            if (rc == STENCIL_OK) rc = rc2;
            if (rc == STENCIL_OK && failed)
                rc = set_error(STENCIL_EHIP, "two-tier launch: a plane hand-off wait gave up (were the workgroups "
                                             "not all resident -- another job on the GPU?); the grid is wrong");
        }
    }
    if (const uint32_t k = uint32_t(iterate_tk_steps(l->prob))) {
        for (; i + k <= iterations && rc == STENCIL_OK; i += k) {
            rc = launch_temporalk(*l, in, out, 0, n, int(k), s);
            std::swap(in, out);
        }
    }
    if (const uint32_t k = uint32_t(iterate_box_steps(l->prob))) {
        for (; i + k <= iterations && rc == STENCIL_OK; i += k) {
            rc = launch_boxk(*l, in, out, 0, n, int(k), s);
            std::swap(in, out);
        }
    }
    if (t2) {
        // A fused pair reads `in` and writes S(S(in)) to `out`, so the buffer
        // holding the result no longer follows the one-sweep parity rule; the
        // caller learns where it is through *final_in_b.
        for (; i + 2 <= iterations && rc == STENCIL_OK; i += 2) {
            rc = launch_fused(*l, in, out, 0, n, s);
            std::swap(in, out);
        }
    }
    for (; i < iterations && rc == STENCIL_OK; ++i) {
        rc = launch_single(*l, in, out, 0, n, s);
        std::swap(in, out);
    }
    if (rc != STENCIL_OK) return rc;
    if (final_in_b) *final_in_b = in == b ? 1 : 0;
    if (elapsed_ms) {
        STENCIL_HIP_CHECK(hipEventRecord(e1, s));
        STENCIL_HIP_CHECK(hipEventSynchronize(e1));
        STENCIL_HIP_CHECK(hipEventElapsedTime(elapsed_ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    clear_error();
    return STENCIL_OK;
}

// ---------------------------------------------------------------------------
// One resident grid (include/stencil_hip.h part 2b).  The reference keeps two
// owner buffers and swaps them every sweep (stencil.cpp:14-21, 88-92;
// boundary_matrix.hpp:59): at BASELINE config 3 (4096^3 fp32) that is 2 x 279
// GB, more than one MI355X holds.  Here one grid plus D spare planes below it:
// a pass of k fused sweeps writes plane z of the new grid into slot z - D
// (down pass) or, from there, back into slot z (up pass), as ceil(nz / S)
// launches over z-ranges of S = D - K*r planes (K = the deepest pass, r the
// radius: a pass reads K*r planes beyond its range), taken bottom-up on the
// down pass and top-down on the up pass.  A launch over [jS, jS + S) reads
// slots [jS - kr, jS + S + kr) and writes slots [jS - D, jS + S - D) (down):
// disjoint, and no later launch reads what it writes; the up pass mirrors it.  Same kernels, same arithmetic: bitwise
// the two-grid job.  Slots are indexed from the home grid's interior plane 0:
// the allocation holds slots [-D - zg, nz + zg), home = slot -zg.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace stencil {
namespace {

int rolling_steps(const stencil_problem& p) {
    if (const int k = iterate_tk_steps(p)) return k;
    if (const int k = iterate_box_steps(p)) return k;
    return iterate_fused(p) ? 2 : 1;
}

int check_rolling(const stencil_layout* l, int64_t shift) {
    if (int rc = check_layout(l)) return rc;
    const stencil_problem& p = l->prob;
    if (p.dims != 3) return set_error(STENCIL_EUNSUPPORTED, "rolling jobs cover 3D grids (z passes)");
    if (p.flags != 0) return set_error(STENCIL_EINVAL, "rolling jobs take no slab halo flags");
    const int64_t reach = int64_t(rolling_steps(p)) * p.radius;  // planes a pass reads beyond its range
    if (shift < reach + 1)
        return set_error(STENCIL_EINVAL, "shift must be at least %lld planes (got %lld)", (long long)(reach + 1),
                         (long long)shift);
    return STENCIL_OK;
}

}  // namespace
}  // namespace stencil

extern "C" {

int stencil_rolling_bytes(const stencil_layout* l, int64_t shift_planes, int64_t* bytes, int32_t* sweeps_per_pass) {
    if (int rc = check_rolling(l, shift_planes)) return rc;
    if (bytes) *bytes = (l->planes + shift_planes) * l->plane * int64_t(elem_size(l->prob)) + 256;
    if (sweeps_per_pass) *sweeps_per_pass = rolling_steps(l->prob);
    clear_error();
    return STENCIL_OK;
}

int stencil_rolling_init_margin(const stencil_layout* l, void* base, int64_t shift_planes, void* stream) {
    if (int rc = check_rolling(l, shift_planes)) return rc;
    if (!base) return set_error(STENCIL_EINVAL, "null grid");
    const size_t pe = size_t(l->plane) * elem_size(l->prob);
    char* home = static_cast<char*>(base) + size_t(shift_planes) * pe;
    const char* ghost = home + size_t(l->zghost + l->prob.nz) * pe;  // the home grid's top ghost plane
    for (int64_t i = 0; i < shift_planes; ++i)
        STENCIL_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(base) + size_t(i) * pe, ghost, pe, hipMemcpyDeviceToDevice,
                                         as_stream(stream)));
    clear_error();
    return STENCIL_OK;
}

int stencil_rolling_iterate(const stencil_layout* l, void* base, int64_t shift_planes, uint32_t iterations,
                            int32_t* position, void* stream, int64_t* launches, float* elapsed_ms) {
    if (int rc = check_rolling(l, shift_planes)) return rc;
    if (!base || !position || (*position != 0 && *position != 1))
        return set_error(STENCIL_EINVAL, "null grid or position not 0 (home) / 1 (shifted)");
    hipStream_t s = as_stream(stream);
    const stencil_problem& p = l->prob;
    const int64_t nz = p.nz, zg = l->zghost, D = shift_planes;
    const int K = rolling_steps(p);
    const int64_t S = D - int64_t(K) * p.radius;
    const size_t pe = size_t(l->plane) * elem_size(p);
    char* shifted = static_cast<char*>(base);
    char* home = shifted + size_t(D) * pe;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (elapsed_ms) {
        STENCIL_HIP_CHECK(hipEventCreate(&e0));
        STENCIL_HIP_CHECK(hipEventCreate(&e1));
        STENCIL_HIP_CHECK(hipEventRecord(e0, s));
    }
    int64_t n = 0;
    const int64_t J = nz > 0 ? (nz + S - 1) / S : 0;
    for (uint32_t done = 0; done < iterations;) {
        int k = int(std::min<uint32_t>(uint32_t(K), iterations - done));
        if (k == 2 && !fused_supported(p)) k = 1;
        const bool down = *position == 0;
        for (int64_t i = 0; i < J; ++i) {
            const int64_t j = down ? i : J - 1 - i;
            const int64_t b = j * S, e = std::min(nz, b + S);
            const int rc = down ? stencil_sweepk(l, home, shifted, b, e, k, stream)
                                : stencil_sweepk(l, shifted, home, b, e, k, stream);
            if (rc != STENCIL_OK) return rc;
            ++n;
        }
        // the slots the pass overwrote that are ghost planes of the grid it
        // produced: the shifted grid's top ghosts (from the home grid's,
        // never written) / the home grid's bottom ghosts (from the shifted
        // grid's, never written)
        if (down)
            STENCIL_HIP_CHECK(hipMemcpyAsync(shifted + size_t(zg + nz) * pe, home + size_t(zg + nz) * pe, size_t(zg) * pe,
                                             hipMemcpyDeviceToDevice, s));
        else
            STENCIL_HIP_CHECK(hipMemcpyAsync(home, shifted, size_t(zg) * pe, hipMemcpyDeviceToDevice, s));
        *position = down ? 1 : 0;
        done += uint32_t(k);
    }
    if (launches) *launches = n;
    if (elapsed_ms) {
        STENCIL_HIP_CHECK(hipEventRecord(e1, s));
        STENCIL_HIP_CHECK(hipEventSynchronize(e1));
        STENCIL_HIP_CHECK(hipEventElapsedTime(elapsed_ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    clear_error();
    return STENCIL_OK;
}

int stencil_plane_sums(const stencil_layout* l, const void* dev, double* plane_sums_host, void* stream) {
    if (int rc = check_layout(l)) return rc;
    const int64_t n = stencil_slow_extent(l);
    if (n == 0) return STENCIL_OK;
    double* d = nullptr;
    STENCIL_HIP_CHECK(hipMalloc(&d, size_t(n) * sizeof(double)));
    const Geom g = geom_of(*l);
    if (l->prob.dtype == STENCIL_F32)
        hipLaunchKernelGGL(plane_sums_kernel<float>, dim3(unsigned(n)), dim3(256), 0, as_stream(stream),
                           static_cast<const float*>(dev), g, l->prob.dims, d);
    else
        hipLaunchKernelGGL(plane_sums_kernel<double>, dim3(unsigned(n)), dim3(256), 0, as_stream(stream),
                           static_cast<const double*>(dev), g, l->prob.dims, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(plane_sums_host, d, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d);
    if (e != hipSuccess) return set_error(STENCIL_EHIP, "plane sums failed: %s", hipGetErrorString(e));
    return STENCIL_OK;
}

int stencil_copy_bandwidth(void* dst, const void* src, int64_t bytes, int reps, void* stream, float* elapsed_ms) {
    if (!dst || !src || bytes <= 0 || (bytes % 16) != 0 || reps <= 0) return set_error(STENCIL_EINVAL, "bad copy args");
    hipStream_t s = as_stream(stream);
    hipEvent_t e0, e1;
    STENCIL_HIP_CHECK(hipEventCreate(&e0));
    STENCIL_HIP_CHECK(hipEventCreate(&e1));
    const int64_t n = bytes / 16;
    const unsigned blocks = unsigned((n + 1023) / 1024);
    STENCIL_HIP_CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, s, static_cast<f32x4*>(dst),
                           static_cast<const f32x4*>(src), n);
    STENCIL_LAUNCH_CHECK();
    STENCIL_HIP_CHECK(hipEventRecord(e1, s));
    STENCIL_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    STENCIL_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (elapsed_ms) *elapsed_ms = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return STENCIL_OK;
}

// ---------------------------------------------------------------------------
// Reference-compatible entry points (stencil_slave.hpp:26-46).
//
// The Sunway kernels read `input`, sweep `iterations` times, and leave the
// final grid in `output` when the count is odd and in `input` when it is even
// (stencil_dma.cpp:556-557,567; stencil.cpp:88-92,134).  Ghost cells are
// never written.  Here: both host grids go to HBM, the GPU sweeps, the final
// grid comes back into the parity-selected host buffer.
// ---------------------------------------------------------------------------
static void reference_entry(StencilArguments* args, int order, bool rma) {
    clear_error();
    if (!args) { set_error(STENCIL_EINVAL, "null arguments"); return; }
    const StencilMatrixView& in = args->input;
    const StencilMatrixView& out = args->output;
    if (in.boundary_width != in.boundary_height || in.boundary_width == 0) {
        set_error(STENCIL_EINVAL, "boundary width and height must be equal and >= 1");
        return;
    }
    if (in.actual_width != out.actual_width || in.actual_height != out.actual_height ||
        in.boundary_width != out.boundary_width || in.data_stride != out.data_stride) {
        set_error(STENCIL_EINVAL, "input and output views differ in shape");
        return;
    }
    const int64_t r = int64_t(in.boundary_width);
    if (in.actual_width < size_t(2 * r) || in.actual_height < size_t(2 * r)) {
        set_error(STENCIL_EINVAL, "view smaller than its ghost ring");
        return;
    }
    const int64_t nx = int64_t(in.actual_width) - 2 * r, ny = int64_t(in.actual_height) - 2 * r;
    // The 64 workers take blocks (ROW, COL) in 0..7 of block_size^2 cells,
    // clipped at the edge; a block past the edge is empty and its worker
    // returns (block_subview, boundary_matrix.hpp:190-218; stencil_dma.cpp:
    // 404-415).  So only [0, 8b)^2 is ever computed: cells at or past 8b keep
    // their initial value and feed the computed ones as fixed neighbours.
    const int64_t reach = 8 * int64_t(args->block_size);
    const int64_t ex = std::min(nx, reach), ey = std::min(ny, reach);
    if (ex == 0 || ey == 0) return;
    stencil_problem p{};
    p.dims = 2;
    p.dtype = STENCIL_F32;
    p.shape = STENCIL_STAR;
    p.radius = int(r);
    p.order = order;
    p.kernel = STENCIL_KERNEL_AUTO;
    p.nx = ex;
    p.ny = ey;
    p.nz = 1;
    stencil_layout l;
    if (stencil_layout_init(&p, &l)) return;
    // Host staging of the computed sub-view incl. its ghost ring.  RMA does
    // not read ghosts: block column 7 / row 7 synthesise x-faces = 1 and
    // y-faces = 0 (stencil_rma.cpp:149-166), which differs from the host
    // cells at 8b when n > 8b.
    const int64_t hw = ex + 2 * r, hh = ey + 2 * r, stride = int64_t(in.data_stride);
    std::vector<float> ha(size_t(hw * hh)), hb(size_t(hw * hh));
    for (int64_t y = 0; y < hh; ++y) {
        std::memcpy(&ha[size_t(y * hw)], in.data + y * stride, size_t(hw) * sizeof(float));
        std::memcpy(&hb[size_t(y * hw)], out.data + y * stride, size_t(hw) * sizeof(float));
    }
    if (rma) {
        for (std::vector<float>* h : {&ha, &hb}) {
            if (ex < nx)
                for (int64_t y = r; y < ey + r; ++y) (*h)[size_t(y * hw + ex + r)] = 1.f;
            if (ey < ny)
                for (int64_t x = r; x < ex + r; ++x) (*h)[size_t((ey + r) * hw + x)] = 0.f;
        }
    }
    void* a = nullptr;
    void* b = nullptr;
    if (stencil_alloc(&l, &a)) return;
    if (stencil_alloc(&l, &b)) { (void)hipFree(a); return; }
    int final_in_b = 0;
    int rc = stencil_upload(&l, a, ha.data(), hw, hh, nullptr);
    if (!rc) rc = stencil_upload(&l, b, hb.data(), hw, hh, nullptr);
    if (!rc) rc = stencil_iterate(&l, a, b, args->iterations, nullptr, &final_in_b, nullptr);
    if (!rc) rc = stencil_download(&l, final_in_b ? b : a, ha.data(), hw, hh, nullptr);
    if (!rc) {
        hipError_t e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) rc = set_error(STENCIL_EHIP, "synchronize: %s", hipGetErrorString(e));
    }
    if (!rc) {
        // only the computed interior is written back: ghost cells are never
        // written (stencil_dma.cpp puts block interiors only)
        const StencilMatrixView& dst = (args->iterations & 1u) ? out : in;
        for (int64_t y = r; y < ey + r; ++y)
            std::memcpy(dst.data + y * stride + r, &ha[size_t(y * hw + r)], size_t(ex) * sizeof(float));
    }
    (void)hipFree(a);
    (void)hipFree(b);
}

void stencil_iterate_dma(StencilArguments* args) { reference_entry(args, STENCIL_ORDER_DMA, false); }
void stencil_iterate_dma_static_unroll(StencilArguments* args) { reference_entry(args, STENCIL_ORDER_NAIVE, false); }
void stencil_iterate_dma_slave_pack(StencilArguments* args) { reference_entry(args, STENCIL_ORDER_DMA, false); }
void stencil_iterate_rma(StencilArguments* args) { reference_entry(args, STENCIL_ORDER_DMA, true); }

}  // extern "C"
