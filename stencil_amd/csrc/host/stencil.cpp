// stencil.cpp -- host engine (mirror of src/stencil/stencil.cpp).
#include "stencil.hpp"

#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>
#include <algorithm>

#include "bmp.hpp"
#include "stencil_hip.h"

namespace {

void check(int rc, const char* what) {
    if (rc != STENCIL_OK)
        throw std::runtime_error(std::string(what) + ": " + stencil_strerror(rc) + ": " +
                                 stencil_last_error_message());
}

int kernel_of(const std::string& k) {
    if (k == "direct") return STENCIL_KERNEL_DIRECT;
    if (k == "zmarch") return STENCIL_KERNEL_ZMARCH;
    if (k == "temporal2") return STENCIL_KERNEL_TEMPORAL2;
    if (k == "temporalk") return STENCIL_KERNEL_TEMPORALK;
    if (k == "persistent") return STENCIL_KERNEL_PERSISTENT;
    return STENCIL_KERNEL_AUTO;
}

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
void u01(uint64_t u, float& f) { f = float(u >> 40) * 0x1.0p-24f; }
void u01(uint64_t u, double& d) { d = double(u >> 11) * 0x1.0p-53; }

// RAII device grid pair.
struct DeviceGrids {
    void* a = nullptr;
    void* b = nullptr;
    ~DeviceGrids() {
        if (a) stencil_free(a);
        if (b) stencil_free(b);
    }
};

}  // namespace

double Stencil::cells() const {
    return double(options.extent_x()) * double(options.extent_y()) * double(options.extent_z());
}

template <class T>
void Stencil::init_typed(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) const {
    // stencil.cpp:190-207: two zero-initialised buffers, x-ghost faces = 1.
    matrix = BoundaryGrid<T>(options.dims, options.extent_x(), options.extent_y(), options.extent_z(), options.radius);
    result = BoundaryGrid<T>(options.dims, options.extent_x(), options.extent_y(), options.extent_z(), options.radius);
    matrix.fill_x_boundaries(T(1));
    result.fill_x_boundaries(T(1));
    if (options.random_init) {
        // Extension: interior = splitmix64(seed + linear index) in [0,1),
        // identical to stencil_fill_initial(STENCIL_INIT_RANDOM).
        for (int64_t z = 0; z < matrix.depth(); ++z)
            for (int64_t y = 0; y < matrix.height(); ++y)
                for (int64_t x = 0; x < matrix.width(); ++x) {
                    const uint64_t lin = (uint64_t(z) * uint64_t(matrix.height()) + uint64_t(y)) * uint64_t(matrix.width()) + uint64_t(x);
                    T v;
                    u01(splitmix64(options.seed + lin), v);
                    matrix.elem_at(z, y, x) = v;
                    result.elem_at(z, y, x) = v;
                }
    }
}

void Stencil::initialize_matrix() {
    if (options.fp64) init_typed(matrix64, result64);
    else init_typed(matrix32, result32);
}

// The job as z-slabs over several GPUs (HIPMultiGPU, or any HIP method with
// --gpus N > 1): one host thread, stencil_slab_* (csrc/slab.hip).  Timed like
// the single-grid run: the rounds on grids already resident on the GPUs.
template <class T>
auto Stencil::run_slabs(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) -> std::chrono::steady_clock::duration {
    if (options.dims != 3) throw std::runtime_error("--gpus / HIPMultiGPU split 3D grids along z (use --dims 3)");
    if (options.share_device && !options.exchange_copy)
        throw std::runtime_error("--share-device needs --exchange copy (RCCL takes one slab per GPU)");
    stencil_problem p{};
    p.dims = 3;
    p.dtype = options.fp64 ? STENCIL_F64 : STENCIL_F32;
    p.shape = options.box ? STENCIL_BOX : STENCIL_STAR;
    p.radius = int(options.radius);
    p.order = STENCIL_ORDER_NAIVE;
    p.kernel = kernel_of(options.kernel);
    p.nx = matrix.width();
    p.ny = matrix.height();
    p.nz = matrix.depth();
    std::vector<int32_t> devices(size_t(options.gpus));
    for (int i = 0; i < options.gpus; ++i) devices[size_t(i)] = options.share_device ? options.device : options.device + i;
    struct Job {
        stencil_slab_job* j = nullptr;
        ~Job() { if (j) stencil_slab_destroy(j); }
    } job;
    check(stencil_slab_create(&p, options.gpus, devices.data(),
                              options.exchange_copy ? STENCIL_EXCHANGE_COPY : STENCIL_EXCHANGE_RCCL, 0, &job.j),
          "stencil_slab_create");
    check(stencil_slab_upload(job.j, matrix.data(), matrix.row_stride(), matrix.rows_with_boundary()), "slab upload");
    if (options.iterations > 0) {
        // untimed warm-up (code-object load, RCCL connection setup, the K-step
        // path's one-time schedule choices): one full round of K fused sweeps
        // and one shorter remainder round, then a fresh upload
        int32_t k = 1;
        check(stencil_slab_info(job.j, 0, nullptr, nullptr, nullptr, &k), "stencil_slab_info");
        check(stencil_slab_run(job.j, uint32_t(std::min<int64_t>(options.iterations, k) + 1), nullptr), "slab warm-up");
        check(stencil_slab_upload(job.j, matrix.data(), matrix.row_stride(), matrix.rows_with_boundary()), "slab upload");
    }
    float ms = 0.f;
    auto const start = std::chrono::steady_clock::now();
    check(stencil_slab_run(job.j, options.iterations, &ms), "stencil_slab_run");
    auto const end = std::chrono::steady_clock::now();
    device_ms = ms;
    BoundaryGrid<T>& dst = (options.iterations & 1u) ? result : matrix;  // parity rule, stencil.cpp:88-92,134
    check(stencil_slab_download(job.j, dst.data(), dst.row_stride(), dst.rows_with_boundary()), "slab download");
    return end - start;
}

template <class T>
auto Stencil::run_typed(InputMethod method, BoundaryGrid<T>& matrix, BoundaryGrid<T>& result)
    -> std::chrono::steady_clock::duration {
    if (method == CPU) return run_cpu(matrix, result);
    initialize_matrix();
    const bool ref_variant = method == DMA || method == DMA_STATIC_UNROLL || method == DMA_SLAVE_PACK || method == RMA;
    if (method == HIP_MULTI_GPU || (options.gpus > 1 && !ref_variant)) return run_slabs(matrix, result);

    stencil_problem p{};
    p.dims = options.dims;
    p.dtype = options.fp64 ? STENCIL_F64 : STENCIL_F32;
    p.shape = options.box ? STENCIL_BOX : STENCIL_STAR;
    p.radius = int(options.radius);
    p.order = (method == DMA || method == RMA || method == DMA_SLAVE_PACK) ? STENCIL_ORDER_DMA : STENCIL_ORDER_NAIVE;
    switch (method) {
    case HIP_DIRECT: p.kernel = STENCIL_KERNEL_DIRECT; break;
    case HIP_ZMARCH: p.kernel = STENCIL_KERNEL_ZMARCH; break;
    case HIP_TEMPORAL2: p.kernel = STENCIL_KERNEL_TEMPORAL2; break;
    case HIP_TEMPORALK: p.kernel = STENCIL_KERNEL_TEMPORALK; break;
    case HIP_PERSISTENT: p.kernel = STENCIL_KERNEL_PERSISTENT; break;
    case HIP: p.kernel = kernel_of(options.kernel); break;
    default: p.kernel = STENCIL_KERNEL_AUTO; break;
    }
    p.nx = matrix.width();
    p.ny = matrix.height();
    p.nz = matrix.depth();
    // The reference's methods compute blocks (ROW, COL) in 0..7 of -b x -b
    // cells only (block_subview, boundary_matrix.hpp:190-218): cells at or
    // past 8b keep their initial value.  RMA synthesises the x = 8b / y = 8b
    // faces as Dirichlet 1 / 0 instead of reading them (stencil_rma.cpp:149-166).
    const bool ref_method = method == DMA || method == DMA_STATIC_UNROLL || method == DMA_SLAVE_PACK || method == RMA;
    if (ref_method && options.dims == 2) {
        const int64_t reach = 8 * int64_t(options.block_size);
        p.nx = std::min<int64_t>(p.nx, reach);
        p.ny = std::min<int64_t>(p.ny, reach);
    }
    if (p.nx == 0 || p.ny == 0) return std::chrono::steady_clock::duration::zero();  // every block empty
    const int64_t r = options.radius, hw = p.nx + 2 * r, hh = p.ny + 2 * r;
    const bool synth = method == RMA && (p.nx < matrix.width() || p.ny < matrix.height());
    stencil_layout l;
    check(stencil_layout_init(&p, &l), "stencil_layout_init");
    std::vector<T> stage;  // RMA: the computed sub-view with its synthesised faces
    auto upload = [&](void* dev, const BoundaryGrid<T>& g) {
        if (!synth) {
            check(stencil_upload(&l, dev, g.data(), g.row_stride(), g.rows_with_boundary(), nullptr), "upload");
            return;
        }
        stage.assign(size_t(hw * hh), T(0));
        for (int64_t y = 0; y < hh; ++y)
            std::copy_n(g.data() + y * g.row_stride(), hw, stage.data() + y * hw);
        if (p.nx < matrix.width())
            for (int64_t y = r; y < p.ny + r; ++y) stage[size_t(y * hw + p.nx + r)] = T(1);
        if (p.ny < matrix.height())
            for (int64_t x = r; x < p.nx + r; ++x) stage[size_t((p.ny + r) * hw + x)] = T(0);
        check(stencil_upload(&l, dev, stage.data(), hw, hh, nullptr), "upload");
        check(stencil_synchronize(nullptr), "synchronize");
    };

    check(stencil_set_device(options.device), "stencil_set_device");
    DeviceGrids d;
    check(stencil_alloc(&l, &d.a), "stencil_alloc");
    check(stencil_alloc(&l, &d.b), "stencil_alloc");
    upload(d.a, matrix);
    upload(d.b, result);
    check(stencil_synchronize(nullptr), "synchronize");

    // Untimed warm-up: the first launch of a kernel in a process pays HIP's
    // lazy code-object load (~0.7 ms); the reference's timer has no such
    // term.  One sweep, then both grids are uploaded again.
    if (options.iterations > 0) {
        int fin = 0;
        check(stencil_iterate(&l, d.a, d.b, 1, nullptr, &fin, nullptr), "warm-up");
        // and the per-shape z-chunk schedule choice, timed on a shape's first
        // fused launch (kernels_strip.hip pick_schedule)
        check(stencil_prepare(&l, d.a, d.b, nullptr), "warm-up");
        upload(d.a, matrix);
        upload(d.b, result);
        check(stencil_synchronize(nullptr), "synchronize");
    }

    // Timed region, like stencil.cpp:33-54 (spawn ... join): the sweeps on
    // grids already resident in device memory, until they have completed.
    int final_in_b = 0;
    float ms = 0.f;
    auto const start = std::chrono::steady_clock::now();
    check(stencil_iterate(&l, d.a, d.b, options.iterations, nullptr, &final_in_b, &ms), "stencil_iterate");
    auto const end = std::chrono::steady_clock::now();
    device_ms = ms;

    // The final grid goes to the buffer the reference's parity rule names
    // (stencil.cpp:88-92,134): `result` after an odd count, else `matrix`.
    BoundaryGrid<T>& dst = (options.iterations & 1u) ? result : matrix;
    if (!synth) {
        check(stencil_download(&l, final_in_b ? d.b : d.a, dst.data(), dst.row_stride(), dst.rows_with_boundary(), nullptr),
              "download");
        check(stencil_synchronize(nullptr), "synchronize");
    } else {  // the computed interior only: the synthesised faces are not host cells
        check(stencil_download(&l, final_in_b ? d.b : d.a, stage.data(), hw, hh, nullptr), "download");
        check(stencil_synchronize(nullptr), "synchronize");
        for (int64_t y = r; y < p.ny + r; ++y)
            std::copy_n(stage.data() + y * hw + r, p.nx, dst.data() + y * dst.row_stride() + r);
    }
    return end - start;
}

auto Stencil::run(InputMethod method) -> std::chrono::steady_clock::duration {
    return options.fp64 ? run_typed(method, matrix64, result64) : run_typed(method, matrix32, result32);
}

auto Stencil::run(std::string_view method_name) -> std::optional<std::chrono::steady_clock::duration> {
    // Name -> method map (stencil.cpp:61-66) plus the GPU-native names.
    static std::unordered_map<std::string_view, InputMethod> const method_map = {
        {"DMA", DMA},
        {"DMAStaticUnroll", DMA_STATIC_UNROLL},
        {"DMASlavePack", DMA_SLAVE_PACK},
        {"RMA", RMA},
        {"HIP", HIP},
        {"HIPDirect", HIP_DIRECT},
        {"HIPZMarch", HIP_ZMARCH},
        {"HIPTemporal2", HIP_TEMPORAL2},
        {"HIPTemporalK", HIP_TEMPORALK},
        {"HIPPersistent", HIP_PERSISTENT},
        {"HIPMultiGPU", HIP_MULTI_GPU},
        {"CPU", CPU},
    };
    auto const iter = method_map.find(method_name);
    if (iter == method_map.end()) return std::nullopt;
    return run(iter->second);
}

// The naive CPU sweep of stencil.cpp:77-131 (check_result's loop), generalised
// to the engine's dims/shapes: `iterations` sweeps ping-ponging a -> b -> a
// ...; returns true when the final grid is in b (stencil.cpp:88-92,134).
// Naive order always (it is the reference's checker and its CPU path).
template <class T>
bool Stencil::naive_sweeps(BoundaryGrid<T>& a, BoundaryGrid<T>& b, unsigned iterations) const {
    BoundaryGrid<T>* in = &a;
    BoundaryGrid<T>* out = &b;
    const int r = int(options.radius);
    const int64_t sx = a.row_stride(), sxy = sx * a.rows_with_boundary();
    T avg;
    if (options.box) {
        int64_t w = 2 * r + 1, n = w * w * (options.dims == 3 ? w : 1);
        avg = T(1) / T(n - 1);
    } else {
        avg = T(1) / T(2 * options.dims * r);  // stencil.cpp:85-86
    }
    bool swapped = false;
    for (unsigned i = 0; i != iterations; ++i) {
        T* src = in->data();
        T* dst = out->data();
        for (int64_t z = 0; z < in->depth(); ++z)
            for (int64_t y = 0; y < in->height(); ++y)
                for (int64_t x = 0; x < in->width(); ++x) {
                    const int64_t zr = options.dims == 3 ? r : 0;
                    const int64_t c = ((z + zr) * in->rows_with_boundary() + (y + r)) * sx + (x + r);
                    T sum = T(0);
                    if (options.box) {
                        // separable partial sums (no reference code):
                        // 3D (P(-r) + .. + P(r)) - centre, 2D W + E
                        auto rowsum = [&](int64_t q) {
                            T acc = src[q - r];
                            for (int dx = -r + 1; dx <= r; ++dx) acc += src[q + dx];
                            return acc;
                        };
                        if (options.dims == 3) {
                            for (int dz = -r; dz <= r; ++dz) {
                                const int64_t pl = c + dz * sxy;
                                T term = rowsum(pl - r * sx);
                                for (int dy = -r + 1; dy <= r; ++dy) term += rowsum(pl + dy * sx);
                                sum = dz == -r ? term : sum + term;
                            }
                            sum = sum - src[c];
                        } else {
                            T w = rowsum(c - r * sx);
                            for (int dy = -r + 1; dy <= r; ++dy)
                                if (dy != 0) w += rowsum(c + dy * sx);
                            T e = src[c - r];
                            for (int dx = -r + 1; dx <= r; ++dx)
                                if (dx != 0) e += src[c + dx];
                            sum = w + e;
                        }
                    } else {
                        for (int k = r; k >= 1; --k) sum += src[c - k];       // left
                        for (int k = 1; k <= r; ++k) sum += src[c + k];       // right
                        for (int k = r; k >= 1; --k) sum += src[c - k * sx];  // top
                        for (int k = 1; k <= r; ++k) sum += src[c + k * sx];  // bottom
                        if (options.dims == 3) {
                            for (int k = r; k >= 1; --k) sum += src[c - k * sxy];
                            for (int k = 1; k <= r; ++k) sum += src[c + k * sxy];
                        }
                    }
                    dst[c] = sum * avg;
                }
        std::swap(in, out);
        swapped = !swapped;
    }
    return swapped;
}

// The method CPU: the reference's own CPU path (check_result's naive loop,
// stencil.cpp:77-131) as a timed method on the host, single-threaded like the
// reference; the final grid lands where the parity rule puts it.
template <class T>
auto Stencil::run_cpu(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) -> std::chrono::steady_clock::duration {
    initialize_matrix();
    auto const start = std::chrono::steady_clock::now();
    naive_sweeps(matrix, result, options.iterations);
    auto const end = std::chrono::steady_clock::now();
    device_ms = std::chrono::duration<double, std::milli>(end - start).count();
    return end - start;
}

// check_result (stencil.cpp:75-151): the naive CPU sweep from a fresh initial
// condition, compared with the method's final grid; absolute tolerance 1e-4,
// first mismatch printed in the reference's format.
template <class T>
bool Stencil::check_typed(const BoundaryGrid<T>& matrix, const BoundaryGrid<T>& result) const {
    BoundaryGrid<T> ga, gb;
    init_typed(ga, gb);
    const bool swapped = naive_sweeps(ga, gb, options.iterations);
    const BoundaryGrid<T>& in = swapped ? gb : ga;
    const BoundaryGrid<T>& compared = swapped ? result : matrix;
    for (int64_t z = 0; z < in.depth(); ++z)
        for (int64_t y = 0; y < in.height(); ++y)
            for (int64_t x = 0; x < in.width(); ++x) {
                const double a = double(in.elem_at(z, y, x)), b = double(compared.elem_at(z, y, x));
                if (std::fabs(a - b) >= 1e-4 || std::isnan(b)) {
                    if (options.dims == 3)
                        std::printf("invalid result at (%u, %u, %u): %.15f vs %.15f\n", unsigned(z), unsigned(y),
                                    unsigned(x), a, b);
                    else
                        std::printf("invalid result at (%u, %u): %.15f vs %.15f\n", unsigned(y), unsigned(x), a, b);
                    return false;
                }
            }
    return true;
}

auto Stencil::check_result() const -> bool {
    return options.fp64 ? check_typed(matrix64, result64) : check_typed(matrix32, result32);
}

template <class T>
bool Stencil::bmp_typed(const BoundaryGrid<T>& matrix, const BoundaryGrid<T>& result, const std::string& path) const {
    // The final grid is where the parity rule put it (stencil.cpp:134).
    const BoundaryGrid<T>& g = (options.iterations & 1u) ? result : matrix;
    if (g.empty()) return false;
    const int64_t z = g.depth() / 2;
    std::vector<BmpPixel> px;
    px.reserve(size_t(g.width() * g.height()));
    for (int64_t y = 0; y < g.height(); ++y)
        for (int64_t x = 0; x < g.width(); ++x) px.push_back(heat_color(double(g.elem_at(z, y, x))));
    return write_bmp24(path, uint32_t(g.width()), uint32_t(g.height()), px);
}

auto Stencil::to_bmp(const std::string& path) const -> bool {
    return options.fp64 ? bmp_typed(matrix64, result64, path) : bmp_typed(matrix32, result32, path);
}
