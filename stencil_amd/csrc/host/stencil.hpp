// stencil.hpp -- host engine, mirror of the reference's class Stencil
// (include/stencil/stencil.hpp:12-59, src/stencil/stencil.cpp).
//
// Same shape: initialize_matrix(), run(method) returning a steady_clock
// duration, run(name) through a name->method map, check_result() against
// the naive CPU sweep.  The "kernels" are GPU launches through the C-ABI in
// include/stencil_hip.h; this file includes no HIP header.
#pragma once

#include <chrono>
#include <optional>
#include <string>
#include <string_view>

#include "grid.hpp"
#include "program_options.hpp"

class Stencil {
public:
    /// Methods. The first four keep the reference's names
    /// (stencil.hpp:15-32, stencil.cpp:61-66); each computes in that
    /// reference variant's arithmetic order, on the GPU.
    enum InputMethod {
        DMA,                ///< stencil_dma.cpp order
        RMA,                ///< stencil_rma.cpp order (= DMA r=1 order)
        DMA_SLAVE_PACK,     ///< stencil_dma_slave_pack.cpp order (= DMA r=1 order)
        DMA_STATIC_UNROLL,  ///< naive order (bit-identical to check_result)
        HIP,                ///< naive order, fastest kernel for the problem (--kernel)
        HIP_DIRECT,         ///< naive order, general one-cell-per-lane kernel
        HIP_ZMARCH,         ///< naive order, 2.5D LDS/register z-marching kernel (3D r=1)
        HIP_TEMPORAL2,      ///< naive order, two fused time steps per launch
        HIP_TEMPORALK,      ///< naive order, 3 or 4 fused time steps per launch (7-point star)
        HIP_PERSISTENT,     ///< naive order, the whole 2D job in one launch (neighbour flags)
        HIP_MULTI_GPU,      ///< naive order, 3D z-slabs over --gpus GPUs, halos over RCCL (stencil_slab_*)
        CPU,                ///< the reference's CPU path: check_result's naive loop, timed, on the host
    };

    Stencil() = default;
    explicit Stencil(ProgramOptions options) : options(options) {}

    void initialize_matrix();

    auto run(InputMethod method) -> std::chrono::steady_clock::duration;
    /// nullopt for an unknown name (the reference asserts, stencil.cpp:69-70).
    auto run(std::string_view method_name) -> std::optional<std::chrono::steady_clock::duration>;

    auto check_result() const -> bool;

    /// Write the final grid of the last run as a 24-bit BMP (2D: the grid;
    /// 3D: the middle z plane), colour map of stencil.cpp:153-188.
    auto to_bmp(const std::string& path) const -> bool;

    /// Device time of the last run (hipEvents around the launches), ms.
    double last_device_ms() const { return device_ms; }
    /// Interior cell count (one iteration updates each once).
    double cells() const;

private:
    ProgramOptions options;
    BoundaryGrid<float> matrix32, result32;
    BoundaryGrid<double> matrix64, result64;
    double device_ms = 0.0;

    template <class T>
    auto run_typed(InputMethod method, BoundaryGrid<T>& matrix, BoundaryGrid<T>& result)
        -> std::chrono::steady_clock::duration;
    template <class T>
    auto run_slabs(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) -> std::chrono::steady_clock::duration;
    template <class T>
    bool check_typed(const BoundaryGrid<T>& matrix, const BoundaryGrid<T>& result) const;
    template <class T>
    bool naive_sweeps(BoundaryGrid<T>& a, BoundaryGrid<T>& b, unsigned iterations) const;
    template <class T>
    auto run_cpu(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) -> std::chrono::steady_clock::duration;
    template <class T>
    void init_typed(BoundaryGrid<T>& matrix, BoundaryGrid<T>& result) const;
    template <class T>
    bool bmp_typed(const BoundaryGrid<T>& matrix, const BoundaryGrid<T>& result, const std::string& path) const;
};
