// grid.hpp -- host-side ghost-padded grid, the 2D/3D generalisation of the
// reference's detail::BoundaryMatrix (include/stencil/boundary_matrix.hpp:31-238).
//
// Dense row-major storage, x fastest, ghost ring of width r on every axis the
// grid has: row stride = nx + 2r (as _data_stride = _actual_width, :58),
// rows per plane = ny + 2r, planes = nz + 2r (3D) or 1 (2D).  This is the
// host image; the device copy uses the padded layout of stencil_layout_init
// and transfers go through stencil_upload/stencil_download.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>

template <class T>
class BoundaryGrid {
public:
    using value_type = T;

    BoundaryGrid() = default;
    BoundaryGrid(int dims, int64_t nx, int64_t ny, int64_t nz, unsigned r)
        : dims_(dims), nx_(nx), ny_(ny), nz_(dims == 3 ? nz : 1), r_(r),
          data_(std::make_unique<T[]>(size_t(elems_with_boundary()))) {}  // zero-initialised

    int dims() const { return dims_; }
    int64_t width() const { return nx_; }
    int64_t height() const { return ny_; }
    int64_t depth() const { return nz_; }
    unsigned boundary() const { return r_; }
    int64_t row_stride() const { return nx_ + 2 * int64_t(r_); }
    int64_t rows_with_boundary() const { return ny_ + 2 * int64_t(r_); }
    int64_t planes_with_boundary() const { return dims_ == 3 ? nz_ + 2 * int64_t(r_) : 1; }
    int64_t elems_with_boundary() const { return row_stride() * rows_with_boundary() * planes_with_boundary(); }
    bool empty() const { return nx_ == 0 || ny_ == 0 || nz_ == 0; }

    T* data() const { return data_.get(); }

    // Coordinates include the ghost ring (0 .. n+2r-1), as elem_with_boundary_at (:115-118).
    T& elem_with_boundary_at(int64_t z, int64_t y, int64_t x) const {
        return data_[size_t((z * rows_with_boundary() + y) * row_stride() + x)];
    }
    // Interior coordinates (0 .. n-1), as elem_at (:120-123).
    T& elem_at(int64_t z, int64_t y, int64_t x) const {
        const int64_t zr = dims_ == 3 ? r_ : 0;
        return elem_with_boundary_at(z + zr, y + r_, x + r_);
    }

    // The reference's boundary condition (stencil.cpp:199-206 with
    // fill_boundary Left/Right over the full height incl. corners,
    // boundary_matrix.hpp:129-145), generalised: every x-ghost cell = value.
    void fill_x_boundaries(T value) {
        for (int64_t z = 0; z < planes_with_boundary(); ++z)
            for (int64_t y = 0; y < rows_with_boundary(); ++y)
                for (int64_t x = 0; x < row_stride(); ++x)
                    if (x < int64_t(r_) || x >= nx_ + int64_t(r_)) elem_with_boundary_at(z, y, x) = value;
    }

private:
    int dims_ = 2;
    int64_t nx_ = 0, ny_ = 0, nz_ = 1;
    unsigned r_ = 0;
    std::unique_ptr<T[]> data_;
};
