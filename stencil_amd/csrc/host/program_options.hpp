// program_options.hpp -- the reference's command-line surface
// (include/stencil/program_options.hpp:8-29, src/program_options.cpp:8-47),
// re-implemented without CLI11 (not available offline), plus long-only
// extension flags for what the reference cannot express (3D, fp64, shapes).
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

struct ProgramOptions {
    // ---- reference options (program_options.cpp:13-37) ----
    /// Side length of the matrix (-s, --matrix-size; required).
    unsigned matrix_size = 0;
    /// Block side length (-b, --block-size; required). The reference splits the
    /// grid into 8x8 CPE blocks of this size; the GPU engine picks its own
    /// tiling and accepts the value for compatibility.
    unsigned block_size = 0;
    /// Number of iterations (-i, --iteration; required).
    unsigned iterations = 0;
    /// Stencil radius (-r, --radius; default 1).
    unsigned radius = 1;
    /// Replicate runs per method (-R, --repeat; default 1).
    unsigned repeat_count = 1;
    /// Methods to run (-m, --methods; one or more; required).
    std::vector<std::string> method_names;
    /// Compare with the naive CPU sweep (-c, --check-result).
    bool check_result = false;

    // ---- extensions (long-only, no reference counterpart) ----
    int dims = 2;                  // --dims 2|3
    int64_t nx = -1, ny = -1, nz = -1;  // --nx/--ny/--nz (default: matrix_size)
    bool fp64 = false;             // --dtype fp32|fp64 (reference: fp32)
    bool box = false;              // --shape star|box
    std::string kernel = "auto";   // --kernel auto|direct|zmarch|temporal2|temporalk|persistent
    int device = 0;                // --device N
    bool random_init = false;      // --init reference|random
    uint64_t seed = 0x5EED;        // --seed N
    bool print_config = false;     // --print-config: print the parsed options and exit 0
    std::string bmp;               // --bmp FILE: dump the final grid of each method (f4)
    int gpus = 1;                  // --gpus N: 3D z-slab job over N GPUs (devices device .. device+N-1)
    bool exchange_copy = false;    // --exchange rccl|copy: halo transport of --gpus jobs
    bool share_device = false;     // --share-device: every slab on --device (needs --exchange copy)

    int64_t extent_x() const { return nx >= 0 ? nx : matrix_size; }
    int64_t extent_y() const { return ny >= 0 ? ny : matrix_size; }
    int64_t extent_z() const { return dims == 3 ? (nz >= 0 ? nz : matrix_size) : 1; }

    /// Parse the program arguments. Returns nullopt (after printing a message
    /// or the help text) on any error and on --help, like the reference
    /// (program_options.cpp:39-44), so main() exits with status 1.
    static auto parse(int argc, char** argv) -> std::optional<ProgramOptions>;
};
