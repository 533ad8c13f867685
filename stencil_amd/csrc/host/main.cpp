// main.cpp -- drop-in for the reference's stencil_main (src/main.cpp:12-62).
// Same control flow and byte-identical stdout lines, so run_expr.py's regex
// (run_expr.py:9) keeps matching; extra engine metrics go to lines that start
// with "[stencil-amd]" and do not match it.
#include <chrono>
#include <cstdio>
#include <exception>
#include <iostream>
#include <ratio>
#include <string>
#include <string_view>

#include "program_options.hpp"
#include "stencil.hpp"
#include "stencil_hip.h"

namespace {

int g_status = 0;

void run_test(std::string_view method_name, ProgramOptions const& options) {
    if (options.check_result) {
        std::cout << "Start to check the correctness of method " << method_name << ".\n";

        Stencil stencil(options);
        if (!stencil.run(method_name)) {
            std::cerr << "Unknown method: " << method_name << "\n";
            g_status = 2;
            return;
        }

        if (stencil.check_result()) {
            std::cout << "The results of method " << method_name << " is correct.\n";
        } else {
            std::cout << "The results of method " << method_name << " is incorrect.\n";
            g_status = 3;
            return;
        }
    }

    std::chrono::steady_clock::duration total_duration = {};
    double total_device_ms = 0.0;
    double cells = 0.0;

    for (unsigned i = 0; i != options.repeat_count; ++i) {
        Stencil stencil(options);
        auto const duration = stencil.run(method_name);
        if (duration && !options.bmp.empty() && i + 1 == options.repeat_count) {
            std::string path = options.bmp;
            if (options.method_names.size() > 1) path += "." + std::string(method_name) + ".bmp";
            if (!stencil.to_bmp(path)) {
                std::cerr << "could not write " << path << "\n";
                g_status = 4;
            }
        }
        if (!duration) {
            std::cerr << "Unknown method: " << method_name << "\n";
            g_status = 2;
            return;
        }
        total_duration += *duration;
        total_device_ms += stencil.last_device_ms();
        cells = stencil.cells();
        std::cout << method_name << " Method spent "
                  << static_cast<std::chrono::duration<double, std::milli>>(*duration).count() << "ms for "
                  << options.iterations << " iterations.\n";
    }

    if (options.repeat_count == 0) return;  // the reference divides by zero here
    std::cout << "The average time taken by " << method_name << " method is "
              << static_cast<std::chrono::duration<double, std::milli>>(total_duration / options.repeat_count).count()
              << "ms for " << options.iterations << " iterations.\n";

    const double dev_ms = total_device_ms / options.repeat_count;
    if (dev_ms > 0.0) {
        const double gcell = cells * options.iterations / (dev_ms * 1e-3) / 1e9;
        const double bytes_per_update = 2.0 * (options.fp64 ? 8.0 : 4.0);
        std::cout << "[stencil-amd] " << method_name << (method_name == "CPU" ? ": host " : ": device ") << dev_ms
                  << " ms, " << gcell
                  << " Gcell-updates/s, " << gcell * bytes_per_update << " GB/s algorithmic\n";
    }
}

void run_all_test(ProgramOptions const& options) {
    for (std::string const& method_name : options.method_names) {
        run_test(method_name, options);
    }
}

}  // namespace

int main(int argc, char** argv) {
    // Parse program arguments.
    if (auto options = ProgramOptions::parse(argc, argv)) {
        if (options->print_config) {
            std::cout << "matrix_size=" << options->matrix_size << " block_size=" << options->block_size
                      << " iterations=" << options->iterations << " radius=" << options->radius
                      << " repeat=" << options->repeat_count << " check=" << options->check_result
                      << " dims=" << options->dims << " nx=" << options->extent_x() << " ny=" << options->extent_y()
                      << " nz=" << options->extent_z() << " dtype=" << (options->fp64 ? "fp64" : "fp32")
                      << " shape=" << (options->box ? "box" : "star") << " kernel=" << options->kernel
                      << " init=" << (options->random_init ? "random" : "reference") << " gpus=" << options->gpus
                      << " exchange=" << (options->exchange_copy ? "copy" : "rccl") << " methods=";
            for (size_t i = 0; i < options->method_names.size(); ++i)
                std::cout << (i ? "," : "") << options->method_names[i];
            std::cout << "\n";
            return 0;
        }
        try {
            run_all_test(*options);
        } catch (std::exception const& e) {
            std::cerr << "error: " << e.what() << "\n";
            return 1;
        }
        return g_status;
    } else {
        return 1;
    }
}
