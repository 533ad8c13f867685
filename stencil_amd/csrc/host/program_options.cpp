// program_options.cpp -- CLI11-compatible parser for the reference's flags
// (src/program_options.cpp:8-47): same short/long names, required-ness,
// defaults, multi-value -m, boolean -c, "--name=value" and "-sVALUE" forms,
// and exit status 1 on any error or --help.  Exact CLI11 message strings are
// not reproduced (CLI11 is not available to compare against).
#include "program_options.hpp"

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <sstream>

namespace {

enum class Kind { Unsigned, Int64, Int, Str, Strs, Flag };

struct Opt {
    char shortname;  // 0 = long-only
    const char* longname;
    Kind kind;
    bool required;
    const char* help;
    std::function<bool(const std::string&)> set;  // returns false on bad value
    bool seen = false;
};

bool parse_unsigned(const std::string& s, unsigned& out) {
    if (s.empty() || s[0] == '-' || s[0] == '+') return false;
    errno = 0;
    char* end = nullptr;
    unsigned long long v = std::strtoull(s.c_str(), &end, 10);
    if (errno || *end || v > 0xFFFFFFFFull) return false;
    out = unsigned(v);
    return true;
}

bool parse_i64(const std::string& s, int64_t& out) {
    if (s.empty()) return false;
    errno = 0;
    char* end = nullptr;
    long long v = std::strtoll(s.c_str(), &end, 10);
    if (errno || *end) return false;
    out = v;
    return true;
}

bool looks_like_option(const std::string& a) {
    if (a.size() < 2 || a[0] != '-') return false;
    // "-5" style negative numbers are values, as in CLI11.
    return !(std::isdigit(static_cast<unsigned char>(a[1])) || a[1] == '.');
}

void print_help(const std::vector<Opt>& opts, const char* prog) {
    std::cout << "Usage: " << prog << " [OPTIONS]\n\nOptions:\n  -h,--help                   Print this help message and exit\n";
    for (const Opt& o : opts) {
        std::ostringstream name;
        name << "  ";
        if (o.shortname) name << '-' << o.shortname << ',';
        name << "--" << o.longname;
        std::string n = name.str();
        if (n.size() < 30) n.resize(30, ' ');
        std::cout << n << o.help << (o.required ? " REQUIRED" : "") << '\n';
    }
}

}  // namespace

auto ProgramOptions::parse(int argc, char** argv) -> std::optional<ProgramOptions> {
    ProgramOptions r{};
    bool methods_cleared = false;
    std::vector<Opt> opts = {
        {'s', "matrix-size", Kind::Unsigned, true, "The side length of the input matrix.",
         [&](const std::string& v) { return parse_unsigned(v, r.matrix_size); }},
        {'i', "iteration", Kind::Unsigned, true, "The number of iterations.",
         [&](const std::string& v) { return parse_unsigned(v, r.iterations); }},
        {'b', "block-size", Kind::Unsigned, true, "The side length of the block into which the matrix is divided.",
         [&](const std::string& v) { return parse_unsigned(v, r.block_size); }},
        {'r', "radius", Kind::Unsigned, false, "The radius of the stencil shape. (default 1)",
         [&](const std::string& v) { return parse_unsigned(v, r.radius); }},
        {'R', "repeat", Kind::Unsigned, false, "The number of replicate runs for each method. (default 1)",
         [&](const std::string& v) { return parse_unsigned(v, r.repeat_count); }},
        {'m', "methods", Kind::Strs, true, "List of methods to be tested.",
         [&](const std::string& v) {
             if (!methods_cleared) { r.method_names.clear(); methods_cleared = true; }
             r.method_names.push_back(v);
             return true;
         }},
        {'c', "check-result", Kind::Flag, false, "Whether to compare the result with the result of the naive implementation.",
         [&](const std::string&) { r.check_result = true; return true; }},
        // ---- extensions ----
        {0, "dims", Kind::Int, false, "[ext] Grid dimensionality: 2 (reference) or 3.",
         [&](const std::string& v) { int64_t x; if (!parse_i64(v, x) || (x != 2 && x != 3)) return false; r.dims = int(x); return true; }},
        {0, "nx", Kind::Int64, false, "[ext] Interior extent along x (default: matrix size).",
         [&](const std::string& v) { return parse_i64(v, r.nx) && r.nx >= 0; }},
        {0, "ny", Kind::Int64, false, "[ext] Interior extent along y (default: matrix size).",
         [&](const std::string& v) { return parse_i64(v, r.ny) && r.ny >= 0; }},
        {0, "nz", Kind::Int64, false, "[ext] Interior extent along z, 3D only (default: matrix size).",
         [&](const std::string& v) { return parse_i64(v, r.nz) && r.nz >= 0; }},
        {0, "dtype", Kind::Str, false, "[ext] Element type: fp32 (reference) or fp64.",
         [&](const std::string& v) { if (v != "fp32" && v != "fp64") return false; r.fp64 = v == "fp64"; return true; }},
        {0, "shape", Kind::Str, false, "[ext] Neighbourhood: star (reference) or box.",
         [&](const std::string& v) { if (v != "star" && v != "box") return false; r.box = v == "box"; return true; }},
        {0, "points", Kind::Int, false, "[ext] Shorthand: 5 (2D r1), 9 (2D r2), 7 (3D r1), 13 (3D r2), 27 (3D box r1).",
         [&](const std::string& v) {
             int64_t p;
             if (!parse_i64(v, p)) return false;
             switch (p) {
             case 5: r.dims = 2; r.radius = 1; r.box = false; return true;
             case 9: r.dims = 2; r.radius = 2; r.box = false; return true;
             case 7: r.dims = 3; r.radius = 1; r.box = false; return true;
             case 13: r.dims = 3; r.radius = 2; r.box = false; return true;
             case 27: r.dims = 3; r.radius = 1; r.box = true; return true;
             default: return false;
             }
         }},
        {0, "kernel", Kind::Str, false, "[ext] GPU kernel family: auto, direct, zmarch, temporal2, temporalk, persistent.",
         [&](const std::string& v) { if (v != "auto" && v != "direct" && v != "zmarch" && v != "temporal2" && v != "temporalk" && v != "persistent") return false; r.kernel = v; return true; }},
        {0, "device", Kind::Int, false, "[ext] HIP device index.",
         [&](const std::string& v) { int64_t d; if (!parse_i64(v, d) || d < 0) return false; r.device = int(d); return true; }},
        {0, "init", Kind::Str, false, "[ext] Initial interior: reference (zeros) or random.",
         [&](const std::string& v) { if (v != "reference" && v != "random") return false; r.random_init = v == "random"; return true; }},
        {0, "print-config", Kind::Flag, false, "[ext] Print the parsed options and exit.",
         [&](const std::string&) { r.print_config = true; return true; }},
        {0, "bmp", Kind::Str, false, "[ext] Write the final grid of each method as a BMP (FILE, or FILE.<method>.bmp for several methods).",
         [&](const std::string& v) { r.bmp = v; return !v.empty(); }},
        {0, "seed", Kind::Int64, false, "[ext] Seed of --init random.",
         [&](const std::string& v) { int64_t s; if (!parse_i64(v, s)) return false; r.seed = uint64_t(s); return true; }},
        {0, "gpus", Kind::Int, false, "[ext] 3D: split the grid into z-slabs over N GPUs (one host thread, RCCL halos).",
         [&](const std::string& v) { int64_t g; if (!parse_i64(v, g) || g < 1 || g > 64) return false; r.gpus = int(g); return true; }},
        {0, "exchange", Kind::Str, false, "[ext] Halo transport of --gpus jobs: rccl (default) or copy (device copies).",
         [&](const std::string& v) { if (v != "rccl" && v != "copy") return false; r.exchange_copy = v == "copy"; return true; }},
        {0, "share-device", Kind::Flag, false, "[ext] Put every slab of a --gpus job on --device (rehearsal; --exchange copy).",
         [&](const std::string&) { r.share_device = true; return true; }},
    };

    auto find_long = [&](const std::string& n) -> Opt* {
        for (Opt& o : opts) if (n == o.longname) return &o;
        return nullptr;
    };
    auto find_short = [&](char c) -> Opt* {
        for (Opt& o : opts) if (o.shortname == c) return &o;
        return nullptr;
    };
    auto fail = [&](const std::string& msg) -> std::optional<ProgramOptions> {
        std::cerr << msg << "\nRun with --help for more information.\n";
        return std::nullopt;
    };

    const char* prog = argc > 0 ? argv[0] : "stencil_main";
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-h" || a == "--help") {
            print_help(opts, prog);
            return std::nullopt;
        }
        Opt* o = nullptr;
        std::string inline_val;
        bool has_inline = false;
        if (a.rfind("--", 0) == 0 && a.size() > 2) {
            std::string name = a.substr(2);
            auto eq = name.find('=');
            if (eq != std::string::npos) { inline_val = name.substr(eq + 1); name = name.substr(0, eq); has_inline = true; }
            o = find_long(name);
        } else if (looks_like_option(a)) {
            o = find_short(a[1]);
            if (o && a.size() > 2) {
                inline_val = a.substr(2);
                if (!inline_val.empty() && inline_val[0] == '=') inline_val = inline_val.substr(1);
                has_inline = true;
            }
        } else {
            return fail("The following argument was not expected: " + a);
        }
        if (!o) return fail("The following argument was not expected: " + a);
        o->seen = true;
        if (o->kind == Kind::Flag) {
            if (has_inline && inline_val != "true" && inline_val != "1")
                return fail("--" + std::string(o->longname) + " is a flag and takes no value");
            o->set("");
            continue;
        }
        if (o->kind == Kind::Strs) {
            int taken = 0;
            if (has_inline) { o->set(inline_val); ++taken; }
            while (i + 1 < argc && !looks_like_option(argv[i + 1])) { o->set(argv[++i]); ++taken; }
            if (!taken) return fail("--" + std::string(o->longname) + ": at least one value is required");
            continue;
        }
        std::string v;
        if (has_inline) v = inline_val;
        else if (i + 1 < argc) v = argv[++i];
        else return fail("--" + std::string(o->longname) + ": 1 required value missing");
        if (!o->set(v)) return fail("--" + std::string(o->longname) + ": invalid value '" + v + "'");
    }
    for (const Opt& o : opts)
        if (o.required && !o.seen) return fail("--" + std::string(o.longname) + " is required");
    return r;
}
