// cumask_probe.hip -- which CUs does a CU-masked stream's kernel run on?
//
// hipExtStreamCreateWithCUMask takes a bit mask over the device's 256 CUs;
// slab.hip's STENCIL_SLAB_XCU assumes the driver stripes a queue's mask over
// the 8 XCDs (bit b -> XCD b % 8).  This probe launches many short workgroups
// on streams with a few mask patterns, records each workgroup's XCC_ID and
// HW_ID (SE / SH / CU fields) and prints the distinct CUs each mask reached.
//   hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe && tools/cumask_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <set>
#include <string>
#include <vector>

__global__ void __launch_bounds__(64) where_kernel(unsigned* out) {
    unsigned xcc = 0, hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(4);  // ~20 us: spread out
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc & 0xf;
        out[2 * blockIdx.x + 1] = hw;
    }
}

static void probe(const char* name, const std::vector<int>& bits, int cus) {
    std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
    for (int b : bits) mask[size_t(b / 32)] |= 1u << (b % 32);
    hipStream_t s;
    if (bits.empty()) {
        (void)hipStreamCreate(&s);
    } else if (hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()) != hipSuccess) {
        std::printf("%s: stream creation failed\n", name);
        return;
    }
    const int nb = 4096;
    unsigned* d = nullptr;
    (void)hipMalloc(&d, size_t(nb) * 2 * sizeof(unsigned));
    hipLaunchKernelGGL(where_kernel, dim3(nb), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    std::vector<unsigned> h(size_t(nb) * 2);
    (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::map<unsigned, std::set<std::string>> per_xcc;
    std::set<std::string> all;
    for (int i = 0; i < nb; ++i) {
        const unsigned xcc = h[2 * size_t(i)], hw = h[2 * size_t(i) + 1];
        const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        char key[64];
        std::snprintf(key, sizeof key, "x%u.se%u.sh%u.cu%u", xcc, se, sh, cu);
        per_xcc[xcc].insert(key);
        all.insert(key);
    }
    std::printf("%s: %zu distinct CUs over %zu XCDs\n", name, all.size(), per_xcc.size());
    for (auto& kv : per_xcc) {
        std::printf("  xcc %u: %zu CUs:", kv.first, kv.second.size());
        int shown = 0;
        for (auto& k : kv.second)
            if (shown++ < 6) std::printf(" %s", k.c_str());
        std::printf("%s\n", kv.second.size() > 6 ? " ..." : "");
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::printf("CUs: %d\n", cus);
    auto range = [](int a, int b) {
        std::vector<int> v;
        for (int i = a; i < b; ++i) v.push_back(i);
        return v;
    };
    probe("no mask", {}, cus);
    probe("bits 0-7", range(0, 8), cus);
    probe("bits 0-15", range(0, 16), cus);
    probe("bits 0-31", range(0, 32), cus);
    std::vector<int> stride32;
    for (int i = 0; i < cus; i += 32) stride32.push_back(i);
    probe("bits 0,32,..,224", stride32, cus);
    probe("bits 8-255 (complement of 0-7)", range(8, cus), cus);
    return 0;
}
