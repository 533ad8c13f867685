/*
 * oracle.c -- CPU restatement of the reference Jacobi sweep.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): never linked into the product.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static inline float u01_f32(uint64_t u) { return (float)(u >> 40) * 0x1.0p-24f; }
static inline double u01_f64(uint64_t u) { return (double)(u >> 11) * 0x1.0p-53; }

#define T float
#define SFX f32
#include "oracle_impl.inc"
#undef T
#undef SFX

#define T double
#define SFX f64
#include "oracle_impl.inc"
#undef T
#undef SFX

static int64_t slow_extent(const oracle_problem* p) { return p->dims == 3 ? p->nz : p->ny; }

int oracle_check(const oracle_problem* p) {
    if (!p) return -1;
    if (p->dims != 2 && p->dims != 3) return -2;
    if (p->dtype != ORACLE_F32 && p->dtype != ORACLE_F64) return -3;
    if (p->shape != ORACLE_STAR && p->shape != ORACLE_BOX) return -4;
    if (p->radius < 1) return -5;
    if (p->order != ORACLE_ORDER_NAIVE && p->order != ORACLE_ORDER_DMA && p->order != ORACLE_ORDER_LEX) return -6;
    if (p->order == ORACLE_ORDER_DMA && (p->dims != 2 || p->shape != ORACLE_STAR)) return -6;
    if (p->order == ORACLE_ORDER_LEX && p->shape != ORACLE_BOX) return -6;
    if (p->nx < 0 || p->ny < 0 || (p->dims == 3 && p->nz < 0)) return -7;
    return 0;
}

int64_t oracle_elems(const oracle_problem* p) {
    const int64_t r = p->radius;
    const int64_t sz = p->dims == 3 ? p->nz + 2 * r : 1;
    return (p->nx + 2 * r) * (p->ny + 2 * r) * sz;
}

int oracle_init(const oracle_problem* p, int init_kind, uint64_t seed, void* buf) {
    int rc = oracle_check(p);
    if (rc) return rc;
    if (p->dtype == ORACLE_F32)
        init_f32(p, init_kind, seed, (float*)buf);
    else
        init_f64(p, init_kind, seed, (double*)buf);
    return 0;
}

int oracle_sweep(const oracle_problem* p, const void* in, void* out, int64_t begin, int64_t end, int nthreads) {
    int rc = oracle_check(p);
    if (rc) return rc;
    if (begin < 0 || end > slow_extent(p) || begin > end) return -8;
    if (p->dtype == ORACLE_F32)
        sweep_f32(p, (const float*)in, (float*)out, begin, end, nthreads);
    else
        sweep_f64(p, (const double*)in, (double*)out, begin, end, nthreads);
    return 0;
}

int oracle_run(const oracle_problem* p, uint32_t iterations, void* a, void* b, int nthreads) {
    int rc = oracle_check(p);
    if (rc) return rc;
    void* in = a;
    void* out = b;
    int swapped = 0;
    for (uint32_t i = 0; i != iterations; ++i) {
        oracle_sweep(p, in, out, 0, slow_extent(p), nthreads);
        void* t = in;
        in = out;
        out = t;
        swapped = !swapped;
    }
    return swapped;
}

#define FOR_INTERIOR(p, BODY)                                                                   \
    do {                                                                                        \
        const int64_t r_ = (p)->radius;                                                         \
        const int64_t sx_ = (p)->nx + 2 * r_, sy_ = (p)->ny + 2 * r_;                           \
        const int64_t nz_ = (p)->dims == 3 ? (p)->nz : 1, zr_ = (p)->dims == 3 ? r_ : 0;        \
        for (int64_t z_ = 0; z_ < nz_; ++z_)                                                    \
            for (int64_t y_ = 0; y_ < (p)->ny; ++y_) {                                          \
                const int64_t row_ = ((z_ + zr_) * sy_ + (y_ + r_)) * sx_ + r_;                 \
                for (int64_t x_ = 0; x_ < (p)->nx; ++x_) {                                      \
                    const int64_t idx = row_ + x_;                                              \
                    BODY                                                                        \
                }                                                                               \
            }                                                                                   \
    } while (0)

uint64_t oracle_fnv1a64_interior(const oracle_problem* p, const void* buf) {
    uint64_t h = 0xcbf29ce484222325ULL;
    const size_t es = p->dtype == ORACLE_F32 ? 4 : 8;
    const unsigned char* base = (const unsigned char*)buf;
    FOR_INTERIOR(p, {
        const unsigned char* e = base + (size_t)idx * es;
        for (size_t k = 0; k < es; ++k) {
            h ^= e[k];
            h *= 0x100000001b3ULL;
        }
    });
    return h;
}

double oracle_sum_interior(const oracle_problem* p, const void* buf) {
    double s = 0.0;
    if (p->dtype == ORACLE_F32) {
        const float* f = (const float*)buf;
        FOR_INTERIOR(p, { s += (double)f[idx]; });
    } else {
        const double* d = (const double*)buf;
        FOR_INTERIOR(p, { s += d[idx]; });
    }
    return s;
}

int oracle_copy_interior(const oracle_problem* p, const void* buf, void* dst) {
    const size_t es = p->dtype == ORACLE_F32 ? 4 : 8;
    const unsigned char* base = (const unsigned char*)buf;
    unsigned char* o = (unsigned char*)dst;
    FOR_INTERIOR(p, {
        memcpy(o, base + (size_t)idx * es, es);
        o += es;
    });
    return 0;
}
