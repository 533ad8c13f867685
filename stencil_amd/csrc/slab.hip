// slab.hip -- multi-GPU z-slab jobs behind the C-ABI (include/stencil_hip.h
// part 3): one process drives N GPUs, RCCL moves the halos.
//
// The reference runs its whole decomposed job behind one kernel call: 64
// CPEs own 8x8 blocks, exchange halo strips by DMA / RMA every iteration and
// meet at a barrier (athread_spawn/join, src/stencil/stencil.cpp:34-53; halo
// DMA stencil_dma.cpp:236-247; barrier 562-563; RMA stencil_rma.cpp:198-255).
// Here the blocks are contiguous z-slabs of the global grid, one per GPU
// (remainder planes to the lowest slabs), each with K ghost planes per shared
// face, where K is the number of sweeps stencil_iterate fuses into one launch
// for the problem (7-point star: 4 or 5; box: 3 or 4): one round = K fused sweeps
// + one exchange of K whole planes with each neighbour (temporal blocking
// across GPUs; the halo planes are advanced on chip).  Per slab and round:
//   stream A (high priority): the K boundary planes of each face, then the
//            exchange -- RCCL ncclSend/ncclRecv inside one ncclGroupStart/End
//            spanning every slab (one thread drives all communicators), or
//            device copies (hipMemcpyPeerAsync: N logical slabs may share a
//            GPU, which RCCL refuses);
//   stream B: the interior planes meanwhile.
// Rounds chain on the two streams through events (stencil_amd/slab.py does
// the same per process with torch.distributed).  Every cell's arithmetic is
// the single-grid kernel's: results are bitwise those of one grid.
//
// RCCL is loaded on first use (dlopen): single-GPU users never load it.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace stencil {
namespace {

// ---- the few RCCL entry points used, resolved at run time -----------------
typedef struct ncclComm* ncclComm_t;
typedef enum { ncclSuccess = 0 } ncclResult_t;
struct ncclUniqueId { char internal[128]; };  // NCCL_UNIQUE_ID_BYTES
enum { ncclChar = 0, ncclUint8 = 1 };  // ncclDataType_t: bytes

struct Rccl {
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        auto sym = [&](auto& f, const char* name) { f = reinterpret_cast<std::decay_t<decltype(f)>>(dlsym(h, name)); };
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = r.CommInitAll && r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.GroupStart && r.GroupEnd && r.Send && r.Recv && r.GetErrorString;
    });
    return r;
}

#define SLAB_NCCL_CHECK(expr)                                                                          \
    do {                                                                                               \
        ncclResult_t e_ = (expr);                                                                      \
        if (e_ != ncclSuccess)                                                                         \
            return set_error(STENCIL_EHIP, "%s failed: %s", #expr, rccl().GetErrorString(e_));        \
    } while (0)

struct Slab {
    int device = 0;
    int index = 0;             // global slab index (= RCCL rank)
    int64_t first = 0, n = 0;  // global first plane, planes owned
    stencil_layout l{};
    void* a = nullptr;
    void* b = nullptr;
    hipStream_t sa = nullptr, sb = nullptr;    // boundary + exchange (high priority) / interior
    hipEvent_t ev_bnd = nullptr, ev_int = nullptr, ev_join = nullptr;
    ncclComm_t comm = nullptr;
    // face-signalled rounds: [0] low-face adds, [1] high-face adds (they run
    // on across launches), [2] the wait kernel's timeout flag
    uint32_t* counters = nullptr;
    uint32_t sig_target = 0;  // adds per face expected once the last queued launch is done
};

}  // namespace
}  // namespace stencil

struct stencil_slab_job {
    stencil_problem global{};
    int exchange = STENCIL_EXCHANGE_RCCL;
    bool periodic = false;
    int k = 1;       // sweeps per round (fused launch depth)
    int depth = 1;   // halo planes exchanged per face
    bool cur_is_a = true;
    bool chained = false;  // round events recorded since the last join
    bool signal = false;   // full rounds as face-signalled single launches
    int nranks = 0;        // rank mode (stencil_slab_create_rank): slabs of the job, this process owns s[0]
    std::vector<stencil::Slab> s;
    // stencil_slab_kernel_timing: hipEvents around slab 0's compute launch of
    // every round (the whole slab in face-signalled rounds, else the interior)
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    int64_t timed_cells = 0;
};

namespace stencil {
namespace {

int set_dev(int d) {
    STENCIL_HIP_CHECK(hipSetDevice(d));
    return STENCIL_OK;
}

// Timing events around slab 0's compute launch (the caller has set slab 0's
// device): begin() before it, end() after it, on the launch's stream.
int time_begin(stencil_slab_job& j, size_t slab, hipStream_t st) {
    if (!j.timing || slab != 0) return STENCIL_OK;
    hipEvent_t a = nullptr, b = nullptr;
    STENCIL_HIP_CHECK(hipEventCreate(&a));
    STENCIL_HIP_CHECK(hipEventCreate(&b));
    j.tev.emplace_back(a, b);
    STENCIL_HIP_CHECK(hipEventRecord(a, st));
    return STENCIL_OK;
}
int time_end(stencil_slab_job& j, size_t slab, hipStream_t st, int64_t cells) {
    if (!j.timing || slab != 0) return STENCIL_OK;
    STENCIL_HIP_CHECK(hipEventRecord(j.tev.back().second, st));
    j.timed_cells = cells;
    return STENCIL_OK;
}
void drop_timing(stencil_slab_job& j) {
    for (auto& e : j.tev) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    j.tev.clear();
    j.timed_cells = 0;
}

// Sweeps stencil_iterate fuses into one launch for `p` (its plan over a
// count that every candidate divides): the round length across slabs.
int fuse_depth(const stencil_problem& p) {
    stencil_layout l;
    if (stencil_layout_init(&p, &l) != STENCIL_OK) return 1;
    for (int k : {5, 4, 3, 2}) {
        int64_t launches = 0;
        int32_t kernel = 0;
        if (stencil_plan(&l, uint32_t(k), &launches, &kernel) == STENCIL_OK && launches == 1 &&
            kernel != STENCIL_KERNEL_PERSISTENT)
            return k;
    }
    return 1;
}

// neighbours of global slab i (its RCCL peers)
int slabs_total(const stencil_slab_job& j) { return j.nranks ? j.nranks : int(j.s.size()); }
int lo_nb(const stencil_slab_job& j, int i) {
    const int n = slabs_total(j);
    return i > 0 ? i - 1 : (j.periodic ? n - 1 : -1);
}
int hi_nb(const stencil_slab_job& j, int i) {
    const int n = slabs_total(j);
    return i < n - 1 ? i + 1 : (j.periodic ? 0 : -1);
}

size_t plane_bytes(const Slab& s) { return size_t(s.l.plane) * (s.l.prob.dtype == STENCIL_F64 ? 8 : 4); }
// first byte of plane z (z may be a ghost/halo plane)
char* plane_ptr(const Slab& s, void* grid, int64_t z) {
    return static_cast<char*>(grid) + size_t(s.l.zghost + z) * plane_bytes(s);
}

// Halo exchange of `grid` (each slab's copy of the same logical grid): every
// slab's K face planes into its neighbours' halo planes, queued on the slabs'
// A streams behind what is already there.
int exchange(stencil_slab_job& j, bool use_a) {
    const int n = int(j.s.size());
    const int64_t d = j.depth;
    if (j.exchange == STENCIL_EXCHANGE_RCCL) {
        const Rccl& r = rccl();
        SLAB_NCCL_CHECK(r.GroupStart());
        for (int i = 0; i < n; ++i) {
            Slab& s = j.s[i];
            void* g = use_a ? s.a : s.b;
            const size_t bytes = size_t(d) * plane_bytes(s);
            const int lo = lo_nb(j, s.index), hi = hi_nb(j, s.index);
            // sends and receives to one peer match in posting order: a slab
            // that is its own neighbour (periodic, N = 1) sends hi -> recv lo
            // first, then lo -> hi
            if (hi >= 0) {
                SLAB_NCCL_CHECK(r.Send(plane_ptr(s, g, s.n - d), bytes, ncclChar, hi, s.comm, s.sa));
            }
            if (lo >= 0) {
                SLAB_NCCL_CHECK(r.Recv(plane_ptr(s, g, -d), bytes, ncclChar, lo, s.comm, s.sa));
                SLAB_NCCL_CHECK(r.Send(plane_ptr(s, g, 0), bytes, ncclChar, lo, s.comm, s.sa));
            }
            if (hi >= 0) {
                SLAB_NCCL_CHECK(r.Recv(plane_ptr(s, g, s.n), bytes, ncclChar, hi, s.comm, s.sa));
            }
        }
        SLAB_NCCL_CHECK(r.GroupEnd());
        return STENCIL_OK;
    }
    // device copies (single-process jobs only: local = global index): slab i's
    // A stream pulls its neighbours' faces once their round is complete (ev_join, recorded on their A streams after joining B)
    for (int i = 0; i < n; ++i) {
        Slab& s = j.s[i];
        if (int rc = set_dev(s.device)) return rc;
        STENCIL_HIP_CHECK(hipEventRecord(s.ev_join, s.sa));
    }
    for (int i = 0; i < n; ++i) {
        Slab& s = j.s[i];
        if (int rc = set_dev(s.device)) return rc;
        void* g = use_a ? s.a : s.b;
        const size_t bytes = size_t(d) * plane_bytes(s);
        const int lo = lo_nb(j, i), hi = hi_nb(j, i);
        if (lo >= 0) {
            Slab& t = j.s[lo];
            STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sa, t.ev_join, 0));
            STENCIL_HIP_CHECK(hipMemcpyPeerAsync(plane_ptr(s, g, -d), s.device, plane_ptr(t, use_a ? t.a : t.b, t.n - d),
                                                 t.device, bytes, s.sa));
        }
        if (hi >= 0) {
            Slab& t = j.s[hi];
            STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sa, t.ev_join, 0));
            STENCIL_HIP_CHECK(hipMemcpyPeerAsync(plane_ptr(s, g, s.n), s.device, plane_ptr(t, use_a ? t.a : t.b, 0),
                                                 t.device, bytes, s.sa));
        }
    }
    return STENCIL_OK;
}

int sync_all(stencil_slab_job& j) {
    for (Slab& s : j.s) {
        if (int rc = set_dev(s.device)) return rc;
        STENCIL_HIP_CHECK(hipStreamSynchronize(s.sa));
        STENCIL_HIP_CHECK(hipStreamSynchronize(s.sb));
    }
    j.chained = false;
    return STENCIL_OK;
}

// One round of `k` fused sweeps: src -> dst on every slab, then the exchange
// of dst's faces.
int slab_round(stencil_slab_job& j, int k) {
    const bool src_a = j.cur_is_a;
    const int64_t edge = j.depth;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab& s = j.s[i];
        if (int rc = set_dev(s.device)) return rc;
        void* src = src_a ? s.a : s.b;
        void* dst = src_a ? s.b : s.a;
        if (j.chained) {
            // interior(r) reads src [0, n): after boundary + exchange(r-1);
            // boundary(r) overwrites planes interior(r-1) read: after it
            STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sb, s.ev_bnd, 0));
            STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sa, s.ev_int, 0));
        }
        const int64_t plane_cells = s.l.prob.nx * s.l.prob.ny;
        if (s.n > 2 * edge) {
            if (int rc = time_begin(j, i, s.sb)) return rc;
            if (int rc = stencil_sweepk(&s.l, src, dst, edge, s.n - edge, k, s.sb)) return rc;
            if (int rc = time_end(j, i, s.sb, plane_cells * (s.n - 2 * edge))) return rc;
            STENCIL_HIP_CHECK(hipEventRecord(s.ev_int, s.sb));
            if (int rc = stencil_sweepk(&s.l, src, dst, 0, edge, k, s.sa)) return rc;
            if (int rc = stencil_sweepk(&s.l, src, dst, s.n - edge, s.n, k, s.sa)) return rc;
        } else {
            if (int rc = time_begin(j, i, s.sa)) return rc;
            if (int rc = stencil_sweepk(&s.l, src, dst, 0, s.n, k, s.sa)) return rc;
            if (int rc = time_end(j, i, s.sa, plane_cells * s.n)) return rc;
            STENCIL_HIP_CHECK(hipEventRecord(s.ev_int, s.sa));
        }
        if (j.exchange == STENCIL_EXCHANGE_COPY)  // the face copies read whole rounds
            STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sa, s.ev_int, 0));
    }
    if (int rc = exchange(j, !src_a)) return rc;
    for (Slab& s : j.s) {
        if (int rc = set_dev(s.device)) return rc;
        STENCIL_HIP_CHECK(hipEventRecord(s.ev_bnd, s.sa));
    }
    j.chained = true;
    j.cur_is_a = !src_a;
    return STENCIL_OK;
}

// One round of `k` fused sweeps as ONE face-signalled launch per slab
// (stencil_sweepk_signal; the slab.py rounds): the launch's
// first z-chunk marches up and its last down, so its face planes are among the
// first stored; the workgroups storing them add to the slab's counters.  The
// exchange stream queues a wait for the counts (stencil_wait_counters) and the
// halo exchange behind it, so the faces leave while the rest of the launch
// runs -- no separate boundary launches.  Order: launch(r) reads the halos
// exchange(r-1) received (B waits for A); exchange(r) receives into the halo
// planes launch(r-1) read, and starts only once launch(r) has signalled, i.e.
// after launch(r-1) ended (one stream).
int slab_round_signal(stencil_slab_job& j, int k) {
    const bool src_a = j.cur_is_a;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab& s = j.s[i];
        if (int rc = set_dev(s.device)) return rc;
        void* src = src_a ? s.a : s.b;
        void* dst = src_a ? s.b : s.a;
        if (j.chained) STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sb, s.ev_bnd, 0));
        int nsig = 0;
        if (int rc = time_begin(j, i, s.sb)) return rc;
        if (int rc = stencil_sweepk_signal(&s.l, src, dst, 0, s.n, k, s.counters, nullptr, &nsig, s.sb)) return rc;
        if (int rc = time_end(j, i, s.sb, s.l.prob.nx * s.l.prob.ny * s.n)) return rc;
        STENCIL_HIP_CHECK(hipEventRecord(s.ev_int, s.sb));
        s.sig_target += uint32_t(nsig);
        if (int rc = stencil_wait_counters(s.counters, s.sig_target, s.sig_target, s.counters + 2, s.sa)) return rc;
    }
    if (int rc = exchange(j, !src_a)) return rc;
    for (Slab& s : j.s) {
        if (int rc = set_dev(s.device)) return rc;
        STENCIL_HIP_CHECK(hipEventRecord(s.ev_bnd, s.sa));
        // the next round's boundary-launch path (remainders) writes planes
        // this launch reads: A must also follow B
        STENCIL_HIP_CHECK(hipStreamWaitEvent(s.sa, s.ev_int, 0));
    }
    j.chained = true;
    j.cur_is_a = !src_a;
    return STENCIL_OK;
}

// Did a face-counter wait give up (10 s)?  Then the halos are wrong.
int check_signal_timeouts(stencil_slab_job& j) {
    for (Slab& s : j.s) {
        if (!s.counters) continue;
        if (int rc = set_dev(s.device)) return rc;
        uint32_t flag = 0;
        STENCIL_HIP_CHECK(hipMemcpy(&flag, s.counters + 2, sizeof(flag), hipMemcpyDeviceToHost));
        if (flag) return set_error(STENCIL_EHIP, "slab on device %d: a face-counter wait timed out", s.device);
    }
    return STENCIL_OK;
}

void release(stencil_slab_job* j) {
    if (!j) return;
    if (!j->s.empty()) {
        (void)hipSetDevice(j->s[0].device);
        drop_timing(*j);
    }
    for (Slab& s : j->s) {
        (void)hipSetDevice(s.device);
        if (s.sa) (void)hipStreamSynchronize(s.sa);
        if (s.sb) (void)hipStreamSynchronize(s.sb);
        if (s.comm && rccl().ok) (void)rccl().CommDestroy(s.comm);
        if (s.a) (void)hipFree(s.a);
        if (s.b) (void)hipFree(s.b);
        if (s.sa) (void)hipStreamDestroy(s.sa);
        if (s.sb) (void)hipStreamDestroy(s.sb);
        if (s.ev_bnd) (void)hipEventDestroy(s.ev_bnd);
        if (s.ev_int) (void)hipEventDestroy(s.ev_int);
        if (s.ev_join) (void)hipEventDestroy(s.ev_join);
        if (s.counters) (void)hipFree(s.counters);
    }
    delete j;
}

}  // namespace
}  // namespace stencil

using namespace stencil;

extern "C" {

}  // extern "C"

namespace stencil {
namespace {

// The slabs this process owns: global slab indices `idx` (of `total`) on
// `devs`; the z split is the same in every process (planes total / N, the first
// nz % N slabs one more), so each rank can build its own share alone.
int build_job(const stencil_problem& g, int total, const std::vector<int>& idx, const std::vector<int>& devs,
              int32_t exchange_kind, int32_t flags, bool rank_mode, stencil_slab_job** out) {
    auto* j = new stencil_slab_job;
    j->global = g;
    j->exchange = exchange_kind;
    j->periodic = flags & STENCIL_SLAB_PERIODIC;
    j->nranks = rank_mode ? total : 0;
    j->k = fuse_depth(g);
    j->depth = std::max<int>(j->k, g.radius);
    // face-signalled rounds where the K-step kernels have them (3D r = 1 naive
    // 7-point star K = 3..5, box K = 2..4); STENCIL_SLAB_SIGNAL=0: boundary +
    // interior launches
    {
        const bool off = api_knob("STENCIL_SLAB_SIGNAL", 1) == 0;
        const bool star = g.shape == STENCIL_STAR && j->k >= 3 && j->k <= 5;
        const bool box = g.shape == STENCIL_BOX && j->k >= 2 && j->k <= 4;
        // and only with one slab per GPU: slabs sharing a GPU multiplex their
        // streams onto its few hardware queues, where a polling wait kernel
        // could sit in front of the launch another slab's wait is polling for
        // (ranks each own one GPU: RCCL refuses two ranks on one device)
        bool distinct = true;
        for (size_t i = 0; i < devs.size(); ++i)
            for (size_t k = 0; k < i; ++k) distinct = distinct && devs[i] != devs[k];
        j->signal = g.radius == 1 && g.order == STENCIL_ORDER_NAIVE && (star || box) && distinct && !off;
    }
    const int64_t base = g.nz / total, rem = g.nz % total;
    j->s.resize(idx.size());
    int rc = STENCIL_OK;
    for (size_t li = 0; li < idx.size() && rc == STENCIL_OK; ++li) {
        const int i = idx[li];
        Slab& s = j->s[li];
        s.index = i;
        s.device = devs[li];
        s.n = base + (i < rem ? 1 : 0);
        s.first = i * base + std::min<int64_t>(i, rem);
        if (s.n < j->depth) {
            rc = set_error(STENCIL_EINVAL, "slab %d owns %lld planes < the %d halo planes: use fewer GPUs", i,
                           (long long)s.n, j->depth);
            break;
        }
        stencil_problem p = g;
        p.nz = s.n;
        p.halo = j->depth;
        p.flags = (lo_nb(*j, i) >= 0 ? STENCIL_HALO_LO : 0) | (hi_nb(*j, i) >= 0 ? STENCIL_HALO_HI : 0);
        if ((rc = stencil_layout_init(&p, &s.l))) break;
        if ((rc = set_dev(s.device))) break;
        if ((rc = stencil_alloc(&s.l, &s.a)) || (rc = stencil_alloc(&s.l, &s.b))) break;
        int lo_prio = 0, hi_prio = 0;
        if (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess ||
            hipStreamCreateWithPriority(&s.sa, hipStreamNonBlocking, hi_prio) != hipSuccess ||
            hipStreamCreateWithFlags(&s.sb, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s.ev_bnd, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.ev_int, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.ev_join, hipEventDisableTiming) != hipSuccess)
            rc = set_error(STENCIL_EHIP, "stream / event creation failed on device %d", s.device);
        if (rc == STENCIL_OK && (hipMalloc(&s.counters, 4 * sizeof(uint32_t)) != hipSuccess ||
                                 hipMemset(s.counters, 0, 4 * sizeof(uint32_t)) != hipSuccess))
            rc = set_error(STENCIL_EHIP, "face counters on device %d", s.device);
    }
    if (rc != STENCIL_OK) {
        release(j);
        return rc;
    }
    *out = j;
    return STENCIL_OK;
}

int check_global(const stencil_problem* global, stencil_problem* g, int32_t flags) {
    *g = *global;
    if (g->dims != 3) return set_error(STENCIL_EUNSUPPORTED, "slab jobs split 3D grids along z");
    if (g->halo != 0 || g->flags != 0) return set_error(STENCIL_EINVAL, "the global problem takes no halo / flags");
    if (flags & ~STENCIL_SLAB_PERIODIC) return set_error(STENCIL_EINVAL, "bad slab flags %d", flags);
    stencil_layout gl;
    return stencil_layout_init(g, &gl);
}

}  // namespace
}  // namespace stencil

extern "C" {

int stencil_slab_create(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange_kind,
                        int32_t flags, stencil_slab_job** job) {
    if (!global || !job || ngpus < 1) return set_error(STENCIL_EINVAL, "null argument or ngpus < 1");
    *job = nullptr;
    if (exchange_kind != STENCIL_EXCHANGE_RCCL && exchange_kind != STENCIL_EXCHANGE_COPY)
        return set_error(STENCIL_EINVAL, "bad exchange kind %d", exchange_kind);
    stencil_problem g;
    if (int rc = check_global(global, &g, flags)) return rc;
    std::vector<int> devs(static_cast<size_t>(ngpus)), idx(static_cast<size_t>(ngpus));
    for (int i = 0; i < ngpus; ++i) {
        devs[size_t(i)] = devices ? devices[i] : i;
        idx[size_t(i)] = i;
    }
    if (exchange_kind == STENCIL_EXCHANGE_RCCL) {
        for (int i = 0; i < ngpus; ++i)
            for (int k = 0; k < i; ++k)
                if (devs[size_t(i)] == devs[size_t(k)])
                    return set_error(STENCIL_EINVAL, "RCCL needs one slab per GPU (device %d twice): use device copies",
                                     devs[size_t(i)]);
        if (!rccl().ok) return set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    }
    stencil_slab_job* j = nullptr;
    if (int rc = build_job(g, ngpus, idx, devs, exchange_kind, flags, false, &j)) return rc;
    if (exchange_kind == STENCIL_EXCHANGE_RCCL) {
        std::vector<ncclComm_t> comms(size_t(ngpus), nullptr);
        const ncclResult_t e = rccl().CommInitAll(comms.data(), ngpus, devs.data());
        if (e != ncclSuccess) {
            const int rc = set_error(STENCIL_EHIP, "ncclCommInitAll(%d) failed: %s", ngpus, rccl().GetErrorString(e));
            release(j);
            return rc;
        }
        for (int i = 0; i < ngpus; ++i) j->s[size_t(i)].comm = comms[size_t(i)];
    }
    *job = j;
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_unique_id(void* id, int64_t bytes) {
    if (!id || bytes < int64_t(sizeof(ncclUniqueId)))
        return set_error(STENCIL_EINVAL, "the id buffer needs %d bytes", int(sizeof(ncclUniqueId)));
    if (!rccl().ok) return set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    ncclUniqueId u;
    const ncclResult_t e = rccl().GetUniqueId(&u);
    if (e != ncclSuccess) return set_error(STENCIL_EHIP, "ncclGetUniqueId failed: %s", rccl().GetErrorString(e));
    std::memcpy(id, &u, sizeof(u));
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_create_rank(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device,
                             const void* id, int64_t id_bytes, int32_t flags, stencil_slab_job** job) {
    if (!global || !job || !id) return set_error(STENCIL_EINVAL, "null argument");
    *job = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(STENCIL_EINVAL, "rank %d of %d", rank, nranks);
    if (id_bytes != int64_t(sizeof(ncclUniqueId)))
        return set_error(STENCIL_EINVAL, "the id holds %d bytes, not %lld", int(sizeof(ncclUniqueId)),
                         (long long)id_bytes);
    stencil_problem g;
    if (int rc = check_global(global, &g, flags)) return rc;
    if (!rccl().ok) return set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    stencil_slab_job* j = nullptr;
    if (int rc = build_job(g, nranks, {rank}, {device}, STENCIL_EXCHANGE_RCCL, flags, true, &j)) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    if (int rc = set_dev(device)) {
        release(j);
        return rc;
    }
    // collective over the ranks: every rank must reach it (a rank whose
    // build_job failed returns before it, and the others wait in RCCL's own
    // bootstrap until it times out)
    const ncclResult_t e = rccl().CommInitRank(&comm, nranks, u, rank);
    if (e != ncclSuccess) {
        const int rc = set_error(STENCIL_EHIP, "ncclCommInitRank(%d of %d) failed: %s", rank, nranks,
                                 rccl().GetErrorString(e));
        release(j);
        return rc;
    }
    j->s[0].comm = comm;
    *job = j;
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_destroy(stencil_slab_job* job) {
    release(job);
    return STENCIL_OK;
}

int stencil_slab_info(const stencil_slab_job* job, int32_t slab, int64_t* first_plane, int64_t* planes,
                      int32_t* device, int32_t* sweeps_per_round) {
    if (!job || slab < 0 || slab >= int(job->s.size())) return set_error(STENCIL_EINVAL, "bad job or slab index");
    const Slab& s = job->s[size_t(slab)];
    if (first_plane) *first_plane = s.first;
    if (planes) *planes = s.n;
    if (device) *device = s.device;
    if (sweeps_per_round) *sweeps_per_round = job->k;
    return STENCIL_OK;
}

int stencil_slab_fill_initial(stencil_slab_job* job, int32_t init_kind, uint64_t seed) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (int rc = sync_all(*job)) return rc;
    for (Slab& s : job->s) {
        if (int rc = set_dev(s.device)) return rc;
        // global linear indices: the slab's interior starts first * nx * ny cells in
        const uint64_t sd = seed + uint64_t(s.first) * uint64_t(s.l.prob.nx) * uint64_t(s.l.prob.ny);
        if (int rc = stencil_fill_initial(&s.l, s.a, init_kind, sd, s.sa)) return rc;
        if (int rc = stencil_fill_initial(&s.l, s.b, init_kind, sd, s.sa)) return rc;
    }
    job->cur_is_a = true;
    // the halos of both grids: the neighbours' faces (ghost planes otherwise)
    if (int rc = exchange(*job, true)) return rc;
    if (int rc = exchange(*job, false)) return rc;
    return sync_all(*job);
}

int stencil_slab_upload(stencil_slab_job* job, const void* host, int64_t host_row, int64_t host_rows) {
    if (!job || !host) return set_error(STENCIL_EINVAL, "null argument");
    const stencil_problem& g = job->global;
    if (host_row < g.nx + 2 * g.radius || host_rows < g.ny + 2 * g.radius)
        return set_error(STENCIL_EINVAL, "host array too small");
    if (int rc = sync_all(*job)) return rc;
    const size_t es = g.dtype == STENCIL_F64 ? 8 : 4;
    for (Slab& s : job->s) {
        if (int rc = set_dev(s.device)) return rc;
        // host planes [first, first + n + 2r) hold this slab's planes -r .. n+r-1
        const char* h = static_cast<const char*>(host) + size_t(s.first) * size_t(host_row * host_rows) * es;
        if (int rc = stencil_upload(&s.l, s.a, h, host_row, host_rows, s.sa)) return rc;
        if (int rc = stencil_upload(&s.l, s.b, h, host_row, host_rows, s.sa)) return rc;
    }
    job->cur_is_a = true;
    if (int rc = exchange(*job, true)) return rc;
    if (int rc = exchange(*job, false)) return rc;
    return sync_all(*job);
}

int stencil_slab_run(stencil_slab_job* job, uint32_t iterations, float* elapsed_ms) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (int rc = sync_all(*job)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t done = 0;
    const uint32_t k = uint32_t(job->k);
    for (; done + k <= iterations; done += k)
        if (int rc = job->signal ? slab_round_signal(*job, int(k)) : slab_round(*job, int(k))) return rc;
    if (done < iterations)  // the remainder as one shorter fused round
        if (int rc = slab_round(*job, int(iterations - done))) return rc;
    if (int rc = sync_all(*job)) return rc;
    if (job->signal)
        if (int rc = check_signal_timeouts(*job)) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    if (elapsed_ms) *elapsed_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_download(stencil_slab_job* job, void* host, int64_t host_row, int64_t host_rows) {
    if (!job || !host) return set_error(STENCIL_EINVAL, "null argument");
    if (int rc = sync_all(*job)) return rc;
    const stencil_problem& g = job->global;
    const int64_t r = g.radius;
    const size_t es = g.dtype == STENCIL_F64 ? 8 : 4;
    const size_t hplane = size_t(host_row * host_rows) * es;
    if (host_row < g.nx + 2 * r || host_rows < g.ny + 2 * r) return set_error(STENCIL_EINVAL, "host array too small");
    std::vector<char> tmp;
    for (size_t i = 0; i < job->s.size(); ++i) {
        Slab& s = job->s[i];
        if (int rc = set_dev(s.device)) return rc;
        // the slab's planes -r .. n+r-1 through a scratch copy; keep its own
        // planes, plus the global ghost planes at the two ends
        tmp.resize(size_t(s.n + 2 * r) * hplane);
        if (int rc = stencil_download(&s.l, job->cur_is_a ? s.a : s.b, tmp.data(), host_row, host_rows, s.sa)) return rc;
        STENCIL_HIP_CHECK(hipStreamSynchronize(s.sa));
        const int64_t z0 = s.index == 0 ? -r : 0;
        const int64_t z1 = s.index + 1 == slabs_total(*job) ? s.n + r : s.n;
        std::memcpy(static_cast<char*>(host) + size_t(s.first + z0 + r) * hplane, tmp.data() + size_t(z0 + r) * hplane,
                    size_t(z1 - z0) * hplane);
    }
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_kernel_timing(stencil_slab_job* job, int32_t enable) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (int rc = sync_all(*job)) return rc;
    if (int rc = set_dev(job->s[0].device)) return rc;
    drop_timing(*job);
    job->timing = enable != 0;
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_kernel_time(stencil_slab_job* job, float* total_ms, int64_t* launches, int64_t* cells_per_launch,
                             int32_t* signalled) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (int rc = sync_all(*job)) return rc;
    if (int rc = set_dev(job->s[0].device)) return rc;
    float sum = 0.f;
    for (auto& e : job->tev) {
        float ms = 0.f;
        STENCIL_HIP_CHECK(hipEventElapsedTime(&ms, e.first, e.second));
        sum += ms;
    }
    if (total_ms) *total_ms = sum;
    if (launches) *launches = int64_t(job->tev.size());
    if (cells_per_launch) *cells_per_launch = job->timed_cells;
    if (signalled) *signalled = job->signal ? 1 : 0;
    clear_error();
    return STENCIL_OK;
}

int stencil_slab_plane_sums(stencil_slab_job* job, double* sums) {
    if (!job || !sums) return set_error(STENCIL_EINVAL, "null argument");
    if (int rc = sync_all(*job)) return rc;
    for (Slab& s : job->s) {
        if (int rc = set_dev(s.device)) return rc;
        if (int rc = stencil_plane_sums(&s.l, job->cur_is_a ? s.a : s.b, sums + s.first, s.sa)) return rc;
        STENCIL_HIP_CHECK(hipStreamSynchronize(s.sa));
    }
    clear_error();
    return STENCIL_OK;
}

}  // extern "C"
