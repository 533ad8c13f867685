// slab.hip -- multi-GPU z-slab jobs behind the C-ABI (include/stencil_hip.h
// part 3): the HIP + RCCL backend of slab_core.hpp (which holds the round
// and exchange logic, shared with the CPU test build in tests/cpu_slab/).
//
// The reference runs its whole decomposed job behind one kernel call: 64
// CPEs own 8x8 blocks, exchange halo strips by DMA / RMA every iteration and
// meet at a barrier (athread_spawn/join, src/stencil/stencil.cpp:34-53; halo
// DMA stencil_dma.cpp:236-247; barrier 562-563; RMA stencil_rma.cpp:198-255).
// Here the blocks are contiguous z-slabs of the global grid, one per GPU,
// exchanging K whole planes with each neighbour per round of K fused sweeps
// (slab_core.hpp: the three round forms -- boundary + interior launches on
// two streams, face-signalled single launches, rolling one-grid passes).
// This file binds them to HIP streams / events / kernels and to RCCL
// ncclSend/ncclRecv inside one ncclGroupStart/End spanning every slab the
// process drives (one thread drives all communicators), or device copies
// (hipMemcpyPeerAsync: N logical slabs may share a GPU, which RCCL refuses).
//
// RCCL is loaded on first use (dlopen): single-GPU users never load it.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "common.hpp"
#include "slab_core.hpp"

namespace stencil {
namespace {

// ---- the few RCCL entry points used, resolved at run time -----------------
typedef struct ncclComm* ncclComm_t;
typedef enum { ncclSuccess = 0, ncclInProgress = 7 } ncclResult_t;
struct ncclUniqueId { char internal[128]; };  // NCCL_UNIQUE_ID_BYTES
enum { ncclChar = 0, ncclUint8 = 1 };  // ncclDataType_t: bytes

struct Rccl {
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
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
        sym(r.CommAbort, "ncclCommAbort");
        sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = r.CommInitAll && r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.CommAbort && r.CommGetAsyncError &&
               r.GroupStart && r.GroupEnd && r.Send && r.Recv && r.GetErrorString;
    });
    return r;
}

#define SLAB_NCCL_CHECK(expr)                                                                          \
    do {                                                                                               \
        ncclResult_t e_ = (expr);                                                                      \
        if (e_ != ncclSuccess)                                                                         \
            return set_error(STENCIL_EHIP, "%s failed: %s", #expr, rccl().GetErrorString(e_));        \
    } while (0)

// one lane spins `ticks` of s_memrealtime (100 MHz): HipDev::debug_delay
__global__ void __launch_bounds__(64) delay_kernel(uint64_t ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

}  // namespace

// ---- the HIP + RCCL backend of slab_core.hpp ------------------------------
struct HipDev {
    using Stream = hipStream_t;
    using Event = hipEvent_t;
    using Comm = ncclComm_t;

    static int set_device(int d) {
        STENCIL_HIP_CHECK(hipSetDevice(d));
        return STENCIL_OK;
    }
    static int layout_init(const stencil_problem* p, stencil_layout* l) { return stencil_layout_init(p, l); }
    // Sweeps stencil_iterate fuses into one launch for `p` (its plan over a
    // count that every candidate divides): the round length across slabs.
    static int fuse_depth(const stencil_problem& p) {
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
    static bool signal_enabled() { return api_knob("STENCIL_SLAB_SIGNAL", 1) != 0; }
    // Confine the exchange of this job (STENCIL_SLAB_XCU CUs per XCD, default
    // 1, for the exchange; the launches off them) when its face-signalled
    // launch takes several rounds of workgroups: more tiles than one round
    // holds with a CU per XCD to spare.  A one-round grid keeps every CU
    // (512^3: 1102 Gcell/s unconfined, 1022 confined; its grid is sized for
    // a spare CU per XCD already).  STENCIL_SLAB_XCU=0: never.
    static bool confine_exchange(const stencil_layout& l, int k) {
        if (xcu() == 0) return false;
        int64_t tiles = 0, wg = 0;
        int slots = 0;
        if (signal_launch_geometry(l, 0, l.prob.nz, k, &tiles, &wg, &slots) != STENCIL_OK) {
            clear_error();
            return false;
        }
        return slots > 0 && tiles > slots - slots / 32;
    }
    // STENCIL_SLAB_WIRE_GBPS=r (debug library, rehearsals): before each
    // exchange, a one-lane spin for one face's bytes at r GB/s on the
    // exchange stream -- the transfer time of a face between distinct GPUs
    // over xGMI, which a rehearsal's transfer to itself does not have
    static int wire_delay(Stream s, size_t face_bytes) {
        const int r = knob("STENCIL_SLAB_WIRE_GBPS", 0);
        if (r <= 0) return STENCIL_OK;
        const uint64_t us = uint64_t(double(face_bytes) / (double(r) * 1e3));
        hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, us * 100);
        STENCIL_HIP_CHECK(hipGetLastError());
        return STENCIL_OK;
    }
    // STENCIL_SLAB_SERIAL=1: every full round as one plain launch of the whole
    // slab followed by the exchange (no overlap)
    static bool serial_rounds() { return api_knob("STENCIL_SLAB_SERIAL", 0) != 0; }
    // STENCIL_SLAB_STAGED=0: many-round slabs run face-signalled rounds (the
    // exchange confined) instead of staged ones
    static bool staged_rounds() { return api_knob("STENCIL_SLAB_STAGED", 1) != 0; }
    // STENCIL_SLAB_PLACEMENTS=n: grid placements a two-grid slab tries at
    // creation (default 1 = the first allocation since round 6: the search
    // gained 0.8 % at C2's 1000 sweeps, profiles/r06/r06d_bench_1000_place*;
    // bench.py opts in with its --placements)
    static int placement_trials() { return std::max(1, api_knob("STENCIL_SLAB_PLACEMENTS", 1)); }
    static bool placement_verbose() { return knob("STENCIL_SLAB_PLACE_VERBOSE", 0) != 0; }
    // STENCIL_SLAB_ROLLING_OVERLAP=0: rolling rounds exchange after the pass
    // (slab_round_rolling) instead of beside it (slab_round_rolling_overlap)
    static bool rolling_overlap() { return api_knob("STENCIL_SLAB_ROLLING_OVERLAP", 1) != 0; }
    // STENCIL_SLAB_NO_PULL_WAIT=1 (debug library, the test that shows the
    // delay below exposing the race): drop the rolling exchange's wait
    static bool pull_wait_enabled() { return knob("STENCIL_SLAB_NO_PULL_WAIT", 0) == 0; }
    // STENCIL_SLAB_SIG_SKEW=n (debug library, the bounded-failure test): the
    // first face-signalled round waits for n face adds more than its launch
    // makes, so its face wait only ends when the job's deadline releases it
    static int debug_signal_skew() { return std::max(0, knob("STENCIL_SLAB_SIG_SKEW", 0)); }
    // STENCIL_SLAB_COPY_DELAY_US (debug library, tests): a one-lane spin of
    // that many microseconds queued before slab 0 pulls its neighbours' faces
    // (the others run on), so that a missing stream dependency of the copy
    // exchange shows every time
    static int debug_delay(Stream s, int slab) {
        const int us = knob("STENCIL_SLAB_COPY_DELAY_US", 0);
        if (us <= 0 || slab != 0) return STENCIL_OK;
        hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, uint64_t(us) * 100);
        STENCIL_HIP_CHECK(hipGetLastError());
        return STENCIL_OK;
    }
    static int free_bytes(int64_t* out) {
        size_t fr = 0, tot = 0;
        STENCIL_HIP_CHECK(hipMemGetInfo(&fr, &tot));
        *out = int64_t(fr);
        return STENCIL_OK;
    }
    static int alloc(int64_t bytes, void** p) {
        if (hipMalloc(p, size_t(bytes)) != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            return set_error(STENCIL_ENOMEM, "hipMalloc of %lld bytes failed", (long long)bytes);
        }
        return STENCIL_OK;
    }
    static void free(void* p) { (void)hipFree(p); }
    // hipMemset runs on the null stream, which the job's non-blocking streams
    // do not follow: the zeroes must land before any of their launches adds
    // to the counters (or a face wait waits for a count the memset erased),
    // so the host waits for them here (creation / reset: the streams are idle)
    static int alloc_counters(uint32_t** c) {
        if (hipMalloc(c, 4 * sizeof(uint32_t)) != hipSuccess || hipMemset(*c, 0, 4 * sizeof(uint32_t)) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess)
            return set_error(STENCIL_EHIP, "face counters");
        return STENCIL_OK;
    }
    static void free_counters(uint32_t* c) { (void)hipFree(c); }
    // the wait kernel's timeout flag in host-coherent memory: the host can
    // release a queued wait by writing it, whatever the device queues hold
    static int alloc_flag(uint32_t** f) {
        if (hipHostMalloc(reinterpret_cast<void**>(f), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
            return set_error(STENCIL_EHIP, "timeout flag");
        __atomic_store_n(*f, 0u, __ATOMIC_SEQ_CST);
        return STENCIL_OK;
    }
    static void free_flag(uint32_t* f) { (void)hipHostFree(f); }
    // counters, flag and face signal back to 0 (the streams are idle)
    static int reset_counters(uint32_t* c, uint32_t* flag, uint64_t* fs) {
        if (c) STENCIL_HIP_CHECK(hipMemset(c, 0, 4 * sizeof(uint32_t)));
        if (flag) __atomic_store_n(flag, 0u, __ATOMIC_SEQ_CST);
        if (fs)
            if (int rc = stencil_face_signal_reset(fs, nullptr)) return rc;
        // the null-stream memset / reset done before the job's streams launch (alloc_counters)
        if (c || fs) STENCIL_HIP_CHECK(hipDeviceSynchronize());
        return STENCIL_OK;
    }
    // a failed job: let every queued face wait return (the polling kernel
    // sees the flag; a command-processor wait sees its target passed)
    static void release_waits(uint32_t* flag, uint64_t* fs) {
        if (flag) __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
        if (fs) {
            hipPointerAttribute_t a{};
            if (hipPointerGetAttributes(&a, fs) == hipSuccess && a.hostPointer)
                __atomic_store_n(static_cast<uint64_t*>(a.hostPointer), uint64_t(1) << 62, __ATOMIC_SEQ_CST);
            (void)hipGetLastError();
        }
    }
    // A slab's streams by role (slab_core.hpp StreamRole): boundary launches
    // at high priority, the interior / whole-slab launches, the exchange.
    // STENCIL_SLAB_XCU=c (c CUs per XCD, 0 = off): the exchange stream is
    // confined to c CUs of every XCD (hipExtStreamCreateWithCUMask), so
    // RCCL's and the copies' kernels run there and not on the CUs a
    // one-per-CU launch beside them counts on; STENCIL_SLAB_XCU_EXCL=1 also
    // keeps the launches' streams off those CUs.
    static int xcu() { return std::max(0, std::min(16, api_knob("STENCIL_SLAB_XCU", 1))); }
    // STENCIL_SLAB_XCU_ALT=c (default 4; 0 = none): the CU budget a staged job
    // with a confined exchange also tries in its tuning rounds, keeping the
    // faster (slab_core.hpp staged_tuning_step)
    static int xcu_alt() {
        const int a = std::max(0, std::min(16, api_knob("STENCIL_SLAB_XCU_ALT", 4)));
        return a == xcu() ? 0 : a;
    }
    static int stream_create(Stream* s, int role, bool confine, int cus = -1) {
        // STENCIL_SLAB_XCU_EXCL=0 (with a confined exchange): the launches may
        // use the exchange's CUs too; cus >= 0: that budget instead of xcu()
        const int c = confine ? (cus >= 0 ? cus : xcu()) : 0;
        const bool excl = c > 0 && api_knob("STENCIL_SLAB_XCU_EXCL", 1) != 0;
        if (role == slab::STREAM_EXCHANGE ? c > 0 : excl) {
            int dev = 0, cus = 0;
            STENCIL_HIP_CHECK(hipGetDevice(&dev));
            STENCIL_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            // CU-mask bit b selects CU b / nxcd of XCD b % nxcd (the driver
            // stripes a queue's mask over the XCDs): bits [0, c * 8) are c CUs
            // on each of the 8 XCDs
            constexpr int kXcds = 8;
            std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
            for (int b = 0; b < cus; ++b) {
                const bool xbit = b < c * kXcds;
                if (xbit == (role == slab::STREAM_EXCHANGE)) mask[size_t(b / 32)] |= 1u << (b % 32);
            }
            if (hipExtStreamCreateWithCUMask(s, uint32_t(mask.size()), mask.data()) != hipSuccess)
                return set_error(STENCIL_EHIP, "CU-masked stream creation failed");
            return STENCIL_OK;
        }
        int lo_prio = 0, hi_prio = 0;
        bool high_priority = role != slab::STREAM_INTERIOR;
        // STENCIL_SLAB_NOPRIO=1 (debug library): every stream at the default priority
        if (knob("STENCIL_SLAB_NOPRIO", 0)) high_priority = false;
        if (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess ||
            hipStreamCreateWithPriority(s, hipStreamNonBlocking, high_priority ? hi_prio : lo_prio) != hipSuccess)
            return set_error(STENCIL_EHIP, "stream creation failed");
        return STENCIL_OK;
    }
    static void stream_destroy(Stream s) { (void)hipStreamDestroy(s); }
    static int stream_sync(Stream s) {
        STENCIL_HIP_CHECK(hipStreamSynchronize(s));
        return STENCIL_OK;
    }
    // Bounded waits: poll the stream / event, and the communicator's
    // asynchronous error, until done or past the deadline (then
    // STENCIL_ETIMEOUT; the caller fails the job).  Spins with a yield: the
    // end of a timed run() waits here.
    static int default_timeout_ms() { return std::max(1, api_knob("STENCIL_SLAB_TIMEOUT_MS", 60000)); }
    template <class Q>
    static int poll_until(Q&& query, Comm c, slab::Clock::time_point deadline, const char* what) {
        for (uint64_t it = 0;; ++it) {
            const hipError_t e = query();
            if (e == hipSuccess) return STENCIL_OK;
            if (e != hipErrorNotReady) return set_error(STENCIL_EHIP, "%s: %s", what, hipGetErrorString(e));
            if ((it & 63) == 63) {
                if (c && rccl().ok) {
                    ncclResult_t r = ncclSuccess;
                    if (rccl().CommGetAsyncError(c, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress)
                        return set_error(STENCIL_EHIP, "%s: RCCL asynchronous error: %s", what, rccl().GetErrorString(r));
                }
                if (slab::Clock::now() > deadline)
                    return set_error(STENCIL_ETIMEOUT, "%s: no progress before the slab job's deadline (a peer stopped "
                                     "answering?): the job is failed and its communicators aborted", what);
            }
            if (it > 4096) std::this_thread::sleep_for(std::chrono::microseconds(20));
            else std::this_thread::yield();
        }
    }
    static int sync_until(Stream s, Comm c, slab::Clock::time_point deadline) {
        return poll_until([&] { return hipStreamQuery(s); }, c, deadline, "slab stream");
    }
    static int event_sync_until(Event e, Comm c, slab::Clock::time_point deadline) {
        return poll_until([&] { return hipEventQuery(e); }, c, deadline, "slab round");
    }
    static int event_create(Event* e, bool timing) {
        STENCIL_HIP_CHECK(timing ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableTiming));
        return STENCIL_OK;
    }
    static void event_destroy(Event e) { (void)hipEventDestroy(e); }
    static int event_record(Event e, Stream s) {
        STENCIL_HIP_CHECK(hipEventRecord(e, s));
        return STENCIL_OK;
    }
    static int stream_wait(Stream s, Event e) {
        STENCIL_HIP_CHECK(hipStreamWaitEvent(s, e, 0));
        return STENCIL_OK;
    }
    static int event_elapsed(float* ms, Event a, Event b) {
        STENCIL_HIP_CHECK(hipEventElapsedTime(ms, a, b));
        return STENCIL_OK;
    }
    static int sweepk(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k, Stream s) {
        return stencil_sweepk(l, src, dst, b, e, k, s);
    }
    static int sweepk_signal(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k,
                             uint32_t* counters, uint64_t* fsig, int* nsig, Stream s) {
        int32_t n = 0;
        const int rc = stencil_sweepk_signal(l, src, dst, b, e, k, counters, fsig, &n, s);
        *nsig = n;
        return rc;
    }
    // STENCIL_SLAB_CPWAIT=1: face-signalled rounds gate the exchange on a HIP
    // signal word waited on by the command processor (no wait kernel resident
    // beside the launch); 0 (default): the polling wait kernel with its timeout
    static int face_signal_create(uint64_t** fs) {
        *fs = nullptr;
        if (api_knob("STENCIL_SLAB_CPWAIT", 0) == 0) return STENCIL_OK;
        if (int rc = stencil_face_signal_create(fs)) return rc;
        if (int rc = stencil_face_signal_reset(*fs, nullptr)) return rc;
        STENCIL_HIP_CHECK(hipDeviceSynchronize());
        return STENCIL_OK;
    }
    static void face_signal_destroy(uint64_t* fs) { (void)stencil_face_signal_destroy(fs); }
    static int wait_face_signal(uint64_t* fs, uint64_t target, Stream s) { return stencil_wait_face_signal(fs, target, s); }
    static int wait_counters(uint32_t* c, uint32_t* flag, uint32_t lo, uint32_t hi, Stream s) {
        return stencil_wait_counters(c, lo, hi, flag, s);
    }
    // Halo-gated face-signalled launches (stencil_sweepk_signal_gated; the
    // 7-point star): only where the workgroups that may wait for an exchange
    // can never hold every CU the exchange's own kernels (RCCL's, the
    // completion store) need -- a confined exchange has CUs of its own, and
    // otherwise the waiting chunks (at most the two face chunks of every
    // tile) must fit one round with a CU per XCD to spare, as the 512^3-class
    // grids do (110 tiles: 220 <= 248).  STENCIL_SLAB_GATE=0: never.
    static bool halo_gate(const stencil_layout& l, int k, bool confined) {
        if (api_knob("STENCIL_SLAB_GATE", 1) == 0 || l.prob.shape != STENCIL_STAR) return false;
        if (confined) return true;
        int64_t tiles = 0, wg = 0;
        int slots = 0;
        if (signal_launch_geometry(l, 0, l.prob.nz, k, &tiles, &wg, &slots) != STENCIL_OK) {
            clear_error();
            return false;
        }
        return slots > 0 && 2 * tiles <= slots - slots / 32;
    }
    static int sweepk_signal_gated(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k,
                                   uint32_t* counters, uint64_t* fsig, uint32_t need, uint32_t* release, int* nsig,
                                   Stream s) {
        int32_t n = 0;
        // STENCIL_SLAB_GATE_SKIP=1 (debug library, the test that shows the
        // gate has teeth): a need every word meets, so nothing waits
        if (knob("STENCIL_SLAB_GATE_SKIP", 0)) need = 0;
        const int rc = stencil_sweepk_signal_gated(l, src, dst, b, e, k, counters, fsig, need, release, &n, s);
        *nsig = n;
        return rc;
    }
    static int exchange_done(uint32_t* counters, uint32_t value, Stream s) {
        return stencil_exchange_done(counters, value, s);
    }
    static int read_timeout(uint32_t* flag, bool* timed_out) {
        *timed_out = __atomic_load_n(flag, __ATOMIC_SEQ_CST) != 0;
        return STENCIL_OK;
    }
    static int copy_d2d(void* dst, const void* src, size_t bytes, Stream s) {
        STENCIL_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
        return STENCIL_OK;
    }
    static int copy_peer(void* dst, int ddev, const void* src, int sdev, size_t bytes, Stream s) {
        STENCIL_HIP_CHECK(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, s));
        return STENCIL_OK;
    }
    static int fill_initial(const stencil_layout* l, void* g, int kind, uint64_t seed, Stream s) {
        return stencil_fill_initial(l, g, kind, seed, s);
    }
    static int upload(const stencil_layout* l, void* g, const void* h, int64_t row, int64_t rows, Stream s) {
        return stencil_upload(l, g, h, row, rows, s);
    }
    static int download(const stencil_layout* l, const void* g, void* h, int64_t row, int64_t rows, Stream s) {
        return stencil_download(l, g, h, row, rows, s);
    }
    static int plane_sums(const stencil_layout* l, const void* g, double* out, Stream s) {
        return stencil_plane_sums(l, g, out, s);
    }
    // communicator (RCCL, dlopen'ed)
    static bool comm_available() { return rccl().ok; }
    static int comm_init_all(Comm* comms, int n, const int* devs) {
        const ncclResult_t e = rccl().CommInitAll(comms, n, devs);
        if (e != ncclSuccess) return set_error(STENCIL_EHIP, "ncclCommInitAll(%d) failed: %s", n, rccl().GetErrorString(e));
        return STENCIL_OK;
    }
    // ncclCommInitRank is a collective: it returns once every rank of the id
    // has joined, and waits for a missing rank forever.  It runs on a helper
    // thread (on the caller's device) and the caller waits at most
    // `timeout_ms`; past that it gets STENCIL_ETIMEOUT and the helper is left
    // behind, blocked in RCCL's bootstrap -- it destroys the communicator
    // itself should the missing ranks join after all (nobody else holds it).
    // A nonblocking communicator could be aborted instead, but its every
    // group end returns before RCCL's kernels are queued, which the rounds'
    // event brackets on the exchange stream cannot allow.
    struct InitCall {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclComm_t comm = nullptr;
        ncclResult_t res = ncclSuccess;
        bool device_ok = true;
    };
    static int comm_init_rank(Comm* comm, int nranks, const void* id, int rank, int64_t timeout_ms) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        int dev = 0;
        STENCIL_HIP_CHECK(hipGetDevice(&dev));
        auto call = std::make_shared<InitCall>();
        try {
            std::thread([call, u, nranks, rank, dev] {
                ncclComm_t c = nullptr;
                ncclResult_t r = ncclSuccess;
                const bool dok = hipSetDevice(dev) == hipSuccess;
                if (dok) r = rccl().CommInitRank(&c, nranks, u, rank);
                std::lock_guard<std::mutex> lk(call->mu);
                if (call->abandoned) {
                    if (dok && r == ncclSuccess && c) (void)rccl().CommDestroy(c);
                    return;
                }
                call->comm = c;
                call->res = r;
                call->device_ok = dok;
                call->done = true;
                call->cv.notify_all();
            }).detach();
        } catch (const std::exception& e) {
            return set_error(STENCIL_EHIP, "communicator creation: no helper thread (%s)", e.what());
        }
        std::unique_lock<std::mutex> lk(call->mu);
        if (!call->cv.wait_for(lk, std::chrono::milliseconds(std::max<int64_t>(1, timeout_ms)),
                               [&] { return call->done; })) {
            call->abandoned = true;
            return set_error(STENCIL_ETIMEOUT,
                             "ncclCommInitRank(rank %d of %d): not every rank joined within %lld ms "
                             "(STENCIL_SLAB_TIMEOUT_MS)", rank, nranks, (long long)timeout_ms);
        }
        if (!call->device_ok) return set_error(STENCIL_EHIP, "communicator creation: hipSetDevice(%d) failed", dev);
        if (call->res != ncclSuccess)
            return set_error(STENCIL_EHIP, "ncclCommInitRank(%d of %d) failed: %s", rank, nranks,
                             rccl().GetErrorString(call->res));
        *comm = call->comm;
        return STENCIL_OK;
    }
    static void comm_destroy(Comm c) {
        if (rccl().ok) (void)rccl().CommDestroy(c);
    }
    // abort: RCCL's kernels still waiting for a peer return (and the comm is freed)
    static void comm_abort(Comm c) {
        if (rccl().ok) (void)rccl().CommAbort(c);
    }
    static void comm_set_timeout(Comm, int64_t) {}  // the bound is enforced by the polling waits
    static int group_start() {
        SLAB_NCCL_CHECK(rccl().GroupStart());
        return STENCIL_OK;
    }
    static int group_end() {
        SLAB_NCCL_CHECK(rccl().GroupEnd());
        return STENCIL_OK;
    }
    static int send(const void* p, size_t bytes, int peer, Comm c, Stream s) {
        SLAB_NCCL_CHECK(rccl().Send(p, bytes, ncclChar, peer, c, s));
        return STENCIL_OK;
    }
    static int recv(void* p, size_t bytes, int peer, Comm c, Stream s) {
        SLAB_NCCL_CHECK(rccl().Recv(p, bytes, ncclChar, peer, c, s));
        return STENCIL_OK;
    }
};

static_assert(sizeof(ncclUniqueId) == STENCIL_SLAB_ID_BYTES, "RCCL id size");

}  // namespace stencil

struct stencil_slab_job : stencil::slab::Job<stencil::HipDev> {};

using stencil::HipDev;
namespace core = stencil::slab;

extern "C" {

int stencil_slab_create(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange_kind,
                        int32_t flags, stencil_slab_job** job) {
    return core::create<HipDev>(global, ngpus, devices, exchange_kind, flags, 0, job);
}

int stencil_slab_create2(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange_kind,
                         int32_t flags, int64_t margin_planes, stencil_slab_job** job) {
    return core::create<HipDev>(global, ngpus, devices, exchange_kind, flags, margin_planes, job);
}

int stencil_slab_unique_id(void* id, int64_t bytes) {
    if (!id || bytes < int64_t(sizeof(stencil::ncclUniqueId)))
        return stencil::set_error(STENCIL_EINVAL, "the id buffer needs %d bytes", int(sizeof(stencil::ncclUniqueId)));
    if (!stencil::rccl().ok) return stencil::set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    stencil::ncclUniqueId u;
    const stencil::ncclResult_t e = stencil::rccl().GetUniqueId(&u);
    if (e != stencil::ncclSuccess)
        return stencil::set_error(STENCIL_EHIP, "ncclGetUniqueId failed: %s", stencil::rccl().GetErrorString(e));
    std::memcpy(id, &u, sizeof(u));
    stencil::clear_error();
    return STENCIL_OK;
}

int stencil_slab_create_rank(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device,
                             const void* id, int64_t id_bytes, int32_t flags, stencil_slab_job** job) {
    return core::create_rank<HipDev>(global, nranks, rank, device, id, id_bytes, flags, 0, job);
}

int stencil_slab_create_rank2(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device,
                              const void* id, int64_t id_bytes, int32_t flags, int64_t margin_planes,
                              stencil_slab_job** job) {
    return core::create_rank<HipDev>(global, nranks, rank, device, id, id_bytes, flags, margin_planes, job);
}

int stencil_slab_destroy(stencil_slab_job* job) {
    core::release<HipDev>(job);
    return STENCIL_OK;
}

int stencil_slab_info(const stencil_slab_job* job, int32_t slab, int64_t* first_plane, int64_t* planes,
                      int32_t* device, int32_t* sweeps_per_round) {
    return core::info<HipDev>(job, slab, first_plane, planes, device, sweeps_per_round);
}

int stencil_slab_rolling_info(const stencil_slab_job* job, int64_t* margin_planes, int64_t* launches_per_pass) {
    return core::rolling_info<HipDev>(job, margin_planes, launches_per_pass);
}

int stencil_slab_fill_initial(stencil_slab_job* job, int32_t init_kind, uint64_t seed) {
    return core::fill_initial<HipDev>(job, init_kind, seed);
}

int stencil_slab_upload(stencil_slab_job* job, const void* host, int64_t host_row, int64_t host_rows) {
    return core::upload<HipDev>(job, host, host_row, host_rows);
}

int stencil_slab_run(stencil_slab_job* job, uint32_t iterations, float* elapsed_ms) {
    const stencil::SustainedScope sustained(iterations >= stencil::kSustainedSweeps);
    return core::run<HipDev>(job, iterations, elapsed_ms);
}

int stencil_slab_download(stencil_slab_job* job, void* host, int64_t host_row, int64_t host_rows) {
    return core::download<HipDev>(job, host, host_row, host_rows);
}

int stencil_slab_kernel_timing(stencil_slab_job* job, int32_t enable) {
    return core::kernel_timing<HipDev>(job, enable);
}

int stencil_slab_kernel_time(stencil_slab_job* job, float* total_ms, int64_t* launches, int64_t* cells_per_launch,
                             int32_t* signalled) {
    return core::kernel_time<HipDev>(job, total_ms, launches, cells_per_launch, signalled);
}

int stencil_slab_exchange_time(stencil_slab_job* job, float* transfer_ms, float* beside_ms, int64_t* exchanges) {
    return core::exchange_time<HipDev>(job, transfer_ms, beside_ms, exchanges);
}

int stencil_slab_plane_sums(stencil_slab_job* job, double* sums) {
    return core::plane_sums<HipDev>(job, sums);
}

int stencil_slab_round_form(const stencil_slab_job* job, int32_t* form) {
    return core::round_form<HipDev>(job, form);
}

int stencil_slab_round_info(const stencil_slab_job* job, int32_t* form, int32_t* gated, int32_t* confined) {
    return core::round_info<HipDev>(job, form, gated, confined);
}

int stencil_slab_exchange_budget(const stencil_slab_job* job, int32_t* cus, int32_t* alt_cus, float* round_ms,
                                 float* alt_round_ms) {
    return core::exchange_budget<HipDev>(job, cus, alt_cus, round_ms, alt_round_ms);
}

int stencil_slab_set_timeout(stencil_slab_job* job, int64_t timeout_ms) {
    return core::set_timeout<HipDev>(job, timeout_ms);
}

}  // extern "C"
