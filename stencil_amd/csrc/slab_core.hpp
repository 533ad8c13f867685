// slab_core.hpp -- the multi-GPU z-slab job (include/stencil_hip.h part 3),
// written once over a device backend.
//
// The reference runs its whole decomposed job behind one kernel call: 64
// CPEs own 8x8 blocks, exchange halo strips by DMA / RMA every iteration and
// meet at a barrier (athread_spawn/join, src/stencil/stencil.cpp:34-53; halo
// DMA stencil_dma.cpp:236-247; barrier 562-563; RMA stencil_rma.cpp:198-255;
// the block cut include/stencil/boundary_matrix.hpp:190-218).  Here the blocks
// are contiguous z-slabs of the global grid, one per GPU (remainder planes to
// the lowest slabs), each with K ghost planes per shared face, where K is the
// number of sweeps stencil_iterate fuses into one launch for the problem
// (7-point star: 4 or 5; box: 3 or 4): one round = K fused sweeps + one
// exchange of K whole planes with each neighbour (temporal blocking across
// GPUs; the halo planes are advanced on chip).  Every cell's arithmetic is
// the single-grid kernel's: results are bitwise those of one grid.
//
// Three round forms:
//   boundary + interior  stream A (high priority): the K boundary planes of
//                        each face, then the exchange; stream B: the interior
//                        meanwhile.
//   face-signalled       ONE launch per slab whose workgroups storing the face
//                        planes add to the slab's counters; the exchange
//                        stream waits for the counts and sends while the rest
//                        of the launch runs.
//   rolling              ONE resident grid per slab plus a margin of spare
//                        planes (stencil_rolling_*): a pass of
//                        K sweeps is ceil(n / S) z-range launches writing the
//                        new grid D planes down (or back up), then the
//                        exchange -- for slabs whose two grids do not fit
//                        (the north star's 4096^3 fp64 on 2 GPUs: one 278 GB
//                        grid per GPU).
// Exchange: RCCL ncclSend/ncclRecv inside one group spanning every slab this
// process drives, or device copies (slabs may then share a GPU).
//
// `Dev` supplies streams, events, memory, the sweeps and the communicator:
// csrc/slab.hip's HipDev (HIP + RCCL, the product) and the CPU test build's
// fake device (tests/cpu_slab/: synchronous plane copies and the oracle's
// sweep, an in-process mailbox for send/recv), which runs this same round
// logic at world 2/3 under `pytest -m "not gpu"`.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <utility>
#include <vector>

#include "errors.hpp"
#include "stencil_hip.h"

namespace stencil {
namespace slab {

template <class Dev>
struct Slab {
    int device = 0;
    int index = 0;             // global slab index (= communicator rank)
    int64_t first = 0, n = 0;  // global first plane, planes owned
    stencil_layout l{};
    // two grids a / b; rolling: `a` is the one allocation (margin + grid), b null
    void* a = nullptr;
    void* b = nullptr;
    typename Dev::Stream sa{}, sb{};  // boundary launches (high priority) / interior
    // the exchange: its own queue, which HipDev may confine to a few CUs per
    // XCD (STENCIL_SLAB_XCU), bracketed by events so that A sees it in order
    typename Dev::Stream sx{};
    typename Dev::Event ev_bnd{}, ev_int{}, ev_join{}, ev_xin{}, ev_xout{};
    // the last kInflight rounds' exchange completions: run() keeps at most
    // that many rounds queued and waits for them with the job's deadline
    std::vector<typename Dev::Event> ring;
    typename Dev::Comm comm{};
    // face-signalled rounds: [0] low-face adds, [1] high-face adds (they run
    // on across launches); tflag: the wait kernel's timeout flag (host-
    // coherent on HIP: the host releases a queued wait by setting it)
    uint32_t* counters = nullptr;
    uint32_t* tflag = nullptr;
    uint32_t sig_target = 0;  // adds per face expected once the last queued launch is done
    // STENCIL_SLAB_CPWAIT: the launch also adds 1 per completed face to this
    // HIP signal word, and the exchange stream waits on it in the command
    // processor (hipStreamWaitValue64) instead of a polling wait kernel
    uint64_t* fsig = nullptr;
    uint64_t fsig_target = 0;
    // halo-gated rounds (Job::gate): exchanges issued on X since the last
    // reset; each one's completion stores its number in counters[3]
    // (Dev::exchange_done), which the next launch's halo-reading workgroups
    // wait for instead of the launch's queue waiting for X's event
    uint32_t xseq = 0;
    // overlapped rolling rounds: the new grid's faces are computed into the
    // send staging xs and travel from there while the pass runs; the
    // neighbours' faces land in the receive staging xr and are copied into
    // the halo slots after the pass (2 x depth planes each: lo face, hi face)
    void* xs = nullptr;
    void* xr = nullptr;
    // staged rounds: the face span F (0 = the default n / 4 until tuned) and
    // the timing events of the tuning rounds (B on its stream, the exchange)
    int64_t face_span = 0;
    typename Dev::Event tb0{}, tb1{}, tx0{}, tx1{}, tr0{};
    // staged rounds with a confined exchange: the alternative CU budget's
    // streams (Dev::xcu_alt CUs per XCD for the exchange, the middle launch
    // off them), swapped in for one timed tuning round and kept where that
    // round ran faster (staged_tuning_step); xcu = CUs per XCD in use,
    // round_ms = the tuning rounds' times with the default / alternative
    typename Dev::Stream sx_alt{}, sb_alt{};
    int xcu = 0;
    float round_ms[2] = {0.f, 0.f};
    float b_ms[2] = {0.f, 0.f}, x_ms[2] = {0.f, 0.f};
    // the grid placement chosen at creation (place_grids): candidates tried
    // and the chosen pair's ms per K-step launch
    int placements = 1;
    float placement_ms = 0.f;
};

template <class Dev>
struct Job {
    stencil_problem global{};
    int exchange = STENCIL_EXCHANGE_RCCL;
    bool periodic = false;
    int k = 1;       // sweeps per round (fused launch depth)
    int depth = 1;   // halo planes exchanged per face
    bool cur_is_a = true;
    bool chained = false;  // round events recorded since the last join
    bool signal = false;   // full rounds as face-signalled single launches
    // face-signalled rounds whose launches gate their halo-reading workgroups
    // on the exchange-completion word (Dev::halo_gate): the launch queue never
    // waits for the exchange queue; gate_chain = the last round issued was
    // such a launch, so the next one may skip the event wait
    bool gate = false;
    bool gate_chain = false;
    bool serial = false;   // full rounds as ONE plain launch, then the exchange (STENCIL_SLAB_SERIAL)
    int nranks = 0;        // rank mode: slabs of the job, this process owns s[0]
    // rolling (STENCIL_SLAB_ROLLING): spare planes below each slab's grid;
    // position 0 = the grid at home (allocation offset `margin` planes), 1 =
    // shifted to the allocation's start
    int64_t margin = 0;
    int position = 0;
    bool roll_overlap = false;  // rolling rounds with the exchange beside the pass (staged faces)
    bool confine = false;       // the exchange on a few CUs of its own, the launches off them
    bool staged = false;        // full rounds: face ranges, then the middle beside the exchange
    int tune_left = 2;          // staged: timed rounds left before the face span is set
    int tune_done = 0;          // staged: timed tuning rounds run (the first: RCCL's connection set-up)
    int xcu_alt = 0;            // staged + confined: the alternative exchange CU budget tried (0: none)
    bool tuning = false;        // this round records the tuning events
    std::vector<Slab<Dev>> s;
    // kernel timing: events around slab 0's compute launch(es) of every round
    bool timing = false;
    std::vector<std::pair<typename Dev::Event, typename Dev::Event>> tev;
    int64_t timed_cells = 0;
    int64_t timed_launches = 0;  // kernel launches inside the timed spans
    // with timing on, the exchange of each timed round on slab 0's X: from
    // the end of what precedes the transfers there (a face wait) to the end
    // of the transfers; xev[i] belongs to the round of tev[i]
    std::vector<std::pair<typename Dev::Event, typename Dev::Event>> xev;
    bool xopen = false;
    // bounded-time failure: every wait for the devices gives up after
    // timeout_ms (a peer that stopped posting leaves RCCL's receive spinning);
    // the job then aborts its communicators and every later call fails with
    // `failed` (destroy is the only thing left to do)
    int64_t timeout_ms = 60000;
    int failed = STENCIL_OK;
    uint64_t rounds = 0;  // rounds issued (the in-flight ring's index)
};

constexpr int kInflight = 8;  // rounds queued ahead of the last completed exchange

// the roles of a slab's streams (Dev::stream_create): boundary launches (high
// priority), the interior / whole-slab launches, the halo exchange
enum StreamRole { STREAM_BOUNDARY = 0, STREAM_INTERIOR = 1, STREAM_EXCHANGE = 2 };

using Clock = std::chrono::steady_clock;

#define SLAB_TRY(expr)               \
    do {                             \
        if (int rc_ = (expr)) return rc_; \
    } while (0)

// ---- geometry -------------------------------------------------------------
template <class Dev>
inline size_t elem_bytes(const Slab<Dev>& s) { return s.l.prob.dtype == STENCIL_F64 ? 8 : 4; }
template <class Dev>
inline size_t plane_bytes(const Slab<Dev>& s) { return size_t(s.l.plane) * elem_bytes(s); }
// first byte of plane z of the grid based at `grid` (z may be a ghost/halo plane)
template <class Dev>
inline char* plane_ptr(const Slab<Dev>& s, void* grid, int64_t z) {
    return static_cast<char*>(grid) + size_t(s.l.zghost + z) * plane_bytes(s);
}
// the grid of slab s at rolling position `pos` (two grids: a for pos 0, b for 1)
template <class Dev>
inline void* grid_at(const Job<Dev>& j, const Slab<Dev>& s, int pos) {
    if (j.margin == 0) return pos == 0 ? s.a : s.b;
    return pos == 0 ? static_cast<char*>(s.a) + size_t(j.margin) * plane_bytes(s) : s.a;
}
template <class Dev>
inline int cur_pos(const Job<Dev>& j) { return j.margin ? j.position : (j.cur_is_a ? 0 : 1); }
template <class Dev>
inline void* cur_grid(const Job<Dev>& j, const Slab<Dev>& s) { return grid_at(j, s, cur_pos(j)); }

// neighbours of global slab i (its communicator peers); -1: a global end
template <class Dev>
inline int slabs_total(const Job<Dev>& j) { return j.nranks ? j.nranks : int(j.s.size()); }
template <class Dev>
inline int lo_nb(const Job<Dev>& j, int i) {
    return i > 0 ? i - 1 : (j.periodic ? slabs_total(j) - 1 : -1);
}
template <class Dev>
inline int hi_nb(const Job<Dev>& j, int i) {
    const int n = slabs_total(j);
    return i < n - 1 ? i + 1 : (j.periodic ? 0 : -1);
}

// ---- timing ---------------------------------------------------------------
template <class Dev>
int time_begin(Job<Dev>& j, size_t slab, typename Dev::Stream st) {
    if (!j.timing || slab != 0) return STENCIL_OK;
    typename Dev::Event a{}, b{};
    SLAB_TRY(Dev::event_create(&a, true));
    if (int rc = Dev::event_create(&b, true)) {
        Dev::event_destroy(a);
        return rc;
    }
    j.tev.emplace_back(a, b);
    return Dev::event_record(a, st);
}
template <class Dev>
int time_end(Job<Dev>& j, size_t slab, typename Dev::Stream st, int64_t cells, int64_t launches) {
    if (!j.timing || slab != 0) return STENCIL_OK;
    j.timed_cells = cells;
    j.timed_launches += launches;
    return Dev::event_record(j.tev.back().second, st);
}
// the exchange span of the round whose launch span is open (slab 0 only;
// fill / upload exchanges, outside any round, are not timed)
template <class Dev>
int xspan_begin(Job<Dev>& j, const Slab<Dev>& s) {
    if (!j.timing || &s != &j.s[0] || j.xev.size() >= j.tev.size()) return STENCIL_OK;
    typename Dev::Event a{}, b{};
    SLAB_TRY(Dev::event_create(&a, true));
    if (int rc = Dev::event_create(&b, true)) {
        Dev::event_destroy(a);
        return rc;
    }
    j.xev.emplace_back(a, b);
    j.xopen = true;
    return Dev::event_record(a, s.sx);
}
template <class Dev>
int xspan_end(Job<Dev>& j, const Slab<Dev>& s) {
    if (!j.xopen || &s != &j.s[0]) return STENCIL_OK;
    j.xopen = false;
    return Dev::event_record(j.xev.back().second, s.sx);
}

template <class Dev>
void drop_timing(Job<Dev>& j) {
    for (auto& e : j.tev) {
        Dev::event_destroy(e.first);
        Dev::event_destroy(e.second);
    }
    j.tev.clear();
    for (auto& e : j.xev) {
        Dev::event_destroy(e.first);
        Dev::event_destroy(e.second);
    }
    j.xev.clear();
    j.xopen = false;
    j.timed_cells = 0;
    j.timed_launches = 0;
}

// ---- exchange -------------------------------------------------------------
// Halo exchange of the grids at rolling position `pos` (each slab's copy of
// the same logical grid): every slab's `depth` face planes into its
// neighbours' halo planes.  Faces are contiguous whole planes: nothing is
// packed.  The transfers run on each slab's exchange stream X, bracketed so
// that they behave as if queued on A behind what is already there: X first
// waits for A (ev_xin), then `pre(slab)` queues what must precede the
// transfers on X (a face-signalled round's wait for its faces), and A finally
// waits for X (ev_xout).  On HIP, X is a queue of its own, which may be
// confined to a few CUs per XCD so that RCCL's or the copies' kernels do not
// take the CUs a one-per-CU launch beside them counts on.
struct NoPre {
    template <class S>
    int operator()(S&) const { return STENCIL_OK; }
};

template <class Dev, class Pre = NoPre>
int exchange(Job<Dev>& j, int pos, Pre&& pre = Pre{}) {
    const int n = int(j.s.size());
    const int64_t d = j.depth;
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::event_record(s.ev_xin, s.sa));
        SLAB_TRY(Dev::stream_wait(s.sx, s.ev_xin));
        SLAB_TRY(pre(s));
        SLAB_TRY(xspan_begin(j, s));
        if (j.tuning) SLAB_TRY(Dev::event_record(s.tx0, s.sx));
        // tests / rehearsals: the transfer's wire time between distinct GPUs (a no-op unless asked for)
        SLAB_TRY(Dev::wire_delay(s.sx, size_t(d) * plane_bytes(s)));
        SLAB_TRY(Dev::event_record(s.ev_join, s.sx));  // this slab's faces are ready
    }
    if (j.exchange == STENCIL_EXCHANGE_RCCL) {
        SLAB_TRY(Dev::group_start());
        int rc = STENCIL_OK;
        for (int i = 0; i < n && rc == STENCIL_OK; ++i) {
            Slab<Dev>& s = j.s[size_t(i)];
            void* g = grid_at(j, s, pos);
            const size_t bytes = size_t(d) * plane_bytes(s);
            const int lo = lo_nb(j, s.index), hi = hi_nb(j, s.index);
            // sends and receives to one peer match in posting order: a slab
            // that is its own neighbour (periodic, N = 1) sends hi -> recv lo
            // first, then lo -> hi
            if (hi >= 0 && rc == STENCIL_OK) rc = Dev::send(plane_ptr(s, g, s.n - d), bytes, hi, s.comm, s.sx);
            if (lo >= 0 && rc == STENCIL_OK) rc = Dev::recv(plane_ptr(s, g, -d), bytes, lo, s.comm, s.sx);
            if (lo >= 0 && rc == STENCIL_OK) rc = Dev::send(plane_ptr(s, g, 0), bytes, lo, s.comm, s.sx);
            if (hi >= 0 && rc == STENCIL_OK) rc = Dev::recv(plane_ptr(s, g, s.n), bytes, hi, s.comm, s.sx);
        }
        const int rc2 = Dev::group_end();
        SLAB_TRY(rc != STENCIL_OK ? rc : rc2);
    } else {
        // device copies (single-process jobs only: local = global index):
        // slab i's X pulls its neighbours' faces once they are ready (ev_join)
        for (int i = 0; i < n; ++i) {
            Slab<Dev>& s = j.s[size_t(i)];
            SLAB_TRY(Dev::set_device(s.device));
            void* g = grid_at(j, s, pos);
            const size_t bytes = size_t(d) * plane_bytes(s);
            const int lo = lo_nb(j, i), hi = hi_nb(j, i);
            SLAB_TRY(Dev::debug_delay(s.sx, i));  // tests: slab 0's pulls slow (a no-op unless asked for)
            if (lo >= 0) {
                Slab<Dev>& t = j.s[size_t(lo)];
                SLAB_TRY(Dev::stream_wait(s.sx, t.ev_join));
                SLAB_TRY(Dev::copy_peer(plane_ptr(s, g, -d), s.device, plane_ptr(t, grid_at(j, t, pos), t.n - d),
                                        t.device, bytes, s.sx));
            }
            if (hi >= 0) {
                Slab<Dev>& t = j.s[size_t(hi)];
                SLAB_TRY(Dev::stream_wait(s.sx, t.ev_join));
                SLAB_TRY(Dev::copy_peer(plane_ptr(s, g, s.n), s.device, plane_ptr(t, grid_at(j, t, pos), 0), t.device,
                                        bytes, s.sx));
            }
        }
    }
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        if (j.tuning) SLAB_TRY(Dev::event_record(s.tx1, s.sx));
        SLAB_TRY(xspan_end(j, s));
        if (j.gate) SLAB_TRY(Dev::exchange_done(s.counters, ++s.xseq, s.sx));
        SLAB_TRY(Dev::event_record(s.ev_xout, s.sx));
    }
    for (int i = 0; i < n; ++i) {
        Slab<Dev>& s = j.s[size_t(i)];
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::stream_wait(s.sa, s.ev_xout));
        if (j.margin && j.exchange == STENCIL_EXCHANGE_COPY && Dev::pull_wait_enabled()) {
            // Rolling slabs: a slab's next pass writes its new grid over the
            // planes its neighbours are still pulling faces from (the grid
            // moves by the shift every round), so every slab waits for its
            // neighbours' pulls first.  Two-grid jobs need no such wait: the
            // next round writes the other grid, and the round after waits on
            // this one.  (RCCL exchanges are ordered by each slab's own X.)
            const int lo = lo_nb(j, i), hi = hi_nb(j, i);
            if (lo >= 0 && lo != i) SLAB_TRY(Dev::stream_wait(s.sa, j.s[size_t(lo)].ev_xout));
            if (hi >= 0 && hi != i && hi != lo) SLAB_TRY(Dev::stream_wait(s.sa, j.s[size_t(hi)].ev_xout));
        }
    }
    return STENCIL_OK;
}

// ---- rounds ---------------------------------------------------------------
// One round of `k` fused sweeps: src -> dst on every slab, then the exchange
// of dst's faces.  Boundary planes on A (the exchange queued behind them),
// the interior on B.
template <class Dev>
int slab_round(Job<Dev>& j, int k) {
    const int src_pos = cur_pos(j), dst_pos = 1 - src_pos;
    const int64_t edge = j.depth;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        void* dst = grid_at(j, s, dst_pos);
        if (j.chained) {
            // interior(r) reads src [0, n): after boundary + exchange(r-1);
            // boundary(r) overwrites planes interior(r-1) read: after it
            SLAB_TRY(Dev::stream_wait(s.sb, s.ev_bnd));
            SLAB_TRY(Dev::stream_wait(s.sa, s.ev_int));
        }
        const int64_t plane_cells = s.l.prob.nx * s.l.prob.ny;
        // serial rounds: the whole slab in one launch on A, the exchange
        // behind it -- nothing runs beside the launch (an overlapped exchange's
        // copy or RCCL kernels take CUs the one-per-CU strip grid counts on)
        if (!j.serial && s.n > 2 * edge) {
            SLAB_TRY(time_begin(j, i, s.sb));
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, edge, s.n - edge, k, s.sb));
            SLAB_TRY(time_end(j, i, s.sb, plane_cells * (s.n - 2 * edge), 1));
            SLAB_TRY(Dev::event_record(s.ev_int, s.sb));
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, 0, edge, k, s.sa));
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, s.n - edge, s.n, k, s.sa));
        } else {
            SLAB_TRY(time_begin(j, i, s.sa));
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, 0, s.n, k, s.sa));
            SLAB_TRY(time_end(j, i, s.sa, plane_cells * s.n, 1));
            SLAB_TRY(Dev::event_record(s.ev_int, s.sa));
        }
        if (j.exchange == STENCIL_EXCHANGE_COPY)  // the face copies read whole rounds
            SLAB_TRY(Dev::stream_wait(s.sa, s.ev_int));
    }
    SLAB_TRY(exchange(j, dst_pos));
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::event_record(s.ev_bnd, s.sa));
    }
    j.chained = true;
    j.cur_is_a = dst_pos == 0;
    return STENCIL_OK;
}

// One round of `k` fused sweeps as ONE face-signalled launch per slab
// (stencil_sweepk_signal): the launch's first z-chunk marches
// up and its last down, so its face planes are among the first stored; the
// workgroups storing them add to the slab's counters.  The exchange stream
// queues a wait for the counts and the halo exchange behind it, so the faces
// leave while the rest of the launch runs.  Order: launch(r) reads the halos
// exchange(r-1) received (B waits for A); exchange(r) receives into the halo
// planes launch(r-1) read, and starts only once launch(r) has signalled,
// i.e. after launch(r-1) ended (one stream).
template <class Dev>
int slab_round_signal(Job<Dev>& j, int k) {
    const int src_pos = cur_pos(j), dst_pos = 1 - src_pos;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        void* dst = grid_at(j, s, dst_pos);
        // the launch reads the halos the last exchange received.  Gated
        // rounds: its halo-reading workgroups wait for that exchange's
        // completion word, and the launch follows the previous round's gated
        // launch on B with no event wait -- that launch's own gated workgroups
        // saw the exchange before it (the grid this launch writes) complete
        // (the cross-queue wait cost ~23 us of a 0.49 ms round at 512^3,
        // DESIGN.md §7).  Otherwise wait for X directly (through A, ev_bnd,
        // costs a third queue hop per round: ~20 us of 500 at 512^3)
        if (j.chained && !(j.gate && j.gate_chain)) SLAB_TRY(Dev::stream_wait(s.sb, s.ev_xout));
        int nsig = 0;
        SLAB_TRY(time_begin(j, i, s.sb));
        if (j.gate)
            SLAB_TRY(Dev::sweepk_signal_gated(&s.l, src, dst, 0, s.n, k, s.counters, s.fsig, s.xseq, s.tflag, &nsig,
                                              s.sb));
        else
            SLAB_TRY(Dev::sweepk_signal(&s.l, src, dst, 0, s.n, k, s.counters, s.fsig, &nsig, s.sb));
        SLAB_TRY(time_end(j, i, s.sb, s.l.prob.nx * s.l.prob.ny * s.n, 1));
        SLAB_TRY(Dev::event_record(s.ev_int, s.sb));
        s.sig_target += uint32_t(nsig);
        if (j.rounds == 0) s.sig_target += uint32_t(Dev::debug_signal_skew());  // tests: a face wait that never ends
        if (s.fsig) s.fsig_target += 2;  // both faces of this launch: +2
    }
    // the wait for the faces goes first on the exchange stream
    SLAB_TRY(exchange(j, dst_pos, [](Slab<Dev>& s) {
        return s.fsig ? Dev::wait_face_signal(s.fsig, s.fsig_target, s.sx)
                      : Dev::wait_counters(s.counters, s.tflag, s.sig_target, s.sig_target, s.sx);
    }));
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::event_record(s.ev_bnd, s.sa));
        // the next round's boundary-launch path (remainders) writes planes
        // this launch reads: A must also follow B
        SLAB_TRY(Dev::stream_wait(s.sa, s.ev_int));
    }
    j.chained = true;
    j.gate_chain = j.gate;
    j.cur_is_a = dst_pos == 0;
    return STENCIL_OK;
}

// One STAGED round of `k` fused sweeps (the default for slabs whose launch
// takes several rounds of workgroups, e.g. 4096^2 planes):
//   A (stream A, every CU): the face ranges [0, F) and [n - F, n) of the new
//     grid, F = n / 4 (at least 2K planes): half the round's work;
//   then, beside each other, the exchange of A's faces (stream X, confined to
//     one CU per XCD) and B (stream B, the other CUs): the middle [F, n - F).
// B starts after A (the launches' z lock-step between neighbouring tiles
// survives; running them concurrently broke it), and the next
// round's A waits for B and for the exchange.  No face signals: A's end is
// the faces' readiness.  The same kernels and sums as one launch of [0, n).
template <class Dev>
inline int64_t staged_face_span(const Job<Dev>& j, const Slab<Dev>& s) {
    if (s.face_span > 0) return s.face_span;
    const int64_t want = std::max<int64_t>((s.n + 3) / 4, 2 * int64_t(j.k));
    return std::min(want, s.n / 2);
}

// The face span after the tuning rounds: B (the middle, beside the exchange)
// is kept 1.25x as long as the measured exchange and no longer, within
// [n / 4, n / 2 - 2K] -- the more of the round's work A does on every CU, the
// less runs on the 248 CUs the confined exchange leaves.  In a rehearsal the
// exchange is a local copy on the confined CUs (NS4096 rank of 4: 9 ms); over
// xGMI it is the wire time.
template <class Dev>
int64_t tuned_face_span(const Job<Dev>& j, const Slab<Dev>& s, float b_ms, float x_ms) {
    const int64_t F = staged_face_span(j, s), mid = s.n - 2 * F;
    const int64_t lo = std::min<int64_t>(std::max<int64_t>((s.n + 3) / 4, 2 * int64_t(j.k)), s.n / 2);
    const int64_t hi = std::max<int64_t>(lo, s.n / 2 - 2 * int64_t(j.k));
    if (mid <= 0 || b_ms <= 0.f) return lo;
    const double per_plane = double(b_ms) / double(mid);
    const int64_t need = int64_t(1.25 * double(x_ms) / per_plane) + 1;
    return std::max(lo, std::min(hi, (s.n - need) / 2));
}

template <class Dev>
int slab_round_staged(Job<Dev>& j, int k) {
    const int src_pos = cur_pos(j), dst_pos = 1 - src_pos;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        void* dst = grid_at(j, s, dst_pos);
        // A(r) writes planes B(r-1) read, and reads the halos exchange(r-1)
        // received (A waits for X in exchange()'s bracket already)
        if (j.chained) SLAB_TRY(Dev::stream_wait(s.sa, s.ev_int));
        const int64_t F = staged_face_span(j, s);
        if (j.tuning) SLAB_TRY(Dev::event_record(s.tr0, s.sa));  // the round's start
        SLAB_TRY(time_begin(j, i, s.sa));
        SLAB_TRY(Dev::sweepk(&s.l, src, dst, 0, F, k, s.sa));
        SLAB_TRY(Dev::sweepk(&s.l, src, dst, s.n - F, s.n, k, s.sa));
        SLAB_TRY(Dev::event_record(s.ev_bnd, s.sa));  // A done: the faces
        SLAB_TRY(Dev::stream_wait(s.sb, s.ev_bnd));
        if (j.tuning) SLAB_TRY(Dev::event_record(s.tb0, s.sb));
        if (s.n > 2 * F) SLAB_TRY(Dev::sweepk(&s.l, src, dst, F, s.n - F, k, s.sb));
        if (j.tuning) SLAB_TRY(Dev::event_record(s.tb1, s.sb));
        SLAB_TRY(time_end(j, i, s.sb, s.l.prob.nx * s.l.prob.ny * s.n, s.n > 2 * F ? 3 : 2));
        SLAB_TRY(Dev::event_record(s.ev_int, s.sb));
    }
    SLAB_TRY(exchange(j, dst_pos));  // X after A (bracket), beside B; A waits for X
    j.chained = true;
    j.cur_is_a = dst_pos == 0;
    return STENCIL_OK;
}

// Launches per pass of a rolling slab: z-ranges of S = margin - K*r planes.
template <class Dev>
inline int64_t rolling_span(const Job<Dev>& j) { return j.margin - int64_t(j.k) * j.global.radius; }

// One rolling pass of `k` sweeps on every slab (the single-GPU scheme of
// stencil_rolling_iterate, api.hip, per slab): from home the new grid goes D
// planes down, launches bottom-up; from the shifted position back up,
// launches top-down.  A launch over [jS, jS + S) reads slots [jS - kr,
// jS + S + kr) and writes [jS - D, jS + S - D) (down): disjoint, and no later
// launch of the pass reads what it writes.  Then the new grid's halo planes:
// a shared face's from the neighbour (the exchange, queued behind the pass on
// the same stream, so it starts once every launch that reads those slots is
// done), a global end's ghost planes by one plane copy from the slots no pass
// writes (the shifted grid's bottom ghosts, the home grid's top ghosts).
template <class Dev>
int slab_round_rolling(Job<Dev>& j, int k) {
    const int64_t S = rolling_span(j);
    const bool down = j.position == 0;
    const int src_pos = j.position, dst_pos = 1 - j.position;
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        void* dst = grid_at(j, s, dst_pos);
        const int64_t J = (s.n + S - 1) / S;
        SLAB_TRY(time_begin(j, i, s.sa));
        for (int64_t q = 0; q < J; ++q) {
            const int64_t jj = down ? q : J - 1 - q;
            const int64_t b = jj * S, e = std::min(s.n, b + S);
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, b, e, k, s.sa));
        }
        SLAB_TRY(time_end(j, i, s.sa, s.l.prob.nx * s.l.prob.ny * s.n, J));
        const int64_t zg = s.l.zghost;
        const size_t pb = plane_bytes(s);
        const bool has_lo = lo_nb(j, s.index) >= 0, has_hi = hi_nb(j, s.index) >= 0;
        if (down && !has_hi)  // the shifted grid's top ghosts from the home grid's (never written)
            SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, s.n), plane_ptr(s, src, s.n), size_t(zg) * pb, s.sa));
        if (!down && !has_lo)  // the home grid's bottom ghosts from the shifted grid's (never written)
            SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, -zg), plane_ptr(s, src, -zg), size_t(zg) * pb, s.sa));
    }
    SLAB_TRY(exchange(j, dst_pos));
    j.position = dst_pos;
    j.chained = false;  // one stream per slab: nothing to chain
    return STENCIL_OK;
}

// The overlapped rolling round (the default for rolling slabs with a shared
// face; STENCIL_SLAB_ROLLING_OVERLAP=0 runs the serial form above).  In the
// serial form the exchange must wait for the whole pass: the new grid's late
// face is written by the pass's last launch, and the halo slots it receives
// into are home-grid planes the last launches still read.  Here, per slab:
//   1. on A, the new grid's faces [0, d) and [n - d, n) are computed first,
//      from the old grid (whole before the pass), into the send staging xs:
//      one stencil_sweepk of d planes each, the same kernels and sums as the
//      pass, so the bits are those the pass writes into the grid;
//   2. on X, the exchange from xs into the neighbours' receive staging xr,
//      as soon as those launches are done -- beside the pass;
//   3. on A, the pass (unchanged, it still writes the face planes);
//   4. on A, after the pass and the exchange, xr into the new grid's halo
//      slots (d planes per shared face), and the global ends' ghost restores.
// The reference overlaps the same way: halo DMA issued before the interior
// rows and waited for after them (stencil_dma.cpp:426, 448), edge results
// put as each edge is computed (stencil_dma.cpp:475-559).
template <class Dev>
inline void* staged_grid(const Slab<Dev>& s, void* buf, int64_t b) {
    // the base whose plane b is buf's first plane (sweepk writes only [b, e))
    return static_cast<char*>(buf) - size_t(s.l.zghost + b) * plane_bytes(s);
}

template <class Dev>
int slab_round_rolling_overlap(Job<Dev>& j, int k) {
    const int64_t S = rolling_span(j);
    const int64_t d = j.depth;
    const bool down = j.position == 0;
    const int src_pos = j.position, dst_pos = 1 - j.position;
    const int n = int(j.s.size());
    // 1. the faces into the send staging
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        const size_t pb = plane_bytes(s);
        SLAB_TRY(time_begin(j, i, s.sa));  // the timed span: the face launches and the pass
        if (lo_nb(j, s.index) >= 0) SLAB_TRY(Dev::sweepk(&s.l, src, staged_grid(s, s.xs, 0), 0, d, k, s.sa));
        if (hi_nb(j, s.index) >= 0)
            SLAB_TRY(Dev::sweepk(&s.l, src, staged_grid(s, static_cast<char*>(s.xs) + size_t(d) * pb, s.n - d), s.n - d,
                                 s.n, k, s.sa));
        SLAB_TRY(Dev::event_record(s.ev_join, s.sa));  // this slab's faces are staged
    }
    // 2. the exchange on X, from the staging, beside the pass
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::stream_wait(s.sx, s.ev_join));
        SLAB_TRY(xspan_begin(j, s));
        SLAB_TRY(Dev::wire_delay(s.sx, size_t(d) * plane_bytes(s)));  // rehearsals: a distinct GPU's wire time
    }
    if (j.exchange == STENCIL_EXCHANGE_RCCL) {
        SLAB_TRY(Dev::group_start());
        int rc = STENCIL_OK;
        for (int i = 0; i < n && rc == STENCIL_OK; ++i) {
            Slab<Dev>& s = j.s[size_t(i)];
            const size_t pb = plane_bytes(s), bytes = size_t(d) * pb;
            char* xs = static_cast<char*>(s.xs);
            char* xr = static_cast<char*>(s.xr);
            const int lo = lo_nb(j, s.index), hi = hi_nb(j, s.index);
            // the posting order of exchange(): a slab that is its own
            // neighbour sends hi -> receives lo first
            if (hi >= 0 && rc == STENCIL_OK) rc = Dev::send(xs + bytes, bytes, hi, s.comm, s.sx);
            if (lo >= 0 && rc == STENCIL_OK) rc = Dev::recv(xr, bytes, lo, s.comm, s.sx);
            if (lo >= 0 && rc == STENCIL_OK) rc = Dev::send(xs, bytes, lo, s.comm, s.sx);
            if (hi >= 0 && rc == STENCIL_OK) rc = Dev::recv(xr + bytes, bytes, hi, s.comm, s.sx);
        }
        const int rc2 = Dev::group_end();
        SLAB_TRY(rc != STENCIL_OK ? rc : rc2);
    } else {
        for (int i = 0; i < n; ++i) {
            Slab<Dev>& s = j.s[size_t(i)];
            SLAB_TRY(Dev::set_device(s.device));
            const size_t bytes = size_t(d) * plane_bytes(s);
            const int lo = lo_nb(j, i), hi = hi_nb(j, i);
            SLAB_TRY(Dev::debug_delay(s.sx, i));
            if (lo >= 0) {  // the low neighbour's high face
                Slab<Dev>& t = j.s[size_t(lo)];
                SLAB_TRY(Dev::stream_wait(s.sx, t.ev_join));
                SLAB_TRY(Dev::copy_peer(s.xr, s.device, static_cast<char*>(t.xs) + bytes, t.device, bytes, s.sx));
            }
            if (hi >= 0) {  // the high neighbour's low face
                Slab<Dev>& t = j.s[size_t(hi)];
                SLAB_TRY(Dev::stream_wait(s.sx, t.ev_join));
                SLAB_TRY(Dev::copy_peer(static_cast<char*>(s.xr) + bytes, s.device, t.xs, t.device, bytes, s.sx));
            }
        }
    }
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(xspan_end(j, s));
        SLAB_TRY(Dev::event_record(s.ev_xout, s.sx));
    }
    // 3. the pass, 4. the halos out of the staging
    for (size_t i = 0; i < j.s.size(); ++i) {
        Slab<Dev>& s = j.s[i];
        SLAB_TRY(Dev::set_device(s.device));
        void* src = grid_at(j, s, src_pos);
        void* dst = grid_at(j, s, dst_pos);
        const int64_t J = (s.n + S - 1) / S;
        for (int64_t q = 0; q < J; ++q) {
            const int64_t jj = down ? q : J - 1 - q;
            const int64_t b = jj * S, e = std::min(s.n, b + S);
            SLAB_TRY(Dev::sweepk(&s.l, src, dst, b, e, k, s.sa));
        }
        const int64_t lo = lo_nb(j, int(s.index)), hi = hi_nb(j, int(s.index));
        SLAB_TRY(time_end(j, i, s.sa, s.l.prob.nx * s.l.prob.ny * s.n, J + (lo >= 0) + (hi >= 0)));
        const int64_t zg = s.l.zghost;
        const size_t pb = plane_bytes(s), bytes = size_t(d) * pb;
        if (down && hi < 0)  // the shifted grid's top ghosts from the home grid's (never written)
            SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, s.n), plane_ptr(s, src, s.n), size_t(zg) * pb, s.sa));
        if (!down && lo < 0)  // the home grid's bottom ghosts from the shifted grid's (never written)
            SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, -zg), plane_ptr(s, src, -zg), size_t(zg) * pb, s.sa));
        SLAB_TRY(Dev::stream_wait(s.sa, s.ev_xout));
        if (lo >= 0) SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, -d), s.xr, bytes, s.sa));
        if (hi >= 0) SLAB_TRY(Dev::copy_d2d(plane_ptr(s, dst, s.n), static_cast<char*>(s.xr) + bytes, bytes, s.sa));
        if (j.exchange == STENCIL_EXCHANGE_COPY && Dev::pull_wait_enabled()) {
            // the neighbours pulled from this slab's xs, which the next
            // round's face launches overwrite
            if (lo >= 0 && lo != int64_t(i)) SLAB_TRY(Dev::stream_wait(s.sa, j.s[size_t(lo)].ev_xout));
            if (hi >= 0 && hi != int64_t(i) && hi != lo) SLAB_TRY(Dev::stream_wait(s.sa, j.s[size_t(hi)].ev_xout));
        }
    }
    j.position = dst_pos;
    j.chained = false;
    return STENCIL_OK;
}

// Did a face-counter wait give up?  Then the halos are wrong.
template <class Dev>
int check_signal_timeouts(Job<Dev>& j) {
    for (Slab<Dev>& s : j.s) {
        if (!s.counters) continue;
        SLAB_TRY(Dev::set_device(s.device));
        bool timed_out = false;
        SLAB_TRY(Dev::read_timeout(s.tflag, &timed_out));
        if (timed_out) return set_error(STENCIL_ETIMEOUT, "slab on device %d: a face-counter wait timed out", s.device);
    }
    return STENCIL_OK;
}

// ---- bounded-time failure ---------------------------------------------------
// A failure the job cannot recover from (a device wait past the deadline, an
// asynchronous RCCL error, a failed launch): abort the communicators (RCCL's
// kernels waiting for a peer that stopped posting then return), release any
// face-signal or face-counter wait still queued, and make every later call
// fail.  Keeps the message of the error that caused it.
template <class Dev>
int fail(Job<Dev>& j, int rc) {
    if (rc == STENCIL_OK || j.failed) return rc;
    j.failed = rc;
    // the waits first: RCCL's kernels may be queued behind them, and an
    // abort that waited for those would wait for the waits
    for (Slab<Dev>& s : j.s) {
        (void)Dev::set_device(s.device);
        Dev::release_waits(s.tflag, s.fsig);
    }
    for (Slab<Dev>& s : j.s) {
        (void)Dev::set_device(s.device);
        if (s.comm) {
            Dev::comm_abort(s.comm);
            s.comm = typename Dev::Comm{};
        }
    }
    return rc;
}

template <class Dev>
int check_alive(const Job<Dev>& j) {
    if (!j.failed) return STENCIL_OK;
    return set_error(j.failed, "the slab job failed earlier (its communicators were aborted): destroy it");
}

// Wait for everything queued on every slab's streams, at most until the job's
// deadline; a failure fails the job.
template <class Dev>
int sync_bounded(Job<Dev>& j) {
    SLAB_TRY(check_alive(j));
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(j.timeout_ms);
    for (Slab<Dev>& s : j.s) {
        if (int rc = Dev::set_device(s.device)) return fail(j, rc);
        for (typename Dev::Stream st : {s.sx, s.sa, s.sb})
            if (int rc = Dev::sync_until(st, s.comm, deadline)) return fail(j, rc);
    }
    j.chained = false;
    j.gate_chain = false;
    return STENCIL_OK;
}

// Before issuing a round: at most kInflight rounds may be queued behind the
// last exchange known complete (this bounds the queues, and a peer that
// stopped posting is noticed while rounds are issued, not only at the end).
template <class Dev>
int throttle(Job<Dev>& j) {
    if (j.rounds < uint64_t(kInflight)) return STENCIL_OK;
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(j.timeout_ms);
    for (Slab<Dev>& s : j.s) {
        if (int rc = Dev::set_device(s.device)) return fail(j, rc);
        if (int rc = Dev::event_sync_until(s.ring[size_t(j.rounds % kInflight)], s.comm, deadline)) return fail(j, rc);
    }
    return STENCIL_OK;
}
template <class Dev>
int mark_round(Job<Dev>& j) {
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::event_record(s.ring[size_t(j.rounds % kInflight)], s.sx));
    }
    ++j.rounds;
    return STENCIL_OK;
}

// ---- lifetime -------------------------------------------------------------
template <class Dev, class JobT>
void release(JobT* j) {
    if (!j) return;
    if (!j->s.empty()) {
        (void)Dev::set_device(j->s[0].device);
        drop_timing(*j);
    }
    // drain the queues within the job's deadline; if they do not drain, fail
    // the job (abort the communicators, release the waits) and try once more;
    // memory still in use then is leaked rather than freed under a kernel
    auto drain = [&]() {
        bool ok = true;
        const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(j->timeout_ms);
        for (Slab<Dev>& s : j->s) {
            (void)Dev::set_device(s.device);
            for (typename Dev::Stream st : {s.sx, s.sa, s.sb})
                if (st) ok = Dev::sync_until(st, s.comm, deadline) == STENCIL_OK && ok;
        }
        return ok;
    };
    bool drained = drain();
    if (!drained) {
        (void)fail(*j, STENCIL_ETIMEOUT);
        drained = drain();
    }
    for (Slab<Dev>& s : j->s) {
        (void)Dev::set_device(s.device);
        if (s.comm) Dev::comm_destroy(s.comm);
        if (!drained) continue;
        for (void* p : {s.a, s.b, s.xs, s.xr})
            if (p) Dev::free(p);
        for (typename Dev::Stream st : {s.sx, s.sa, s.sb, s.sx_alt, s.sb_alt})
            if (st) Dev::stream_destroy(st);
        for (typename Dev::Event e : {s.ev_bnd, s.ev_int, s.ev_join, s.ev_xin, s.ev_xout, s.tb0, s.tb1, s.tx0, s.tx1, s.tr0})
            if (e) Dev::event_destroy(e);
        for (typename Dev::Event e : s.ring)
            if (e) Dev::event_destroy(e);
        if (s.counters) Dev::free_counters(s.counters);
        if (s.tflag) Dev::free_flag(s.tflag);
        if (s.fsig) Dev::face_signal_destroy(s.fsig);
    }
    delete j;
}

// Sweeps stencil_iterate fuses into one launch for `p`: the round length.
// Margin (spare planes) of a rolling slab whose layout is `l`: `want` > 0 as
// asked; 0 = as deep as the device's free memory allows beside the grid, less
// a reserve for the communicator, at most 512 planes.
template <class Dev>
int rolling_margin(const Job<Dev>& j, const stencil_layout& l, int64_t want, int64_t* out) {
    const int64_t reach = int64_t(j.k) * j.global.radius;
    const int64_t pb = l.plane * (l.prob.dtype == STENCIL_F64 ? 8 : 4);
    int64_t m = want;
    if (m <= 0) {
        int64_t free_b = 0;
        SLAB_TRY(Dev::free_bytes(&free_b));
        const int64_t reserve = int64_t(4) << 30;
        m = std::min<int64_t>(512, (free_b - l.bytes - reserve - 256) / pb);
        if (m < 4 * (reach + 1))
            return set_error(STENCIL_ENOMEM, "rolling slab: %lld GB grid + a margin of %lld planes do not fit %lld GB free",
                             (long long)(l.bytes / 1000000000), (long long)(4 * (reach + 1)),
                             (long long)(free_b / 1000000000));
    }
    if (m < reach + 1)
        return set_error(STENCIL_EINVAL, "rolling slab margin must be at least %lld planes (got %lld)",
                         (long long)(reach + 1), (long long)m);
    *out = m;
    return STENCIL_OK;
}

// Where a slab's two grids live: the same launch runs 4-8 %
// apart depending on which physical pages its grids occupy.  Up to
// Dev::placement_trials() candidate pairs (each allocated while the earlier
// ones are held, within a quarter of the free memory), one K-step launch of
// the whole slab timed on each in two interleaved passes, the fastest pair
// kept and the rest freed.  Values do not matter (the grids are filled
// before the job starts); every rank chooses alone, no collective.
template <class Dev>
int place_grids(const Job<Dev>& j, Slab<Dev>& s) {
    const int trials = Dev::placement_trials();
    if (trials <= 1 || !s.a || !s.b) return STENCIL_OK;
    const int64_t bytes = s.l.bytes + 256;
    int64_t free_b = 0;
    SLAB_TRY(Dev::free_bytes(&free_b));
    const int64_t extra = std::min<int64_t>(trials - 1, free_b / 4 / std::max<int64_t>(1, 2 * bytes));
    if (extra <= 0) return STENCIL_OK;
    std::vector<std::pair<void*, void*>> cand{{s.a, s.b}};
    typename Dev::Event e0{}, e1{};
    int rc = Dev::event_create(&e0, true);
    if (rc == STENCIL_OK) rc = Dev::event_create(&e1, true);
    for (int64_t i = 0; i < extra && rc == STENCIL_OK; ++i) {
        void* a = nullptr;
        void* b = nullptr;
        if (Dev::alloc(bytes, &a) != STENCIL_OK) break;  // no room: fewer candidates
        if (Dev::alloc(bytes, &b) != STENCIL_OK) {
            Dev::free(a);
            break;
        }
        cand.emplace_back(a, b);
    }
    clear_error();
    std::vector<float> best(cand.size(), 1e30f);
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(j.timeout_ms);
    for (auto& c : cand)
        for (void* g : {c.first, c.second})
            if (rc == STENCIL_OK) rc = Dev::fill_initial(&s.l, g, STENCIL_INIT_REFERENCE, 0, s.sa);
    for (int w = 0; w < 8 && rc == STENCIL_OK; ++w)  // clock up before the first candidate is timed
        rc = Dev::sweepk(&s.l, cand[0].first, cand[0].second, 0, s.n, j.k, s.sa);
    for (int pass = 0; pass < 2 && rc == STENCIL_OK; ++pass)
        for (size_t i = 0; i < cand.size() && rc == STENCIL_OK; ++i)
            for (int t = 0; t < 3 && rc == STENCIL_OK; ++t) {  // one untimed, two timed launches
                if (t) rc = Dev::event_record(e0, s.sa);
                if (rc == STENCIL_OK) rc = Dev::sweepk(&s.l, cand[i].first, cand[i].second, 0, s.n, j.k, s.sa);
                if (t && rc == STENCIL_OK) rc = Dev::event_record(e1, s.sa);
                if (t && rc == STENCIL_OK) rc = Dev::sync_until(s.sa, typename Dev::Comm{}, deadline);
                float ms = 0.f;
                if (t && rc == STENCIL_OK) rc = Dev::event_elapsed(&ms, e0, e1);
                if (t && rc == STENCIL_OK) best[i] = std::min(best[i], ms);
            }
    size_t pick = 0;
    for (size_t i = 1; i < cand.size(); ++i)
        if (best[i] < best[pick]) pick = i;
    if (rc != STENCIL_OK) pick = 0;  // keep the first pair; the error is returned
    if (e0) Dev::event_destroy(e0);
    if (e1) Dev::event_destroy(e1);
    for (size_t i = 0; i < cand.size(); ++i)
        if (i != pick) {
            Dev::free(cand[i].first);
            Dev::free(cand[i].second);
        }
    if (Dev::placement_verbose()) {
        std::fprintf(stderr, "[slab %d] placement: %zu candidates, ms per launch:", s.index, cand.size());
        for (float v : best) std::fprintf(stderr, " %.4f", double(v));
        std::fprintf(stderr, "; chose %zu\n", pick);
    }
    s.a = cand[pick].first;
    s.b = cand[pick].second;
    s.placement_ms = rc == STENCIL_OK ? best[pick] : 0.f;
    s.placements = int(cand.size());
    return rc;
}

// The slabs this process owns: global slab indices `idx` (of `total`) on
// `devs`; the z split is the same in every process (planes total / N, the first
// nz % N slabs one more), so each rank can build its own share alone.
template <class Dev, class JobT>
int build_job(const stencil_problem& g, int total, const std::vector<int>& idx, const std::vector<int>& devs,
              int32_t exchange_kind, int32_t flags, int64_t margin, bool rank_mode, JobT** out) {
    auto* j = new JobT;
    j->global = g;
    j->exchange = exchange_kind;
    j->periodic = flags & STENCIL_SLAB_PERIODIC;
    j->nranks = rank_mode ? total : 0;
    j->k = Dev::fuse_depth(g);
    j->depth = std::max<int>(j->k, g.radius);
    const bool rolling = flags & STENCIL_SLAB_ROLLING;
    // face-signalled rounds where the K-step kernels have them (3D r = 1 naive
    // 7-point star K = 3..5, box K = 2..4), two-grid slabs only; the product's
    // STENCIL_SLAB_SIGNAL=0: boundary + interior launches
    {
        const bool star = g.shape == STENCIL_STAR && j->k >= 3 && j->k <= 5;
        const bool box = g.shape == STENCIL_BOX && j->k >= 2 && j->k <= 4;
        // and only with one slab per GPU: slabs sharing a GPU multiplex their
        // streams onto its few hardware queues, where a polling wait kernel
        // could sit in front of the launch another slab's wait is polling for
        // (ranks each own one GPU: RCCL refuses two ranks on one device)
        bool distinct = true;
        for (size_t i = 0; i < devs.size(); ++i)
            for (size_t q = 0; q < i; ++q) distinct = distinct && devs[i] != devs[q];
        j->serial = !rolling && Dev::serial_rounds();
        j->signal = g.radius == 1 && g.order == STENCIL_ORDER_NAIVE && (star || box) && distinct && !rolling &&
                    !j->serial && Dev::signal_enabled();
        // A face-signalled launch that takes several rounds of workgroups
        // (4096^2 planes: ~6400 tiles) runs with the exchange -- its face
        // wait and RCCL's kernels -- confined to a few CUs the launch does not
        // use: a helper wave resident on a CU the launch's dispatch is
        // waiting for holds up the whole launch (NS4096 rank of 4: 61 ms per
        // launch unconfined, 54 confined, 50 alone).  Decided
        // from the global problem's largest slab, the same on every rank.
        if (j->signal && g.nz / total >= j->depth) {
            stencil_problem p = g;
            p.nz = g.nz / total + (g.nz % total ? 1 : 0);
            p.halo = j->depth;
            p.flags = STENCIL_HALO_LO | STENCIL_HALO_HI;
            stencil_layout l{};
            if (Dev::layout_init(&p, &l) == STENCIL_OK) j->confine = Dev::confine_exchange(l, j->k);
            // such grids run STAGED rounds by default (below): the face ranges
            // first, then the middle, the exchange beside the middle
            if (j->confine && Dev::staged_rounds()) {
                j->staged = true;
                j->signal = false;
                j->xcu_alt = Dev::xcu_alt();
            }
            // halo-gated launches where a waiting workgroup can never hold
            // the CU the exchange's kernels need (Dev::halo_gate)
            if (j->signal) j->gate = Dev::halo_gate(l, j->k, j->confine);
        }
    }
    j->timeout_ms = Dev::default_timeout_ms();
    const int64_t base = g.nz / total, rem = g.nz % total;
    // the smallest slab of the job decides, the same in every process: ranks
    // of one job all reject it here, before any of them enters the
    // communicator's collective init (a rank that failed alone would leave
    // the others waiting in the bootstrap)
    if (base < j->depth) {
        const int rc = set_error(STENCIL_EINVAL, "%d slabs of %lld planes: the smallest owns %lld planes < the %d halo "
                                 "planes: use fewer GPUs", total, (long long)g.nz, (long long)base, j->depth);
        delete j;
        return rc;
    }
    j->s.resize(idx.size());
    int rc = STENCIL_OK;
    for (size_t li = 0; li < idx.size() && rc == STENCIL_OK; ++li) {
        const int i = idx[li];
        Slab<Dev>& s = j->s[li];
        s.index = i;
        s.device = devs[li];
        s.n = base + (i < rem ? 1 : 0);
        s.first = i * base + std::min<int64_t>(i, rem);
        stencil_problem p = g;
        p.nz = s.n;
        p.halo = j->depth;
        p.flags = (lo_nb(*j, i) >= 0 ? STENCIL_HALO_LO : 0) | (hi_nb(*j, i) >= 0 ? STENCIL_HALO_HI : 0);
        if ((rc = Dev::layout_init(&p, &s.l))) break;
        if ((rc = Dev::set_device(s.device))) break;
        if (rolling) {
            // the overlapped rounds' face staging first (2 x d planes to send,
            // 2 x d to receive), then the margin from what memory is left
            j->roll_overlap = Dev::rolling_overlap() && (total > 1 || j->periodic);
            if (j->roll_overlap) {
                const int64_t sb = 2 * int64_t(j->depth) * int64_t(plane_bytes(s));
                if ((rc = Dev::alloc(sb, &s.xs)) || (rc = Dev::alloc(sb, &s.xr))) break;
            }
            int64_t m = 0;
            if ((rc = rolling_margin(*j, s.l, margin, &m))) break;
            // one margin for the job (the largest slab decides when sized from free memory)
            if (li == 0 || m < j->margin) j->margin = m;
            const int64_t bytes = (s.l.planes + m) * int64_t(plane_bytes(s)) + 256;
            if ((rc = Dev::alloc(bytes, &s.a))) break;
        } else {
            if ((rc = Dev::alloc(s.l.bytes + 256, &s.a)) || (rc = Dev::alloc(s.l.bytes + 256, &s.b))) break;
        }
        // staged rounds: the face launches (A) take every CU -- nothing runs
        // beside them -- and only the middle launch (B) and the exchange are
        // confined
        if ((rc = Dev::stream_create(&s.sa, STREAM_BOUNDARY, j->confine && !j->staged)) ||
            (rc = Dev::stream_create(&s.sb, STREAM_INTERIOR, j->confine)) ||
            (rc = Dev::stream_create(&s.sx, STREAM_EXCHANGE, j->confine)) || (rc = Dev::event_create(&s.ev_bnd, false)) ||
            (rc = Dev::event_create(&s.ev_int, false)) || (rc = Dev::event_create(&s.ev_join, false)) ||
            (rc = Dev::event_create(&s.ev_xin, false)) || (rc = Dev::event_create(&s.ev_xout, false)))
            break;
        if (j->staged)
            for (auto* e : {&s.tb0, &s.tb1, &s.tx0, &s.tx1, &s.tr0})
                if ((rc = Dev::event_create(e, true))) break;
        if (rc) break;
        s.xcu = j->confine ? Dev::xcu() : 0;
        if (j->staged && j->confine && j->xcu_alt > 0 &&
            ((rc = Dev::stream_create(&s.sb_alt, STREAM_INTERIOR, true, j->xcu_alt)) ||
             (rc = Dev::stream_create(&s.sx_alt, STREAM_EXCHANGE, true, j->xcu_alt))))
            break;
        s.ring.assign(size_t(kInflight), typename Dev::Event{});
        for (auto& e : s.ring)
            if ((rc = Dev::event_create(&e, false))) break;
        if (rc) break;
        if ((rc = Dev::alloc_counters(&s.counters)) || (rc = Dev::alloc_flag(&s.tflag))) break;
        if (j->signal && (rc = Dev::face_signal_create(&s.fsig))) break;
        if (!rolling && (rc = place_grids(*j, s))) break;
    }
    if (rc != STENCIL_OK) {
        release<Dev>(j);
        return rc;
    }
    *out = j;
    return STENCIL_OK;
}

template <class Dev>
int check_global(const stencil_problem* global, stencil_problem* g, int32_t flags) {
    *g = *global;
    if (g->dims != 3) return set_error(STENCIL_EUNSUPPORTED, "slab jobs split 3D grids along z");
    if (g->halo != 0 || g->flags != 0) return set_error(STENCIL_EINVAL, "the global problem takes no halo / flags");
    if (flags & ~(STENCIL_SLAB_PERIODIC | STENCIL_SLAB_ROLLING)) return set_error(STENCIL_EINVAL, "bad slab flags %d", flags);
    stencil_layout gl;
    return Dev::layout_init(g, &gl);
}

// ---- the C-ABI's bodies -----------------------------------------------------
template <class Dev, class JobT>
int create(const stencil_problem* global, int32_t ngpus, const int32_t* devices, int32_t exchange_kind, int32_t flags,
           int64_t margin, JobT** job) {
    if (!global || !job || ngpus < 1) return set_error(STENCIL_EINVAL, "null argument or ngpus < 1");
    *job = nullptr;
    if (exchange_kind != STENCIL_EXCHANGE_RCCL && exchange_kind != STENCIL_EXCHANGE_COPY)
        return set_error(STENCIL_EINVAL, "bad exchange kind %d", exchange_kind);
    stencil_problem g;
    SLAB_TRY(check_global<Dev>(global, &g, flags));
    std::vector<int> devs(static_cast<size_t>(ngpus)), idx(static_cast<size_t>(ngpus));
    for (int i = 0; i < ngpus; ++i) {
        devs[size_t(i)] = devices ? devices[i] : i;
        idx[size_t(i)] = i;
    }
    if (exchange_kind == STENCIL_EXCHANGE_RCCL) {
        for (int i = 0; i < ngpus; ++i)
            for (int q = 0; q < i; ++q)
                if (devs[size_t(i)] == devs[size_t(q)])
                    return set_error(STENCIL_EINVAL, "RCCL needs one slab per GPU (device %d twice): use device copies",
                                     devs[size_t(i)]);
        if (!Dev::comm_available()) return set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    }
    JobT* j = nullptr;
    SLAB_TRY((build_job<Dev, JobT>(g, ngpus, idx, devs, exchange_kind, flags, margin, false, &j)));
    if (exchange_kind == STENCIL_EXCHANGE_RCCL) {
        std::vector<typename Dev::Comm> comms(static_cast<size_t>(ngpus), typename Dev::Comm{});
        if (int rc = Dev::comm_init_all(comms.data(), ngpus, devs.data())) {
            release<Dev>(j);
            return rc;
        }
        for (int i = 0; i < ngpus; ++i) {
            j->s[size_t(i)].comm = comms[size_t(i)];
            Dev::comm_set_timeout(comms[size_t(i)], j->timeout_ms);
        }
    }
    *job = j;
    clear_error();
    return STENCIL_OK;
}

template <class Dev, class JobT>
int create_rank(const stencil_problem* global, int32_t nranks, int32_t rank, int32_t device, const void* id,
                int64_t id_bytes, int32_t flags, int64_t margin, JobT** job) {
    if (!global || !job || !id) return set_error(STENCIL_EINVAL, "null argument");
    *job = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(STENCIL_EINVAL, "rank %d of %d", rank, nranks);
    if (id_bytes != STENCIL_SLAB_ID_BYTES)
        return set_error(STENCIL_EINVAL, "the id holds %d bytes, not %lld", int(STENCIL_SLAB_ID_BYTES),
                         (long long)id_bytes);
    stencil_problem g;
    SLAB_TRY(check_global<Dev>(global, &g, flags));
    if (!Dev::comm_available()) return set_error(STENCIL_EUNSUPPORTED, "librccl could not be loaded");
    JobT* j = nullptr;
    SLAB_TRY((build_job<Dev, JobT>(g, nranks, {rank}, {device}, STENCIL_EXCHANGE_RCCL, flags, margin, true, &j)));
    if (int rc = Dev::set_device(device)) {
        release<Dev>(j);
        return rc;
    }
    // collective over the ranks: every rank must reach it (build_job's
    // checks that depend on the global problem fail on every rank alike); a
    // rank that never arrives fails it with STENCIL_ETIMEOUT after the job's
    // deadline
    typename Dev::Comm comm{};
    if (int rc = Dev::comm_init_rank(&comm, nranks, id, rank, j->timeout_ms)) {
        release<Dev>(j);
        return rc;
    }
    j->s[0].comm = comm;
    Dev::comm_set_timeout(comm, j->timeout_ms);
    *job = j;
    clear_error();
    return STENCIL_OK;
}

template <class Dev, class JobT>
int info(const JobT* job, int32_t slab, int64_t* first_plane, int64_t* planes, int32_t* device, int32_t* sweeps) {
    if (!job || slab < 0 || slab >= int(job->s.size())) return set_error(STENCIL_EINVAL, "bad job or slab index");
    const Slab<Dev>& s = job->s[size_t(slab)];
    if (first_plane) *first_plane = s.first;
    if (planes) *planes = s.n;
    if (device) *device = s.device;
    if (sweeps) *sweeps = job->k;
    return STENCIL_OK;
}

template <class Dev, class JobT>
int rolling_info(const JobT* job, int64_t* margin, int64_t* launches_per_pass) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (margin) *margin = job->margin;
    if (launches_per_pass) {
        int64_t most = 0;
        if (job->margin)
            for (const Slab<Dev>& s : job->s) most = std::max(most, (s.n + rolling_span(*job) - 1) / rolling_span(*job));
        *launches_per_pass = most;
    }
    return STENCIL_OK;
}

// The margin's spare slots of a rolling slab get a copy of the home grid's
// plane -1 (as stencil_rolling_init_margin copies a ghost plane): every plane
// then has the same x/y ghost ring, the reference initial condition's
// invariant, and the shifted grid's bottom planes [-zg, 0) -- slots no pass
// writes -- hold the global bottom ghost plane on the first slab (a halo
// elsewhere, received before it is read).  Called before the halo exchange.
template <class Dev>
int init_margin(const Job<Dev>& j, Slab<Dev>& s) {
    if (!j.margin) return STENCIL_OK;
    void* home = grid_at(j, s, 0);
    const size_t pb = plane_bytes(s);
    for (int64_t i = 0; i < j.margin; ++i)
        SLAB_TRY(Dev::copy_d2d(static_cast<char*>(s.a) + size_t(i) * pb, plane_ptr(s, home, -1), pb, s.sa));
    // the face staging's planes likewise: the face launches write only the
    // interior, the x/y ghost ring they send is this copy's
    for (void* buf : {s.xs, s.xr})
        if (buf)
            for (int64_t i = 0; i < 2 * j.depth; ++i)
                SLAB_TRY(Dev::copy_d2d(static_cast<char*>(buf) + size_t(i) * pb, plane_ptr(s, home, -1), pb, s.sa));
    return STENCIL_OK;
}

// Counters and face signals back to zero (a job whose face-counter wait
// timed out earlier starts clean: the timeout flag is sticky otherwise).
template <class Dev>
int reset_signals(Job<Dev>& j) {
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        SLAB_TRY(Dev::reset_counters(s.counters, s.tflag, s.fsig));
        s.sig_target = 0;
        s.fsig_target = 0;
        s.xseq = 0;
    }
    return STENCIL_OK;
}

#define SLAB_FAIL(j, expr)                       \
    do {                                         \
        if (int rc_ = (expr)) return fail(j, rc_); \
    } while (0)

template <class Dev, class JobT>
int fill_initial(JobT* job, int32_t init_kind, uint64_t seed) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    SLAB_TRY(sync_bounded(*job));
    SLAB_FAIL(*job, reset_signals(*job));
    job->cur_is_a = true;
    job->position = 0;
    for (Slab<Dev>& s : job->s) {
        SLAB_FAIL(*job, Dev::set_device(s.device));
        // global linear indices: the slab's interior starts first * nx * ny cells in
        const uint64_t sd = seed + uint64_t(s.first) * uint64_t(s.l.prob.nx) * uint64_t(s.l.prob.ny);
        SLAB_FAIL(*job, Dev::fill_initial(&s.l, grid_at(*job, s, 0), init_kind, sd, s.sa));
        if (job->margin)
            SLAB_FAIL(*job, init_margin(*job, s));
        else
            SLAB_FAIL(*job, Dev::fill_initial(&s.l, s.b, init_kind, sd, s.sa));
    }
    // the halos: the neighbours' faces (ghost planes otherwise)
    SLAB_FAIL(*job, exchange(*job, 0));
    if (!job->margin) SLAB_FAIL(*job, exchange(*job, 1));
    SLAB_TRY(sync_bounded(*job));
    clear_error();
    return STENCIL_OK;
}

// Rolling slabs need every plane's x/y ghost ring to be the same and the
// bottom ghost planes to be equal: no sweep writes a
// ghost cell, and a pass lands plane z of the new grid in a slot whose ring
// came from an older plane or from the margin's copies of plane -1.  The
// reference initial condition has this; an uploaded grid must too.
// Host planes [z0, z1) (host plane index = global plane + r) are compared
// with ONE anchor, plane z0: the ring cells of every plane, and every cell of
// the global bottom ghost planes (host planes < r).  Only ring cells are
// visited: full rows y < r and y >= ny + r, the x < r / x >= nx + r ends of
// the others (the 4096^3 grids this form exists for have 2^24 interior cells
// a plane).
template <class T>
int check_rolling_rings(const T* h, const stencil_problem& g, int64_t row, int64_t rows, int64_t z0, int64_t z1) {
    const int64_t r = g.radius, w = g.nx + 2 * r, hgt = g.ny + 2 * r;
    const size_t hp = size_t(row) * size_t(rows);
    const T* anchor = h + size_t(z0) * hp;
    auto cmp = [&](int64_t z, int64_t y, int64_t x) {
        const T a = h[size_t(z) * hp + size_t(y * row + x)];
        const T b = anchor[size_t(y * row + x)];
        if (std::memcmp(&a, &b, sizeof(T)) == 0) return STENCIL_OK;
        return set_error(STENCIL_EINVAL,
                         "rolling slab upload: host plane %lld cell (x %lld, y %lld) differs from plane %lld -- "
                         "rolling slabs need the same x/y ghost ring in every plane and equal bottom "
                         "ghost planes (use two grids: no STENCIL_SLAB_ROLLING)",
                         (long long)(z - r), (long long)(x - r), (long long)(y - r), (long long)(z0 - r));
    };
    for (int64_t z = z0 + 1; z < z1; ++z) {
        const bool full = z < r;  // a global bottom ghost plane: every cell
        for (int64_t y = 0; y < hgt; ++y) {
            if (full || y < r || y >= g.ny + r) {
                for (int64_t x = 0; x < w; ++x) SLAB_TRY(cmp(z, y, x));
            } else {
                for (int64_t x = 0; x < r; ++x) SLAB_TRY(cmp(z, y, x));
                for (int64_t x = g.nx + r; x < w; ++x) SLAB_TRY(cmp(z, y, x));
            }
        }
    }
    return STENCIL_OK;
}

template <class Dev, class JobT>
int upload(JobT* job, const void* host, int64_t host_row, int64_t host_rows) {
    if (!job || !host) return set_error(STENCIL_EINVAL, "null argument");
    const stencil_problem& g = job->global;
    if (host_row < g.nx + 2 * g.radius || host_rows < g.ny + 2 * g.radius)
        return set_error(STENCIL_EINVAL, "host array too small");
    if (job->margin) {
        // every rank checks the whole global array (ring cells only), so a bad
        // grid fails every rank alike, before any exchange
        const int64_t z1 = g.nz + 2 * g.radius;
        const int rc = g.dtype == STENCIL_F64
                           ? check_rolling_rings(static_cast<const double*>(host), g, host_row, host_rows, 0, z1)
                           : check_rolling_rings(static_cast<const float*>(host), g, host_row, host_rows, 0, z1);
        SLAB_TRY(rc);
    }
    SLAB_TRY(sync_bounded(*job));
    SLAB_FAIL(*job, reset_signals(*job));
    const size_t es = g.dtype == STENCIL_F64 ? 8 : 4;
    job->cur_is_a = true;
    job->position = 0;
    for (Slab<Dev>& s : job->s) {
        SLAB_FAIL(*job, Dev::set_device(s.device));
        // host planes [first, first + n + 2r) hold this slab's planes -r .. n+r-1
        const char* h = static_cast<const char*>(host) + size_t(s.first) * size_t(host_row * host_rows) * es;
        SLAB_FAIL(*job, Dev::upload(&s.l, grid_at(*job, s, 0), h, host_row, host_rows, s.sa));
        if (job->margin)
            SLAB_FAIL(*job, init_margin(*job, s));
        else
            SLAB_FAIL(*job, Dev::upload(&s.l, s.b, h, host_row, host_rows, s.sa));
    }
    SLAB_FAIL(*job, exchange(*job, 0));
    if (!job->margin) SLAB_FAIL(*job, exchange(*job, 1));
    SLAB_TRY(sync_bounded(*job));
    clear_error();
    return STENCIL_OK;
}

// After each timed tuning round of a staged job (the streams are idle):
//   1st round: RCCL's lazy connection set-up -- nothing kept;
//   2nd round: B, the exchange and the round with the default CU budget.
//     Where the exchange ran at least 0.8x as long as B and an alternative
//     budget exists (confined exchanges: Dev::xcu_alt CUs per XCD), the
//     alternative's streams are swapped in for one more tuning round;
//     otherwise the face span is set from this round;
//   3rd round: the same with the alternative; each slab keeps the budget
//     whose round was faster (the alternative only if 2 % faster) and sets
//     its face span from that round's B and exchange.
// The rehearsals' emulated wire decided the 1-CU budget; RCCL's
// P2P kernels over real xGMI links may need more CUs to fill a link -- this
// lets the first multi-GPU run measure it instead of assuming it.
template <class Dev>
int staged_tuning_step(Job<Dev>& j) {
    const int step = ++j.tune_done;
    if (step == 1) return STENCIL_OK;
    const int m = step == 2 ? 0 : 1;
    bool slow_exchange = false;
    for (Slab<Dev>& s : j.s) {
        SLAB_TRY(Dev::set_device(s.device));
        float rb = 0.f, rx = 0.f;
        SLAB_TRY(Dev::event_elapsed(&s.b_ms[m], s.tb0, s.tb1));
        SLAB_TRY(Dev::event_elapsed(&s.x_ms[m], s.tx0, s.tx1));
        SLAB_TRY(Dev::event_elapsed(&rb, s.tr0, s.tb1));
        SLAB_TRY(Dev::event_elapsed(&rx, s.tr0, s.tx1));
        s.round_ms[m] = std::max(rb, rx);
        slow_exchange = slow_exchange || s.x_ms[m] >= 0.8f * s.b_ms[m];
    }
    if (m == 0 && slow_exchange && j.xcu_alt > 0) {
        for (Slab<Dev>& s : j.s) {
            std::swap(s.sx, s.sx_alt);
            std::swap(s.sb, s.sb_alt);
            s.xcu = j.xcu_alt;
        }
        j.tune_left = 1;  // one more timed round, with the alternative
        return STENCIL_OK;
    }
    for (Slab<Dev>& s : j.s) {
        int keep = 0;
        if (m == 1) {
            keep = s.round_ms[1] < 0.98f * s.round_ms[0] ? 1 : 0;
            if (!keep) {
                std::swap(s.sx, s.sx_alt);
                std::swap(s.sb, s.sb_alt);
                s.xcu = Dev::xcu();
            }
        }
        s.face_span = tuned_face_span(j, s, s.b_ms[keep], s.x_ms[keep]);
    }
    j.tune_left = 0;
    return STENCIL_OK;
}

template <class Dev>
int one_round(Job<Dev>& j, int k, bool full) {
    SLAB_TRY(throttle(j));
    if (!(full && j.signal)) j.gate_chain = false;  // only a gated launch may follow a gated launch unsynchronised
    if (j.margin)
        SLAB_FAIL(j, j.roll_overlap ? slab_round_rolling_overlap(j, k) : slab_round_rolling(j, k));
    else if (full && j.signal)
        SLAB_FAIL(j, slab_round_signal(j, k));
    else if (full && j.staged) {
        // the first two staged rounds are timed (the first also carries
        // RCCL's lazy connection set-up): the second sets the face span
        j.tuning = j.tune_left > 0;
        SLAB_FAIL(j, slab_round_staged(j, k));
        if (j.tuning) {
            j.tuning = false;
            SLAB_TRY(sync_bounded(j));
            --j.tune_left;
            SLAB_FAIL(j, staged_tuning_step(j));
        }
    }
    else
        SLAB_FAIL(j, slab_round(j, k));
    SLAB_FAIL(j, mark_round(j));
    return STENCIL_OK;
}

template <class Dev, class JobT>
int run(JobT* job, uint32_t iterations, float* elapsed_ms) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    SLAB_TRY(sync_bounded(*job));
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t done = 0;
    const uint32_t k = uint32_t(job->k);
    for (; done + k <= iterations; done += k) SLAB_TRY(one_round(*job, int(k), true));
    if (done < iterations)  // the remainder as one shorter fused round
        SLAB_TRY(one_round(*job, int(iterations - done), false));
    SLAB_TRY(sync_bounded(*job));
    if (job->signal) SLAB_FAIL(*job, check_signal_timeouts(*job));
    const auto t1 = std::chrono::steady_clock::now();
    if (elapsed_ms) *elapsed_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    clear_error();
    return STENCIL_OK;
}

template <class Dev, class JobT>
int download(JobT* job, void* host, int64_t host_row, int64_t host_rows) {
    if (!job || !host) return set_error(STENCIL_EINVAL, "null argument");
    const stencil_problem& g = job->global;
    const int64_t r = g.radius;
    const size_t es = g.dtype == STENCIL_F64 ? 8 : 4;
    const size_t hplane = size_t(host_row * host_rows) * es;
    if (host_row < g.nx + 2 * r || host_rows < g.ny + 2 * r) return set_error(STENCIL_EINVAL, "host array too small");
    SLAB_TRY(sync_bounded(*job));
    std::vector<char> tmp;
    for (Slab<Dev>& s : job->s) {
        SLAB_FAIL(*job, Dev::set_device(s.device));
        // the slab's planes -r .. n+r-1 through a scratch copy; keep its own
        // planes, plus the global ghost planes at the two ends
        tmp.resize(size_t(s.n + 2 * r) * hplane);
        SLAB_FAIL(*job, Dev::download(&s.l, cur_grid(*job, s), tmp.data(), host_row, host_rows, s.sa));
        SLAB_TRY(sync_bounded(*job));
        const int64_t z0 = s.index == 0 ? -r : 0;
        const int64_t z1 = s.index + 1 == slabs_total(*job) ? s.n + r : s.n;
        std::memcpy(static_cast<char*>(host) + size_t(s.first + z0 + r) * hplane, tmp.data() + size_t(z0 + r) * hplane,
                    size_t(z1 - z0) * hplane);
    }
    clear_error();
    return STENCIL_OK;
}

template <class Dev, class JobT>
int kernel_timing(JobT* job, int32_t enable) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    SLAB_TRY(sync_bounded(*job));
    SLAB_TRY(Dev::set_device(job->s[0].device));
    drop_timing(*job);
    job->timing = enable != 0;
    clear_error();
    return STENCIL_OK;
}

// The round form of the job's full rounds (STENCIL_SLAB_FORM_*).
template <class Dev>
int round_form_of(const Job<Dev>& j) {
    return j.signal ? STENCIL_SLAB_FORM_SIGNALLED
           : j.staged ? STENCIL_SLAB_FORM_STAGED
           : j.margin ? STENCIL_SLAB_FORM_ROLLING
           : j.serial ? STENCIL_SLAB_FORM_SERIAL
                      : STENCIL_SLAB_FORM_BOUNDARY_INTERIOR;
}

template <class Dev, class JobT>
int kernel_time(JobT* job, float* total_ms, int64_t* launches, int64_t* cells_per_launch, int32_t* signalled) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    SLAB_TRY(sync_bounded(*job));
    SLAB_TRY(Dev::set_device(job->s[0].device));
    float sum = 0.f;
    for (auto& e : job->tev) {
        float ms = 0.f;
        SLAB_TRY(Dev::event_elapsed(&ms, e.first, e.second));
        sum += ms;
    }
    if (total_ms) *total_ms = sum;
    // a timed span is one launch, or (rolling) the pass's launches: reported
    // per span, so `cells_per_launch` is what one span covers
    if (launches) *launches = int64_t(job->tev.size());
    if (cells_per_launch) *cells_per_launch = job->timed_cells;
    if (signalled) *signalled = job->signal ? 1 : 0;  // stencil_slab_round_form: the form
    clear_error();
    return STENCIL_OK;
}

// The exchanges of the timed rounds against their launch spans: the summed
// transfer time on slab 0's X (from the end of its face wait, or of the face
// launches it follows, to the end of the transfers) and the part of it that
// ran while the same round's timed launch span was running (both on one
// device clock).  Serial rounds: ~0 beside.
template <class Dev, class JobT>
int exchange_time(JobT* job, float* transfer_ms, float* beside_ms, int64_t* exchanges) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    SLAB_TRY(sync_bounded(*job));
    SLAB_TRY(Dev::set_device(job->s[0].device));
    double tsum = 0.0, bsum = 0.0;
    int64_t n = 0;
    const size_t m = std::min(job->tev.size(), job->xev.size() - (job->xopen ? 1 : 0));
    for (size_t i = 0; i < m; ++i) {
        float L = 0.f, a = 0.f, b = 0.f;
        SLAB_TRY(Dev::event_elapsed(&L, job->tev[i].first, job->tev[i].second));
        SLAB_TRY(Dev::event_elapsed(&a, job->tev[i].first, job->xev[i].first));
        SLAB_TRY(Dev::event_elapsed(&b, job->tev[i].first, job->xev[i].second));
        tsum += std::max(0.f, b - a);
        bsum += std::max(0.f, std::min(L, b) - std::max(0.f, a));
        ++n;
    }
    if (transfer_ms) *transfer_ms = float(tsum);
    if (beside_ms) *beside_ms = float(bsum);
    if (exchanges) *exchanges = n;
    clear_error();
    return STENCIL_OK;
}

template <class Dev, class JobT>
int round_form(const JobT* job, int32_t* form) {
    if (!job || !form) return set_error(STENCIL_EINVAL, "null argument");
    *form = round_form_of(*job);
    return STENCIL_OK;
}

template <class Dev, class JobT>
int round_info(const JobT* job, int32_t* form, int32_t* gated, int32_t* confined) {
    if (!job) return set_error(STENCIL_EINVAL, "null job");
    if (form) *form = round_form_of(*job);
    if (gated) *gated = job->signal && job->gate ? 1 : 0;
    if (confined) *confined = job->confine ? 1 : 0;
    return STENCIL_OK;
}

// The exchange's CU budget of slab 0 (staged, confined jobs): CUs per XCD
// in use, the alternative tried (0: none), and the tuning rounds' times with
// the default and with the alternative (0: not run).
template <class Dev, class JobT>
int exchange_budget(const JobT* job, int32_t* cus, int32_t* alt_cus, float* round_ms, float* alt_round_ms) {
    if (!job || job->s.empty()) return set_error(STENCIL_EINVAL, "null job");
    const Slab<Dev>& s = job->s[0];
    if (cus) *cus = s.xcu;
    if (alt_cus) *alt_cus = job->xcu_alt;
    if (round_ms) *round_ms = s.round_ms[0];
    if (alt_round_ms) *alt_round_ms = s.round_ms[1];
    return STENCIL_OK;
}

template <class Dev, class JobT>
int set_timeout(JobT* job, int64_t ms) {
    if (!job || ms < 1) return set_error(STENCIL_EINVAL, "null job or timeout < 1 ms");
    job->timeout_ms = ms;
    for (Slab<Dev>& s : job->s)
        if (s.comm) Dev::comm_set_timeout(s.comm, ms);
    return STENCIL_OK;
}

template <class Dev, class JobT>
int plane_sums(JobT* job, double* sums) {
    if (!job || !sums) return set_error(STENCIL_EINVAL, "null argument");
    SLAB_TRY(sync_bounded(*job));
    for (Slab<Dev>& s : job->s) {
        SLAB_FAIL(*job, Dev::set_device(s.device));
        SLAB_FAIL(*job, Dev::plane_sums(&s.l, cur_grid(*job, s), sums + s.first, s.sa));
        SLAB_TRY(sync_bounded(*job));
    }
    clear_error();
    return STENCIL_OK;
}

#undef SLAB_FAIL
#undef SLAB_TRY

}  // namespace slab
}  // namespace stencil
