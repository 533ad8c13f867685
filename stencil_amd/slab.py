"""Z-slab decomposition of the Jacobi sweep across processes (one per GPU).

The reference decomposes its grid into an 8x8 mesh of CPE blocks and
exchanges 4 halo strips per iteration by DMA through main memory or by RMA
into the neighbour's LDM (src/stencil/slave/stencil_dma.cpp:236-247,
stencil_rma.cpp:198-255), with a 64-core barrier per iteration
(stencil_dma.cpp:562-563).  Across GPUs the natural cut is contiguous slabs of
the slow axis (z in 3D, y in 2D): each rank owns planes [z0, z0 + n) plus r
ghost planes per side, and one iteration exchanges r whole, contiguous planes
with rank-1 and rank+1 -- no packing, and on an 8-GPU MI355X node every
neighbour pair has its own xGMI link.

Per round, on each rank (overlap=True):
  stream A: update the boundary planes (high priority) -> post send/recv of
            them to the neighbours (torch.distributed P2P; RCCL on GPUs, gloo
            on CPUs);
  stream B: update the interior planes meanwhile;
  chain:    round r+1's interior waits for round r's boundary launches, its
            boundary launches for round r's interior and the received halos
            (events between the two streams; see _round).
On GPUs with the 7-point star's K-step kernel (the default), a round is
instead ONE launch over the whole slab (_round_signal): its first z-chunk
marches up and its last one down, so both K-plane faces are stored first and
counted in device counters; the exchange stream waits for the counts and sends
the faces while the launch finishes the interior.
A round is one sweep (halo depth r), or -- when the backend has a fused
multi-step kernel and K-deep halos -- K sweeps in one launch per plane range
(temporal blocking across GPUs: the exchange of K planes every K sweeps, the
halo planes themselves advanced to t+K-1 .. t+1 on chip by the fused kernel;
K = the library's fuse depth: 4 for the 7-point star, 3 or 4 for the 27-point box).
Every cell's arithmetic is the single-GPU kernel's, so results are bitwise
identical for any number of ranks (tests/test_slab_gloo.py, tests/test_gpu_*).

`backend` is the per-rank compute object: stencil_amd.engine.JacobiEngine on
a GPU.  The driver only needs sweep(), plane_view(), fill_initial() and the
two grids a/b from it, so the CPU tests drive the identical exchange logic
with the oracle as a stand-in backend.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def partition(n: int, world: int, rank: int) -> tuple[int, int]:
    """(first, count) of rank's contiguous share of n planes; the remainder
    goes to the lowest ranks."""
    base, rem = divmod(n, world)
    count = base + (1 if rank < rem else 0)
    first = rank * base + min(rank, rem)
    return first, count


class TorchDistExchanger:
    """Halo exchange with the slab neighbours over torch.distributed P2P."""

    def __init__(self, rank: int, world: int, group=None):
        self.rank, self.world, self.group = rank, world, group

    def exchange(self, send_lo, send_hi, recv_lo, recv_hi):
        ops = []
        if self.rank > 0:
            ops.append(dist.P2POp(dist.isend, send_lo, self.rank - 1, self.group))
            ops.append(dist.P2POp(dist.irecv, recv_lo, self.rank - 1, self.group))
        if self.rank < self.world - 1:
            ops.append(dist.P2POp(dist.isend, send_hi, self.rank + 1, self.group))
            ops.append(dist.P2POp(dist.irecv, recv_hi, self.rank + 1, self.group))
        if not ops:
            return []
        return dist.batch_isend_irecv(ops)


class HostStagedExchanger(TorchDistExchanger):
    """The same exchange through host memory over a CPU backend (gloo): lets
    N ranks share one GPU, which RCCL refuses.  Used only to rehearse the
    multi-rank path on a single-GPU box (bench.py --exchange host); blocking,
    so it does not overlap."""

    def exchange(self, send_lo, send_hi, recv_lo, recv_hi):
        if send_lo.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
        host = [t.cpu() for t in (send_lo, send_hi)]
        rl, rh = torch.empty_like(host[0]), torch.empty_like(host[1])
        for w in super().exchange(host[0], host[1], rl, rh):
            w.wait()
        if self.rank > 0:
            recv_lo.copy_(rl)
        if self.rank < self.world - 1:
            recv_hi.copy_(rh)
        return []


class SelfP2PExchanger(TorchDistExchanger):
    """LoopbackExchanger's periodic halos, but through torch.distributed P2P
    with this rank as its own peer (world size 1, RCCL): exercises the RCCL
    send/recv path of TorchDistExchanger -- batch_isend_irecv posted on the
    boundary stream, completion waited for on that stream -- on a one-GPU box
    (bench.py --exchange nccl-self).  Sends and receives to one peer match in
    posting order: send_hi -> recv_lo, send_lo -> recv_hi."""

    def exchange(self, send_lo, send_hi, recv_lo, recv_hi):
        me = self.rank
        ops = [dist.P2POp(dist.isend, send_hi, me, self.group), dist.P2POp(dist.irecv, recv_lo, me, self.group),
               dist.P2POp(dist.isend, send_lo, me, self.group), dist.P2POp(dist.irecv, recv_hi, me, self.group)]
        return dist.batch_isend_irecv(ops)


class LoopbackExchanger:
    """Rehearsal on ONE GPU of a rank with two neighbours: the slab's own
    boundary planes become its halos (periodic in z), copied device to device
    on the calling stream.  The numbers change (periodic instead of
    Dirichlet z faces); the per-round launch and stream structure of an
    interior rank does not (bench.py --exchange loopback)."""

    def __init__(self, rank: int = 0, world: int = 1):
        self.rank, self.world = rank, world

    def exchange(self, send_lo, send_hi, recv_lo, recv_hi):
        recv_lo.copy_(send_hi, non_blocking=True)
        recv_hi.copy_(send_lo, non_blocking=True)
        return []


@dataclass
class SlabInfo:
    rank: int
    world: int
    first: int   # global index of the first owned plane
    count: int   # owned planes


class SlabJacobi:
    """One rank's share of a slab-decomposed Jacobi job."""

    def __init__(self, backend, slab: SlabInfo, exchanger, overlap: bool = True):
        self.be = backend
        self.slab = slab
        self.ex = exchanger
        self.overlap = overlap
        self.r = backend.r
        self.depth = backend.depth  # planes exchanged per side
        self.fused = bool(getattr(backend, "fused", False)) and self.depth >= 2
        # sweeps per fused round: what the backend fuses, at most the halo depth
        self.k = min(int(getattr(backend, "fuse_steps", 2)), self.depth) if self.fused else 1
        n = slab.count
        if slab.world > 1 and n < self.depth:
            raise ValueError(f"rank {slab.rank} owns {n} planes < halo depth {self.depth}; use fewer ranks")
        self.cur, self.nxt = backend.a, backend.b
        self.on_gpu = self.cur.device.type == "cuda"
        self._timing = None  # list of (start, end) events around interior sweeps
        self._ev_bnd = self._ev_int = None  # last round's boundary / interior completion
        # Face-signalled rounds (_round_signal): one launch per round whose
        # face-owning workgroups signal device counters [lo, hi, timeout].
        self.signalled = (self.on_gpu and self.fused and overlap and slab.world > 1 and n >= 2 * self.k
                          and bool(getattr(backend, "supports_signal", False)) and self.use_signal)
        self._sig = torch.zeros(4, dtype=torch.int32, device=self.cur.device) if self.signalled else None
        self._sig_rounds = 0
        # the exchange stream waits for the faces through the one-lane wait
        # kernel (stencil_wait_counters, 10 s timeout) or, with
        # use_face_signal, hipStreamWaitValue64 on a signal word -- which HIP
        # also runs as a kernel (__amd_rocclr_streamOpsWait in the trace,
        # profiles/r01j_sig_kernel_stats.csv) and which never times out
        self._fsig = None
        if self.signalled and self.use_face_signal and hasattr(backend, "face_signal"):
            self._fsig = backend.face_signal()
        if self.on_gpu:
            # The boundary stream has the high priority, so the boundary
            # planes and their exchange come first and stay off the critical
            # path.  Traced on one GPU (bench.py --exchange loopback): with
            # the interior first, the boundary launches only get the CUs the
            # interior leaves free and share HBM with it, and take ~480 us of
            # a ~500 us round -- an RCCL exchange behind them would then set
            # the round time; boundary first costs the interior ~25 us.
            self.stream_bnd = torch.cuda.Stream(device=self.cur.device, priority=-1)
            self.stream_int = torch.cuda.Stream(device=self.cur.device)

    # -------------------------------------------------------------- helpers
    def _halo_views(self, grid):
        n, d, be = self.slab.count, self.depth, self.be
        return (be.plane_view(grid, 0, d), be.plane_view(grid, n - d, d),
                be.plane_view(grid, -d, d), be.plane_view(grid, n, d))

    def init(self, kind: str = "reference", seed: int = 0, plane_elems: int = 0) -> None:
        """Initial condition of the global grid restricted to this slab.
        `plane_elems` = interior cells per slow-axis unit, so the random
        interior uses global linear indices (seed shifted by first*plane)."""
        s = seed + self.slab.first * plane_elems
        self.be.fill_initial(self.be.a, kind, s)
        self.be.fill_initial(self.be.b, kind, s)
        self.cur, self.nxt = self.be.a, self.be.b
        self._exchange_blocking(self.cur)

    def _exchange_blocking(self, grid) -> None:
        if self.slab.world == 1:
            return
        if self.on_gpu:
            torch.cuda.current_stream().synchronize()
        for w in self.ex.exchange(*self._halo_views(grid)):
            w.wait()
        if self.on_gpu:
            torch.cuda.current_stream().synchronize()

    # ----------------------------------------------------------------- step
    def _round(self, update, edge: int) -> None:
        """One exchange round: `update(src, dst, b, e, stream)` advances planes
        [b, e); `edge` = boundary planes updated first on each side."""
        src, dst = self.cur, self.nxt
        n = self.slab.count
        serial = self.slab.world == 1 or not self.overlap or n <= 2 * edge or not self.on_gpu
        if serial:
            # These branches launch on the caller's stream: join the round
            # streams first.  A remainder pair/single after face-signalled
            # rounds otherwise reads src while the last signalled launch on
            # stream_int still writes it, and its halos while the exchange on
            # stream_bnd still receives them (the nz = 2K failures of
            # test_signalled_rounds_every_k, round 1).
            self.finish()
        if self.slab.world == 1:
            update(src, dst, 0, n, None)
        elif not self.overlap or n <= 2 * edge:
            update(src, dst, 0, n, None)
            for w in self.ex.exchange(*self._halo_views(dst)):
                w.wait()
        elif not self.on_gpu:
            update(src, dst, 0, edge, None)
            update(src, dst, n - edge, n, None)
            works = self.ex.exchange(*self._halo_views(dst))
            update(src, dst, edge, n - edge, None)
            for w in works:
                w.wait()
        else:
            # Rounds chain on the two streams directly, not through the
            # caller's stream (each cross-queue hop costs ~15 us on MI355X:
            # a main-stream join per round measured 30 us of idle GPU between
            # rounds).  Dependencies of round r (src = dst of round r-1):
            #   interior(r) reads src [0, n): after boundary(r-1)   (sa event)
            #   boundary(r) reads src incl. the halos received by exchange(r-1)
            #     (on sa already) and planes interior(r-1) wrote, and
            #     overwrites planes interior(r-1) read: after interior(r-1)
            #   exchange(r) after boundary(r) (same stream); the P2P's
            #   completion is waited for on sa, ahead of boundary(r+1).
            # finish() joins both streams into the caller's stream.
            sa, sb = self.stream_bnd, self.stream_int
            if self._ev_bnd is None:
                main = torch.cuda.current_stream()
                sa.wait_stream(main)
                sb.wait_stream(main)
            else:
                sb.wait_event(self._ev_bnd)
                sa.wait_event(self._ev_int)
            with torch.cuda.stream(sb):
                if self._timing is not None:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev0.record(sb)
                update(src, dst, edge, n - edge, sb)
                if self._timing is not None:
                    ev1.record(sb)
                    self._timing.append((ev0, ev1))
                self._ev_int = torch.cuda.Event()
                self._ev_int.record(sb)
            with torch.cuda.stream(sa):
                update(src, dst, 0, edge, sa)
                update(src, dst, n - edge, n, sa)
                self._ev_bnd = torch.cuda.Event()
                self._ev_bnd.record(sa)
                for w in self.ex.exchange(*self._halo_views(dst)):
                    w.wait()  # sa waits for the P2P
        self.cur, self.nxt = dst, src

    def _round_signal(self) -> None:
        """One K-step round as ONE launch over the whole slab (GPU, fused):
        its first z-chunk marches up and its last down, so the face planes
        are among the first it stores, and the workgroups that store them
        add to device counters (stencil_sweepk_signal).  The exchange stream
        queues a wait for the counts, then the P2P -- the faces leave while
        the rest of the launch runs, with no separate boundary launches.
        Dependencies: launch(r) reads the halos exchange(r-1) received (sb
        waits for it); exchange(r) receives into the planes launch(r-1) read
        as halos -- ordered because launch(r) only starts, and only signals,
        after launch(r-1) (one stream)."""
        src, dst = self.cur, self.nxt
        n, k = self.slab.count, self.k
        sa, sb = self.stream_bnd, self.stream_int
        if self._ev_bnd is None:
            main = torch.cuda.current_stream()
            sa.wait_stream(main)
            sb.wait_stream(main)
        else:
            sb.wait_event(self._ev_bnd)
        with torch.cuda.stream(sb):
            if self._timing is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record(sb)
            nsig = self.be.sweepk_signal(src, dst, 0, n, k, self._sig, stream=sb, face_signal=self._fsig)
            if self._timing is not None:
                ev1.record(sb)
                self._timing.append((ev0, ev1))
            self._ev_int = torch.cuda.Event()
            self._ev_int.record(sb)
        self._sig_rounds += 1
        target = self._sig_rounds * nsig
        with torch.cuda.stream(sa):
            if self._fsig is not None:
                self._fsig.wait(2 * self._sig_rounds, stream=sa)
            else:
                self.be.wait_counters(self._sig, target, target, stream=sa)
            for w in self.ex.exchange(*self._halo_views(dst)):
                w.wait()  # sa waits for the P2P
            self._ev_bnd = torch.cuda.Event()
            self._ev_bnd.record(sa)
        self.cur, self.nxt = dst, src

    def signal_timeouts(self) -> int:
        """Nonzero if a face-counter wait gave up (10 s): results invalid."""
        if self._sig is None:
            return 0
        torch.cuda.synchronize(self.cur.device)
        return int(self._sig[2].item())

    def finish(self) -> None:
        """Join the round streams into the caller's stream (after run())."""
        if self.on_gpu and self._ev_bnd is not None:
            main = torch.cuda.current_stream()
            main.wait_stream(self.stream_bnd)
            main.wait_stream(self.stream_int)
        self._ev_bnd = self._ev_int = None

    def _step(self) -> None:
        self._round(lambda s, d, b, e, st: self.be.sweep(s, d, b, e, stream=st), max(self.r, self.depth))

    def _step2(self) -> None:
        self._round(lambda s, d, b, e, st: self.be.sweep2(s, d, b, e, stream=st), self.depth)

    def _stepk(self, k: int) -> None:
        self._round(lambda s, d, b, e, st: self.be.sweepk(s, d, b, e, k, stream=st), self.depth)

    def step(self) -> None:
        """One sweep."""
        self._step()
        self.finish()

    def step2(self) -> None:
        """Two sweeps, fused (needs backend.fused and halo depth >= 2)."""
        self._step2()
        self.finish()

    def stepk(self, k: int) -> None:
        """k sweeps fused in one launch per plane range (halo depth >= k)."""
        self._stepk(k)
        self.finish()

    def step2_split(self) -> None:
        """Two single sweeps per exchange of 2 planes (halo depth >= 2): the
        first sweep also advances the 1-deep halo planes of shared faces, the
        second the owned planes -- communication-avoiding temporal blocking
        with the single-sweep kernel (used where no fused kernel is faster).
        The result lands back in the current grid."""
        self.finish()  # this round joins through the caller's stream
        src, dst = self.cur, self.nxt
        n, be, sl = self.slab.count, self.be, self.slab
        lo = -1 if sl.rank > 0 else 0
        hi = n + 1 if sl.rank < sl.world - 1 else n
        B = 2  # planes exchanged = second-sweep boundary thickness
        if sl.world == 1:
            be.sweep(src, dst, 0, n)
            be.sweep(dst, src, 0, n)
        elif not self.overlap or not self.on_gpu or n <= 2 * B + 2:
            be.sweep(src, dst, lo, hi)
            be.sweep(dst, src, 0, n)
            for w in self.ex.exchange(*self._halo_views(src)):
                w.wait()
        else:
            main = torch.cuda.current_stream()
            sa, sb = self.stream_bnd, self.stream_int
            sa.wait_stream(main)
            sb.wait_stream(main)
            first_done = torch.cuda.Event()
            with torch.cuda.stream(sa):
                be.sweep(src, dst, lo, B + 1, stream=sa)
                be.sweep(src, dst, n - B - 1, hi, stream=sa)
                first_done.record(sa)
                be.sweep(dst, src, 0, B, stream=sa)
                be.sweep(dst, src, n - B, n, stream=sa)
                works = self.ex.exchange(*self._halo_views(src))
            with torch.cuda.stream(sb):
                if self._timing is not None:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev0.record(sb)
                # reads src planes [B, n-B): disjoint from what stream A's
                # second sweep writes ([0, B) and [n-B, n))
                be.sweep(src, dst, B + 1, n - B - 1, stream=sb)
                if self._timing is not None:  # time the interior launch alone
                    ev1.record(sb)
                    self._timing.append((ev0, ev1))
                sb.wait_event(first_done)
                be.sweep(dst, src, B, n - B, stream=sb)
            for w in works:
                w.wait()
            main.wait_stream(sa)
            main.wait_stream(sb)

    # ------------------------------------------------------- kernel timing
    def start_kernel_timing(self) -> None:
        """Record HIP events on the interior stream around every interior
        sweep (the dominant kernel) until stop_kernel_timing()."""
        self._timing = []

    def stop_kernel_timing(self) -> tuple[float, int]:
        """(total ms of the recorded interior sweeps, number of launches)."""
        ev, self._timing = self._timing or [], None
        if not ev:
            return 0.0, 0
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev), len(ev)

    @property
    def mode(self) -> str:
        """'fused' (k sweeps per launch), 'split2' (two single sweeps per
        2-plane exchange) or 'single' (one sweep per 1-plane exchange)."""
        if self.fused:
            return "fused"
        if self.depth >= 2 * self.r and self.r == 1 and self.split2:
            return "split2"
        return "single"

    split2 = True  # allow the communication-avoiding 2-sweep rounds
    use_signal = True  # face-signalled single-launch rounds where the backend has them
    use_face_signal = False  # wait on the HIP signal word (hipStreamWaitValue64) instead of the counters

    def run(self, iterations: int) -> None:
        mode = self.mode
        if mode == "fused":
            k = self.k
            if self.signalled and iterations >= k:
                self.finish()
                self._sig.zero_()  # on the caller's stream, before the rounds join it
                if self._fsig is not None:
                    self._fsig.reset()
                self._sig_rounds = 0
            for _ in range(iterations // k):
                if self.signalled:
                    self._round_signal()
                else:
                    self._stepk(k) if k != 2 else self._step2()
            rem = iterations % k
            if rem >= 2:
                self._step2()
                rem -= 2
            if rem:
                self._step()
        elif mode == "split2":
            for _ in range(iterations // 2):
                self.step2_split()
            if iterations % 2:
                self._step()
        else:
            for _ in range(iterations):
                self._step()
        self.finish()

    def launches_per_round(self) -> int:
        """Sweeps per timed interior launch (the bench's roofline unit)."""
        return self.k if self.fused else 1
