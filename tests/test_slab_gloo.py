"""Multi-process slab decomposition (stencil_amd/slab.py) on CPU with gloo.

The exchange/overlap logic is the product code; the per-rank compute backend
here is the oracle (a test double standing in for JacobiEngine -- on GPUs the
same driver runs the HIP kernels, tests/test_gpu_slab.py).  Results gathered
from world_size 2 and 3 must be bitwise equal to a single-process run, for
single sweeps (halo depth 1) and for fused two-step rounds (halo depth 2).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import binding as ob
from stencil_amd.slab import SlabInfo, SlabJacobi, TorchDistExchanger, partition

NX, NY, NZ = 11, 9, 14


class OracleSlabBackend:
    """Per-rank grid pair in the oracle's dense layout with `depth` halo
    planes per z side; sweeps run the oracle on plane ranges."""

    def __init__(self, n, depth, lo_halo, hi_halo, fused, fuse_steps=2):
        self.r, self.depth, self.n, self.fuse_steps = 1, depth, n, fuse_steps
        self.lo_halo, self.hi_halo, self.fused = lo_halo, hi_halo, fused
        # the oracle's interior spans local planes -(depth-1) .. n+depth-2
        self.p = ob.problem(3, "fp64", "star", 1, "naive", NX, NY, n + 2 * (depth - 1))
        shape = ob.dense_shape(self.p)
        self.unit = shape[1] * shape[2]
        self.a = torch.zeros(int(np.prod(shape)), dtype=torch.float64)
        self.b = torch.zeros_like(self.a)

    def _np(self, t):
        return t.numpy().reshape(ob.dense_shape(self.p))

    def fill_initial(self, grid, kind, seed):
        d = self.depth
        g = ob.init(self.p, kind, seed - (d - 1) * NX * NY)
        ghost = g[0].copy()  # a Dirichlet ghost plane: x-ghosts 1, rest 0
        if not self.lo_halo:
            g[:d] = ghost
        if not self.hi_halo:
            g[self.n + d:] = ghost
        self._np(grid)[...] = g

    def plane_view(self, grid, first, count):
        start = (self.depth + first) * self.unit
        return grid[start:start + count * self.unit]

    def sweep(self, src, dst, b, e, stream=None):
        o = self.depth - 1
        ob.sweep(self.p, self._np(src), self._np(dst), b + o, e + o)

    def sweepk(self, src, dst, b, e, k, stream=None):
        """k sweeps: intermediate step j (1..k-1) also advances the shared-face
        halo planes k-j deep, as the fused kernels do."""
        o = self.depth - 1
        cur = self._np(src)
        for j in range(1, k):
            lo = -(k - j) if self.lo_halo else 0
            hi = self.n + (k - j) if self.hi_halo else self.n
            t = cur.copy()  # ghost planes stay as in src (Dirichlet copy)
            ob.sweep(self.p, cur, t, max(b - (k - j), lo) + o, min(e + (k - j), hi) + o)
            cur = t
        ob.sweep(self.p, cur, self._np(dst), b + o, e + o)

    def sweep2(self, src, dst, b, e, stream=None):
        self.sweepk(src, dst, b, e, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, iterations, depth, fused, init, split2=True, fuse_steps=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = partition(NZ, world, rank)
    be = OracleSlabBackend(count, depth, rank > 0, rank < world - 1, fused, fuse_steps)
    slab = SlabJacobi(be, SlabInfo(rank, world, first, count), TorchDistExchanger(rank, world))
    slab.split2 = split2
    slab.init(init, seed=31, plane_elems=NX * NY)
    slab.run(iterations)
    g = be._np(slab.cur)
    o = depth - 1
    np.save(os.path.join(outdir, f"r{rank}.npy"), g[1 + o:1 + o + count, 1:-1, 1:-1])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("depth,fused,split2", [(1, False, True), (2, False, False), (2, False, True),
                                                (2, True, False)])
@pytest.mark.parametrize("iterations", [4, 5])
def test_slab_matches_single_process(world, depth, fused, split2, iterations):
    """single sweeps (depth 1 or 2), split2 rounds (two single sweeps per
    2-plane exchange) and fused rounds, each bitwise equal to one process."""
    p = ob.problem(3, "fp64", "star", 1, "naive", NX, NY, NZ)
    want = ob.interior(p, ob.run(p, iterations, "random", 31))
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, iterations, depth, fused, "random", split2),
                           nprocs=world, join=True, start_method="fork")
        got = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)], axis=0)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("depth,k", [(3, 3), (4, 3), (4, 4)])
@pytest.mark.parametrize("iterations", [7, 8])
def test_slab_k_step_rounds(world, depth, k, iterations):
    """k fused sweeps per k-plane exchange (the TEMPORALK rounds), remainder
    as a pair and/or a single sweep: bitwise equal to one process."""
    p = ob.problem(3, "fp64", "star", 1, "naive", NX, NY, NZ)
    want = ob.interior(p, ob.run(p, iterations, "random", 31))
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, iterations, depth, True, "random", False, k),
                           nprocs=world, join=True, start_method="fork")
        got = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)], axis=0)
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))


def test_partition():
    assert [partition(14, 3, r) for r in range(3)] == [(0, 5), (5, 5), (10, 4)]
    assert sum(partition(4096, 8, r)[1] for r in range(8)) == 4096
    assert [partition(7, 7, r) for r in range(7)] == [(r, 1) for r in range(7)]
