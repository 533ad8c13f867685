"""Face-signalled launches (stencil_sweepk_signal, whole 512^3 fp64 slab,
K=4) back to back, with the exchange-stream gate of each round:
  none    -- no gate (the launch alone)
  kernel  -- a one-lane wait kernel polling the device counters
  cp      -- the command processor waiting on the face signal
             (HIP signal memory, hipStreamWaitValue64)
Rounds interleave over 4 trials; prints ms per launch."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from stencil_amd import _lib
from stencil_amd.engine import FaceSignal, JacobiEngine, StencilSpec

n = int(os.environ.get("N", "512"))
k = int(os.environ.get("K", "4"))
e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=k), n, n, n, device=0, flags=_lib.HALO_LO | _lib.HALO_HI)
e.reset("random", 1)
sig = torch.zeros(4, dtype=torch.int32, device="cuda")
fs = FaceSignal()
sa = torch.cuda.Stream(priority=int(os.environ.get("PRIO", "-1")))
MASK = int(os.environ.get("MASK", "0"))  # 1: launches on CUs 0..254, the exchange stream on CU 255
if MASK:
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count

    def masked(bits):
        words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
        for b in bits:
            words[b // 32] |= 1 << (b % 32)
        h = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words) == 0
        return torch.cuda.ExternalStream(h.value)
    sb_masked = masked(range(ncu - 1))
    sa = masked([ncu - 1])
    torch.cuda.set_stream(sb_masked)
    print("CU masks: launches", ncu - 1, "CUs, exchange stream 1 CU", flush=True)
tiny = torch.zeros(64, device="cuda")
halo = torch.empty(k * e.unit, dtype=e.b.dtype, device=e.b.device)


def rounds(reps, gate):
    cur = torch.cuda.current_stream()
    sig.zero_()
    fs.reset()
    sa.wait_stream(cur)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    if gate == "sa_busy":  # one CP wait pending on sa over all launches
        fs.wait(2 * reps, stream=sa)
    if gate == "sa_evt":  # one event wait pending on sa over all launches
        evq = torch.cuda.Event()
    for r in range(reps if gate == "sa_evt" else 0):
        e.sweepk_signal(e.a, e.b, 0, n, k, sig, stream=cur)
    if gate == "sa_evt":
        evq.record(cur)
        sa.wait_event(evq)
        with torch.cuda.stream(sa):
            tiny.add_(1.0)
        cur.wait_stream(sa)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps
    for r in range(reps):
        m = e.sweepk_signal(e.a, e.b, 0, n, k, sig, stream=cur,
                            face_signal=fs if gate.startswith("cp") or gate in ("fs_only", "sa_busy") else None)
        if gate in ("none", "fs_only", "sa_busy"):
            continue
        with torch.cuda.stream(sa):
            if gate.startswith("cp"):
                fs.wait(2 * (r + 1), stream=sa)
            else:
                e.wait_counters(sig, (r + 1) * m, (r + 1) * m, stream=sa)
            if gate == "cp_tiny":
                tiny.add_(1.0)
            elif gate != "cp_only":
                halo.copy_(e.plane_view(e.b, 0, k))
    cur.wait_stream(sa)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for zc in os.environ.get("ZC", "default").split(","):
    if zc == "default":
        os.environ.pop("STENCIL_TK_ZCHUNK", None)
    else:
        os.environ["STENCIL_TK_ZCHUNK"] = zc
    res = {}
    for trial in range(3):
        for gate in ("none", "sa_busy"):
            rounds(3, gate)
            res.setdefault(gate, []).append(round(rounds(30, gate), 4))
    for gate, v in res.items():
        print(f"zchunk {zc}: {gate:7s} ms per launch {v}", flush=True)
print("face signal after the last trial:", fs.value())

