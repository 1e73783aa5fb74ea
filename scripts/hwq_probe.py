"""What a spinning communication kernel does to the rest of a process (one MI355X).

    python scripts/hwq_probe.py queues <mode>      # which streams a spinning receive blocks
    python scripts/hwq_probe.py gemms              # decode GEMMs beside a spinning receive

queues: a receive kernel that is never matched (parallel/rccl_standin's device kernel, as an RCCL
p2p receive posted before its send) spins in the stream under test; one small kernel is then
enqueued on the default stream and on 7 pool streams, and the probe reports the streams whose
kernel did not finish within 1 s -- they share the spinner's hardware queue (HIP deals a
process's streams over GPU_MAX_HW_QUEUES queues; a queue runs in order).  Modes:
  pool          the spinner in a pool stream
  masked_all    a CU-masked stream whose mask is every CU (hipExtStreamCreateWithCUMask)
  masked_part   a CU-masked stream on CUs 0..N-9 (every CU but 8)
  priority      a high-priority pool stream
  priority_multi / masked_multi   the same, probing three more streams of the spinner's kind
Run with GPU_MAX_HW_QUEUES in the environment to probe other queue counts.

gemms: the Llama-3-8B decode projections at M = 256 (gemm_wide, the engine's split choice) alone
and beside a spinner holding 4 CUs (no LDS; 40 KiB of LDS per block, which a 144 KiB gemm_wide
workgroup cannot share), then the same with the split-K grids sized to leave those CUs free
(knobs.wide_target_wgs).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def spinner(k, stream, lds_kib, timeout_s, channels):
    import ctypes
    from distributed_llms_amd.parallel import rccl_standin as rs
    words = k.p2p_host_words(2)
    wv = (ctypes.c_int * 2).from_address(words)
    inbox = torch.zeros(k.p2p_inbox_bytes(rs.CHUNK, rs.SLOTS), dtype=torch.uint8, device="cuda")
    dst = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    k.p2p_standin(0, 0, 0, 0, dst.data_ptr(), inbox.data_ptr(), dst.numel(), 0, rs.CHUNK, rs.SLOTS, channels,
                  words, timeout_s, words + 4, lds_kib << 10, stream.cuda_stream)
    return wv, (inbox, dst)


def queues(mode):
    from distributed_llms_amd import _ext
    k, m = _ext.kernels(), _ext.rccl_native()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    bufs = [torch.zeros(1 << 16, device="cuda") for _ in range(8)]
    pool = [torch.cuda.Stream() for _ in range(7)]
    if mode == "pool":
        spin = torch.cuda.Stream()
    elif mode == "masked_all":
        spin = torch.cuda.ExternalStream(m.cu_masked_stream(0))
    elif mode == "masked_part":
        mask = [0] * ((cus + 31) // 32)
        for c in range(cus - 8):
            mask[c // 32] |= 1 << (c % 32)
        spin = torch.cuda.ExternalStream(m.cu_masked_stream(0, mask))
    elif mode in ("priority", "priority_multi"):
        lo, hi = torch.cuda.Stream.priority_range()
        spin = torch.cuda.Stream(priority=hi)
    elif mode == "masked_multi":
        spin = torch.cuda.ExternalStream(m.cu_masked_stream(0))
    else:
        raise SystemExit(f"unknown mode {mode}")
    extra, names = [], []
    if mode == "priority_multi":         # three more high-priority streams (torch's high-priority pool)
        extra = [torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1]) for _ in range(3)]
        names = ["hi 1..3"]
    elif mode == "masked_multi":         # three more CU-masked streams
        extra = [torch.cuda.ExternalStream(m.cu_masked_stream(0)) for _ in range(3)]
        names = ["masked 1..3"]
    bufs += [torch.zeros(1 << 16, device="cuda") for _ in extra]
    torch.cuda.synchronize()
    wv, keep = spinner(k, spin, 0, 10.0, 2)
    time.sleep(0.05)
    others = [torch.cuda.current_stream()] + pool + extra
    evs = []
    for i, s in enumerate(others):
        with torch.cuda.stream(s):
            bufs[i].add_(1)
            e = torch.cuda.Event()
            e.record(s)
        evs.append(e)
    t0 = time.time()
    while time.time() - t0 < 1.0 and not all(e.query() for e in evs):
        time.sleep(0.01)
    blocked = [i for i, e in enumerate(evs) if not e.query()]
    live = not spin.query()
    wv[0] = 1
    spin.synchronize()
    for e in evs:
        e.synchronize()
    print(f"queues mode={mode} GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '(default)')}: "
          f"blocked {blocked} of [default, pool 0..6{', ' + names[0] if names else ''}] "
          f"(spinner live during probe: {live})", flush=True)


def _spin_main(lds_kib, channels, timeout_s, ready, stop):
    from distributed_llms_amd import _ext
    k = _ext.kernels()
    s = torch.cuda.Stream()
    wv, keep = spinner(k, s, lds_kib, timeout_s, channels)
    time.sleep(0.05)
    ready.set()
    stop.wait(timeout_s + 30)
    wv[0] = 1
    s.synchronize()


class SpinnerProc:
    """The spinner in another process: shares CUs with the timed work, none of its hardware
    queues, normal priority (a high-priority in-process spinner starves normal queues)."""

    def __init__(self, lds_kib, channels, timeout_s=60.0):
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        self.ready, self.stop = ctx.Event(), ctx.Event()
        self.p = ctx.Process(target=_spin_main, args=(lds_kib, channels, timeout_s, self.ready, self.stop), daemon=True)

    def __enter__(self):
        self.p.start()
        assert self.ready.wait(120)
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.p.join(timeout=90)
        return False


def _time(fn, n=20):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    ev[-1][1].synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2] * 1e3


def gemms():
    from distributed_llms_amd import _ext, knobs
    from distributed_llms_amd.ops import gemm
    torch.manual_seed(0)
    m = 256
    shapes = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
              "down": (4096, 14336, False)}
    x = {kk: torch.randn(m, kk, device="cuda", dtype=torch.bfloat16) for kk in (4096, 14336)}
    ws = {nm: [torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(4)]
          for nm, (n, kk, _) in shapes.items()}
    it = {"i": 0}

    def run(nm):
        n, kk, sw = shapes[nm]
        w = ws[nm][it["i"] % 4]
        it["i"] += 1
        return gemm.linear_wide(x[kk], w, swiglu=sw)

    from distributed_llms_amd.ops.gemm import release_cus_for_comm, reserve_cus_for_comm
    for lds, reserve in ((0, 0), (40, 0), (40, 16)):
        if reserve:
            reserve_cus_for_comm(reserve)
        try:
            solo = {nm: _time(lambda nm=nm: run(nm)) for nm in shapes}
            with SpinnerProc(lds, 4):
                beside = {nm: min(_time(lambda nm=nm: run(nm)) for _ in range(3)) for nm in shapes}
            for nm, (n, kk, sw) in shapes.items():
                s = gemm.wide_splits(m, n, kk, sw)
                tiles = (n // 128) * (-(-m // gemm.wide_row_tile(m, n, kk, sw)))
                print(f"gemms spinner LDS {lds:2d} KiB reserved CUs {reserve:2d} {nm:8s} wgs={tiles * s:4d} solo {solo[nm]:7.1f} us  "
                      f"beside a 4-CU spinner (other process) {beside[nm]:7.1f} us  ({beside[nm] / solo[nm]:.2f}x)", flush=True)
        finally:
            if reserve:
                release_cus_for_comm()


if __name__ == "__main__":
    if sys.argv[1] == "queues":
        queues(sys.argv[2])
    else:
        gemms()
