"""Host-side cost of one decode microbatch on the pipeline driver (stage 0), CPU only.

Per microbatch the driver runs: Scheduler.schedule(slot) -> build_host_batch -> HostBatch.pack
(meta to the next stage), and when the microbatch's tokens come back Scheduler.complete.  A
follower runs HostBatch.unpack.  At pp=8 a stage's GPU time per decode microbatch of 256
sequences is ~0.9 ms (4 Llama-3-8B layers), so this host path must stay well below that.
Decode bookkeeping is native (csrc/runtime/slot_batcher.cpp); the per-sequence Python version
it replaced measured schedule 108 + build 240 + pack 20 + complete 520 = 888 us here (8-CPU
Xeon container, B = 256, 9 slots).

    python bench/host_overhead.py [--batch 256] [--slots 9] [--ctx 192] [--steps 50]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

from distributed_llms_amd.engine.batch import HostBatch, build_host_batch
from distributed_llms_amd.engine.llm_engine import make_block_manager
from distributed_llms_amd.engine.scheduler import Scheduler
from distributed_llms_amd.engine.sequence import SamplingParams, Sequence


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--slots", type=int, default=9)
    ap.add_argument("--ctx", type=int, default=192)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--max-blocks", type=int, default=16)
    a = ap.parse_args()
    bs = 32
    nseq = a.batch * a.slots
    bm = make_block_manager(nseq * (a.ctx // bs + 4) + 8, bs)
    sch = Scheduler(bm, a.slots, a.batch, max_prefill_tokens=1 << 30, max_seq_len=4096)
    rng = np.random.default_rng(0)
    params = SamplingParams(max_new_tokens=10_000, ignore_eos=True)
    for _ in range(nseq):
        sch.add(Sequence(rng.integers(100, 30000, a.ctx).tolist(), params))
    # admit everything (one prefill step per slot), then run decode microbatches slot by slot
    for slot in range(a.slots):
        st = sch.schedule(slot)
        sch.complete(st, np.full(len(st.seqs), 7, np.int32))
    t = {"schedule": [], "build": [], "pack": [], "unpack": [], "complete": []}
    for i in range(a.steps * a.slots):
        slot = i % a.slots
        t0 = time.perf_counter()
        st = sch.schedule(slot)
        t1 = time.perf_counter()
        hb = build_host_batch(st, bm, bs, a.max_blocks, i)
        t2 = time.perf_counter()
        arr = hb.pack()
        t3 = time.perf_counter()
        HostBatch.unpack(arr)
        t4 = time.perf_counter()
        toks = np.concatenate([np.array([i, len(st.seqs)], np.int32), np.full(len(st.seqs), 11, np.int32)])
        sch.complete(st, toks[2:2 + int(toks[1])], time.perf_counter())
        t5 = time.perf_counter()
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
            t[k].append(v * 1e6)
    tot = 0.0
    print(f"decode microbatch host path, B={a.batch}, slots={a.slots}, ctx~{a.ctx} (median us over {a.steps * a.slots})")
    for k, v in t.items():
        m = statistics.median(v)
        tot += m if k != "unpack" else 0.0
        print(f"  {k:9s} {m:8.1f}")
    print(f"  driver total (schedule + build + pack + complete) {tot:.1f} us")


if __name__ == "__main__":
    main()
