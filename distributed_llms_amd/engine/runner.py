"""Stage executor: a ModelStage + its paged KV pool + decode-graph runner.

Used by the single-GPU engine and by every pipeline worker.
"""
from __future__ import annotations

import logging
from typing import Optional

import torch

from .. import knobs
from ..config import EngineConfig, ModelConfig, pipeline_slots
from ..models.stage import KVCache, ModelStage
from ..utils.tracing import get_tracer
from .batch import HostBatch, to_device_meta
from .graphs import DecodeGraphRunner

log = logging.getLogger("dllm.runner")


def plan_kv_blocks(mcfg: ModelConfig, num_layers: int, ecfg: EngineConfig, device,
                   num_kv_heads: Optional[int] = None) -> int:
    """KV blocks for a stage: enough for max_batch x max_seq_len (+ scratch), capped by free HBM.
    ``num_kv_heads``: the heads this rank caches (its share under tensor parallelism)."""
    bs = ecfg.kv_block_size
    if ecfg.num_kv_blocks > 0:
        return ecfg.num_kv_blocks
    per_seq = -(-ecfg.max_seq_len // bs)
    # microbatch slots in flight (the pipeline driver's, config.pipeline_slots)
    slots = pipeline_slots(ecfg, ecfg.num_workers, device)
    want = ecfg.max_batch * slots * per_seq + 2
    per_block = max(1, KVCache.bytes_per_block(num_layers, num_kv_heads or mcfg.num_kv_heads, mcfg.head_dim, bs))
    dev = torch.device(device)
    if dev.type == "cuda":
        free, _total = torch.cuda.mem_get_info(dev)
        cap = int(free * ecfg.kv_cache_fraction) // per_block
    else:
        cap = max(64, (2 << 30) // per_block)     # CPU: at most ~2 GiB of KV
    n = min(want, cap)
    if n < 2:
        raise RuntimeError("not enough memory for the KV cache")
    return n


class StageRunner:
    """``num_slots`` > 1 gives every microbatch slot its own decode-graph set (static buffers,
    graph pool, attention workspace), so slots can be replayed concurrently on separate streams."""

    def __init__(self, stage: ModelStage, ecfg: EngineConfig, num_blocks: Optional[int] = None,
                 num_slots: int = 1):
        self.stage = stage
        self.ecfg = ecfg
        self.tracer = get_tracer()
        # before any launch / graph capture: defaults (+ DLLM_KNOBS), then this config's overrides --
        # a previous engine's overrides in the same process must not leak into this one
        knobs.reset()
        if ecfg.kernel_knobs:
            knobs.update(ecfg.kernel_knobs)
        self.block_size = ecfg.kv_block_size
        nb = num_blocks or plan_kv_blocks(stage.cfg, stage.num_layers, ecfg, stage.device, stage.hkv)
        stage.allocate_kv(nb, self.block_size)
        self.num_blocks = nb
        self.max_blocks = -(-ecfg.max_seq_len // self.block_size)
        self._busy = None                 # [(start, end) events or host seconds] while metering
        self.graph_sets = []
        if ecfg.use_graphs and stage.device.type == "cuda":
            sizes = [b for b in ecfg.graph_batch_sizes if b <= ecfg.max_batch] or [ecfg.max_batch]
            if max(sizes) < ecfg.max_batch:
                sizes.append(ecfg.max_batch)
            self.graph_sets = [DecodeGraphRunner(stage, ecfg.max_batch, self.max_blocks, sizes)
                               for _ in range(max(1, num_slots))]
        log.info("stage [%d,%d) kv blocks=%d (%.1f GiB) weights=%.2f GiB", stage.layer_start, stage.layer_end,
                 nb, stage.kv.nbytes / 2**30, stage.weight_bytes() / 2**30)

    @property
    def graphs(self) -> Optional[DecodeGraphRunner]:
        return self.graph_sets[0] if self.graph_sets else None

    @torch.inference_mode()
    def execute(self, hb: HostBatch, hidden: Optional[torch.Tensor] = None, slot: int = 0,
                ids_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``ids_dev`` (first stage, decode): input token ids already on the device (they replace
        ``hb.ids``, a placeholder then)."""
        tr = self.tracer
        run = self._execute if self._busy is None else self._metered
        if not tr.enabled:
            return run(hb, hidden, slot, ids_dev)
        kind = "prefill" if hb.is_prefill else "decode"
        gspan = tr.gpu_span(kind, cat="stage") if self.stage.device.type == "cuda" else tr.span(kind, cat="stage")
        with tr.span(f"stage.{kind}", cat="host", rows=hb.num_tokens, seqs=hb.num_seqs, slot=slot), gspan:
            return run(hb, hidden, slot, ids_dev)

    def _execute(self, hb: HostBatch, hidden: Optional[torch.Tensor], slot: int,
                 ids_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        st = self.stage
        gr = self.graph_sets[slot % len(self.graph_sets)] if self.graph_sets else None
        if (not hb.is_prefill) and gr is not None and gr.can_run(hb.num_seqs, hb.max_ctx):
            return gr.run(hb, hidden, ids_dev=ids_dev)
        ids, meta = to_device_meta(hb, st.device)
        if ids_dev is not None:
            ids = ids_dev.to(torch.int32)
        return st.forward(ids if st.is_first else hidden, meta)

    # ---- busy metering: the stage's device time per microbatch (bench.py's stage_busy_frac)
    def meter(self, on: bool = True):
        self._busy = [] if on else None

    def _metered(self, hb, hidden, slot, ids_dev):
        if self.stage.device.type != "cuda":
            import time
            t0 = time.perf_counter()
            out = self._execute(hb, hidden, slot, ids_dev)
            self._busy.append(time.perf_counter() - t0)
            return out
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = self._execute(hb, hidden, slot, ids_dev)
        b.record()
        self._busy.append((a, b))
        return out

    def busy_seconds(self) -> float:
        """Sum of the metered microbatches' execution spans (synchronises the recorded events)."""
        tot = 0.0
        for e in self._busy or ():
            if isinstance(e, float):
                tot += e
            else:
                e[1].synchronize()
                tot += e[0].elapsed_time(e[1]) * 1e-3
        return tot

    def warmup_graphs(self, batch_sizes=None, ctx_buckets=(256,)):
        """Pre-capture decode graphs (keeps capture cost out of timed regions)."""
        for gr in self.graph_sets:
            for b in (batch_sizes or gr.batch_sizes):
                for c in ctx_buckets:
                    bb, cb = gr.bucket(b, c)
                    if (bb, cb) not in gr.graphs:
                        gr.capture(bb, cb)
