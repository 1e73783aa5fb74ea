"""Kernel-dispatch knobs: every A/B switch of the GPU op layer, in one place.

The defaults are the measured best on MI355X (each field cites its profile).  They change only
through :func:`update` -- called with ``EngineConfig.kernel_knobs`` when an engine or a pipeline
rank is built (so the values a run used are part of its config and of the bench JSON line) --
or, for experiments, from ONE environment variable read once at import::

    DLLM_KNOBS="wide_variant=1,defer_qkv=1"        # or a JSON object

Nothing else in the package reads kernel switches from the environment.  The op layer reads
``knobs.K.<field>`` at call time, so an update applies to every launch after it (HIP graphs
captured before an update keep the dispatch they were captured with).

Environment variables the package still reads (all documented in README "Environment"):
DLLM_KNOBS, DLLM_TRACE, DLLM_ROCTX, DLLM_JSON_LOGS, DLLM_DEVICE, DLLM_DIST_ADDR, DLLM_TRANSPORT,
DLLM_SHARE_GPU, DLLM_DATA_BACKEND, DLLM_PP_UNITS, DLLM_PP_FINE, DLLM_OFFLOAD_ARCH, DLLM_PART_TYPE.
"""
from __future__ import annotations

import contextlib
import dataclasses
import json
import os
from dataclasses import dataclass
from typing import Any, Dict, Mapping, Optional


@dataclass
class Knobs:
    # ---- dense GEMM dispatch (ops/gemm.py; profiles/wide_gemm.md)
    # which decode-sized GEMMs gemm_wide serves: "auto" (the cutovers below), "all", "none", or a
    # comma list of roles gate_up / down / proj
    wide: str = "auto"
    # gemm_wide variant for unsplit grids (33: LDS-DMA interleaved + asm fragment reads with one
    # lgkmcnt per MFMA row) and for split-K grids (1); in-engine A/B 27,123 vs 27,014 / 26,896 tok/s
    wide_variant: int = 33
    wide_variant_split: int = 1
    wide_gate_up_max_m: int = 256     # SwiGLU-fused gate|up on gemm_wide up to this M (then split-K gemm_pp / gemm_pf)
    wide_down_max_m: int = 384        # MLP down (K >= 8192, K > N) up to this M (512: split gemm_pp 59 vs 66 us)
    wide_proj_max_m: int = 256        # qkv / LM head up to this M (o: wide_o_max_m; down: wide_down_max_m)
    wide_target_wgs: int = 256        # split-K: about one workgroup per CU
    # medium M (mixed prefill + decode steps, short prompts; profiles/round5_medium_m_gemm.md): above
    # the decode cutovers a projection runs on gemm_pf only where its 256 x 256 grid fills the CUs
    # (ops/gemm.pf_fills: >= one tile per CU, rounds at least pf_min_eff full or >= 4 rounds), else
    # on gemm_pp with split-K; the square o-projection stays on gemm_wide up to wide_o_max_m
    pf_min_eff: float = 0.85
    wide_o_max_m: int = 512
    # decode SwiGLU gate|up from this M up to 256 on gemm_pp's 128-column tile with nontemporal
    # weights instead of gemm_wide, for grids of CUs / 2 .. CUs tiles (0 = off; not while comm kernels
    # reserve CUs).  8B at B = 256: 62.1 vs 64.1 us, engine +0.45 % tok/s over three interleaved pairs;
    # at M = 224: 8B 61.4 vs 65.7, 70B (256-column tile) 206 vs 244; at M = 192 the 8B loses
    # (profiles/round6_gate_up_pp.md)
    pp_gate_up_min_m: int = 200
    # decode down projections with K >= this (225 <= M <= 256) on split gemm_pp 128-column tiles with
    # nontemporal weights (0 = off): the 70B down (K = 28672) 126 vs 135 us, engine +0.85 % tok/s
    # (profiles/round6_gate_up_pp.md); the 8B down (K = 14336) stays on gemm_wide
    pp_down_min_k: int = 16384
    wide_small_bm: int = 128          # row-tile override for small split grids (0: off): the 8B o-projection at M = 256 as 2 x 128-row tiles x 4 K slices, engine +0.75 % tok/s (profiles/round6_gate_up_pp.md)
    wide_small_bm_maxw: int = 4096 * 4096
    # 256 x 256 decode GEMM (gemm_sq.hip): roles ("all", "none", or gate_up / down / proj / head),
    # from this M up to 256, unsplit grids only unless sq_split
    sq: str = "all"
    sq_min_m: int = 225
    sq_split: bool = False
    sq_variant: int = 4
    # prefill-sized GEMMs (above the decode kernels' ranges) on the hand-written 256 x 256 kernels
    # instead of hipBLASLt, from this M (0 = hipBLASLt): the persistent schedule-2 kernel gemm_pf
    # (pp_persistent; else gemm_pp schedule 2).  At T = 32768 (profiles/round4_gemm_counters.md):
    # gate|up + SwiGLU 1396 TFLOP/s vs 1345 for hipBLASLt + silu_mul; qkv / o / down 1415-1474 vs
    # hipBLASLt's 1511-1591.  In-engine (Llama-3-8B B = 256, two interleaved pairs): every prefill
    # GEMM hand-written 27,532 / 27,513 tok/s vs 27,792 / 27,753 with hipBLASLt on qkv / o / down
    # (-0.9 %) -- taken, so that no vendor GEMM runs in the forward path
    pp_swiglu_min_m: int = 257
    pp_proj_min_m: int = 257
    pp_persistent: bool = True
    # gemm_pf pulls its tiles from per-XCD device queues (a workgroup that starts late -- its CU held
    # by a co-resident RCCL / stand-in kernel -- finds them taken) instead of the static w + i P walk:
    # "on", "off", or "auto" = on while a transport with spinning comm kernels is live
    # (ops/gemm.reserve_cus_for_comm).  Alone on the GPU the static walk is 0.3 % faster end to end
    # (TTFT 343 vs 346 ms, two interleaved pairs, gpurun_out/r5j_bench.log)
    pf_dynamic: str = "auto"
    # decode LM head (N > 65536) at pp_head_min_m <= M <= 256 on gemm_pp schedule 2 with nontemporal
    # weights: 230 vs 265 us for gemm_sq at M = 256 (Llama-3-8B); 0 = off
    pp_head_min_m: int = 225
    # the LM head while comm kernels may hold CUs (a GPU pipeline stage with RCCL): "sq" (gemm_sq,
    # unaffected by a spinning receive) or "pp" (the nontemporal gemm_pp, faster alone)
    head_beside_comm: str = "sq"
    # ---- attention (ops/__init__.py)
    attn_target_waves: int = 1024     # decode split-KV: waves to aim for (profiles/attn_decode_sweep.txt)
    prefill_attn: int = 0             # prefill kernel: 0 = auto (9 from prefill_w32_min_q query rows at head_dim 128 -- 7 while comm kernels hold CUs -- else 4); 4 = LDS-shared K/V tiles on 16x16 MFMAs, 6 / 7 = the same on 32x32x16 MFMAs (7: P.V overlapping the softmax), 9 = 7 persistent (one workgroup per CU), 3 = register-tiled (> 32k fallback)
    prefill_w32_min_q: int = 384      # auto: the 32x32 kernel from this many query rows (128 x 256-token prompts: v4 209-215 us, v9 210-212; 96 x 384: 267-272 vs 260-262; profiles/round6_attention.md)
    # prefill q-RoPE in the attention kernel's q load (rope_cache appends K / V only): no rotated-q
    # round trip through HBM (268 MB per layer at T = 32768)
    prefill_fused_rope: bool = True
    # ---- model / engine
    fused_rope: bool = True           # decode: RoPE + KV append fused into attention
    # split-K qkv partials summed inside the fused RoPE + attention kernel (no splitk_reduce launch):
    # +0.2-0.6 % tok/s in 4 of 4 interleaved in-engine pairs on two boxes (round 3,
    # profiles/round3_gemm_experiments.md; a round-2 build measured -3 %)
    defer_qkv: bool = True
    defer_o: bool = True              # split-K o-proj reduce fused into the next add + RMSNorm
    lookahead: bool = True            # single-GPU engine: issue step n+1 before step n's tokens land
    pp_lookahead: bool = True         # pipeline driver: the same across stages
    # RCCL transport comm streams (send / recv / ring / ids copy): "pool" (torch pool streams) or
    # "priority" (one native high-priority stream per role: a queue of its own, but a spinning
    # high-priority kernel starves the compute queues -- pp2 73 % of IPC, pp4 stalled;
    # parallel/rccl_transport.comm_stream, profiles/round5_comm_queues.md)
    comm_queue: str = "pool"
    # CUs a GPU pipeline stage's spinning comm kernels may hold at once (receive + send + ids ring):
    # gemm_wide's split-K grids leave them free (ops/gemm.reserve_cus_for_comm)
    comm_reserved_cus: int = 16
    # device RCCL stand-in (parallel/rccl_standin.py, rehearsal only): LDS each channel workgroup
    # holds -- 20 KiB like RCCL's own p2p kernel (rcclGenericKernel on gfx950: 19,744 B of LDS,
    # 261-280 VGPRs, 256 threads; profiles/round5_comm_queues.md), which keeps a 144 KiB gemm_wide
    # workgroup off its CU -- and channels
    standin_lds_kib: int = 20
    standin_channels: int = 4
    # ---- MoE (ops/moe.py)
    moe_variant: int = 0
    moe_wide_min_pairs: int = 8       # token-expert pairs per expert from which the tiled GEMM serves
    moe_fused_router: bool = True
    # prefill V append eight tokens per workgroup, 16-byte stores into the transposed V cache
    # (norm_elementwise.hip v_group_kernel); False = the per-token 2-byte scatter.
    v_group_append: bool = True
    # grouped expert GEMM ring depth: 6 / 5 LDS slots at 64 / 128-row tiles (False: 3 slots)
    moe_deep_ring: bool = True
    # ---- FP8 W8A8 (ops/quant.py)
    fp8_bm128: bool = True
    fp8_group_m: int = 4096


K = Knobs()


def _coerce(name: str, value: Any) -> Any:
    typ = type(getattr(Knobs(), name))
    if typ is bool:
        if isinstance(value, str):
            return value.strip().lower() in ("1", "true", "yes", "on")
        return bool(value)
    return typ(value)


def update(overrides: Optional[Mapping[str, Any]] = None, **kw) -> Knobs:
    """Apply overrides (unknown names raise).  Returns the live knob object."""
    items = dict(overrides or {})
    items.update(kw)
    names = {f.name for f in dataclasses.fields(Knobs)}
    unknown = set(items) - names
    if unknown:
        raise ValueError(f"unknown kernel knobs: {sorted(unknown)} (known: {sorted(names)})")
    for k, v in items.items():
        setattr(K, k, _coerce(k, v))
    return K


@contextlib.contextmanager
def override(**kw):
    """Temporarily apply overrides (restored on exit, also on an exception)."""
    saved = dataclasses.asdict(K)
    update(kw)
    try:
        yield K
    finally:
        update(saved)


def reset() -> Knobs:
    """Back to the defaults (then the DLLM_KNOBS overrides)."""
    for f in dataclasses.fields(Knobs):
        setattr(K, f.name, f.default)
    update(parse(os.environ.get("DLLM_KNOBS", "")))
    return K


def parse(spec: str) -> Dict[str, Any]:
    """``"a=1,b=x"`` or a JSON object -> dict."""
    spec = (spec or "").strip()
    if not spec:
        return {}
    if spec.startswith("{"):
        return dict(json.loads(spec))
    out = {}
    for part in spec.split(","):
        if part.strip():
            k, _, v = part.partition("=")
            out[k.strip()] = v.strip()
    return out


def as_dict() -> Dict[str, Any]:
    return dataclasses.asdict(K)


def changed() -> Dict[str, Any]:
    """The knobs that differ from the defaults (what a bench line records)."""
    d = Knobs()
    return {f.name: getattr(K, f.name) for f in dataclasses.fields(Knobs) if getattr(K, f.name) != getattr(d, f.name)}


reset()
