"""Stage planner: contiguous, cost-balanced stage ranges.

The reference groups parameters by ``key.split('.')[1]`` and greedily drops whole layers
onto the currently smallest shard (``src/model/shard_manager.py:33-61``), which for
equal-size layers is round-robin (shard0 = layers 0,2,4 -- D12) and useless for a
pipeline.  Here each stage owns ONE contiguous range, chosen by dynamic programming to
minimise the most expensive stage.

Two granularities:
* whole layers (:func:`plan_stages`) -- checkpoint shards (``shards/shard_{i}.pt`` hold whole
  blocks), cost = weight bytes (+ the LM head on the last stage);
* half layers (:func:`plan_units`, ``group`` 2) -- runtime pipelines: unit 2l = attention half of
  layer l (norm, qkv, RoPE + KV append, attention, o-proj), unit 2l+1 = its MLP half.  Llama-3-8B
  on 8 stages at batch 256 is capped at ~80 % balance by whole-layer cuts (32 layers + an LM head
  worth ~1.35 layers of time) and at ~93 % by half-layer cuts;
* sub-layer units (``group`` 5, opt-in for GPU pipelines of dense models) -- unit 5l + j of layer
  l is j = 0 norm + qkv projection, 1 RoPE + KV append + attention, 2 o-projection, 3 / 4 the MLP
  over the first / second half of the intermediate columns (models/stage.py).  A cut inside a half
  hands over the residual stream plus the pending qkv / attention output / partial MLP sum, and
  the DP prices each such cut on both stages it separates (CUT_US, fitted to measured stage
  times).  Measured on MI355X (profiles/pp_stage_balance.md) the cuts' own costs eat the balance
  they buy (pp8 slowest stage -1.3 %, pp2 / pp4 slower), so pipelines default to halves.
Costs come from a decode time model calibrated on MI355X kernel profiles
(profiles/llama3_8b_b256_kernels_current.md): each GEMM takes max(weight bytes / HBM rate, FLOPs /
achieved MFMA rate), attention reads the KV of ``ctx`` tokens per sequence, plus fixed per-half
elementwise/norm time.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from ..config import ModelConfig

# ---- decode time model (MI355X, bf16, wide decode GEMMs; calibrated on the Llama-3-8B batch-256
# profile, profiles/llama3_8b_b256_kernels_current.md: attention half 100.6 us, MLP half 99.7 us,
# LM head 254 us + argmax 19 us per step)
HBM_B_PER_US = 5.0e6          # weight streaming, bytes / us
KV_B_PER_US = 5.5e6           # attention KV read (nontemporal), bytes / us
ATTN_GEMM_FLOP_PER_US = 4.0e8 # qkv + o projections at decode M (0.40 PF achieved, split-K)
MLP_GEMM_FLOP_PER_US = 9.5e8  # gate_up (SwiGLU fused) + down (0.95 PF)
HEAD_FLOP_PER_US = 9.85e8     # LM head + argmax (0.99 PF)
ATTN_FIXED_US = 11.4          # qkv split-K reduce + residual/RMSNorm
MLP_FIXED_US = 6.3            # residual/RMSNorm (SwiGLU is in the GEMM epilogue)
# a stage cut inside a half (sub-layer units): the receiving side re-normalises the residual
# stream, half-width MLP GEMMs fill fewer CUs, partial sums are materialised, the hop is wider
CUT_US = {1: 6.0, 2: 15.0, 4: 45.0}   # by position j of the cut (after unit 5l + j - 1); fitted to
# bench/pp_stage_times.py on MI355X (profiles/pp_stage_balance.md)

HALF_GROUP, FINE_GROUP = 2, 5


@dataclass(frozen=True)
class StagePlan:
    ranges: Tuple[Tuple[int, int], ...]     # [start, end) layers touched per stage
    costs: Tuple[float, ...]
    units: Optional[Tuple[Tuple[int, int], ...]] = None   # [start, end) units per stage
    group: int = HALF_GROUP                 # units per layer (2: halves, 5: sub-layer units)

    @property
    def num_stages(self) -> int:
        return len(self.ranges)

    def stage_of_layer(self, layer: int) -> int:
        for i, (a, b) in enumerate(self.ranges):
            if a <= layer < b:
                return i
        raise KeyError(layer)

    def unit_range(self, stage: int) -> Tuple[int, int]:
        if self.units is not None:
            return self.units[stage]
        a, b = self.ranges[stage]
        return self.group * a, self.group * b

    def imbalance(self) -> float:
        return max(self.costs) / (sum(self.costs) / len(self.costs))

    def to_json(self):
        d = {"ranges": [list(r) for r in self.ranges], "costs": [round(c, 1) for c in self.costs]}
        if self.units is not None:
            d["units"] = [list(u) for u in self.units]
            d["group"] = self.group
        return d


def layer_costs(cfg: ModelConfig, dtype_bytes: int = 2) -> List[float]:
    return [cfg.layer_param_count() * dtype_bytes] * cfg.num_layers


def head_cost(cfg: ModelConfig, dtype_bytes: int = 2) -> float:
    return cfg.head_param_count() * dtype_bytes


def _partition(costs: Sequence[float], n: int, head: float, first_extra: float = 0.0,
               cut: Optional[Sequence[float]] = None) -> List[Tuple[int, int]]:
    """Exact min-max contiguous partition of ``costs`` into ``n`` parts (head added to the last).
    ``cut[i]``: extra cost a cut before unit i puts on BOTH stages it separates."""
    L = len(costs)
    if not 1 <= n <= L:
        raise ValueError(f"cannot split {L} units into {n} stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)

    def seg(a, b, s):
        c = pre[b] - pre[a]
        if cut is not None:
            c += (cut[a] if a > 0 else 0.0) + (cut[b] if b < L else 0.0)
        if s == 0:
            c += first_extra
        if s == n - 1:
            c += head
        return c

    INF = float("inf")
    best = [[INF] * (L + 1) for _ in range(n)]
    arg = [[0] * (L + 1) for _ in range(n)]
    for j in range(1, L + 1):
        best[0][j] = seg(0, j, 0)
    for s in range(1, n):
        for j in range(s + 1, L + 1):
            for i in range(s, j):
                v = max(best[s - 1][i], seg(i, j, s))
                if v < best[s][j] - 1e-9:
                    best[s][j], arg[s][j] = v, i
    bounds = [L]
    j = L
    for s in range(n - 1, 0, -1):
        j = arg[s][j]
        bounds.append(j)
    bounds.append(0)
    bounds.reverse()
    return [(bounds[i], bounds[i + 1]) for i in range(n)]


def plan_stages(cfg: ModelConfig, num_stages: int, costs: Optional[Sequence[float]] = None,
                head: Optional[float] = None, first_extra: float = 0.0) -> StagePlan:
    """Whole-layer plan (checkpoint shards), cost = bytes."""
    costs = list(costs) if costs is not None else layer_costs(cfg)
    head = head_cost(cfg) if head is None else head
    ranges = _partition(costs, num_stages, head, first_extra)
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    cs = [pre[b] - pre[a] + (first_extra if i == 0 else 0) + (head if i == num_stages - 1 else 0)
          for i, (a, b) in enumerate(ranges)]
    return StagePlan(tuple(ranges), tuple(cs))


def unit_costs_us(cfg: ModelConfig, batch: int = 256, ctx: int = 192) -> Tuple[List[float], float]:
    """Per half-layer decode time estimates (us) and the LM head's."""
    h, i = cfg.hidden_size, cfg.intermediate_size
    attn_p = h * cfg.qkv_size + cfg.q_size * h
    if cfg.is_moe:
        mlp_p_read = cfg.num_experts * 3 * h * i           # every expert is read at decode batch sizes
        mlp_p_flop = cfg.experts_per_token * 3 * h * i
    else:
        mlp_p_read = mlp_p_flop = (2 if cfg.arch == "gpt2" else 3) * h * i
    kv_b = batch * ctx * 2 * cfg.kv_size * 2
    attn = max(2 * attn_p / HBM_B_PER_US, 2 * batch * attn_p / ATTN_GEMM_FLOP_PER_US) + kv_b / KV_B_PER_US \
        + ATTN_FIXED_US
    mlp = max(2 * mlp_p_read / HBM_B_PER_US, 2 * batch * mlp_p_flop / MLP_GEMM_FLOP_PER_US) + MLP_FIXED_US
    head_p = cfg.vocab_size * h
    head = max(2 * head_p / HBM_B_PER_US, 2 * batch * head_p / HEAD_FLOP_PER_US)
    return [attn, mlp] * cfg.num_layers, head


def unit_costs_cpu(cfg: ModelConfig, ctx: int = 192) -> Tuple[List[float], float]:
    """Per half-layer costs of a CPU stage, in multiply-adds per decoded token.

    A CPU stage has no fixed per-kernel floor worth modelling: its GEMMs stream their weights
    (small batches) or are FLOP bound (large ones), and both scale with the parameter count, so
    the LM head weighs what its parameters weigh -- GPT-2 small's (50257 x 768) is worth ~5.5
    layers, which the GPU model above prices at ~1.  Attention adds its q.k and p.v work over
    ``ctx`` cached tokens."""
    h, i = cfg.hidden_size, cfg.intermediate_size
    attn = h * cfg.qkv_size + cfg.q_size * h + 2 * ctx * cfg.q_size
    mlp = (cfg.num_experts if cfg.is_moe else 1) * 3 * h * i
    if cfg.arch == "gpt2":
        mlp = 2 * h * i                                      # fc + proj, no gate
    return [float(attn), float(mlp)] * cfg.num_layers, float(cfg.vocab_size * h)


def unit_costs_fine_us(cfg: ModelConfig, batch: int = 256, ctx: int = 192) -> Tuple[List[float], float]:
    """Per sub-layer unit decode time estimates (us): the half-layer model with the attention half
    divided between qkv (its GEMM share + the split-K reduce and norm), the attention core (KV
    read) and the o-projection (its GEMM share), and the MLP half in two equal column halves."""
    halves, head = unit_costs_us(cfg, batch, ctx)
    h = cfg.hidden_size
    qkv_p, o_p = h * cfg.qkv_size, cfg.q_size * h
    kv_b = batch * ctx * 2 * cfg.kv_size * 2
    attn_core = kv_b / KV_B_PER_US
    gemm = halves[0] - attn_core - ATTN_FIXED_US
    qkv = gemm * qkv_p / (qkv_p + o_p) + ATTN_FIXED_US
    o = gemm * o_p / (qkv_p + o_p)
    mlp = halves[1]
    return [qkv, attn_core, o, mlp / 2, mlp / 2] * cfg.num_layers, head


def unit_costs_fine_cpu(cfg: ModelConfig, ctx: int = 192) -> Tuple[List[float], float]:
    """:func:`unit_costs_cpu` per sub-layer unit (multiply-adds per decoded token)."""
    h, i = cfg.hidden_size, cfg.intermediate_size
    qkv, attn, o = h * cfg.qkv_size, 2 * ctx * cfg.q_size, cfg.q_size * h
    mlp = 3 * h * i / 2
    return [float(qkv), float(attn), float(o), mlp, mlp] * cfg.num_layers, float(cfg.vocab_size * h)


def fine_units_ok(cfg: ModelConfig) -> bool:
    """Sub-layer units need a dense SwiGLU MLP whose halves keep the GEMM shape rules."""
    return cfg.arch != "gpt2" and not cfg.is_moe and cfg.intermediate_size % 256 == 0


def explicit_plan(cfg: ModelConfig, spec: str, num_stages: int) -> StagePlan:
    """A hand-placed plan: ``spec`` = "g:a,b;b,c;..." -- unit ranges in units of g per layer
    (``DLLM_PP_UNITS``; operations / experiments)."""
    g, _, body = spec.partition(":")
    group = int(g)
    units = tuple(tuple(int(x) for x in r.split(",")) for r in body.split(";"))
    if len(units) != num_stages or units[0][0] != 0 or units[-1][1] != group * cfg.num_layers or \
            any(a[1] != b[0] or a[0] >= a[1] for a, b in zip(units, units[1:] + ((units[-1][1], 0),))):
        raise ValueError(f"DLLM_PP_UNITS={spec!r} is not a contiguous {num_stages}-stage cover")
    ranges = tuple((a // group, (b + group - 1) // group) for a, b in units)
    return StagePlan(ranges, tuple(0.0 for _ in units), units, group)


def plan_units(cfg: ModelConfig, num_stages: int, batch: int = 256, ctx: int = 192,
               device: str = "cuda", fine: bool = False) -> StagePlan:
    """Runtime-pipeline plan (see module doc): half-layer units, or sub-layer units with ``fine``
    (GPU stages of a dense model; ignored elsewhere).  ``device`` picks the cost model (GPU decode
    time model, or :func:`unit_costs_cpu` for CPU stages).  ``DLLM_PP_UNITS`` overrides the plan
    (:func:`explicit_plan`)."""
    import os
    spec = os.environ.get("DLLM_PP_UNITS", "")
    if spec and num_stages > 1:
        return explicit_plan(cfg, spec, num_stages)
    cpu = str(device).startswith("cpu")
    cut = None
    group = HALF_GROUP
    if fine and num_stages > 1 and fine_units_ok(cfg):
        group = FINE_GROUP
        if cpu:
            costs, head = unit_costs_fine_cpu(cfg, ctx)
        else:
            costs, head = unit_costs_fine_us(cfg, batch, ctx)
            cut = [CUT_US.get(i % group, 0.0) for i in range(len(costs) + 1)]
    elif cpu:
        costs, head = unit_costs_cpu(cfg, ctx)
    else:
        costs, head = unit_costs_us(cfg, batch, ctx)
    units = _partition(costs, num_stages, head, cut=cut)
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    L = len(costs)
    cs = [pre[b] - pre[a] + (head if k == num_stages - 1 else 0)
          + ((cut[a] if a > 0 else 0.0) + (cut[b] if b < L else 0.0) if cut is not None else 0.0)
          for k, (a, b) in enumerate(units)]
    ranges = tuple((a // group, (b + group - 1) // group) for a, b in units)
    return StagePlan(ranges, tuple(cs), tuple(units), group)
