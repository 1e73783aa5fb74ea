"""Stage planner: contiguous, cost-balanced layer ranges.

The reference groups parameters by ``key.split('.')[1]`` and greedily drops whole
layers onto the currently smallest shard (``src/model/shard_manager.py:33-61``), which
for equal-size layers is round-robin (shard0 = layers 0,2,4 -- D12) and useless for a
pipeline.  Here each stage owns ONE contiguous block range, and the split minimises the
most expensive stage under a decode cost model in bytes read per step:

  block    = its weight bytes (+ KV bytes of the expected context, optional)
  stage 0  += one embedding row gather (negligible)
  last     += final norm + LM head (the 8B head is ~2.4 blocks of bytes)

Solved exactly by dynamic programming over (layers, stages) (L <= 80, stages <= 8).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from ..config import ModelConfig


@dataclass(frozen=True)
class StagePlan:
    ranges: Tuple[Tuple[int, int], ...]     # [start, end) per stage
    costs: Tuple[float, ...]

    @property
    def num_stages(self) -> int:
        return len(self.ranges)

    def stage_of_layer(self, layer: int) -> int:
        for i, (a, b) in enumerate(self.ranges):
            if a <= layer < b:
                return i
        raise KeyError(layer)

    def imbalance(self) -> float:
        return max(self.costs) / (sum(self.costs) / len(self.costs))

    def to_json(self):
        return {"ranges": [list(r) for r in self.ranges], "costs": list(self.costs)}


def layer_costs(cfg: ModelConfig, dtype_bytes: int = 2, active_experts_only: bool = True) -> List[float]:
    per = cfg.layer_param_count()
    if cfg.is_moe and active_experts_only:
        # decode reads only the routed experts' weights for small batches; at large batches
        # all experts are touched -- keep the full count, it is what HBM capacity needs anyway
        pass
    return [per * dtype_bytes] * cfg.num_layers


def head_cost(cfg: ModelConfig, dtype_bytes: int = 2) -> float:
    return cfg.head_param_count() * dtype_bytes


def plan_stages(cfg: ModelConfig, num_stages: int, costs: Optional[Sequence[float]] = None,
                head: Optional[float] = None, first_extra: float = 0.0) -> StagePlan:
    L = cfg.num_layers
    if not 1 <= num_stages <= L:
        raise ValueError(f"cannot split {L} layers into {num_stages} stages")
    costs = list(costs) if costs is not None else layer_costs(cfg)
    head = head_cost(cfg) if head is None else head
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)

    def seg(a, b, s):
        c = pre[b] - pre[a]
        if s == 0:
            c += first_extra
        if s == num_stages - 1:
            c += head
        return c

    INF = float("inf")
    # best[s][j]: min over splits of layers [0, j) into s+1 stages of the max stage cost
    best = [[INF] * (L + 1) for _ in range(num_stages)]
    arg = [[0] * (L + 1) for _ in range(num_stages)]
    for j in range(1, L + 1):
        best[0][j] = seg(0, j, 0)
    for s in range(1, num_stages):
        for j in range(s + 1, L + 1):
            for i in range(s, j):
                v = max(best[s - 1][i], seg(i, j, s))
                if v < best[s][j] - 1e-9:
                    best[s][j], arg[s][j] = v, i
    bounds = [L]
    j = L
    for s in range(num_stages - 1, 0, -1):
        j = arg[s][j]
        bounds.append(j)
    bounds.append(0)
    bounds.reverse()
    ranges = tuple((bounds[i], bounds[i + 1]) for i in range(num_stages))
    cs = tuple(seg(a, b, i) for i, (a, b) in enumerate(ranges))
    return StagePlan(ranges, cs)
