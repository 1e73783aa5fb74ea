"""Dense GEMM dispatch for y = x @ w^T (w is [N, K], nn.Linear layout).

Large M (prefill) is a plain library GEMM (hipBLASLt via torch).  Small M
(decode, M <= 256) goes to the hand-written MFMA weight-streaming kernel in
``csrc/kernels/gemm.hip`` once it is built with that entry point.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    return F.linear(x, w, bias)
