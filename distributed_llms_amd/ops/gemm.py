"""Dense GEMM dispatch for y = x @ w^T (w is [N, K], nn.Linear layout).

* M <= 64 (decode): hand-written weight-streaming MFMA kernel (csrc/kernels/gemm_skinny.hip),
  8 waves per workgroup split K and reduce in LDS; optional fused SwiGLU epilogue.
* larger M (prefill) or shapes the kernel does not tile: plain library GEMM (hipBLASLt via
  torch).  That is the only non-HIP GPU path and it is purely shape-based.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext

SKINNY_MAX_M = 64
# Engine dispatch threshold: the skinny kernel is used for M <= ENGINE_SKINNY_M.  Set from
# measurements (bench/gemm_bench.py, profiles/gemm_skinny_v2.txt): v2 ties hipBLASLt only at
# M = 1, so the engine keeps the library GEMM until the kernel wins.
ENGINE_SKINNY_M = 0


def skinny_ok(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor, swiglu: bool = False,
              force: bool = False) -> bool:
    lim = SKINNY_MAX_M if force else ENGINE_SKINNY_M
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and 1 <= m <= lim
            and k % 128 == 0 and n % (32 if swiglu else 16) == 0 and x.is_contiguous() and w.is_contiguous())


def _launch(x, w, bias, y, m, n, k, mode):
    _ext.kernels().gemm_skinny(y.data_ptr(), x.data_ptr(), w.data_ptr(), 0 if bias is None else bias.data_ptr(),
                               m, n, k, mode, torch.cuda.current_stream().cuda_stream)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           force_skinny: bool = False) -> torch.Tensor:
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if w.shape[1] != k:
        raise ValueError(f"linear: x[..., {k}] vs w {tuple(w.shape)}")
    if skinny_ok(m, n, k, x, w, force=force_skinny) and (bias is None or bias.dtype == torch.bfloat16):
        y = torch.empty(*x.shape[:-1], n, dtype=x.dtype, device=x.device)
        _launch(x, w, bias, y, m, n, k, 0)
        return y
    return F.linear(x, w, bias)


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor, force_skinny: bool = False) -> Optional[torch.Tensor]:
    """silu(x Wg^T) * (x Wu^T) with W = [Wg; Wu] in one launch; None if the shape is not eligible."""
    k = x.shape[-1]
    n = w_gate_up.shape[0]
    m = x.numel() // k
    if not skinny_ok(m, n, k, x, w_gate_up, swiglu=True, force=force_skinny):
        return None
    y = torch.empty(*x.shape[:-1], n // 2, dtype=x.dtype, device=x.device)
    _launch(x, w_gate_up, None, y, m, n, k, 1)
    return y
