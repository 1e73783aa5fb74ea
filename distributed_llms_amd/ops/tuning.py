"""Pre-tuned hipBLASLt/rocBLAS solution choices for the library GEMMs (PyTorch TunableOp).

``bench/tune_gemms.py`` runs TunableOp over every GEMM shape the engine issues (decode graph
buckets, prefill chunk, LM head) on an MI355X and writes ``tuning/tunableop_gfx950.csv``.
At start-up the engine loads that file READ-ONLY (tuning disabled: nothing is timed at run time,
and a shape that is not in the file simply uses the library heuristic), so the choice is fixed
before any HIP graph is captured.  The file carries TunableOp validators (torch, HIP,
hipBLASLt, rocBLAS versions, gfx arch); on a mismatching stack TunableOp ignores it.

Disable with the ``tunableop`` kernel knob (distributed_llms_amd/knobs.py).
"""
from __future__ import annotations

import logging
import os
import tempfile

import torch

log = logging.getLogger("dllm.tuning")

TUNED_CSV = os.environ.get("DLLM_TUNABLEOP_FILE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "tunableop_gfx950.csv")
_state = {"done": False, "ok": False}


def enable_tuned_gemms(path: str = TUNED_CSV) -> bool:
    """Idempotent; returns True when the tuned table is active."""
    if _state["done"]:
        return _state["ok"]
    _state["done"] = True
    from .. import knobs
    if not knobs.K.tunableop or not torch.cuda.is_available() or not os.path.exists(path):
        return False
    tun = torch.cuda.tunable
    try:
        # TunableOp dumps its table at process exit to its filename: point that at a scratch
        # path so the in-tree file is never rewritten
        tun.set_filename(os.path.join(tempfile.gettempdir(), f"dllm_tunableop_{os.getpid()}.csv"))
        tun.enable(True)
        tun.tuning_enable(False)
        if hasattr(tun, "record_untuned_enable"):
            tun.record_untuned_enable(False)
        ok = bool(tun.read_file(path))
    except Exception as e:  # pragma: no cover - depends on the torch build
        log.warning("TunableOp table not loaded: %s", e)
        ok = False
    if not ok:
        tun.enable(False)
    _state["ok"] = ok
    log.info("tuned GEMM table %s: %s", path, "active" if ok else "not used")
    return ok
