"""Loader for the in-tree native extensions.

``_C_kernels``  HIP/CDNA4 kernels for gfx950 (csrc/kernels/*.hip), pybind11 module.
``_C_runtime``  host C++ runtime: paged-KV block manager, wire-frame codec (csrc/runtime).
``_C_rccl``     native RCCL p2p transport (csrc/comm).

Both are built in-tree by ``python -m distributed_llms_amd.csrc.build`` (also run by
``__graft_entry__.build()``).  GPU ops never fall back silently: if the kernel module is
missing when a CUDA tensor reaches an op, :func:`kernels` raises.
"""
from __future__ import annotations

import importlib
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_kernels = None
_runtime = None
_kernels_err = None
_runtime_err = None


def _import(name):
    # torch must be imported first so its libamdhip64.so.7 is the one our module binds to.
    import torch  # noqa: F401
    return importlib.import_module(f"distributed_llms_amd.{name}")


def kernels():
    """The HIP kernel module; raises (loudly) if it is not built."""
    global _kernels, _kernels_err
    if _kernels is None:
        try:
            _kernels = _import("_C_kernels")
        except ImportError as e:  # pragma: no cover - exercised on misconfigured boxes
            _kernels_err = e
            raise RuntimeError(
                "distributed_llms_amd._C_kernels is not built (or failed to load): "
                f"{e}. Run `python -m distributed_llms_amd.csrc.build`.") from e
    return _kernels


def runtime():
    global _runtime, _runtime_err
    if _runtime is None:
        try:
            _runtime = _import("_C_runtime")
        except ImportError as e:
            _runtime_err = e
            raise RuntimeError(
                "distributed_llms_amd._C_runtime is not built: "
                f"{e}. Run `python -m distributed_llms_amd.csrc.build`.") from e
    return _runtime


_rccl = None


def rccl():
    """The native RCCL p2p module; raises if it is not built.  ``DLLM_RCCL_STANDIN=1`` (tests /
    rehearsal only) returns parallel/rccl_standin.py instead: the same interface over the
    torch.distributed store, so the transport's multi-rank path runs where RCCL cannot."""
    if os.environ.get("DLLM_RCCL_STANDIN", "0") == "1":
        from .parallel import rccl_standin
        rccl_standin.warn_selected()
        return rccl_standin
    return rccl_native()


def rccl_native():
    """The native module itself (also the stand-in's HIP-IPC helpers)."""
    global _rccl
    if _rccl is None:
        try:
            _rccl = _import("_C_rccl")
        except ImportError as e:
            raise RuntimeError(
                "distributed_llms_amd._C_rccl is not built (or failed to load): "
                f"{e}. Run `python -m distributed_llms_amd.csrc.build`.") from e
    return _rccl


def has_kernels() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def has_runtime() -> bool:
    try:
        runtime()
        return True
    except RuntimeError:
        return False
