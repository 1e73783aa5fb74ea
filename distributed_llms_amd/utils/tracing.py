"""Tracing: roctx ranges + a host-side ns timeline + GPU-timed spans.

The reference has ``print`` only (``src/master/node.py:36,70,...``; "latency profiling" is
future work at ``plan.md:297-300``).  Here:

* every span is also a ``roctxRangePushA``/``roctxRangePop`` pair when the ROCm roctx library
  is loadable, so ``rocprofv3 --marker-trace`` shows engine steps / stage hops next to kernels;
* spans land in a bounded in-memory timeline (``perf_counter_ns``), exportable as Chrome-trace
  JSON (``chrome://tracing`` / Perfetto);
* ``gpu_span`` brackets work with HIP events on the current stream, so a stage's *device*
  busy time (and hence its pipeline bubble %) is measured, not inferred from host time.

Disabled (the default) the hooks cost one attribute check: ``span`` returns a shared no-op
context.  Enable with ``DLLM_TRACE=1`` or ``get_tracer().enable()``.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from collections import deque
from typing import Dict, List, Optional

_NULL = contextlib.nullcontext()


def _load_roctx():
    for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                return lib
            except (OSError, AttributeError):
                continue
    return None


class _Span:
    __slots__ = ("tr", "name", "cat", "args", "t0")

    def __init__(self, tr: "Tracer", name: str, cat: str, args):
        self.tr, self.name, self.cat, self.args = tr, name, cat, args

    def __enter__(self):
        if self.tr._roctx is not None:
            self.tr._roctx.roctxRangePushA(self.name.encode())
        self.t0 = time.perf_counter_ns()
        return self

    def __exit__(self, *exc):
        t1 = time.perf_counter_ns()
        if self.tr._roctx is not None:
            self.tr._roctx.roctxRangePop()
        self.tr._push({"name": self.name, "cat": self.cat, "ph": "X", "ts": self.t0 / 1e3,
                       "dur": (t1 - self.t0) / 1e3, "tid": threading.get_ident() & 0xFFFF, "args": self.args})
        return False


class _GpuSpan:
    """Records start/end HIP events on the current stream; resolved lazily in ``flush_gpu``."""
    __slots__ = ("tr", "name", "cat", "args", "ev")

    def __init__(self, tr, name, cat, args):
        self.tr, self.name, self.cat, self.args = tr, name, cat, args

    def __enter__(self):
        import torch
        self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.ev[0].record()
        return self

    def __exit__(self, *exc):
        self.ev[1].record()
        with self.tr._lock:
            self.tr._pending_gpu.append((self.name, self.cat, self.args, self.ev))
        return False


class Tracer:
    def __init__(self, enabled: Optional[bool] = None, capacity: int = 1 << 16, roctx: Optional[bool] = None):
        self.enabled = (os.environ.get("DLLM_TRACE", "0") == "1") if enabled is None else enabled
        self._lock = threading.Lock()
        self._events: deque = deque(maxlen=capacity)
        self._pending_gpu: List = []
        self._gpu_busy: Dict[str, float] = {}   # cat -> accumulated device ms
        self._gpu_first: Dict[str, float] = {}
        self._roctx = None
        want_roctx = (os.environ.get("DLLM_ROCTX", "1") == "1") if roctx is None else roctx
        if want_roctx:
            self._roctx = _load_roctx()
        self.pid = os.getpid()

    # -- control ---------------------------------------------------------------------------
    def enable(self, on: bool = True):
        self.enabled = on
        return self

    def clear(self):
        with self._lock:
            self._events.clear()
            self._pending_gpu.clear()
            self._gpu_busy.clear()

    @property
    def has_roctx(self) -> bool:
        return self._roctx is not None

    # -- recording -------------------------------------------------------------------------
    def _push(self, ev: dict):
        with self._lock:
            self._events.append(ev)

    def span(self, name: str, cat: str = "host", **args):
        if not self.enabled:
            return _NULL
        return _Span(self, name, cat, args)

    def gpu_span(self, name: str, cat: str = "gpu", **args):
        """Device-timed span on the current HIP stream (no host sync until ``flush_gpu``)."""
        if not self.enabled:
            return _NULL
        return _GpuSpan(self, name, cat, args)

    def mark(self, name: str, **args):
        if not self.enabled:
            return
        if self._roctx is not None:
            self._roctx.roctxMarkA(name.encode())
        self._push({"name": name, "cat": "mark", "ph": "i", "s": "t", "ts": time.perf_counter_ns() / 1e3,
                    "tid": threading.get_ident() & 0xFFFF, "args": args})

    def counter(self, name: str, **values):
        if self.enabled:
            self._push({"name": name, "ph": "C", "ts": time.perf_counter_ns() / 1e3, "args": values})

    def flush_gpu(self):
        """Synchronise the recorded HIP events and fold them into the per-category busy time."""
        with self._lock:
            pend, self._pending_gpu = self._pending_gpu, []
        for name, cat, args, (a, b) in pend:
            b.synchronize()
            ms = a.elapsed_time(b)
            with self._lock:
                self._gpu_busy[cat] = self._gpu_busy.get(cat, 0.0) + ms
                self._events.append({"name": name, "cat": cat, "ph": "X", "ts": 0.0, "dur": ms * 1e3,
                                     "tid": 0xFFFF, "args": dict(args, device=True)})

    # -- reporting -------------------------------------------------------------------------
    def events(self) -> List[dict]:
        with self._lock:
            return list(self._events)

    def gpu_busy_ms(self, cat: str = "gpu") -> float:
        self.flush_gpu()
        return self._gpu_busy.get(cat, 0.0)

    def utilization(self, wall_s: float, cat: str = "gpu") -> Dict[str, float]:
        """Device busy fraction of a category over a wall-clock window; 1 - busy = bubble."""
        busy = self.gpu_busy_ms(cat) / 1e3
        if busy == 0.0:   # CPU stages: host spans of that category are the busy time
            busy = sum(e["dur"] for e in self.events() if e.get("cat") == cat and e.get("ph") == "X") / 1e6
        frac = busy / wall_s if wall_s > 0 else 0.0
        return {"busy_s": busy, "wall_s": wall_s, "busy_frac": frac, "bubble_frac": max(0.0, 1.0 - frac)}

    def host_summary(self) -> Dict[str, Dict[str, float]]:
        """Per span name: count, total and mean host ms."""
        out: Dict[str, Dict[str, float]] = {}
        for e in self.events():
            if e.get("ph") != "X" or e.get("args", {}).get("device"):
                continue
            d = out.setdefault(e["name"], {"count": 0, "total_ms": 0.0})
            d["count"] += 1
            d["total_ms"] += e["dur"] / 1e3
        for d in out.values():
            d["mean_ms"] = d["total_ms"] / max(1, d["count"])
        return out

    def export_chrome(self, path: str, process_name: Optional[str] = None):
        self.flush_gpu()
        evs = []
        for e in self.events():
            e = dict(e)
            e["pid"] = self.pid
            evs.append(e)
        if process_name:
            evs.append({"name": "process_name", "ph": "M", "pid": self.pid, "args": {"name": process_name}})
        with open(path, "w") as f:
            json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
        return path


_TRACER: Optional[Tracer] = None


def get_tracer() -> Tracer:
    global _TRACER
    if _TRACER is None:
        _TRACER = Tracer()
    return _TRACER
