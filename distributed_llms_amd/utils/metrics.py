"""Request / engine metrics: tok/s, latency percentiles, TTFT, ITL.

The reference has ``print`` statements only (``src/master/node.py:36,70,...``); Prometheus
and ``/metrics`` appear only in its docs (``implementation.md:34-41,146-157``).  Here every
component can keep a :class:`RequestMetrics` and dump ``summary()`` as JSON; the master's
STATUS reply carries it, and :func:`prometheus_text` renders the same numbers in the
Prometheus text exposition format.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional


def percentile(xs: List[float], q: float) -> Optional[float]:
    if not xs:
        return None
    s = sorted(xs)
    k = (len(s) - 1) * q / 100.0
    f = int(k)
    c = min(f + 1, len(s) - 1)
    return s[f] + (s[c] - s[f]) * (k - f)


class RequestMetrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.t0 = time.perf_counter()
        self.latencies: List[float] = []
        self.ttfts: List[float] = []
        self.tokens = 0
        self.requests = 0

    def record(self, n_tokens: int, latency_s: float, ttft_s: Optional[float] = None):
        with self._lock:
            self.tokens += n_tokens
            self.requests += 1
            self.latencies.append(latency_s)
            if ttft_s is not None:
                self.ttfts.append(ttft_s)

    def record_seqs(self, seqs):
        for s in seqs:
            self.record(len(s.output), s.latency() or 0.0, s.ttft())

    def summary(self) -> Dict[str, Optional[float]]:
        with self._lock:
            el = time.perf_counter() - self.t0
            lat, tt = list(self.latencies), list(self.ttfts)
            return {
                "requests": self.requests, "output_tokens": self.tokens, "elapsed_s": el,
                "output_tok_per_s": self.tokens / el if el > 0 else None,
                "latency_p50_s": percentile(lat, 50), "latency_p90_s": percentile(lat, 90),
                "latency_p99_s": percentile(lat, 99), "ttft_p50_s": percentile(tt, 50),
                "ttft_p99_s": percentile(tt, 99),
            }


def request_timing(ttfts: List[float], itls: List[float]) -> Dict[str, Optional[float]]:
    """Bench-line fields: time to first token and inter-token latency percentiles, in ms."""
    ms = lambda v: None if v is None else round(1000.0 * v, 3)
    return {"ttft_p50_ms": ms(percentile(ttfts, 50)), "ttft_p99_ms": ms(percentile(ttfts, 99)),
            "itl_p50_ms": ms(percentile(itls, 50)), "itl_p99_ms": ms(percentile(itls, 99))}


def seq_timing(seqs):
    """(ttfts, itls) in seconds of finished sequences."""
    ttfts = [t for t in (s.ttft() for s in seqs) if t is not None]
    itls = [d for s in seqs for d in s.itl()]
    return ttfts, itls


def itl_stats(seqs) -> Dict[str, Optional[float]]:
    xs = [d for s in seqs for d in s.itl()]
    return {"itl_p50_s": percentile(xs, 50), "itl_p99_s": percentile(xs, 99)}


def prometheus_text(summary: Dict[str, Optional[float]], prefix: str = "dllm") -> str:
    lines = []
    for k, v in summary.items():
        if v is None:
            continue
        lines.append(f"# TYPE {prefix}_{k} gauge")
        lines.append(f"{prefix}_{k} {float(v):.6g}")
    return "\n".join(lines) + "\n"


# per-worker gauges of the master's STATUS fan-out (HBM used, KV blocks, queue depth)
_WORKER_GAUGES = ("hbm_used_bytes", "hbm_total_bytes", "kv_free_blocks", "running", "waiting", "steps",
                  "hop_tx_bytes", "hop_rx_bytes", "hop_tx_bytes_per_s", "hop_rx_bytes_per_s")


def _label(v) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")


def cluster_prometheus_text(status: Dict, prefix: str = "dllm") -> str:
    """Render ``MasterNode.status()`` as Prometheus gauges: the request metrics, the master's
    pending requests, and one labelled series per worker for every numeric gauge it reported."""
    out = [prometheus_text(status.get("metrics") or {}, prefix).rstrip("\n")]
    if "pending_requests" in status:
        out += [f"# TYPE {prefix}_pending_requests gauge", f"{prefix}_pending_requests {int(status['pending_requests'])}"]
    out += [f"# TYPE {prefix}_workers gauge", f"{prefix}_workers {len(status.get('workers') or {})}"]
    stage_of = {w: i for i, w in enumerate(status.get("stage_workers") or [])}
    rows = {g: [] for g in _WORKER_GAUGES}
    for wid, w in sorted((status.get("workers") or {}).items()):
        remote = w.get("remote") or {}
        labels = f'worker="{_label(wid)}",stage="{stage_of.get(wid, -1)}",role="{_label(remote.get("role", ""))}"'
        for g in _WORKER_GAUGES:
            v = remote.get(g)
            if isinstance(v, (int, float)) and not isinstance(v, bool):
                rows[g].append(f"{prefix}_worker_{g}{{{labels}}} {float(v):.6g}")
    for g, lines in rows.items():
        if lines:
            out.append(f"# TYPE {prefix}_worker_{g} gauge")
            out += lines
    return "\n".join(x for x in out if x) + "\n"
