"""HTTP front end of the master: the serving entry point for clients that are not Python.

The reference has an interactive REPL only (``run_master.py:26-42``); a ``/status`` HTTP
endpoint and Prometheus metrics appear in its docs (``implementation.md:34-41,80-83``).
Here ``run_master.py --http PORT`` serves, from a threaded stdlib HTTP server (no extra
dependency; every request thread only submits to the master's request futures):

  GET  /health                 {"state": "ready" | "degraded" | "idle", "workers": n}
  GET  /status                 the master's STATUS fan-out (workers, KV occupancy, metrics)
  GET  /metrics                Prometheus text: request metrics + per-worker gauges (HBM, KV blocks,
                               running / waiting sequences, microbatches executed)
  POST /generate               {"prompt": str | "prompt_ids": [int], "max_new_tokens", "temperature",
                                "top_k", "top_p", "ignore_eos"} -> {"tokens", "text", "latency_s", ...}
  POST /v1/completions         OpenAI-style: {"prompt": str | [int] | [str...], "max_tokens", ...}
                               -> {"object": "text_completion", "choices": [...], "usage": {...}}
  "stream": true               (either POST, one prompt) server-sent events: one ``data: {...}`` event
                               per pipeline step that produced tokens (TOKENS messages from stage 0),
                               then ``data: [DONE]``

Batches of prompts submitted together are scheduled together (continuous batching on stage 0).
"""
from __future__ import annotations

import json
import logging
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Tuple

from ..utils.metrics import cluster_prometheus_text

log = logging.getLogger("dllm.http")

_PARAM_KEYS = ("temperature", "top_k", "top_p", "ignore_eos", "seed")


def _sampling(body: Dict[str, Any], default_max: int = 64, max_key: str = "max_new_tokens") -> Dict[str, Any]:
    p = {k: body[k] for k in _PARAM_KEYS if k in body}
    p["max_new_tokens"] = int(body.get(max_key, body.get("max_new_tokens", default_max)))
    if p["max_new_tokens"] < 1:
        raise ValueError("max tokens must be >= 1")
    return p


class _Handler(BaseHTTPRequestHandler):
    server_version = "dllm-master/1"
    master = None            # set by serve_http
    timeout_s = 600.0

    # -------------------------------------------------------------- plumbing
    def log_message(self, fmt, *args):      # route through logging, not stderr
        log.debug("%s " + fmt, self.address_string(), *args)

    def _send(self, code: int, obj: Any, ctype: str = "application/json"):
        data = obj.encode() if isinstance(obj, str) else json.dumps(obj, default=str).encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self) -> Dict[str, Any]:
        n = int(self.headers.get("Content-Length") or 0)
        if n > 64 << 20:
            raise ValueError("request body too large")
        raw = self.rfile.read(n) if n else b"{}"
        body = json.loads(raw or b"{}")
        if not isinstance(body, dict):
            raise ValueError("JSON object expected")
        return body

    # -------------------------------------------------------------- routes
    def do_GET(self):
        m = self.master
        try:
            if self.path == "/health":
                self._send(200, {"state": m.state, "workers": len(m.workers)})
            elif self.path == "/status":
                self._send(200, m.status())
            elif self.path == "/metrics":
                self._send(200, cluster_prometheus_text(m.status()), "text/plain; version=0.0.4")
            else:
                self._send(404, {"error": f"no route {self.path}"})
        except Exception as e:  # noqa: BLE001 - reported to the client
            self._send(500, {"error": repr(e)})

    def do_POST(self):
        try:
            body = self._body()
            if body.get("stream") and self.path in ("/generate", "/v1/completions"):
                return self._stream(body)
            if self.path == "/generate":
                self._send(200, self._generate(body))
            elif self.path == "/v1/completions":
                self._send(200, self._completions(body))
            else:
                self._send(404, {"error": f"no route {self.path}"})
        except (ValueError, KeyError, TypeError) as e:
            self._send(400, {"error": repr(e)})
        except Exception as e:  # noqa: BLE001 - worker failures, timeouts
            self._send(503, {"error": repr(e)})

    def _stream(self, body: Dict[str, Any]):
        """Server-sent events: token chunks as stage 0 produces them, then [DONE]."""
        completions = self.path == "/v1/completions"
        prompt = body["prompt_ids"] if "prompt_ids" in body else body.get("prompt", "")
        ids = self._ids(prompt)
        if not ids:
            raise ValueError("empty prompt")
        params = _sampling(body, default_max=16 if completions else 64,
                           max_key="max_tokens" if completions else "max_new_tokens")
        gen = self.master.stream(ids, timeout=self.timeout_s, **params)
        first = next(gen, None)                       # errors before the first byte -> HTTP status
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.send_header("Cache-Control", "no-cache")
        self.send_header("Connection", "close")
        self.end_headers()
        tok = self.master.tokenizer

        def event(chunk):
            if completions:
                obj = {"object": "text_completion", "model": self.master.model_spec,
                       "choices": [{"index": 0, "text": tok.decode(chunk), "tokens": chunk, "finish_reason": None}]}
            else:
                obj = {"tokens": chunk, "text": tok.decode(chunk)}
            self.wfile.write(b"data: " + json.dumps(obj).encode() + b"\n\n")
            self.wfile.flush()

        try:
            if first is not None:
                event(first)
            for chunk in gen:
                event(chunk)
            self.wfile.write(b"data: [DONE]\n\n")
        except Exception as e:  # noqa: BLE001 - mid-stream failure: report in-band
            self.wfile.write(b"data: " + json.dumps({"error": repr(e)}).encode() + b"\n\n")
        self.wfile.flush()
        self.close_connection = True

    def _ids(self, prompt) -> List[int]:
        if isinstance(prompt, str):
            return self.master.tokenizer.encode(prompt)
        if isinstance(prompt, list) and all(isinstance(t, int) for t in prompt):
            return list(prompt)
        raise ValueError("prompt must be a string or a list of token ids")

    def _run(self, prompts: List[List[int]], params: Dict[str, Any]) -> List[Dict[str, Any]]:
        if not prompts or any(not p for p in prompts):
            raise ValueError("empty prompt")
        m = self.master
        futs = [m.submit(p, params) for p in prompts]          # submitted together -> batched together
        out = []
        for f in futs:
            r = m._finish(f, self.timeout_s)
            r["text"] = m.tokenizer.decode(r["tokens"])
            out.append(r)
        return out

    def _generate(self, body: Dict[str, Any]) -> Dict[str, Any]:
        ids = body["prompt_ids"] if "prompt_ids" in body else self._ids(body.get("prompt", ""))
        return self._run([self._ids(ids)], _sampling(body))[0]

    def _completions(self, body: Dict[str, Any]) -> Dict[str, Any]:
        prompt = body.get("prompt", "")
        if isinstance(prompt, list) and prompt and not all(isinstance(t, int) for t in prompt):
            prompts = [self._ids(p) for p in prompt]           # a batch of prompts
        else:
            prompts = [self._ids(prompt)]
        res = self._run(prompts, _sampling(body, default_max=16, max_key="max_tokens"))
        choices = [{"index": i, "text": r["text"], "tokens": r["tokens"],
                    "finish_reason": "length" if r.get("finish_reason") in ("length", "max_seq_len") else "stop"}
                   for i, r in enumerate(res)]
        ptok = sum(len(p) for p in prompts)
        ctok = sum(len(r["tokens"]) for r in res)
        return {"id": res[0].get("task_id"), "object": "text_completion", "created": int(time.time()),
                "model": self.master.model_spec, "choices": choices,
                "usage": {"prompt_tokens": ptok, "completion_tokens": ctok, "total_tokens": ptok + ctok}}


def serve_http(master, host: str = "127.0.0.1", port: int = 8000,
               timeout_s: float = 600.0) -> Tuple[ThreadingHTTPServer, threading.Thread]:
    """Start the HTTP front end on a daemon thread; returns (server, thread).  port 0 = any free port
    (``server.server_address[1]``).  ``server.shutdown()`` stops it."""
    handler = type("Handler", (_Handler,), {"master": master, "timeout_s": timeout_s})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    th = threading.Thread(target=srv.serve_forever, name="dllm-http", daemon=True)
    th.start()
    log.info("HTTP API on http://%s:%d", host, srv.server_address[1])
    return srv, th
