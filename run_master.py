#!/usr/bin/env python
"""Master entrypoint (reference: run_master.py -- hard-coded 0.0.0.0:65432, facebook/opt-125m, 2 shards,
REPL verbs assign / distribute / inference / exit).  Same verbs, plus flags and a non-interactive mode.

    python run_master.py --model synthetic:llama3-8b --workers 1
    python run_master.py --model /path/to/hf_checkpoint --workers 2 --port 65432
    python run_master.py --model synthetic:gpt2-small --workers 2 --device cpu --auto --bench 16

    python run_master.py --model synthetic:llama3-8b --workers 2 --auto --http 8000   # HTTP serving

REPL: assign | distribute | inference | generate <n> | status | metrics | http <port> | exit
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llms_amd.config import EngineConfig  # noqa: E402
from distributed_llms_amd.master.node import MasterNode  # noqa: E402
from distributed_llms_amd.utils.logging import setup_logging  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=65432)
    ap.add_argument("--model", default="synthetic:gpt2-small")
    ap.add_argument("--workers", type=int, default=2, help="pipeline stages (= shards = workers)")
    ap.add_argument("--config", default=None, help="EngineConfig JSON/YAML file")
    ap.add_argument("--cache-dir", default="./models")
    ap.add_argument("--max-batch", type=int, default=None)
    ap.add_argument("--max-seq-len", type=int, default=None)
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--quant", choices=["none", "fp8"], default=None,
                    help="fp8: workers run W8A8 e4m3 projections / experts (ops/quant.py)")
    ap.add_argument("--heartbeat-timeout", type=float, default=None)
    ap.add_argument("--auto", action="store_true", help="wait for workers, assign + distribute, no REPL prompt")
    ap.add_argument("--auto-recover", action="store_true", help="re-distribute after a worker failure")
    ap.add_argument("--spares", type=int, default=0,
                    help="hot-spare workers to wait for beyond --workers: registered and heartbeating but "
                         "unassigned, so --auto-recover re-plans onto one at once when a stage dies")
    ap.add_argument("--bench", type=int, default=0, help="with --auto: submit N synthetic requests, print metrics")
    ap.add_argument("--bench-warmup", type=int, default=1, help="untimed warmup rounds before --bench")
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--gen-len", type=int, default=16)
    ap.add_argument("--wait-timeout", type=float, default=300.0)
    ap.add_argument("--http", type=int, default=-1, metavar="PORT",
                    help="serve the HTTP API (/generate, /v1/completions, /status, /metrics, /health) on PORT "
                         "once the pipeline is loaded (0 = any free port); with --auto, serve until Ctrl-C")
    ap.add_argument("--http-host", default="127.0.0.1")
    ap.add_argument("--log-level", default="INFO")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    setup_logging(a.log_level)
    cfg = EngineConfig.from_file(a.config) if a.config else EngineConfig()
    cfg = cfg.apply_overrides(host=a.host, port=a.port, model=a.model, num_workers=a.workers,
                              max_batch=a.max_batch, max_seq_len=a.max_seq_len, dtype=a.dtype,
                              heartbeat_timeout=a.heartbeat_timeout, quant=a.quant)
    master = MasterNode(a.host, a.port, cfg, auto_recover=a.auto_recover).start()
    print(f"Initializing model {a.model} into {a.workers} shard(s)...", flush=True)
    path = master.initialize_model(a.model, num_shards=a.workers, cache_dir=a.cache_dir)
    print(f"Model ready: {path}", flush=True)
    print(f"Master listening on {a.host}:{master.port}; start workers with:\n"
          f"  python run_worker.py --master 127.0.0.1:{master.port} [--device cuda:N]", flush=True)
    try:
        if a.auto:
            master.wait_for_workers(a.workers + a.spares, timeout=a.wait_timeout)
            print("assignments:", master.assign_shards(), flush=True)
            acks = master.distribute_shards()
            print("loaded:", json.dumps({w: x.get("layer_range") for w, x in acks.items()}), flush=True)
            if a.http >= 0:
                from distributed_llms_amd.master.http_api import serve_http
                srv, _ = serve_http(master, a.http_host, a.http)
                print(f"HTTP API on http://{a.http_host}:{srv.server_address[1]}", flush=True)
                if not a.bench:
                    while master.running:        # serve until Ctrl-C
                        time.sleep(1.0)
            if a.bench:
                import numpy as np
                rng = np.random.default_rng(0)
                vocab = master.model_config.vocab_size
                prompts = rng.integers(3, min(vocab, 30000), size=(a.bench, a.prompt_len)).tolist()
                for _ in range(a.bench_warmup):     # untimed: first-use costs (graph replays, allocator)
                    master.generate(prompts, max_new_tokens=a.gen_len, ignore_eos=True)
                t0 = time.perf_counter()
                res = master.generate(prompts, max_new_tokens=a.gen_len, ignore_eos=True)
                el = time.perf_counter() - t0
                toks = sum(len(r["tokens"]) for r in res)
                lat = sorted(r["latency_s"] for r in res)
                print(json.dumps({"requests": len(res), "output_tokens": toks, "elapsed_s": round(el, 3),
                                  "output_tok_per_s": round(toks / el, 2),
                                  "p50_latency_ms": round(1000 * lat[len(lat) // 2], 2)}), flush=True)
            return 0
        while True:
            cmd = input("\nEnter command (assign/distribute/inference/stream/generate/status/metrics/exit): ").strip()
            if cmd == "assign":
                print("Shard assignments:", master.assign_shards())
            elif cmd == "distribute":
                acks = master.distribute_shards()
                print("Shards distributed:", {w: x.get("layer_range") for w, x in acks.items()})
            elif cmd == "inference":
                text = input("Enter text for inference: ")
                res = master.run_inference(text, max_new_tokens=32)
                print("Inference result:", json.dumps({k: res[k] for k in ("tokens", "text", "latency_s")}))
            elif cmd == "stream":
                # tokens printed as the pipeline produces them (TOKENS messages from stage 0)
                text = input("Enter text for inference: ")
                ids = master.tokenizer.encode(text)
                for chunk in master.stream(ids, max_new_tokens=32):
                    print(master.tokenizer.decode(chunk), end="", flush=True)
                print()
            elif cmd.startswith("generate"):
                n = int(cmd.split()[1]) if len(cmd.split()) > 1 else 8
                res = master.generate([[5, 6, 7, 8]] * n, max_new_tokens=16)
                print([r["tokens"] for r in res])
            elif cmd == "status":
                print(json.dumps(master.status(), indent=1, default=str))
            elif cmd == "metrics":
                print(json.dumps(master.metrics.summary(), indent=1))
            elif cmd.startswith("http"):
                from distributed_llms_amd.master.http_api import serve_http
                srv, _ = serve_http(master, a.http_host, int(cmd.split()[1]) if len(cmd.split()) > 1 else 8000)
                print(f"HTTP API on http://{a.http_host}:{srv.server_address[1]}")
            elif cmd == "exit":
                break
            else:
                print("Unknown command")
    except (KeyboardInterrupt, EOFError):
        pass
    finally:
        master.stop()
        print("Master node stopped", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
