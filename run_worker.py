#!/usr/bin/env python
"""Worker entrypoint (reference: run_worker.py -- WorkerNode(master_address="localhost:65432").start()).

    python run_worker.py --master 127.0.0.1:65432 --device cuda:0
    python run_worker.py --master 127.0.0.1:65432 --device cpu
One worker per GPU; the master assigns each a contiguous layer slice (pipeline stage).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_llms_amd.utils.logging import setup_logging  # noqa: E402
from distributed_llms_amd.worker.node import WorkerNode  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--master", default="localhost:65432")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=65433)
    ap.add_argument("--device", default="auto", help="cuda:N | cpu | auto")
    ap.add_argument("--heartbeat", type=float, default=5.0)
    ap.add_argument("--fail-after", type=int, default=0, help="fault injection: exit after N engine steps")
    ap.add_argument("--no-peer-server", action="store_true")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    setup_logging(a.log_level)
    worker = WorkerNode(a.host, a.port, master_address=a.master, device=a.device, heartbeat_interval=a.heartbeat,
                        fail_after_steps=a.fail_after, serve_peers=not a.no_peer_server)
    print(f"Worker node initialized and connecting to master at {a.master}", flush=True)
    try:
        worker.start(block=True)
    except KeyboardInterrupt:
        pass
    finally:
        worker.stop()
        print("Worker node stopped", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
