"""Probe: can two processes on ONE GPU form a native RCCL edge (RcclTransport, 2-stage pipeline)?
RCCL normally refuses two ranks on one device; if it accepts, run hops through the transport and
check them.  Prints a verdict line; never hangs (communicator deadlines + join timeouts).

    python scripts/rccl_2rank_probe.py
"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(rank, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    g = dist.new_group([0, 1], backend="gloo")
    try:
        from distributed_llms_amd.parallel.rccl_transport import RcclTransport
        t = RcclTransport([0, 1], rank, g, "cuda:0", max_rows=64, hidden=128, timeout_s=20.0)
        ok = True
        for i in range(7):
            if rank == 0:
                t.send_hidden(torch.full((64, 128), float(i), dtype=torch.bfloat16, device="cuda"))
                ids = t.recv_ids(64, "cuda").host()
                ok &= bool((ids == i).all())
            else:
                h = t.recv_hidden(64, 128, torch.bfloat16, "cuda")
                ok &= bool((h == float(i)).all().item())
                t.send_ids(torch.full((64,), i, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        t.drain()
        t.close()
        q.put((rank, "ok" if ok else "WRONG DATA", t.hop_stats()))
    except Exception as e:                       # noqa: BLE001
        q.put((rank, f"error: {type(e).__name__}: {str(e)[:300]}", {}))
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q), daemon=True) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, msg, hs = q.get(timeout=120)
            res[r] = (msg, hs)
    except Exception as e:                       # noqa: BLE001
        print("probe: no answer from a rank:", e)
    for p in ps:
        p.join(timeout=30)
    for r in sorted(res):
        print(f"rank {r}: {res[r][0]} {res[r][1]}")


if __name__ == "__main__":
    main()
