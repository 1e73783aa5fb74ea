"""Control-plane transport vs the reference's framing (BASELINE comparator (b), config 1 plumbing).

The reference's one working data path frames a message as a 10-byte ASCII header
length, a pickled header dict and the raw payload, and receives the payload in 4 KiB pieces
with ``payload += chunk`` (D18: O(n^2) copying).  This bench re-creates that ALGORITHM in a few
lines (no reference code is imported or copied) and times it against ``network/protocol.py``
(24-byte binary prefix via the native codec, JSON header, ``recv_into`` one preallocated
buffer) over a localhost TCP socket pair:

* one-way payload throughput for payloads from 1 KiB to 256 MiB (a shard file is ~0.2-2 GB);
* round-trip latency of a small control message (HEARTBEAT-sized ping-pong).

    python bench/protocol_bench.py [--max-mb 256] [--ref-max-mb 16] [--out profiles/...md]
"""
from __future__ import annotations

import argparse
import os
import pickle
import socket
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llms_amd.network.protocol import MessageProtocol  # noqa: E402

REF_HDR = 10


# ---------------------------------------------------------------- the reference's algorithm
def ref_send(sock, command, payload=None, metadata=None):
    header = dict(metadata or {}, command=command)
    if payload is not None:
        header["payload_size"] = len(payload)
    h = pickle.dumps(header)
    sock.sendall(f"{len(h):<{REF_HDR}}".encode() + h)
    if payload is not None:
        sock.sendall(payload)


def _ref_recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("closed")
        buf += chunk
    return buf


def ref_recv(sock):
    hlen = int(_ref_recv_exact(sock, REF_HDR).decode().strip())
    header = pickle.loads(_ref_recv_exact(sock, hlen))      # trusted here: our own bytes
    payload = None
    if "payload_size" in header:
        payload = b""
        while len(payload) < header["payload_size"]:         # 4 KiB pieces, concatenated: O(n^2)
            chunk = sock.recv(min(4096, header["payload_size"] - len(payload)))
            if not chunk:
                raise ConnectionError("closed")
            payload += chunk
    return header, payload


# ---------------------------------------------------------------- harness
def _pair():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    cli = socket.create_connection(srv.getsockname())
    conn, _ = srv.accept()
    srv.close()
    for s in (cli, conn):
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return cli, conn


def one_way(send, recv, size, reps):
    cli, conn = _pair()
    payload = os.urandom(min(size, 1 << 20)) * max(1, size >> 20) if size >= (1 << 20) else os.urandom(size)
    payload = payload[:size]
    times = []
    got = []

    def reader():
        for _ in range(reps):
            h, p = recv(conn)
            got.append(len(p))
            conn.sendall(b"k")                               # ack: the receive is complete

    th = threading.Thread(target=reader)
    th.start()
    for _ in range(reps):
        t0 = time.perf_counter()
        send(cli, "LOAD_SHARD", payload, {"shard_id": 0})
        assert cli.recv(1) == b"k"
        times.append(time.perf_counter() - t0)
    th.join()
    cli.close()
    conn.close()
    assert all(g == size for g in got)
    return min(times)


def ping_pong(send, recv, reps=2000):
    cli, conn = _pair()

    def echo():
        for _ in range(reps):
            h, _ = recv(conn)
            send(conn, "HEARTBEAT", None, {"timestamp": h.get("timestamp")})

    th = threading.Thread(target=echo)
    th.start()
    ts = []
    for i in range(reps):
        t0 = time.perf_counter()
        send(cli, "HEARTBEAT", None, {"timestamp": i})
        recv(cli)
        ts.append(time.perf_counter() - t0)
    th.join()
    cli.close()
    conn.close()
    return statistics.median(ts)


def ours_send(sock, command, payload=None, metadata=None):
    MessageProtocol.send_message(sock, command, payload=payload, metadata=metadata)


def ours_recv(sock):
    return MessageProtocol.receive_message(sock, timeout=600)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mb", type=int, default=256)
    ap.add_argument("--ref-max-mb", type=int, default=16, help="the O(n^2) receive gets slow fast")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sizes = [1 << 10, 64 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20]
    sizes = [s for s in sizes if s <= (a.max_mb << 20)]
    rows = []
    for s in sizes:
        reps = 5 if s >= (16 << 20) else 20
        t_ours = one_way(ours_send, ours_recv, s, reps)
        t_ref = one_way(ref_send, ref_recv, s, 3 if s >= (4 << 20) else reps) if s <= (a.ref_max_mb << 20) else None
        rows.append((s, t_ours, t_ref))
        print(f"{s >> 10:>8} KiB  ours {s / t_ours / 1e6:9.1f} MB/s  "
              + (f"reference-style {s / t_ref / 1e6:9.1f} MB/s  ({t_ref / t_ours:.1f}x)" if t_ref else ""), flush=True)
    rt_ours, rt_ref = ping_pong(ours_send, ours_recv), ping_pong(ref_send, ref_recv)
    print(f"control round trip: ours {rt_ours * 1e6:.1f} us, reference-style {rt_ref * 1e6:.1f} us", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("# Control-plane framing vs the reference's (localhost TCP, 8-CPU dev container)\n\n")
            f.write("`python bench/protocol_bench.py` -- one-way payload transfer (send until the receiver has\n"
                    "the whole payload in memory), best of several; the reference-style column re-creates its\n"
                    "algorithm (pickled header behind a 10-byte ASCII length, payload received in 4 KiB pieces\n"
                    "concatenated with `+=`, SURVEY D18).\n\n")
            f.write("| payload | ours MB/s | reference-style MB/s | speedup |\n|---|---|---|---|\n")
            for s, to, tr in rows:
                size = f"{s >> 20} MiB" if s >= (1 << 20) else f"{s >> 10} KiB"
                f.write(f"| {size} | {s / to / 1e6:,.0f} | " + (f"{s / tr / 1e6:,.0f} | {tr / to:.1f}x |\n" if tr else
                                                               "(not run: quadratic) | |\n"))
            f.write(f"\nSmall control message round trip (HEARTBEAT ping-pong, median of 2000): ours "
                    f"{rt_ours * 1e6:.1f} us, reference-style {rt_ref * 1e6:.1f} us.\n")


if __name__ == "__main__":
    main()
