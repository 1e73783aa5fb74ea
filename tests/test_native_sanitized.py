"""Host runtime under UBSan + libstdc++ assertions: ``_C_runtime`` (paged-KV block
manager, decode-slot batcher, wire-frame codec) is rebuilt with -fsanitize=undefined (no recovery) and
_GLIBCXX_ASSERTIONS, loaded into a fresh interpreter under its package name, and driven through a
randomized workload that includes every error path.  Any undefined behaviour or container
bounds violation aborts the child process, failing the test.  CPU only."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent('''
    import importlib.util, random, sys, zlib
    import numpy as np
    so = sys.argv[1]
    spec = importlib.util.spec_from_file_location("distributed_llms_amd._C_runtime", so)
    rt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rt)
    sys.modules["distributed_llms_amd._C_runtime"] = rt
    rng = random.Random(0)

    # ---- block manager: random alloc / grow / free with invariant checks
    for bs in (1, 16, 32):
        nb = 257
        bm = rt.BlockManager(nb, bs)
        live = {}
        for step in range(4000):
            op = rng.random()
            if op < 0.55:
                s = rng.randrange(64)
                n = live.get(s, 0) + rng.randrange(1, 4 * bs)
                if bm.ensure_capacity(s, n):
                    live[s] = n
            elif op < 0.75 and live:
                s = rng.choice(list(live))
                bm.free_sequence(s)
                del live[s]
            elif live:
                seqs = np.array(list(live)[: rng.randrange(1, len(live) + 1)], np.int64)
                width = max(bm.blocks_for(live[int(q)]) for q in seqs) + rng.randrange(3)
                out = np.full((len(seqs), width), -1, np.int32)
                bm.fill_block_tables(seqs, out, 0)
                start = np.array([rng.randrange(live[int(q)]) for q in seqs], np.int32)
                cnt = np.array([min(live[int(q)] - st, rng.randrange(1, 8)) for q, st in zip(seqs, start)], np.int32)
                slots = np.zeros(int(cnt.sum()), np.int32)
                assert bm.fill_slots(seqs, start, cnt, slots) == int(cnt.sum())
                assert (slots // bs >= 0).all() and (slots // bs < nb).all()
                lens = np.array([live[int(q)] + rng.randrange(0, 2 * bs) for q in seqs], np.int64)
                r = bm.ensure_capacity_batch(seqs, lens)   # grows seqs[:r] (all when r == -1)
                for q, l in list(zip(seqs, lens))[: len(seqs) if r == -1 else r]:
                    live[int(q)] = int(l)
            used = sum(bm.blocks_for(v) for v in live.values())
            assert bm.num_free() == nb - used, (bm.num_free(), nb, used)
        # error paths
        for bad in (lambda: bm.fill_slots(np.array([10 ** 6], np.int64), np.array([0], np.int32),
                                          np.array([1], np.int32), np.zeros(1, np.int32)),
                    lambda: bm.fill_block_tables(np.array([0, 1], np.int64), np.zeros((1, 1), np.int32), 0),
                    lambda: rt.BlockManager(0, 16)):
            try:
                bad()
            except Exception:
                pass

    # ---- slot batcher: random admit / decode (sync + lookahead) / complete / abort over a small
    # KV pool, so preemption and capacity failures happen
    for bs in (1, 4, 16):
        bm = rt.BlockManager(24 + 8 * bs, bs)
        nslots, max_seq = 3, 24 + rng.randrange(40)
        sb = rt.SlotBatcher(bm, nslots, max_seq)
        nxt = 1
        inflight = {s: [] for s in range(nslots)}
        for step in range(3000):
            slot = rng.randrange(nslots)
            op = rng.random()
            if op < 0.2 and sb.num_running(slot) < 12:
                n = rng.randrange(1, max_seq - 1)
                if bm.ensure_capacity(nxt, n):
                    sb.admit(slot, nxt, n, rng.randrange(1000), rng.randrange(1, 30),
                             rng.choice([-1, 3, 7]), rng.choice([0, 0, 5000]), 0, 10000)
                nxt += 1
            elif op < 0.6:
                look = bool(inflight[slot]) and rng.random() < 0.5
                if not look and inflight[slot]:
                    continue
                mb = -(-max_seq // bs) + rng.randrange(2)
                r = sb.build_decode(slot, mb, step, look)
                if r is not None:
                    packed, rows, keep = r
                    assert packed[2] == len(rows) and packed[3] == mb
                    inflight[slot].append(rows)
            elif op < 0.9 and inflight[slot]:
                rows = inflight[slot].pop(0)
                sb.complete(slot, rows, np.array([rng.randrange(10) for _ in rows], np.int32), float(step))
            elif op < 0.95:
                ids = sb.running_ids(slot)
                if len(ids) and not inflight[slot]:
                    sb.abort(int(ids[rng.randrange(len(ids))]))
            for sid, why in sb.take_finished():
                sb.take_output(sid)
            for sid in sb.take_preempted():
                sb.take_output(sid)
            assert bm.num_free() >= 0
        for bad in (lambda: sb.admit(99, 1, 1, 1, 1), lambda: sb.take_output(10 ** 9),
                    lambda: sb.build_decode(0, 0, 0, False), lambda: rt.SlotBatcher(bm, 1, 1)):
            try:
                bad()
            except Exception:
                pass

    # ---- frame codec: round trips, corrupted prefixes, wrong sizes
    for i in range(3000):
        hdr = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300)))
        plen = rng.randrange(0, 1 << 40)
        fr = rt.encode_frame_head(rng.randrange(0, 0xFFFF), rng.randrange(256), hdr, plen)
        pre = fr[:rt.FRAME_PREFIX_SIZE]
        try:
            cid, flags, hl, pl, crc = rt.decode_frame_prefix(pre)
            assert hl == len(hdr) and pl == plen and crc == zlib.crc32(hdr)
            assert rt.check_header_crc(hdr, crc) and rt.crc32(hdr) == crc
        except ValueError:
            pass                                  # payload beyond the codec's cap
        bad = bytearray(pre)
        bad[rng.randrange(len(bad))] ^= 1 << rng.randrange(8)
        for blob in (bytes(bad), pre[:rng.randrange(24)], pre + b"x"):
            try:
                rt.decode_frame_prefix(blob)
            except ValueError:
                pass
    print("sanitized runtime ok")
''')


def test_runtime_under_ubsan(tmp_path):
    from distributed_llms_amd.csrc import build
    try:
        so = build.build_runtime_sanitized(str(tmp_path / "ubsan"))
    except Exception as e:          # no sanitizer runtime in this toolchain
        pytest.skip(f"sanitizer build unavailable: {e}")
    r = subprocess.run([sys.executable, "-c", CHILD, so], cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"))
    assert r.returncode == 0 and "sanitized runtime ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
