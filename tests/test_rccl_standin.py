"""RcclTransport's MULTI-RANK code path, executed on CPU processes against the stand-in
communicators (parallel/rccl_standin.py: the native module's interface, bytes over the
torch.distributed store).

Real RCCL cannot run two ranks on one device, and CPU hosts have none -- without the stand-in the
transport's per-edge unique-id exchange, communicator init order, send / recv / ring streams, slot
rings and ids ring closure would first run on the driver's 8-GPU node.  Here every stage of a
2 / 4 / 8-process pipeline builds its RcclTransport (kind "rccl", 2-rank edge communicators) and
the generated ids must equal the single-process engine's bit for bit.  The fallback tests inject a
failure on ONE rank -- at unique-id creation (before the exchange) and inside a communicator's
construction (after it) -- and every rank must agree on torch.distributed and still complete
(dist_engine.make_transport).  Reference flow: /root/reference/src/master/node.py:256-269.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams

PROMPTS = [[i + 1, i + 5, 7, 9, 3 * i + 2] for i in range(11)]
PARAMS = SamplingParams(max_new_tokens=6, ignore_eos=True)


def _ecfg(**kw):
    d = dict(model="tiny-llama", dtype="float32", device="cpu", max_batch=4, max_seq_len=128,
             use_graphs=False, num_kv_blocks=256, comm_timeout_s=8.0)
    d.update(kw)
    return EngineConfig(**d)


@pytest.fixture(scope="module")
def expected():
    return LLMEngine(_ecfg()).generate(PROMPTS, PARAMS)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, pp, port, env, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DLLM_TRANSPORT="rccl", DLLM_RCCL_STANDIN="1", **env)
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llms_amd.parallel.dist_engine import RankRole, init_distributed
    try:
        ctx = init_distributed(pp=pp, backend="gloo")
        role = RankRole(ctx, _ecfg(num_workers=pp))
        t = role.transport
        info = (t.kind, getattr(t, "comm_ranks", []))
        res = []
        for _ in range(2):   # two rounds: the rings and sequence numbers carry over
            seqs = [role.add_request(p, PARAMS) for p in PROMPTS] if role.is_driver else []
            role.run_round()
            res.append([s.output for s in seqs])
        role.shutdown()
        dist.barrier()
        out_q.put((rank, info, res if role.is_driver else None, None))
        dist.destroy_process_group()
    except Exception as e:      # noqa: BLE001 - reported to the test
        import traceback
        out_q.put((rank, None, None, traceback.format_exc()))
        raise


def _run(world, pp, env=None, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, pp, port, env or {}, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            r, info, res, err = q.get(timeout=timeout)
            assert err is None, f"rank {r} failed:\n{err}"
            results[r] = (info, res)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return results


@pytest.mark.slow
@pytest.mark.parametrize("world,pp", [(2, 2), (4, 4), (4, 2), (8, 8)])
def test_rccl_transport_multirank_matches_single(expected, world, pp):
    results = _run(world, pp)
    for r, (info, res) in results.items():
        kind, comm_ranks = info
        assert kind == "rccl"
        stage = r % pp
        # 2-rank edge communicators: in-edge, out-edge, and the ring closure on the end stages
        n_comms = (stage > 0) + (stage < pp - 1) + (1 if stage in (0, pp - 1) else 0)
        assert comm_ranks == [2] * n_comms
        if r % pp == 0:
            for rnd in res:
                assert rnd == expected


@pytest.mark.slow
@pytest.mark.parametrize("phase", ["uid", "init"])
def test_rccl_transport_failure_on_one_rank_falls_back_everywhere(expected, phase):
    """One rank's native transport fails; every rank must fall back to torch.distributed (the
    same kind on all stages) and the run completes with the same tokens."""
    results = _run(4, 4, env={"DLLM_RCCL_STANDIN_FAIL": f"{phase}:1"})
    kinds = {info[0] for info, _ in results.values()}
    assert kinds == {"torch"}
    for rnd in results[0][1]:
        assert rnd == expected


def test_standin_resolution(monkeypatch):
    from distributed_llms_amd.parallel.dist_engine import resolve_transport
    monkeypatch.setenv("DLLM_TRANSPORT", "rccl")
    monkeypatch.delenv("DLLM_RCCL_STANDIN", raising=False)
    assert resolve_transport("auto", "cpu", False) == "torch"
    monkeypatch.setenv("DLLM_RCCL_STANDIN", "1")
    assert resolve_transport("auto", "cpu", False) == "rccl"
    monkeypatch.delenv("DLLM_TRANSPORT")
    assert resolve_transport("auto", "cpu", False) == "torch"
