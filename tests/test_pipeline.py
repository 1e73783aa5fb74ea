"""Pipeline parallelism on CPU: in-process loopback stages and multi-process gloo ranks.

Both must reproduce the single-process engine's greedy tokens exactly (same fp32 math,
layers just split across stages).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.parallel.planner import plan_stages
from distributed_llms_amd.parallel.pipeline import run_loopback_pipeline

PROMPTS = [[i + 1, i + 5, 7, 9, 3 * i + 2] for i in range(13)]
PARAMS = SamplingParams(max_new_tokens=7, ignore_eos=True)


def _ecfg(**kw):
    d = dict(model="tiny-llama", dtype="float32", device="cpu", max_batch=4, max_seq_len=128,
             use_graphs=False, num_kv_blocks=256)
    d.update(kw)
    return EngineConfig(**d)


@pytest.fixture(scope="module")
def expected():
    return LLMEngine(_ecfg()).generate(PROMPTS, PARAMS)


@pytest.mark.parametrize("stages", [2, 3, 4])
def test_loopback_pipeline_matches_single(expected, stages):
    outs, drv, plan = run_loopback_pipeline(_ecfg(), stages, PROMPTS, PARAMS)
    assert outs == expected
    assert plan.num_stages == stages
    assert drv.num_slots >= stages


def test_planner_contiguous_and_balanced():
    cfg = get_model_config("llama3-8b")
    for n in (1, 2, 4, 8):
        plan = plan_stages(cfg, n)
        assert plan.ranges[0][0] == 0 and plan.ranges[-1][1] == 32
        for (a, b), (c, d) in zip(plan.ranges, plan.ranges[1:]):
            assert b == c and a < b
    p8 = plan_stages(cfg, 8)
    # the LM head (~2.4 blocks of bytes) pushes layers off the last stage
    assert p8.ranges[-1][1] - p8.ranges[-1][0] < 4
    assert p8.imbalance() < 1.2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, pp, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from distributed_llms_amd.parallel.dist_engine import RankRole, init_distributed
    import torch.distributed as dist
    ctx = init_distributed(pp=pp, backend="gloo")
    role = RankRole(ctx, _ecfg(num_workers=pp))
    res = []
    for rnd in range(2):   # two rounds: followers must return on ROUND_END and serve again
        seqs = [role.add_request(p, PARAMS) for p in PROMPTS] if role.is_driver else []
        role.run_round()
        res.append([s.output for s in seqs])
    role.shutdown()
    dist.barrier()
    out_q.put((rank, res if role.is_driver else None))
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("world,pp", [(2, 2), (4, 2), (2, 1)])
def test_multiprocess_gloo_pipeline(expected, world, pp):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, pp, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, res = q.get(timeout=300)
        results[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    drivers = [r for r in range(world) if r % pp == 0]
    for r in drivers:
        for rnd in results[r]:
            assert rnd == expected
