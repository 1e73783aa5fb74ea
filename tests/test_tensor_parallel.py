"""Tensor parallelism (parallel/tensor_parallel.py): shard algebra on CPU, then multi-process gloo
TP groups that must generate the single-process engine's greedy tokens."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.ops import reference as ref
from distributed_llms_amd.parallel import tensor_parallel as T

PROMPTS = [[i + 1, i + 5, 7, 9, 3 * i + 2] for i in range(9)]
PARAMS = SamplingParams(max_new_tokens=6, ignore_eos=True)


@pytest.mark.parametrize("name,size", [("tiny-llama", 2), ("tiny-mixtral", 2), ("llama3-8b", 8)])
def test_row_and_column_shards_sum_to_the_full_projection(name, size):
    cfg = get_model_config(name)
    if name == "llama3-8b":      # shapes only: a scaled-down stand-in with the same head structure
        import dataclasses
        cfg = dataclasses.replace(cfg, hidden_size=256, intermediate_size=512, head_dim=16)
    w = W.synth_block(cfg, 0, 3, torch.float32, "cpu")
    x = torch.randn(5, cfg.hidden_size)
    a = torch.randn(5, cfg.num_heads * cfg.head_dim)
    shards = [T.shard_block(cfg, w, r, size) for r in range(size)]
    hq = cfg.num_heads // size
    # o projection: row-parallel partials of the rank's own q heads sum to the full product
    o = sum(a[:, r * hq * cfg.head_dim:(r + 1) * hq * cfg.head_dim] @ s["wo"].t() for r, s in enumerate(shards))
    torch.testing.assert_close(o, a @ w["wo"].t(), rtol=1e-4, atol=1e-4)
    # qkv: column shards are the rank's q heads | k heads | v heads of the full output
    full = x @ w["wqkv"].t()
    d, hkv = cfg.head_dim, cfg.num_kv_heads // size
    for r, s in enumerate(shards):
        y = x @ s["wqkv"].t()
        q0, k0, v0 = r * hq * d, cfg.q_size + r * hkv * d, cfg.q_size + cfg.kv_size + r * hkv * d
        torch.testing.assert_close(y, torch.cat([full[:, q0:q0 + hq * d], full[:, k0:k0 + hkv * d],
                                                 full[:, v0:v0 + hkv * d]], 1))
    if cfg.is_moe:
        i = cfg.intermediate_size
        for e in range(cfg.num_experts):
            gu = w["experts_gate_up"][e]
            ref_e = (torch.nn.functional.silu(x @ gu[:i].t()) * (x @ gu[i:].t())) @ w["experts_down"][e].t()
            part = 0
            for s in shards:
                g = s["experts_gate_up"][e]
                il = g.shape[0] // 2
                part = part + (torch.nn.functional.silu(x @ g[:il].t()) * (x @ g[il:].t())) @ s["experts_down"][e].t()
            torch.testing.assert_close(part, ref_e, rtol=1e-4, atol=1e-4)
    else:
        ref_mlp = ref.linear(ref.silu_mul(x @ w["w_gate_up"].t()), w["w_down"])
        part = sum(ref.linear(ref.silu_mul(x @ s["w_gate_up"].t()), s["w_down"]) for s in shards)
        torch.testing.assert_close(part, ref_mlp, rtol=1e-4, atol=1e-4)


def test_expert_parallel_shards_sum_to_the_full_moe():
    """moe="ep": each rank holds whole experts; with routing over all experts and the other ranks'
    tokens contributing zero, the group's partial MoE outputs sum to the full sparse MLP."""
    cfg = get_model_config("tiny-mixtral")
    w = W.synth_block(cfg, 0, 5, torch.float32, "cpu")
    x = torch.randn(7, cfg.hidden_size)
    from distributed_llms_amd import ops
    full = ops.moe_forward(x, w["router"], w["experts_gate_up"], w["experts_down"], cfg.experts_per_token)
    for size in (2, 4):
        shards = [T.shard_block(cfg, w, r, size, moe="ep") for r in range(size)]
        assert shards[0]["experts_gate_up"].shape[0] == cfg.num_experts // size
        parts = [ops.moe_forward(x, s["router"], s["experts_gate_up"], s["experts_down"], cfg.experts_per_token,
                                 T.TPGroup(r, size, moe="ep").expert_offset(cfg.num_experts))
                 for r, s in enumerate(shards)]
        torch.testing.assert_close(sum(parts), full, rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError):
        T.check_divisible(cfg, 8, moe="ep")                  # 4 experts


def test_divisibility_is_checked():
    with pytest.raises(ValueError):
        T.check_divisible(get_model_config("tiny-llama"), 4)          # 2 kv heads
    with pytest.raises(ValueError):
        T.check_divisible(get_model_config("tiny-gpt2"), 2)
    T.check_divisible(get_model_config("llama3-70b"), 8)


def _ecfg(model, **kw):
    d = dict(model=model, dtype="float32", device="cpu", max_batch=4, max_seq_len=128, use_graphs=False,
             num_kv_blocks=128)
    d.update(kw)
    return EngineConfig(**d)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, tp, model, port, out_q, pp=1, moe="tp"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llms_amd.parallel.dist_engine import RankRole, init_distributed
    try:
        ctx = init_distributed(pp=pp, backend="gloo", tp=tp, moe=moe)
        role = RankRole(ctx, _ecfg(model, num_workers=pp))
        res = []
        for rnd in range(2):       # followers return on ROUND_END and serve the next round
            seqs = [role.add_request(p, PARAMS) for p in PROMPTS] if role.is_driver else []
            role.run_round()
            res.append([s.output for s in seqs])
        role.shutdown()
        dist.barrier()
        out_q.put((rank, res if role.is_driver else None, None))
        dist.destroy_process_group()
    except BaseException as e:       # pragma: no cover - surfaced in the parent
        out_q.put((rank, None, repr(e)))
        raise


@pytest.mark.slow
@pytest.mark.parametrize("model,world,tp,moe", [("tiny-llama", 2, 2, "tp"), ("tiny-mixtral", 2, 2, "tp"),
                                                ("tiny-llama", 4, 2, "tp"), ("tiny-mixtral", 2, 2, "ep"),
                                                ("tiny-mixtral", 4, 2, "ep")])
def test_multiprocess_tensor_parallel_matches_single(model, world, tp, moe):
    """dp x tp groups (and, for Mixtral, expert parallelism inside the group: moe="ep") generate the
    single-process engine's greedy tokens."""
    expected = LLMEngine(_ecfg(model)).generate(PROMPTS, PARAMS)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, tp, model, port, q, 1, moe)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, res, err = q.get(timeout=300)
        assert err is None, f"rank {r}: {err}"
        results[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(0, world, tp):               # every replica's leader
        for rnd in results[r]:
            assert rnd == expected


@pytest.mark.slow
@pytest.mark.parametrize("model,world,pp,tp", [("tiny-llama", 4, 2, 2), ("tiny-mixtral", 4, 2, 2)])
def test_pipeline_of_tensor_parallel_stages_matches_single(model, world, pp, tp):
    """pp x tp: every stage is a TP group; lane t (the t-th TP rank of each stage) carries its own
    activation hops and sampled-ids ring; the stage-0 TP peer replays the driver's issues."""
    expected = LLMEngine(_ecfg(model)).generate(PROMPTS, PARAMS)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, tp, model, port, q, pp)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, res, err = q.get(timeout=300)
        assert err is None, f"rank {r}: {err}"
        results[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r in results if results[r] is not None] == [0]     # one driver: stage 0, TP rank 0
    for rnd in results[0]:
        assert rnd == expected


def test_shards_own_their_storage():
    """Every TP / EP shard is a copy, not a view into the full tensor (a leading-dim slice is
    'contiguous', and a view would keep the whole layer / LM head resident on every rank)."""
    from distributed_llms_amd.models import weights as W
    from distributed_llms_amd.parallel.tensor_parallel import shard_block, shard_vocab
    for name, moe in (("tiny-llama", "tp"), ("tiny-mixtral", "tp"), ("tiny-mixtral", "ep")):
        cfg = get_model_config(name)
        full = {n: W.synth_tensor(1, 0, n, s, torch.float32, "cpu") for n, s in W.block_shapes(cfg).items()}
        for r in range(2):
            for n, t in shard_block(cfg, full, r, 2, moe).items():
                if t is not full.get(n):
                    assert t.untyped_storage().nbytes() == t.numel() * t.element_size(), (name, moe, n)
    head = torch.randn(64, 16)
    sh = shard_vocab(head, 1, 4)
    assert torch.equal(sh, head[16:32]) and sh.untyped_storage().nbytes() == sh.numel() * 4
