"""bench.py driver contract on CPU: the exact `python -m torch.distributed.run ... bench.py --gpus N`
form (gloo backend here), one JSON line from rank 0 with the required keys."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.slow
@pytest.mark.parametrize("n,par,trace", [(2, "pp", True), (3, "pp", False), (8, "pp", False), (2, "dp", False),
                                         (2, "tp", False)])
def test_torchrun_bench_cpu(n, par, trace, tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "1", "--model", "tiny-llama", "--batch", "3",
           "--prompt-len", "6", "--gen-len", "4", "--parallelism", par]
    if trace:
        cmd += ["--trace", str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == n and rec["value"] > 0 and rec["config"]["parallelism"] == f"{par}{n}"
    if par == "pp":                 # CPU stages run one slot per stage (config.pipeline_slots)
        assert rec["microbatch_slots"] == n
        assert rec["config"]["global_batch"] == 3 * n
        # every stage but the last sends activations; the last sends the ids back to stage 0
        assert len(rec["hop_tx_MBps"]) == n and all(v > 0 for v in rec["hop_tx_MBps"])
        assert rec["transport"] == "torch" and all(v > 0 for v in rec["meta_MBps"][:-1])
    assert rec["ttft_p50_ms"] > 0 and rec["itl_p50_ms"] > 0 and rec["ttft_p99_ms"] >= rec["ttft_p50_ms"]
    if par == "tp":                 # one TP group: one engine's batch
        assert rec["config"]["global_batch"] == 3
    if trace:   # every rank wrote a timeline; every stage reports its busy fraction
        assert sorted(os.listdir(tmp_path)) == [f"trace_rank{r}.json" for r in range(n)]
        assert len(rec["stage_busy_frac"]) == n and all(0 < b <= 1.0 for b in rec["stage_busy_frac"])
        # the per-rank host-cost summary (scripts/trace_host_summary.py) reads those timelines
        out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_host_summary.py"), str(tmp_path)],
                             capture_output=True, text=True, timeout=120).stdout
        assert all(f"rank {r}:" in out for r in range(n)) and "stage.decode" in out


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 4])
def test_torchrun_bench_over_rccl_transport_cpu(n):
    """The driver's N-GPU bench path with the pipeline data plane on the native RCCL transport's
    multi-rank branch (2-rank edge communicators, rings, ids ring closure), its byte movement
    replaced by the stand-in communicator (parallel/rccl_standin.py): the bench JSON must report
    the rccl transport on every rank and the edge communicators it built."""
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT, DLLM_TRANSPORT="rccl", DLLM_RCCL_STANDIN="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "1", "--model", "tiny-llama", "--batch", "3",
           "--prompt-len", "6", "--gen-len", "4", "--parallelism", "pp"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert KEYS <= set(rec) and rec["n_gpus"] == n and rec["value"] > 0
    assert rec["transport"] == "rccl-standin"      # the stand-in is named in the result
    # n - 1 stage edges + the ids ring closure, every rank on at least one 2-rank communicator
    assert rec["rccl_comms"] == n and rec["rccl_ranks"] == n and rec["rccl_comm_nranks"] == [2]
    assert all(v > 0 for v in rec["hop_tx_MBps"])


def test_single_process_bench_json_cpu():
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--model",
                        "tiny-llama", "--batch", "2", "--prompt-len", "5", "--gen-len", "3"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert KEYS <= set(rec) and rec["n_gpus"] == 1
    assert rec["ttft_p50_ms"] > 0 and rec["itl_p50_ms"] > 0 and rec["kernel_knobs"] == {}


def test_open_loop_rate_mode_cpu():
    """bench.py --rate: Poisson arrivals into the running engine; p50 request latency (ms, lower
    is better) with p99 / TTFT / ITL and the offered vs achieved request rate."""
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--model",
                        "tiny-llama", "--batch", "4", "--prompt-len", "5", "--gen-len", "4", "--rate", "40"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["higher_is_better"] is False and rec["unit"] == "ms" and rec["requests"] == 12
    assert 0 < rec["p50_latency_ms"] <= rec["p99_latency_ms"] and rec["value"] == rec["p50_latency_ms"]
    assert rec["ttft_p50_ms"] > 0 and rec["offered_rate_rps"] == 40 and rec["achieved_rate_rps"] > 0


@pytest.mark.slow
def test_torchrun_bench_hybrid_dp_pp_cpu():
    """world 4 = 2 pipelines x 2 stages: each pipeline owns its own scheduler, KV pool and
    stage-to-stage transport; the job reports the sum over pipelines."""
    n = 4
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "1", "--model", "tiny-llama", "--batch", "3",
           "--prompt-len", "6", "--gen-len", "4", "--parallelism", "pp", "--pp", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["config"]["parallelism"] == "dp2xpp2" and rec["n_gpus"] == 4
    assert rec["microbatch_slots"] == 2 and rec["config"]["global_batch"] == 2 * 3 * 2   # CPU: pp slots


def test_pp_stage_times_cpu():
    """bench/pp_stage_times.py builds every stage of the half-layer and sub-layer plans and times
    its decode step (CPU, tiny model): both plans print, with per-stage times."""
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "pp_stage_times.py"), "--model", "tiny-llama",
                        "--pp", "2", "--batch", "4", "--ctx", "40", "--iters", "1", "--device", "cpu"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "pp2 half-layer" in r.stdout and "pp2 sub-layer" in r.stdout and r.stdout.count("stage us") == 2


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 4])
def test_plain_bench_gpus_n_launches_its_own_ranks_cpu(n):
    """The literal `python bench.py --gpus N` (no torchrun, no launcher environment) starts its N
    rank processes itself and relays rank 0's single JSON line (review round 5, item 1)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                               "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup", "1",
           "--model", "tiny-llama", "--batch", "3", "--prompt-len", "6", "--gen-len", "4"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert KEYS <= set(rec) and rec["n_gpus"] == n and rec["value"] > 0
    assert rec["config"]["parallelism"] == f"pp{n}" and rec["latency_kind"].startswith("round")
    assert len(rec["stage_busy_frac"]) == n


def test_plain_bench_gpus_n_fails_loudly_when_a_rank_fails_cpu():
    """A rank that cannot start (here: an unknown model) makes the self-launched job exit non-zero
    with no JSON line, instead of hanging the others."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--model", "no-such-model", "--launch-timeout", "300"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode != 0 and not _json_lines(r.stdout)
