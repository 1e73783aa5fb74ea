"""Master + workers over localhost sockets on CPU (BASELINE config 1 plumbing), with real
``run_worker.py`` processes: registration, contiguous stage plan, torch.distributed (gloo)
pipeline, request routing, heartbeat eviction and recovery."""
import os
import subprocess
import sys
import threading
import time

import pytest

from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.master.node import MasterNode, WorkerFailure

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [[3, 5, 7, 9, 11], [20, 21, 22], [100, 4, 4, 4, 4, 4, 4, 4, 9]]

pytestmark = pytest.mark.slow


def _cfg(model):
    return EngineConfig(model=model, dtype="float32", device="cpu", max_batch=8, max_seq_len=128,
                        use_graphs=False, num_kv_blocks=128, heartbeat_interval=0.5, heartbeat_timeout=4.0)


def _spawn_worker(port, extra=()):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    return subprocess.Popen([sys.executable, os.path.join(ROOT, "run_worker.py"), "--master", f"127.0.0.1:{port}",
                             "--device", "cpu", "--port", "0", "--heartbeat", "0.5", "--log-level", "WARNING",
                             *extra], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


@pytest.fixture
def cluster():
    procs = []
    masters = []

    def make(model, n, auto_recover=False, extra=None):
        m = MasterNode("127.0.0.1", 0, _cfg(model), auto_recover=auto_recover).start()
        masters.append(m)
        m.initialize_model(model, num_shards=n)
        for i in range(n):
            procs.append(_spawn_worker(m.port, (extra or {}).get(i, ())))
        m.wait_for_workers(n, timeout=120)
        return m

    yield make, procs
    for m in masters:
        m.stop()
    for p in procs:
        try:
            p.wait(timeout=15)
        except subprocess.TimeoutExpired:
            p.kill()


@pytest.mark.parametrize("model", ["synthetic:tiny-gpt2", "synthetic:tiny-llama"])
def test_two_worker_pipeline_matches_single_process(cluster, model):
    make, _ = cluster
    m = make(model, 2)
    assert m.assign_shards() == {"w0": [0], "w1": [1]}
    acks = m.distribute_shards(timeout=300)
    assert [acks[w]["layer_range"] for w in ("w0", "w1")] == [[0, 2], [2, 4]]
    res = m.generate(PROMPTS, max_new_tokens=6, ignore_eos=True, timeout=120)
    ref = LLMEngine(_cfg(model)).generate(PROMPTS, SamplingParams(max_new_tokens=6, ignore_eos=True))
    assert [r["tokens"] for r in res] == ref
    text = m.run_inference("hello", max_new_tokens=4, timeout=60, ignore_eos=True)
    assert len(text["tokens"]) == 4 and isinstance(text["text"], str)
    # token streaming (TOKENS messages from the stage-0 driver): several chunks, same tokens
    chunks = list(m.stream(PROMPTS[2], max_new_tokens=6, ignore_eos=True, timeout=120))
    assert sum(chunks, []) == ref[2] and len(chunks) >= 2
    st = m.status()
    assert st["state"] == "ready" and st["metrics"]["requests"] == 5
    assert {w["remote"]["role"] for w in st["workers"].values()} == {"driver", "follower"}


def test_single_worker_engine(cluster):
    make, _ = cluster
    m = make("synthetic:tiny-llama", 1)
    m.assign_shards()
    m.distribute_shards(timeout=300)
    res = m.generate(PROMPTS, max_new_tokens=5, ignore_eos=True, timeout=120)
    ref = LLMEngine(_cfg("synthetic:tiny-llama")).generate(PROMPTS, SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert [r["tokens"] for r in res] == ref
    chunks = list(m.stream(PROMPTS[1], max_new_tokens=5, ignore_eos=True, timeout=120))
    assert sum(chunks, []) == ref[1] and len(chunks) >= 2


def test_worker_failure_eviction_and_recovery(cluster):
    """A stage worker dies mid-generation (fault injection): the master evicts it, keeps the
    in-flight requests parked, re-admits a replacement, and re-runs them from their prompts --
    they complete with the tokens a fault-free run gives (plan.md:430-436 retry + recovery)."""
    make, procs = cluster
    # stage-0 worker dies after 3 engine steps (fault injection)
    m = make("synthetic:tiny-llama", 2, auto_recover=True, extra={0: ("--fail-after", "3")})
    m.assign_shards()
    m.distribute_shards(timeout=300)
    futs = [m.submit(p, {"max_new_tokens": 40, "ignore_eos": True}) for p in PROMPTS]
    streamed = {}

    def consume(key, prompt):      # stream() submits on its first iteration, in this thread
        streamed[key] = list(m.stream(prompt, max_new_tokens=40, ignore_eos=True, timeout=240))
    import threading
    th_inflight = threading.Thread(target=consume, args=("inflight", PROMPTS[0]))
    th_inflight.start()            # in flight when the stage dies: parked, re-run, resumed
    t0 = time.time()
    while m.state != "degraded" and time.time() - t0 < 30:
        time.sleep(0.2)
    assert m.state == "degraded"
    assert m.running                                    # the master survives
    assert not any(f.done() for f in futs)              # parked, not failed
    late = m.submit(PROMPTS[1], {"max_new_tokens": 40, "ignore_eos": True})   # held while degraded
    th_late = threading.Thread(target=consume, args=("late", PROMPTS[2]))
    th_late.start()
    time.sleep(0.5)
    assert not late.done() and m.state == "degraded"
    procs.append(_spawn_worker(m.port))                 # a replacement worker joins
    res = [m._finish(f, 180) for f in futs]
    assert m.state == "ready"
    ref = LLMEngine(_cfg("synthetic:tiny-llama")).generate(PROMPTS, SamplingParams(max_new_tokens=40, ignore_eos=True))
    assert [r["tokens"] for r in res] == ref
    assert m._finish(late, 180)["tokens"] == ref[1]     # the held request ran after recovery
    th_inflight.join(240)
    th_late.join(240)
    assert sum(streamed["inflight"], []) == ref[0]      # greedy stream resumed exactly
    assert sum(streamed["late"], []) == ref[2]          # a held stream too
    res = m.generate(PROMPTS[:2], max_new_tokens=4, ignore_eos=True, timeout=120)
    assert [r["tokens"] for r in res] == [r[:4] for r in ref[:2]]


def test_checkpoint_shards_distributed_by_path(cluster, tmp_path):
    from distributed_llms_amd.checkpoint.shard_manager import write_synthetic_checkpoint
    d = write_synthetic_checkpoint("tiny-gpt2", str(tmp_path / "ckpt"), seed=7)
    make, _ = cluster
    m = make(d, 2)
    m.assign_shards()
    m.distribute_shards(timeout=300)
    res = m.generate(PROMPTS, max_new_tokens=5, ignore_eos=True, timeout=120)
    from distributed_llms_amd.checkpoint.shard_manager import iter_checkpoint
    from distributed_llms_amd.models.stage import ModelStage
    from distributed_llms_amd.config import get_model_config
    cfg = get_model_config(d)
    st = ModelStage(cfg, 0, cfg.num_layers, "cpu", __import__("torch").float32).load_hf_state(dict(iter_checkpoint(d)))
    ref = LLMEngine(_cfg(d), st).generate(PROMPTS, SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert [r["tokens"] for r in res] == ref


def test_http_api_generate_completions_status_metrics(cluster):
    """HTTP front end (run_master.py --http): /generate and /v1/completions route through the same
    request futures as the Python API (identical greedy tokens), /status /metrics /health report."""
    import json
    import urllib.request

    from distributed_llms_amd.master.http_api import serve_http

    make, _ = cluster
    m = make("synthetic:tiny-llama", 2)
    m.assign_shards()
    m.distribute_shards(timeout=300)
    srv, _ = serve_http(m, "127.0.0.1", 0)
    base = f"http://127.0.0.1:{srv.server_address[1]}"

    def post(path, body):
        req = urllib.request.Request(base + path, data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            return json.loads(r.read())

    try:
        expect = m.generate([PROMPTS[0]], max_new_tokens=5, ignore_eos=True, timeout=120)[0]["tokens"]
        g = post("/generate", {"prompt_ids": PROMPTS[0], "max_new_tokens": 5, "ignore_eos": True})
        assert g["tokens"] == expect and isinstance(g["text"], str)
        c = post("/v1/completions", {"prompt": [PROMPTS[0], PROMPTS[1]], "max_tokens": 5, "ignore_eos": True})
        assert c["object"] == "text_completion" and len(c["choices"]) == 2
        assert c["choices"][0]["tokens"] == expect and c["usage"]["completion_tokens"] == 10
        t = post("/v1/completions", {"prompt": "hello world", "max_tokens": 3, "ignore_eos": True})
        assert len(t["choices"][0]["tokens"]) == 3
        with urllib.request.urlopen(base + "/health", timeout=30) as r:
            assert json.loads(r.read())["state"] == "ready"
        with urllib.request.urlopen(base + "/metrics", timeout=30) as r:
            text = r.read().decode()
        assert "dllm_requests" in text and "dllm_workers 2" in text and "dllm_pending_requests 0" in text
        assert 'dllm_worker_kv_free_blocks{worker="' in text and 'stage="0"' in text and 'stage="1"' in text
        assert "dllm_worker_steps{" in text
        with urllib.request.urlopen(base + "/status", timeout=60) as r:
            assert json.loads(r.read())["state"] == "ready"
        # server-sent events: chunks concatenate to the same greedy tokens
        req = urllib.request.Request(base + "/v1/completions",
                                     data=json.dumps({"prompt": PROMPTS[0], "max_tokens": 5, "ignore_eos": True,
                                                      "stream": True}).encode())
        with urllib.request.urlopen(req, timeout=120) as r:
            assert r.headers["Content-Type"] == "text/event-stream"
            events = [ln[len(b"data: "):] for ln in r.read().split(b"\n\n") if ln.startswith(b"data: ")]
        assert events[-1] == b"[DONE]" and len(events) >= 2
        streamed = [t for e in events[:-1] for t in json.loads(e)["choices"][0]["tokens"]]
        assert streamed == expect
        bad = urllib.request.Request(base + "/generate", data=b'{"prompt_ids": []}')
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(bad, timeout=30)
        assert ei.value.code == 400
    finally:
        srv.shutdown()


def test_recovery_timeout_fails_parked_and_later_requests():
    """Recovery that never gets its replacement workers gives up: requests parked while it ran fail
    with WorkerFailure, the state becomes "failed", and later submits raise instead of parking into
    a list nobody drains (advisor round 4: park only while a recovery thread runs)."""
    from distributed_llms_amd.master.node import MasterNode, WorkerFailure
    m = MasterNode("127.0.0.1", 0, auto_recover=True).start()
    try:
        m.num_shards = 2
        m.stage_workers = ["w0", "w1"]
        with m._lock:                      # what _evict does when a stage worker dies
            m.state = "degraded"
            m._recovering = True
        th = threading.Thread(target=m._recover_when_possible, kwargs={"timeout": 1.0}, daemon=True)
        th.start()
        parked = m.submit([1, 2, 3], {"max_new_tokens": 2})
        assert not parked.done() and len(m._retry) == 1
        th.join(10)
        assert not th.is_alive()
        assert m.state == "failed" and not m._recovering and m._retry == []
        with pytest.raises(WorkerFailure):
            parked.result(timeout=5)
        with pytest.raises(WorkerFailure):
            m.submit([4, 5], {"max_new_tokens": 2})
    finally:
        m.stop(shutdown_workers=False)


def test_eviction_during_resubmit_leaves_the_newer_recovery_in_charge():
    """Advisor round 5: a stage worker evicted while a recovery thread re-submits the parked requests
    starts a second recovery.  The first thread, finishing, must neither clear ``_recovering`` nor
    declare the pipeline failed (which would fail the newly parked requests): the newer thread
    recovers and re-submits them."""
    import concurrent.futures as cf
    from distributed_llms_amd.master.node import MasterNode
    m = MasterNode("127.0.0.1", 0, auto_recover=True).start()
    try:
        m.num_shards = 1
        m.workers["w9"] = {"socket": None, "last_heartbeat": time.time()}   # a registered spare
        sent = []
        m.assign_shards = lambda: None
        m._send_request = lambda ids, params, fut, stream, hint, attempts: (sent.append(ids), fut.set_result(ids))
        calls = {"n": 0}

        def distribute_shards(*a, **k):
            calls["n"] += 1
            m.state = "ready"

        m.distribute_shards = distribute_shards
        orig_resubmit = m._resubmit_parked
        late = cf.Future()

        def resubmit_with_eviction():
            orig_resubmit()
            if calls["n"] == 1:            # what _evict does when a re-admitted stage worker dies now
                with m._lock:
                    m.state = "degraded"
                    m._recovering = True
                    m._recovery_gen += 1
                    m._retry.append({"ids": [7, 8], "params": {}, "attempts": 0, "hint": None,
                                     "future": late, "stream": None})

        m._resubmit_parked = resubmit_with_eviction
        first = cf.Future()
        with m._lock:
            m.state = "degraded"
            m._recovering = True
            m._recovery_gen += 1
            m._retry.append({"ids": [1, 2], "params": {}, "attempts": 0, "hint": None, "future": first,
                             "stream": None})
        th1 = threading.Thread(target=m._recover_when_possible, kwargs={"timeout": 5.0, "gen": m._recovery_gen},
                               daemon=True)
        th1.start()
        th1.join(10)
        assert not th1.is_alive() and first.result(timeout=1) == [1, 2]
        # the older thread left the newer recovery's state alone
        assert m.state == "degraded" and m._recovering and not late.done()
        th2 = threading.Thread(target=m._recover_when_possible, kwargs={"timeout": 5.0, "gen": m._recovery_gen},
                               daemon=True)
        th2.start()
        th2.join(10)
        assert m.state == "ready" and not m._recovering
        assert late.result(timeout=1) == [7, 8] and sent == [[1, 2], [7, 8]]
    finally:
        m.workers.pop("w9", None)
        m.stop(shutdown_workers=False)


def test_degraded_without_recovery_thread_does_not_park():
    from distributed_llms_amd.master.node import MasterNode, WorkerFailure
    m = MasterNode("127.0.0.1", 0, auto_recover=True).start()
    try:
        m.state = "degraded"               # no recovery thread running (e.g. it already returned)
        with pytest.raises(WorkerFailure):
            m.submit([1, 2], {"max_new_tokens": 1})
        assert m._retry == []
    finally:
        m.stop(shutdown_workers=False)


def test_hot_spare_takes_over_without_a_new_registration(cluster):
    """Shard redundancy (plan.md:434): a spare worker registered beside the stages stays
    unassigned; when a stage worker dies, recovery re-plans onto the spare at once -- no replacement
    has to join -- and the parked requests complete with the fault-free tokens."""
    make, procs = cluster
    m = make("synthetic:tiny-llama", 2, auto_recover=True, extra={1: ("--fail-after", "3")})
    procs.append(_spawn_worker(m.port))                 # the hot spare
    m.wait_for_workers(3, timeout=120)
    m.assign_shards()
    m.distribute_shards(timeout=300)
    st = m.status()
    assert len(st["spare_workers"]) == 1 and st["spare_workers"][0] not in m.stage_workers
    spare = st["spare_workers"][0]
    futs = [m.submit(p, {"max_new_tokens": 30, "ignore_eos": True}) for p in PROMPTS]
    res = [m._finish(f, 240) for f in futs]            # no worker is started after the failure
    assert m.state == "ready" and m.recoveries == 1 and spare in m.stage_workers
    ref = LLMEngine(_cfg("synthetic:tiny-llama")).generate(PROMPTS, SamplingParams(max_new_tokens=30, ignore_eos=True))
    assert [r["tokens"] for r in res] == ref
