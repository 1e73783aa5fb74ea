"""Tracing subsystem: spans, marks, Chrome export, engine integration."""
import json

import pytest
import torch

from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.utils.tracing import Tracer, get_tracer


def test_disabled_tracer_is_noop():
    tr = Tracer(enabled=False, roctx=False)
    with tr.span("x"):
        pass
    tr.mark("m")
    assert tr.events() == []


def test_spans_marks_and_chrome_export(tmp_path):
    tr = Tracer(enabled=True, capacity=8)
    with tr.span("outer", cat="host", a=1):
        with tr.span("inner"):
            pass
    tr.mark("tick", step=3)
    tr.counter("kv", used=5)
    evs = tr.events()
    names = [e["name"] for e in evs]
    assert names == ["inner", "outer", "tick", "kv"]
    outer = evs[1]
    assert outer["ph"] == "X" and outer["dur"] >= evs[0]["dur"] and outer["args"] == {"a": 1}
    summ = tr.host_summary()
    assert summ["outer"]["count"] == 1
    p = tr.export_chrome(str(tmp_path / "t.json"), process_name="test")
    doc = json.load(open(p))
    assert any(e["name"] == "outer" for e in doc["traceEvents"])
    for _ in range(20):   # bounded ring
        tr.mark("m")
    assert len(tr.events()) == 8


def test_engine_steps_are_traced():
    tr = get_tracer()
    tr.clear()
    tr.enable(True)
    try:
        eng = LLMEngine(EngineConfig(model="tiny-llama", dtype="float32", device="cpu", max_batch=4,
                                     max_seq_len=64, use_graphs=False, num_kv_blocks=64))
        eng.generate([[1, 2, 3], [4, 5]], SamplingParams(max_new_tokens=4, ignore_eos=True))
        s = tr.host_summary()
        assert s["stage.prefill"]["count"] >= 1
        assert s["stage.decode"]["count"] >= 3
    finally:
        tr.enable(False)
        tr.clear()


@pytest.mark.gpu
def test_gpu_span_measures_device_time():
    tr = Tracer(enabled=True)
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    with tr.gpu_span("mm", cat="stage"):
        for _ in range(20):
            a = a @ a
            a = a / a.norm()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    u = tr.utilization(wall, cat="stage")
    assert 0 < u["busy_s"] <= wall * 1.05
    assert 0.0 <= u["bubble_frac"] < 1.0
