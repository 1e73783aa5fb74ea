"""The HIP-IPC pipeline transport's slot protocol (parallel/ipc_transport.py), on CPU.

The transport sends no credits back: it relies on the driver never having more than
``inflight_window`` microbatches in flight (parallel/pipeline.py), so that a ring of
``window + 1`` slots is never overwritten before its consumer read it.  These tests check that
invariant against the real PipelineDriver (loopback transport, CPU) and, with a small
adversarial model of sender and receiver, that the ring depth the transport picks is enough
while a shallower one is not."""
import pytest

from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.parallel import ipc_transport as ipct
from distributed_llms_amd.parallel import pipeline as pl


def worst_case_overwrites(window: int, slots: int, messages: int = 64) -> int:
    """Sender runs as far ahead as the window allows (issue n once n - window was consumed);
    counts copies that land on a slot whose previous message was not consumed yet."""
    written = {}            # slot -> message currently stored
    consumed = set()
    bad = 0
    sent = 0
    for m in range(messages):                       # receiver consumes in order
        while sent < messages and (sent - window < 0 or (sent - window) in consumed):
            slot = sent % slots
            prev = written.get(slot)
            if prev is not None and prev not in consumed:
                bad += 1
            written[slot] = sent
            sent += 1
        assert written[m % slots] == m or bad
        consumed.add(m)
    return bad


@pytest.mark.parametrize("window", [1, 2, 4, 6, 18])
def test_ring_of_window_plus_one_slots_is_never_overwritten(window):
    assert worst_case_overwrites(window, window + 1) == 0


@pytest.mark.parametrize("window", [2, 4, 18])
def test_shallower_ring_would_be_overwritten(window):
    assert worst_case_overwrites(window, window - 1) > 0


@pytest.mark.parametrize("pp", [2, 4, 8])
def test_window_matches_driver_slots(pp):
    ecfg = EngineConfig(model="tiny-llama", num_workers=pp)
    assert pl.pipeline_slots(ecfg, pp, "cuda:0") == pp + 1
    assert pl.inflight_window(ecfg, pp, "cuda:0") == 2 * (pp + 1)
    assert pl.inflight_window(ecfg, pp, "cpu") == 2 * pp


@pytest.mark.parametrize("stages", [2, 3])
def test_driver_never_exceeds_the_inflight_window(stages, monkeypatch):
    """Run the real pipeline (stage threads over the loopback transport, CPU) and record the
    driver's in-flight count at every issue."""
    seen = []
    orig = pl.PipelineDriver._issue

    def spy(self, step, ids_dev=None):
        seen.append((len(self.inflight) + 1, self.num_slots))
        return orig(self, step, ids_dev)

    monkeypatch.setattr(pl.PipelineDriver, "_issue", spy)
    ecfg = EngineConfig(model="tiny-llama", dtype="float32", device="cpu", max_batch=4, max_seq_len=128,
                        num_kv_blocks=128, use_graphs=False)
    prompts = [[i + 1, 2 * i + 3, 5, 7] for i in range(12)]
    pl.run_loopback_pipeline(ecfg, stages, prompts, SamplingParams(max_new_tokens=6, ignore_eos=True),
                             device="cpu")
    assert seen and all(n <= 2 * slots for n, slots in seen)
    assert max(n for n, _ in seen) > 1                 # the pipeline did overlap microbatches


def test_transport_validates_before_touching_the_gpu():
    with pytest.raises(ValueError, match="window"):
        ipct.IpcTransport([0, 1], 0, None, "cuda:0", 8, 8, window=0)
    with pytest.raises(ValueError, match="GPU stage"):
        ipct.IpcTransport([0, 1], 0, None, "cpu", 8, 8)
