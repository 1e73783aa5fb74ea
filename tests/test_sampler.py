"""Sampling on the last stage (engine/sampler.py): greedy rows, temperature + top-k / top-p rows
mixed in one batch (CPU; the greedy path's argmax kernel is covered in test_kernels_gpu)."""
import torch

from distributed_llms_amd.engine.sampler import sample


def test_top_k_one_and_tiny_top_p_are_greedy():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(6, 50, generator=g)
    ref = logits.argmax(-1).to(torch.int32)
    assert torch.equal(sample(logits, [1.0] * 6, top_k=[1] * 6, generator=g), ref)
    assert torch.equal(sample(logits, [1.0] * 6, top_p=[1e-6] * 6, generator=g), ref)


def test_mixed_rows_stay_inside_their_top_k():
    g = torch.Generator().manual_seed(1)
    logits = torch.randn(8, 40, generator=g)
    temps = [0.0, 1.0, 1.0, 0.7, 2.0, 1.0, 0.0, 1.5]
    ks = [0, 3, 0, 5, 2, 1, 4, 40]
    top = torch.argsort(logits, dim=-1, descending=True)
    for _ in range(20):
        ids = sample(logits, temps, top_k=ks, generator=g)
        for i, (t, k) in enumerate(zip(temps, ks)):
            if t <= 0:
                assert ids[i] == logits[i].argmax()
            elif k > 0:
                assert int(ids[i]) in top[i, :k].tolist()


def test_top_k_draws_cover_the_k_set():
    """k = 3 at a high temperature: over many draws every one of the 3 best ids appears, no other."""
    g = torch.Generator().manual_seed(2)
    logits = torch.tensor([[5.0, 4.9, 4.8, 4.7, -1.0, 0.0]])
    seen = {int(sample(logits, [10.0], top_k=[3], generator=g)[0]) for _ in range(200)}
    assert seen == {0, 1, 2}
