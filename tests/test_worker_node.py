"""WorkerNode / ModelShard (reference: tests/worker/test_node.py -- 12 tests, 8 passed there, one hung
forever on start() (D20)).  Same cases against the real implementation."""
import io
import socket
import unittest
from unittest.mock import MagicMock, patch

import pytest
import torch

from distributed_llms_amd.config import get_model_config
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.network.protocol import MessageProtocol, pack_tensors, unpack_tensors
from src.worker.node import ModelShard, WorkerNode

CFG = get_model_config("tiny-llama")


def _shard_params(layers):
    sd = W.synth_hf_state_dict(CFG, seed=0)
    keep = {k: v for k, v in sd.items() if W.layer_of(k) in layers
            or (0 in layers and W.is_embed_key(k))
            or (CFG.num_layers - 1 in layers and W.layer_of(k) is None and not W.is_embed_key(k))}
    return keep


class TestModelShard(unittest.TestCase):
    def setUp(self):
        self.shard = ModelShard(1, _shard_params({0, 1}), CFG, device="cpu")

    def test_init(self):
        self.assertEqual(self.shard.shard_id, 1)
        self.assertEqual(self.shard.layer_range, (0, 2))

    def test_to_device(self):
        self.shard.to_device()
        for p in self.shard.parameters.values():
            self.assertEqual(p.device.type, "cpu")

    def test_compute(self):
        out = self.shard.compute({"input_ids": torch.tensor([[1, 2, 3]])})
        self.assertEqual(tuple(out["hidden_states"].shape), (1, 3, CFG.hidden_size))


class TestWorkerNode(unittest.TestCase):
    def setUp(self):
        self.worker = WorkerNode(device="cpu", port=0)

    def tearDown(self):
        self.worker.stop()

    def test_init(self):
        w = WorkerNode()
        self.assertEqual(w.host, "0.0.0.0")
        self.assertEqual(w.port, 65433)
        self.assertIsNone(w.master_address)
        self.assertEqual(w.shards, {})
        self.assertFalse(w.running)

    def test_start_nonblocking_and_stop(self):
        self.worker.start(block=False)          # the reference's start() never returned (D20)
        self.assertTrue(self.worker.running)
        self.assertIsNotNone(self.worker.server_socket)
        self.worker.stop()
        self.assertFalse(self.worker.running)

    def test_load_and_unload_shard(self):
        buf = io.BytesIO()
        torch.save(_shard_params({0, 1}), buf)            # torch.save bytes (the reference shipped these, D10)
        self.assertTrue(self.worker.load_shard(1, buf.getvalue(), config=CFG))
        self.assertIn(1, self.worker.shards)
        st = pack_tensors(_shard_params({2, 3}))         # safetensors bytes
        self.assertTrue(self.worker.load_shard(2, st, config=CFG))
        self.assertTrue(self.worker.unload_shard(1))
        self.assertNotIn(1, self.worker.shards)
        self.assertFalse(self.worker.unload_shard(1))

    def test_schedule_computation_chains_shards(self):
        self.worker.load_shard(0, _shard_params({0, 1}), config=CFG)
        self.worker.load_shard(1, _shard_params({2, 3}), config=CFG)
        ids = torch.tensor([[4, 5, 6, 7]])
        out = self.worker.schedule_computation({"input_ids": ids}, [0, 1])
        self.assertEqual(tuple(out["logits"].shape), (1, 4, CFG.vocab_size))
        full = ModelShard(9, W.synth_hf_state_dict(CFG, seed=0), CFG, device="cpu")
        torch.testing.assert_close(out["logits"], full.compute({"input_ids": ids})["logits"])

    def test_shard_unloading_during_computation(self):
        self.worker.load_shard(1, _shard_params({0, 1}), config=CFG)
        self.worker.unload_shard(1)
        with self.assertRaises(KeyError):
            self.worker.schedule_computation({"input_ids": torch.tensor([1])}, [1])


def test_peer_tcp_path():
    """The reference's one working path: client -> worker raw TCP LOAD_SHARD + RUN_INFERENCE (§3.5)."""
    w = WorkerNode(device="cpu", port=0)
    w.start(block=False)
    try:
        s = socket.create_connection(("127.0.0.1", w.port), timeout=30)
        MessageProtocol.send_message(s, "LOAD_SHARD", pack_tensors(_shard_params({0, 1, 2, 3})),
                                     {"shard_id": 0, "config": CFG.to_hf_config(), "layer_range": [0, 4]})
        h, _ = MessageProtocol.receive_message(s, timeout=60)
        assert h["command"] == "SHARD_LOADED" and h["shard_id"] == 0
        MessageProtocol.send_message(s, "RUN_INFERENCE", pack_tensors({"input_ids": torch.tensor([[1, 2, 3]])}),
                                     {"task_id": "t1", "shard_ids": [0]})
        h, p = MessageProtocol.receive_message(s, timeout=60)
        assert h["command"] == "RESULT" and h["task_id"] == "t1"
        assert tuple(unpack_tensors(p)["logits"].shape) == (1, 3, CFG.vocab_size)
        MessageProtocol.send_message(s, "STATUS", metadata={"req": "r"})
        h, _ = MessageProtocol.receive_message(s, timeout=30)
        assert h["command"] == "STATUS_REPLY" and h["status"]["shards"] == [0]
        s.close()
    finally:
        w.stop()


def test_shard_request_migrates_a_shard_between_workers():
    """SHARD_REQUEST (declared but never sent or handled by the reference, protocol.py:18): a
    replacement worker pulls a resident shard from a peer and computes the same result;
    TASK_ASSIGN runs like SCHEDULE_COMPUTATION."""
    a, b = WorkerNode(device="cpu", port=0), WorkerNode(device="cpu", port=0)
    a.start(block=False)
    b.start(block=False)
    try:
        sa = socket.create_connection(("127.0.0.1", a.port), timeout=30)
        MessageProtocol.send_message(sa, "LOAD_SHARD", pack_tensors(_shard_params({0, 1, 2, 3})),
                                     {"shard_id": 0, "config": CFG.to_hf_config(), "layer_range": [0, 4]})
        assert MessageProtocol.receive_message(sa, timeout=60)[0]["command"] == "SHARD_LOADED"
        MessageProtocol.send_message(sa, "SHARD_REQUEST", metadata={"shard_id": 0})
        h, blob = MessageProtocol.receive_message(sa, timeout=60)
        assert h["command"] == "LOAD_SHARD" and h["layer_range"] == [0, 4] and blob
        MessageProtocol.send_message(sa, "SHARD_REQUEST", metadata={"shard_id": 7})
        assert MessageProtocol.receive_message(sa, timeout=30)[0]["command"] == "ERROR"
        sb = socket.create_connection(("127.0.0.1", b.port), timeout=30)
        MessageProtocol.send_message(sb, "LOAD_SHARD", blob, {k: h[k] for k in ("shard_id", "config", "layer_range")})
        assert MessageProtocol.receive_message(sb, timeout=60)[0]["command"] == "SHARD_LOADED"
        x = pack_tensors({"input_ids": torch.tensor([[5, 6, 7]])})
        outs = []
        for s, cmd in ((sa, "SCHEDULE_COMPUTATION"), (sb, "TASK_ASSIGN")):
            MessageProtocol.send_message(s, cmd, x, {"task_id": cmd, "shard_ids": [0]})
            hh, p = MessageProtocol.receive_message(s, timeout=60)
            assert hh["command"] == "RESULT" and hh["task_id"] == cmd
            outs.append(unpack_tensors(p)["logits"])
        torch.testing.assert_close(outs[0], outs[1])
        sa.close()
        sb.close()
    finally:
        a.stop()
        b.stop()
