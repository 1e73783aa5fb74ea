"""Wire protocol (reference: tests/network/test_protocol.py -- 8 tests, all failing there because
the instance methods were called statically, D2).  Same cases, plus real-socket round trips."""
import socket
import threading
import unittest
from unittest.mock import MagicMock, patch

import pytest

from distributed_llms_amd.network.protocol import HEADER_SIZE, MessageProtocol, pack_ids, unpack_ids
from src.network.protocol import MessageProtocol as CompatProtocol


def _frame(command="TEST", payload=None, metadata=None):
    head = MessageProtocol.encode(command, payload, metadata)
    return head + (payload or b"")


class _FakeSock:
    """recv_into-capable fake socket over a byte string, with optional timeout / early close."""

    def __init__(self, data: bytes, close_after=None, timeout_at=None):
        self.data, self.pos = data, 0
        self.close_after, self.timeout_at = close_after, timeout_at

    def settimeout(self, t):
        pass

    def recv_into(self, view, n):
        if self.timeout_at is not None and self.pos >= self.timeout_at:
            raise socket.timeout()
        end = len(self.data) if self.close_after is None else min(len(self.data), self.close_after)
        k = min(n, end - self.pos, 7)   # short reads on purpose
        if k <= 0:
            return 0
        view[:k] = self.data[self.pos:self.pos + k]
        self.pos += k
        return k

    def recv(self, n, flags=0):
        # short reads even with MSG_WAITALL (what a signal or a peer close can cause): the
        # receiver must loop
        buf = bytearray(n)
        k = self.recv_into(memoryview(buf), n)
        return bytes(buf[:k])


class TestMessageProtocol(unittest.TestCase):
    @patch("socket.socket")
    def setUp(self, mock_socket):
        self.mock_socket = mock_socket.return_value
        self.protocol = MessageProtocol      # static use, exactly as the reference tests do

    def test_send_message(self):
        self.assertTrue(self.protocol.send_message(self.mock_socket, "TEST_COMMAND"))
        self.mock_socket.sendall.assert_called()

    def test_send_message_with_payload(self):
        self.assertTrue(self.protocol.send_message(self.mock_socket, "TEST_COMMAND", payload=b"test_payload"))
        self.assertEqual(self.mock_socket.sendall.call_count, 2)

    def test_receive_message_header_only(self):
        h, p = MessageProtocol.receive_message(_FakeSock(_frame("HEARTBEAT", metadata={"timestamp": 1.5})))
        self.assertEqual(h["command"], "HEARTBEAT")
        self.assertEqual(h["timestamp"], 1.5)
        self.assertIsNone(p)

    def test_receive_message_with_payload(self):
        payload = bytes(range(256)) * 40
        h, p = MessageProtocol.receive_message(_FakeSock(_frame("LOAD_SHARD", payload, {"shard_id": 3})))
        self.assertEqual(h["shard_id"], 3)
        self.assertEqual(h["payload_size"], len(payload))
        self.assertEqual(p, payload)

    def test_receive_timeout(self):
        with self.assertRaises(TimeoutError):
            MessageProtocol.receive_message(_FakeSock(_frame("X"), timeout_at=0))

    def test_receive_invalid_header(self):
        with self.assertRaises(ValueError):
            MessageProtocol.receive_message(_FakeSock(b"\x00" * HEADER_SIZE + b"junk"))

    def test_receive_bad_crc(self):
        f = bytearray(_frame("PING", metadata={"a": 1}))
        f[-2] ^= 0xFF
        with self.assertRaises(ValueError):
            MessageProtocol.receive_message(_FakeSock(bytes(f)))

    def test_receive_connection_closed(self):
        f = _frame("RESULT", b"x" * 100)
        with self.assertRaises(ConnectionError):
            MessageProtocol.receive_message(_FakeSock(f, close_after=len(f) - 10))
        self.assertEqual(MessageProtocol.receive_message(_FakeSock(b"")), ({}, None))


def test_instance_and_compat_forms_agree():
    a = MessageProtocol().encode("REGISTER", None, {"capabilities": {"x": 1}})
    b = CompatProtocol.encode("REGISTER", None, {"capabilities": {"x": 1}})
    assert a == b
    assert set(MessageProtocol.MESSAGE_TYPES) >= {"REGISTER", "LOAD_SHARD", "RUN_INFERENCE", "RESULT",
                                                  "HEARTBEAT", "SHARD_REQUEST", "TASK_ASSIGN"}


def test_socketpair_large_payload_and_concurrent_senders():
    a, b = socket.socketpair()
    big = bytes(bytearray(range(256)) * (1 << 14))   # 4 MiB
    got = []

    def reader():
        for _ in range(21):
            got.append(MessageProtocol.receive_message(b, timeout=30))

    th = threading.Thread(target=reader)
    th.start()
    senders = [threading.Thread(target=lambda i=i: [MessageProtocol.send_message(a, "HEARTBEAT", metadata={"i": i})
                                                    for _ in range(10)]) for i in range(2)]
    for s in senders:
        s.start()
    MessageProtocol.send_message(a, "LOAD_SHARD", big, {"shard_id": 0})
    for s in senders:
        s.join()
    th.join(timeout=60)
    cmds = [h["command"] for h, _ in got]
    assert cmds.count("HEARTBEAT") == 20 and cmds.count("LOAD_SHARD") == 1
    assert [p for h, p in got if h["command"] == "LOAD_SHARD"][0] == big
    a.close()
    b.close()


def test_ids_roundtrip():
    assert unpack_ids(pack_ids([1, 2, 300000])) == [1, 2, 300000]


def test_python_codec_matches_native():
    from distributed_llms_amd import _ext
    from distributed_llms_amd.network.protocol import _PyCodec
    nat, py = _ext.runtime(), _PyCodec()
    h = b'{"command":"X","k":[1,2]}'
    assert nat.encode_frame_head(7, 0, h, 123) == py.encode_frame_head(7, 0, h, 123)
    assert tuple(nat.decode_frame_prefix(py.encode_frame_head(7, 0, h, 123)[:24])) == \
        py.decode_frame_prefix(py.encode_frame_head(7, 0, h, 123)[:24])


def test_setup_zmq_socket_binds_servers_and_connects_clients():
    """Reference API (src/network/protocol.py:27-36) with D1 fixed: ROUTER binds, REQ connects."""
    import threading
    mp = MessageProtocol()
    srv = mp.setup_zmq_socket("ROUTER", "tcp://127.0.0.1:0")
    port = srv.getsockname()[1]
    got = {}

    def serve():
        conn, _ = srv.accept()
        got["msg"] = MessageProtocol.receive_message(conn, timeout=10)
        MessageProtocol.send_message(conn, "REGISTER_ACK", metadata={"worker_id": 7})
        conn.close()

    t = threading.Thread(target=serve)
    t.start()
    cli = mp.setup_zmq_socket("REQ", f"tcp://127.0.0.1:{port}")
    assert MessageProtocol.send_message(cli, "REGISTER", metadata={"capabilities": {"device": "cpu"}})
    hdr, _ = MessageProtocol.receive_message(cli, timeout=10)
    t.join(10)
    cli.close()
    srv.close()
    assert got["msg"][0]["command"] == "REGISTER" and hdr["worker_id"] == 7
    import pytest
    with pytest.raises(ValueError):
        mp.setup_zmq_socket("BOGUS", "tcp://127.0.0.1:1")
