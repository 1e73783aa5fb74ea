"""Control-plane wire protocol (master <-> worker, client <-> worker).

Keeps the reference's command vocabulary and call shapes
(``src/network/protocol.py:12-20`` MESSAGE_TYPES, ``send_message(sock, command,
payload=None, metadata=None) -> bool``, ``receive_message(sock, timeout=60) ->
(header, payload)``) but replaces its framing:

* reference: 10 ASCII bytes of header length + ``pickle(header)`` + payload, received in
  4 KiB chunks with ``payload += chunk`` (O(n^2), D18) and unpickled from the socket
  (arbitrary code execution on untrusted input);
* here: a 24-byte binary prefix (magic, version, command id, header length, payload
  length, header CRC-32 -- encoded/validated by the native codec in ``_C_runtime``), a
  JSON header, and the raw payload read by one ``MSG_WAITALL`` receive straight into the
  result (O(n), no zero-fill, no copy; short reads continue with ``recv_into``).  Nothing
  received is ever unpickled (bench/protocol_bench.py: ~20x (1 MiB) to ~150-300x (16 MiB) the reference framing's
  throughput from 1 to 16 MiB, profiles/protocol_vs_reference.md).

``send_message``/``receive_message`` are static, so both ``MessageProtocol.send_message(sock,
...)`` (how the reference's tests call it, D2) and instance calls work.
"""
from __future__ import annotations

import json
import socket
import struct
import threading
import zlib
from typing import Any, Dict, Optional, Tuple

HEADER_SIZE = 24                      # fixed frame prefix (the reference's was a 10-byte length field)
MAX_PAYLOAD = 1 << 40

# Command ids are the wire encoding; names are the API (superset of the reference's).
COMMANDS = [
    "REGISTER", "LOAD_SHARD", "RUN_INFERENCE", "RESULT", "HEARTBEAT", "SHARD_REQUEST", "TASK_ASSIGN",
    "SHARD_LOADED", "UNLOAD_SHARD", "SHARD_UNLOADED", "SCHEDULE_COMPUTATION", "ERROR",
    "REGISTER_ACK", "PLAN", "STATUS", "STATUS_REPLY", "SHUTDOWN", "TOKENS", "ABORT", "PING", "PONG",
]
_CMD_ID = {c: i for i, c in enumerate(COMMANDS)}
EXTENDED_ID = 0xFFFF                  # unknown command names travel in the header


def _codec():
    try:
        from .. import _ext
        return _ext.runtime()
    except Exception:   # pragma: no cover - pure-Python fallback only when the runtime is unbuilt
        return None


class _PyCodec:
    """Bit-identical pure-Python twin of csrc/runtime/frame_codec.cpp (used if unbuilt)."""
    _fmt = struct.Struct("<IBBHIQI")
    MAGIC = 0x4D4C4C44

    def encode_frame_head(self, cid, flags, header, plen):
        return self._fmt.pack(self.MAGIC, 1, flags, cid, len(header), plen, zlib.crc32(header)) + header

    def decode_frame_prefix(self, prefix):
        magic, ver, flags, cid, hl, pl, crc = self._fmt.unpack(prefix)
        if magic != self.MAGIC:
            raise ValueError("bad frame magic")
        if ver != 1:
            raise ValueError("unsupported frame version")
        if hl > (16 << 20) or pl > MAX_PAYLOAD:
            raise ValueError("frame length out of bounds")
        return cid, flags, hl, pl, crc

    def check_header_crc(self, header, crc):
        return zlib.crc32(header) == crc


_CODEC = None


def _get_codec():
    """The native frame codec (cached: resolving it per frame cost ~5 us), else the Python twin."""
    global _CODEC
    if _CODEC is None:
        c = _codec()
        _CODEC = c if c is not None else _PyCodec()
    return _CODEC


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    """n bytes (fewer only if the peer closed).  One MSG_WAITALL receive straight into the result
    in the common case (no zero-fill, no copy); after a short read (signal, peer close) the rest
    goes into one preallocated buffer with recv_into -- O(n) either way."""
    if n == 0:
        return b""
    b = sock.recv(n, socket.MSG_WAITALL)
    if len(b) == n or not b:
        return b
    buf = bytearray(n)
    buf[:len(b)] = b
    got = len(b) + _recv_exact_into(sock, memoryview(buf)[len(b):])
    return bytes(buf[:got])


def _recv_exact_into(sock: socket.socket, view: memoryview) -> int:
    got = 0
    n = len(view)
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            return got
        got += k
    return got


class MessageProtocol:
    """Framed messages over a stream socket.  Instances are cheap; methods are static."""

    MESSAGE_TYPES = {
        "REGISTER": "Worker registration (capabilities: device, HBM bytes, arch)",
        "LOAD_SHARD": "Load a model shard / layer range (by path, or file bytes as payload)",
        "RUN_INFERENCE": "Submit a generation request (token ids payload)",
        "RESULT": "Generated token ids for a request",
        "HEARTBEAT": "Health check",
        "SHARD_REQUEST": "Request a shard re-load (recovery / migration)",
        "TASK_ASSIGN": "Assign a computation task",
        "SHARD_LOADED": "Shard load acknowledgement",
        "UNLOAD_SHARD": "Free a shard",
        "SHARD_UNLOADED": "Shard unload acknowledgement",
        "SCHEDULE_COMPUTATION": "Run a stateless forward over loaded shards",
        "ERROR": "Error report",
        "REGISTER_ACK": "Registration accepted (worker id, config)",
        "STATUS": "Status query",
        "STATUS_REPLY": "Status response",
        "SHUTDOWN": "Stop the worker",
        "TOKENS": "Streamed tokens for a request",
        "ABORT": "Cancel a request",
    }
    _send_locks: Dict[int, threading.Lock] = {}
    _locks_guard = threading.Lock()

    def __init__(self, zmq_context=None):
        # the reference took a pyzmq context; the transport here is plain TCP
        self.zmq_context = zmq_context

    # socket "types" of the reference's setup_zmq_socket (src/network/protocol.py:27-36), mapped
    # to TCP roles.  The reference bound only PUB/PUSH/REP, so its ROUTER master connected to
    # nobody; here every server-side type binds and every client-side type connects.
    SERVER_TYPES = ("ROUTER", "REP", "PUB", "PUSH", "SERVER")
    CLIENT_TYPES = ("REQ", "DEALER", "SUB", "PULL", "CLIENT")

    def setup_zmq_socket(self, socket_type: str, address: str, timeout: Optional[float] = 10.0,
                         backlog: int = 64) -> socket.socket:
        """``address`` like ``tcp://host:port``.  Server types return a listening socket (accept
        connections yourself); client types return a connected stream socket."""
        kind = str(socket_type).upper()
        hostport = address.split("://", 1)[-1]
        host, _, port = hostport.rpartition(":")
        host = host.strip("[]") or "0.0.0.0"
        if kind in self.SERVER_TYPES:
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind(("0.0.0.0" if host == "*" else host, int(port)))
            s.listen(backlog)
            return s
        if kind in self.CLIENT_TYPES:
            s = socket.create_connection((host, int(port)), timeout=timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            return s
        raise ValueError(f"unknown socket type {socket_type!r}")

    @staticmethod
    def _lock_for(sock) -> threading.Lock:
        key = id(sock)
        lk = MessageProtocol._send_locks.get(key)
        if lk is None:
            with MessageProtocol._locks_guard:
                lk = MessageProtocol._send_locks.setdefault(key, threading.Lock())
        return lk

    @staticmethod
    def encode(command: str, payload: Optional[bytes] = None, metadata: Optional[Dict[str, Any]] = None) -> bytes:
        header = {"command": command}
        if metadata:
            header.update(metadata)
        if payload is not None:
            header["payload_size"] = len(payload)
        hb = _JSON.encode(header).encode()
        cid = _CMD_ID.get(command, EXTENDED_ID)
        return _get_codec().encode_frame_head(cid, 0, hb, 0 if payload is None else len(payload))

    @staticmethod
    def send_message(sock, command: str, payload: Optional[bytes] = None,
                     metadata: Optional[Dict[str, Any]] = None) -> bool:
        """Send one frame; thread-safe per socket (heartbeat and replies may interleave)."""
        try:
            head = MessageProtocol.encode(command, payload, metadata)
            with MessageProtocol._lock_for(sock):
                sock.sendall(head)
                if payload is not None and len(payload):
                    sock.sendall(payload)
            return True
        except socket.timeout:
            return False
        except (OSError, ValueError, TypeError):
            return False

    @staticmethod
    def receive_message(sock, timeout: Optional[float] = 60) -> Tuple[Dict[str, Any], Optional[bytes]]:
        """Receive one frame. ({}, None) on orderly close before a frame starts;
        TimeoutError on timeout; ConnectionError on close mid-frame; ValueError on a bad frame."""
        try:
            sock.settimeout(timeout)
            prefix = _recv_exact(sock, HEADER_SIZE)
            if not prefix:
                return {}, None
            if len(prefix) < HEADER_SIZE:
                raise ConnectionError("connection closed while receiving frame prefix")
            codec = _get_codec()
            cid, _flags, hl, pl, crc = codec.decode_frame_prefix(prefix)
            hbytes = _recv_exact(sock, hl)
            if len(hbytes) < hl:
                raise ConnectionError("connection closed while receiving header")
            if not codec.check_header_crc(hbytes, crc):
                raise ValueError("frame header CRC mismatch")
            header = json.loads(hbytes.decode("utf-8"))
            if not isinstance(header, dict) or "command" not in header:
                raise ValueError("frame header must be a JSON object with a command")
            if cid != EXTENDED_ID and (cid >= len(COMMANDS) or COMMANDS[cid] != header["command"]):
                raise ValueError("command id / header mismatch")
            payload = None
            if "payload_size" in header:
                if int(header["payload_size"]) != pl:
                    raise ValueError("payload_size mismatch")
                payload = _recv_exact(sock, pl)
                if len(payload) < pl:
                    raise ConnectionError("connection closed while receiving payload")
            return header, payload
        except socket.timeout:
            raise TimeoutError("timeout while receiving message")


def _json_default(o):  # numpy scalars / arrays in headers
    try:
        import numpy as np
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"not JSON serialisable: {type(o)}")


_JSON = json.JSONEncoder(separators=(",", ":"), default=_json_default)


# -------------------------------------------------------------- payload helpers
def pack_ids(ids) -> bytes:
    import numpy as np
    return np.asarray(ids, dtype=np.int32).tobytes()


def unpack_ids(b: Optional[bytes]):
    import numpy as np
    if not b:
        return []
    return np.frombuffer(b, dtype=np.int32).tolist()


def pack_tensors(tensors: Dict[str, "torch.Tensor"]) -> bytes:
    """Tensors -> safetensors bytes (no pickle on the wire)."""
    from safetensors.torch import save
    return save({k: v.detach().contiguous().cpu() for k, v in tensors.items()})


def unpack_tensors(b: bytes) -> Dict[str, "torch.Tensor"]:
    from safetensors.torch import load
    return load(b)
