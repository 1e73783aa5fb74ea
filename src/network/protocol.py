"""Re-export of :mod:`distributed_llms_amd.network.protocol` (reference path ``src/network/protocol.py``)."""
from distributed_llms_amd.network.protocol import HEADER_SIZE, MessageProtocol  # noqa: F401
