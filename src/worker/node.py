"""Re-export of :mod:`distributed_llms_amd.worker.node` (reference path ``src/worker/node.py``)."""
from distributed_llms_amd.network.protocol import MessageProtocol  # noqa: F401
from distributed_llms_amd.worker.node import ModelShard, WorkerNode  # noqa: F401
