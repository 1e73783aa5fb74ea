"""Re-export of :mod:`distributed_llms_amd.master.node` (reference path ``src/master/node.py``)."""
from distributed_llms_amd.master.node import MasterNode, WorkerFailure  # noqa: F401
