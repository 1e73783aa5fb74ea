"""Re-export (reference path ``src/model/shard_manager.py``)."""
from distributed_llms_amd.checkpoint.shard_manager import ModelShardManager  # noqa: F401
