"""Re-export (reference path ``src/model/loader.py``)."""
from distributed_llms_amd.checkpoint.loader import load_model, load_tokenizer  # noqa: F401
