"""Re-export (reference path ``src/model/downloader.py``)."""
from distributed_llms_amd.checkpoint.loader import download_model  # noqa: F401
