"""Structured (JSON-lines) logging with rank / role context."""
from __future__ import annotations

import json
import logging
import os
import sys
import time


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(time.time(), 3), "lvl": record.levelname, "logger": record.name, "msg": record.getMessage(),
             "pid": os.getpid()}
        for k in ("RANK", "DLLM_ROLE"):
            if k in os.environ:
                d[k.lower()] = os.environ[k]
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def setup_logging(level: str = "INFO", json_lines: bool = None):
    json_lines = os.environ.get("DLLM_JSON_LOGS", "0") == "1" if json_lines is None else json_lines
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_lines else
                   logging.Formatter("%(asctime)s %(levelname)s %(name)s[%(process)d]: %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(getattr(logging, str(level).upper(), logging.INFO))
