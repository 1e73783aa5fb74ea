"""rocprofv3 counter smoke tests (north star: "tiling validated with rocprof
counters on gfx950").  Each runs bench/kernel_counters.py for one kernel under one --pmc pass
(kernel trace only -- never combined with sys/runtime tracing) and checks a tiling property:

* wide decode GEMM (split-K down projection): the XOR-swizzled LDS image has no bank conflicts,
  and MFMAs issue;
* paged decode attention: HBM reads equal the K/V bytes of the batch (no over-fetch).
"""
import csv
import glob
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCPROF = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"


def _collect(tmp_path, counters, only):
    if not os.path.exists(ROCPROF):
        pytest.skip("rocprofv3 not available")
    out = tmp_path / "prof"
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = [ROCPROF, "--pmc", *counters, "--kernel-trace", "-d", str(out), "-o", "run", "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "bench", "kernel_counters.py"), "--only", only, "--reps", "2"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    files = glob.glob(str(out / "**" / "*counter_collection.csv"), recursive=True)
    assert files, "no counter output"
    per = {}
    for row in csv.DictReader(open(files[0])):
        per.setdefault(row["Kernel_Name"], {}).setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
        per[row["Kernel_Name"]][row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    return per


def _kernel(per, needle):
    hits = {k: v for k, v in per.items() if needle in k}
    assert hits, f"{needle} not profiled; saw {list(per)[:8]}"
    return next(iter(hits.values()))


def test_wide_gemm_lds_conflict_free_and_mfma_busy(tmp_path):
    per = _collect(tmp_path, ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"], "gemm")
    for d in _kernel(per, "gemm_wide_kernel").values():
        assert d["SQ_LDS_IDX_ACTIVE"] > 0
        assert d["SQ_LDS_BANK_CONFLICT"] <= 0.01 * d["SQ_LDS_IDX_ACTIVE"]
        assert d["SQ_VALU_MFMA_BUSY_CYCLES"] > 0


def test_decode_attention_reads_each_kv_byte_once(tmp_path):
    per = _collect(tmp_path, ["FETCH_SIZE"], "attn")
    kv_bytes = 256 * 192 * 8 * 128 * 2 * 2          # bench/kernel_counters.py attention shape
    for d in _kernel(per, "attn_decode_kernel").values():
        read = 2 * d["FETCH_SIZE"] * 1024             # gfx950 FETCH_SIZE = half of wide streaming reads
        assert 0.9 * kv_bytes <= read <= 1.15 * kv_bytes, (read, kv_bytes)
