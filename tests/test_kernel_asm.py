"""Static checks of the compiled gfx950 code (CPU: hipcc cross-compiles, nothing runs).

gemm_gu.hip's register-A kernels load activations with inline-asm global loads whose destination
registers hipcc believes written at issue; a first build let the allocator reuse such registers as
address registers before the data landed (a GPU memory fault).  This test compiles the file to
assembly and runs scripts/check_async_loads.py over every gemm_gua_kernel instantiation: no
non-MFMA instruction may touch a VGPR with an asm load still in flight, and the K loop keeps its
counted waits (no compiler-inserted vmcnt(0) before the tail)."""
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_gua_kernels_have_no_async_load_hazards(tmp_path):
    src = ROOT / "distributed_llms_amd" / "csrc" / "kernels" / "gemm_gu.hip"
    out = tmp_path / "gu.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only", "-S",
                    str(src), f"-I{src.parent}", "-o", str(out)], check=True, capture_output=True, timeout=600)
    res = subprocess.run([sys.executable, str(ROOT / "scripts" / "check_async_loads.py"), str(out)],
                         check=True, capture_output=True, text=True).stdout
    lines = [l for l in res.splitlines() if "hazards" in l]
    assert len(lines) >= 7, res                      # 3 plain + 3 slab + 1 SwiGLU instantiations
    for l in lines:
        assert re.search(r"hazards 0 ", l), l
        waits = [int(x) for x in re.findall(r"\d+", l.split("vmcnt", 1)[1])]
        assert waits[0] > 0 and 0 not in waits[:-1], l   # counted waits; vmcnt(0) only at the end
