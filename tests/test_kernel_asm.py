"""Static checks of the compiled gfx950 code (CPU: hipcc cross-compiles, nothing runs).

gemm_rw.hip loads its weight fragments with inline-asm buffer loads straight into VGPRs: hipcc
believes the destination written at issue, so any instruction that touches such a register before
the covering ``s_waitcnt vmcnt`` -- a compiler-inserted copy, an address computation, an MFMA --
reads bytes that have not landed (wrong results, or a fault if the value feeds an address).  The
test compiles the file to assembly and runs scripts/check_async_loads.py over every gemm_rw
instantiation: no instruction may touch a VGPR with an asm load still in flight, the waits are
counted (the K loop never drains with vmcnt(0); only the epilogue does), and the main loop holds
no register copies (v_mov / v_accvgpr_mov: the window structure keeps every value in place)."""
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def rw_asm(tmp_path_factory):
    src = ROOT / "distributed_llms_amd" / "csrc" / "kernels" / "gemm_rw.hip"
    out = tmp_path_factory.mktemp("asm") / "rw.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only", "-S",
                    str(src), f"-I{src.parent}", "-o", str(out)], check=True, capture_output=True, timeout=900)
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_rw_kernels_have_no_async_load_hazards(rw_asm):
    res = subprocess.run([sys.executable, str(ROOT / "scripts" / "check_async_loads.py"), str(rw_asm)],
                         check=True, capture_output=True, text=True).stdout
    lines = [l for l in res.splitlines() if "hazards" in l]
    assert len(lines) == 64, res                 # (3 + 3 + 2 ring depths) x 4 modes x 2 weight layouts
    for l in lines:
        assert re.search(r"hazards 0 ", l), res
        waits = [int(x) for x in re.findall(r"\d+", l.split("vmcnt", 1)[1])]
        assert waits[-1] == 0 and any(w > 0 for w in waits), l


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_rw_main_loop_has_no_register_copies(rw_asm):
    s = rw_asm.read_text()
    names = re.findall(r"^(_ZN4dllm14gemm_rw_kernel\w+):", s, re.M)
    assert names
    for name in names:
        body = s[s.index(name + ":"): s.index(".Lfunc_end", s.index(name + ":"))]
        # the K loop's basic blocks: hipcc annotates every block of a loop ("Loop Header" /
        # "in Loop: Header=...")
        loop, inside = [], False
        for l in body.split("\n"):
            if re.match(r"^\.LBB\S*:|^; %bb", l):
                inside = "Loop Header" in l or "in Loop:" in l
                continue
            if inside and l.strip() and not l.strip().startswith((";", ".")):
                loop.append(l.strip())
        copies = [l for l in loop if l.startswith(("v_mov_b", "v_accvgpr_mov", "v_accvgpr_write", "v_accvgpr_read"))]
        assert not copies, (name, copies[:4])
        assert sum(l.startswith("v_mfma_f32_32x32x16_bf16") for l in loop) >= 32


@pytest.fixture(scope="module")
def pp_asm(tmp_path_factory):
    src = ROOT / "distributed_llms_amd" / "csrc" / "kernels" / "gemm_pp.hip"
    out = tmp_path_factory.mktemp("asm") / "pp.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only", "-S",
                    str(src), f"-I{src.parent}", "-o", str(out)], check=True, capture_output=True, timeout=900)
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_pf_persistent_kernel_keeps_the_pipeline_full(pp_asm):
    """gemm_pf (persistent schedule 2): no scratch spills (a spill reload in the tile loop waits on
    vmcnt, i.e. drains the LDS-DMA pipeline the persistent form exists to keep full), and no
    vmcnt(0) anywhere before the final drain -- the tile-boundary epilogue included."""
    s = pp_asm.read_text()
    names = re.findall(r"^(_ZN4dllm14gemm_pf_kernel\w+):", s, re.M)
    assert len(names) == 2
    for name in names:
        start = s.index(name + ":")
        body = s[start: s.index(".Lfunc_end", start)]
        meta = s[s.index(".amdhsa_kernel " + name):]
        scratch = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1))
        assert scratch == 0, (name, scratch)
        assert "scratch_" not in body
        waits = re.findall(r"s_waitcnt vmcnt\((\d+)\)", body)
        assert waits.count("0") <= 1, (name, waits)
        assert body.count("v_mfma_f32_16x16x32_bf16") >= 128
