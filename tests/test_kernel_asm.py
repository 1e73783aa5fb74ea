"""Static checks of the compiled gfx950 code (CPU: hipcc cross-compiles, nothing runs).

The persistent prefill GEMM (gemm_pf in gemm_pp.hip) keeps its LDS-DMA pipeline running across
output tiles, so the tile-boundary epilogue must not drain it: hipcc, left alone, copied all 256
accumulators to VGPRs at the K loop's exit, spilled, and waited vmcnt(0) on the reloads.  The
test compiles the file to assembly and checks every gemm_pf instantiation for scratch, spill
reloads and vmcnt(0) waits before the final drain."""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


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
    assert len(names) >= 2
    for name in names:
        start = s.index(name + ":")
        body = s[start: s.index(".Lfunc_end", start)]
        meta = s[s.index(".amdhsa_kernel " + name):]
        scratch = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1))
        assert scratch == 0, (name, scratch)
        assert "scratch_" not in body
        lines = body.split("\n")
        # template <MODE, SCH, DYN> mangles as ILi<MODE>ELi<SCH>ELb<DYN>E
        m = re.search(r"gemm_pf_kernelILi\d+ELi\d+ELb(\d)E", name)
        dyn = bool(m and m.group(1) == "1")
        # vmcnt(0) is allowed once (the final drain) -- and, in the dynamic-tile-queue form (template
        # flag DYN), on the queue's own blocking paths (start, steal, retire: right behind its atomic
        # or relaxed sc1 head load, lane 0 only), never in the K loop's pipeline itself
        drains = [i for i, l in enumerate(lines) if "s_waitcnt vmcnt(0)" in l
                  and not (dyn and any("global_atomic_add" in p or " sc1" in p
                                       for p in lines[max(0, i - 4): i]))]
        assert len(drains) <= 1, (name, [lines[i - 2: i + 1] for i in drains])
        if dyn:                            # the K loop's fetch is the asynchronous inline-asm one
            assert "global_atomic_add" in body and "off sc0" in body
        assert body.count("v_mfma_f32_16x16x32_bf16") >= 128
