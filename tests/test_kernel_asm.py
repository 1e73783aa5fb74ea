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


@pytest.fixture(scope="module")
def attn_asm(tmp_path_factory):
    from distributed_llms_amd.csrc.build import kernel_flags
    src = ROOT / "distributed_llms_amd" / "csrc" / "kernels" / "attention.hip"
    out = tmp_path_factory.mktemp("asm") / "attn.s"
    subprocess.run([HIPCC, *kernel_flags(str(src)), "--offload-device-only", "-S", str(src), f"-I{src.parent}",
                    "-o", str(out)], check=True, capture_output=True, timeout=900)
    return out.read_text()


def _kernel_body(s, name):
    start = s.index(name + ":")
    return s[start: s.index(".Lfunc_end", start)]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_attention_softmax_stays_in_valu(attn_asm):
    """The online softmax's column max / sum cross the four 16-lane rows with v_permlane16/32_swap
    (no ds_bpermute LDS round trip on the dependency chain), its fmaxf calls are not preceded by
    NaN-quieting self-max instructions (attention.hip builds with -fno-honor-nans), and no decode or
    prefill kernel spills."""
    s = attn_asm
    names = re.findall(r"^(_ZN4dllm(?:18attn_decode_kernel|23attn_prefill_lds_kernel|20attn_prefill2_kernel)\w+):",
                       s, re.M)
    assert len(names) >= 20
    for name in names:
        body = _kernel_body(s, name)
        meta = s[s.index(".amdhsa_kernel " + name):]
        assert int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1)) == 0, name
        assert "ds_bpermute" not in body, name
        assert "v_permlane32_swap" in body and "v_permlane16_swap" in body, name
        quiet = re.findall(r"v_max_f32_e32 (v\d+), (v\d+), (v\d+)", body)
        assert not [q for q in quiet if q[1] == q[2]], (name, "NaN-quieting v_max x, x")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_decode_patch_is_a_scalar_branch(attn_asm):
    """The fused decode kernel patches the new key into ONE chunk's registers: the lane selects sit
    in blocks behind a wave-uniform branch, apart from the chunk's MFMAs, so the steady-state chunk
    carries only the softmax's few selects (the branch-free form ran ~140 per chunk)."""
    name = re.search(r"^(_ZN4dllm18attn_decode_kernelILi128ELi4ELb1ELi5E\w+):", attn_asm, re.M).group(1)
    blocks = re.split(r"\n(?=\.LBB\w+:|\s*; %bb)", _kernel_body(attn_asm, name))
    mfma_blocks = [b for b in blocks if "v_mfma" in b]
    assert mfma_blocks
    for b in mfma_blocks:
        assert b.count("v_cndmask_b32") <= 16, b.count("v_cndmask_b32")
    assert any(b.count("v_cndmask_b32") >= 32 and "v_mfma" not in b for b in blocks)   # the patch itself


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_prefill_w32_kernels_keep_softmax_in_registers(attn_asm):
    """Prefill attention on 32x32x16 MFMAs (versions 6 / 7): no spills, the column max crosses the two
    lane halves with v_permlane32_swap (no LDS shuffle), no NaN-quieting self-max, and the pipelined
    form (7) runs its softmax exponentials in the same basic block as the previous tile's P.V MFMAs
    (interleaved, not sunk behind the rescale branch), with no accumulator copies in the tile loop."""
    names = re.findall(r"^(_ZN4dllm23attn_prefill_w32_kernel\w+):", attn_asm, re.M)
    assert len(names) == 10
    for name in names:
        body = _kernel_body(attn_asm, name)
        meta = attn_asm[attn_asm.index(".amdhsa_kernel " + name):]
        assert int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1)) == 0, name
        assert "ds_bpermute" not in body and "v_permlane32_swap" in body, name
        quiet = re.findall(r"v_max_f32_e32 (v\d+), (v\d+), (v\d+)", body)
        assert not [q for q in quiet if q[1] == q[2]], name
        assert body.count("v_mfma_f32_32x32x16_bf16") >= 32, name
        if "Lb1E" in name:                          # template <G, PIPE = true>
            blocks = re.split(r"\n(?=\.LBB\w+:|\s*; %bb)", body)
            fused = [b for b in blocks if b.count("v_exp_f32") >= 32 and b.count("v_mfma_f32_32x32x16_bf16") >= 16]
            assert fused, name
            assert fused[0].count("sched_barrier") >= 15 or fused[0].count("v_exp_f32") >= 32
            loop_movs = sum(b.count("v_mov_b64") for b in blocks if "v_mfma" in b or "v_exp" in b)
            assert loop_movs < 8, (name, loop_movs)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_prefill_persistent_kernel_stages_without_flat_loads(attn_asm):
    """Version 9 (attn_prefill_w32p_kernel, v7 persistent): the same fused softmax / P.V block as v7,
    no spills, and no flat loads -- a block id picked between the block table and the LDS id list
    through one pointer compiles to flat_load_dword, whose wait (vmcnt(0) lgkmcnt(0)) drains the
    LDS-DMA issued just before it, once per staged tile piece."""
    names = re.findall(r"^(_ZN4dllm24attn_prefill_w32p_kernel\w+):", attn_asm, re.M)
    assert len(names) == 5
    for name in names:
        body = _kernel_body(attn_asm, name)
        meta = attn_asm[attn_asm.index(".amdhsa_kernel " + name):]
        assert int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1)) == 0, name
        assert "flat_load" not in body and "scratch_" not in body, name
        blocks = re.split(r"\n(?=\.LBB\w+:|\s*; %bb)", body)
        assert [b for b in blocks if b.count("v_exp_f32") >= 32 and b.count("v_mfma_f32_32x32x16_bf16") >= 16], name
        loop_movs = sum(b.count("v_mov_b64") for b in blocks if "v_mfma" in b or "v_exp" in b)
        assert loop_movs < 8, (name, loop_movs)
