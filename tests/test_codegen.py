"""Codegen guards for the hot kernels (CPU: hipcc cross-compiles gfx950 to assembly here).

The attention inner loop is issue-bound: its tile body must stay 64 v_exp_f32 +
32 v_cvt_pk_bf16_f32 + a handful of address ops, with no register shuffles.  An unrelated edit once
made the compiler re-allocate the loop with ~30 extra v_mov per tile (attention +27 % in time), so the
tile bodies and the spill counts of the layer kernels are checked on every CPU test run."""

import collections
import re
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parent.parent / "multimodalpfn_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1"]

pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")


def _asm(src: str, extra=()):
    out = subprocess.run([HIPCC, *FLAGS, *extra, "-x", "hip", "-S", "--cuda-device-only", str(CSRC / src), "-o", "-"],
                         capture_output=True, text=True, check=True, timeout=600)
    return out.stdout


def _resources(src: str, extra=()):
    out = subprocess.run([HIPCC, *FLAGS, *extra, "-x", "hip", "-c", str(CSRC / src), "-o", "/dev/null",
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, check=True,
                         timeout=600)
    res, name = {}, None
    for ln in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            name = m.group(1)
        m = re.search(r"VGPRs Spill: (\d+)", ln)
        if m and name:
            res[name] = int(m.group(1))
    return res


def _function(asm: str, needle: str) -> str:
    start = re.search(rf"^\S*{needle}\S*:", asm, re.M)
    assert start, needle
    end = asm.find(".Lfunc_end", start.end())
    return asm[start.end():end]


def _blocks(body: str) -> list[collections.Counter]:
    """Instruction counts per basic block (label to label)."""
    out = []
    for ln in body.splitlines():
        if re.match(r"^\.LBB\S+:", ln):
            out.append(collections.Counter())
        elif out:
            m = re.match(r"^\s+([a-z_0-9]+)", ln)
            if m:
                out[-1][m.group(1)] += 1
    return out


@pytest.mark.parametrize("qk,smfma", [("Lb0ELb0E", "v_mfma_f32_32x32x16_bf16"), ("Lb0ELb1E", "v_mfma_f32_32x32x16_bf16"),
                                      ("Lb1ELb1E", "v_mfma_f32_32x32x16_f16")])
def test_attention_tile_bodies_have_no_register_shuffles(qk, smfma):
    """The pipelined loop (attention_pipe.hip) is one basic block of four tiles: per tile 64 v_exp_f32,
    32 v_cvt_pk_bf16_f32, 16 + 8 MFMAs and a handful of address / loop ops, no register shuffles (bf16 Q / K with
    bf16 or fp16 O -- the bf16 and the fp16 mode's forward --, and the fp16 Q / K of the kernel-level tap, whose
    8 score MFMAs per tile are the f16 form)."""
    body = _function(_asm("attention_pipe.hip", ["-fno-honor-nans"]), f"attn_pipe_kernelILi0E{qk}")
    pvm = "v_mfma_f32_32x32x16_bf16"
    loops = [c for c in _blocks(body) if c["v_exp_f32_e32"] >= 256 and c["v_exp_f32_e32"] % 64 == 0
             and (c[smfma] + c[pvm] * (smfma != pvm)) * 4 == c["v_exp_f32_e32"] and c["v_cndmask_b32_e64"] == 0]
    assert len(loops) == 1, [(c["v_exp_f32_e32"], c[smfma], c[pvm]) for c in _blocks(body)]
    c = loops[0]
    tiles = c["v_exp_f32_e32"] // 64
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    movs = c["v_mov_b32_e32"] + c["v_mov_b64_e32"]
    assert c[smfma] + c[pvm] * (smfma != pvm) == 16 * tiles and c[pvm] >= 8 * tiles
    assert c["v_mfma_f32_16x16x32_bf16"] == 8 * tiles and c["v_cvt_pk_bf16_f32"] == 32 * tiles
    assert movs <= tiles and valu <= 100 * tiles, (valu, movs)


@pytest.mark.parametrize("variant,cvt", [(1, "v_cvt_scalef32_pk_fp8_f32"), (2, "v_cvt_scalef32_pk_bf8_f32")])
def test_fp8_attention_tile_bodies(variant, cvt):
    """The fp8 P.V variants (config E): per tile 64 exps, 8 score MFMAs (bf16), one 32x32x64 P.V and one
    16x16x128 row-sum MFMA per chain (block-scaled f8f6f4), 32 scaled conversions, no register shuffles
    (a defined `old` word of the packed conversions once cost 16 v_mov per tile)."""
    body = _function(_asm("attention_pipe.hip", ["-fno-honor-nans"]), f"attn_pipe_kernelILi{variant}ELb0ELb1E")
    loops = [c for c in _blocks(body) if c["v_exp_f32_e32"] >= 256 and c["v_exp_f32_e32"] % 64 == 0
             and c["v_mfma_f32_32x32x16_bf16"] * 8 == c["v_exp_f32_e32"]]
    assert len(loops) == 1, [(c["v_exp_f32_e32"], c["v_mfma_f32_32x32x16_bf16"]) for c in _blocks(body)]
    c = loops[0]
    tiles = c["v_exp_f32_e32"] // 64
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    movs = c["v_mov_b32_e32"] + c["v_mov_b64_e32"]
    assert c["v_mfma_scale_f32_32x32x64_f8f6f4"] == 2 * tiles and c["v_mfma_scale_f32_16x16x128_f8f6f4"] == 2 * tiles
    assert c[cvt] == 32 * tiles and c["v_cvt_pk_bf16_f32"] == 0
    assert movs <= tiles and valu <= 100 * tiles, (valu, movs)


@pytest.mark.parametrize("src,needle,limit", [
    ("attention_pipe.hip", "attn_pipe_kernel", 0),
    ("mlp_rows.hip", "mlp_rows_kernelILi2ELb1ELi4ELb0ELb0E", 0),
    ("mlp_rows.hip", "mlp_rows_kernelILi2ELb1ELi4ELb1ELb0E", 0),
    ("mlp_rows.hip", "mlp_rows_kernelILi2ELb0E", 0),
    ("mlp_rows.hip", "mlp_rows_kernelILi2ELb1ELi4ELb0ELb1E", 96),  # CAP tail: one-time prologue spills
    ("rowgemm.hip", "rowgemm_qkv2_kernel", 0),
    ("featrow.hip", "feat_rows_kernelILi3ELb0E", 16),  # one-time spills (finished heads' O^T fragments)
    ("featrow.hip", "feat_rows_kernelILi3ELb1E", 32),  # PREC_F16: X^T fragments live to the residual (46 before the saddr DMA)
])
def test_layer_kernels_spills(src, needle, limit):
    extra = ["-fno-honor-nans"] if src in ("attention.hip", "attention_pipe.hip", "featrow.hip") else []
    res = _resources(src, extra)
    hits = {k: v for k, v in res.items() if needle in k}
    assert hits, (needle, list(res))
    assert max(hits.values()) <= limit, hits


@pytest.mark.parametrize("variant,mm", [("Lb0E", "v_mfma_f32_16x16x32_bf16"), ("Lb1E", "v_mfma_f32_16x16x32_f16")])
def test_mlp_gelu_rides_in_the_up_projection(variant, mm):
    """The previous chunk's GELU once sank past the `if (MORE) hmma` branch into the down-projection's
    block, whose MFMAs consume it.  Now each chunk is one block (up-projection of the next
    chunk + this chunk's GELU + down-projection, 48 MFMAs, 16 exps); only the pre-loop up-projection of
    chunk 0 (24 MFMAs) has no GELU to carry."""
    body = _function(_asm("mlp_rows.hip"), f"mlp_rows_kernelILi2ELb1ELi4E{variant}Lb0E")
    exps = lambda c: sum(v for k, v in c.items() if k.startswith("v_exp_f"))  # noqa: E731 (fp16 mode: v_exp_f16)
    blocks = [c for c in _blocks(body) if c[mm] >= 24]
    bare = [c for c in blocks if exps(c) == 0 and c[mm] < 72]
    # a block is one chunk (48 MFMAs, 16 exps) or several back to back (the three-chunk unroll as one block
    # once the chunk's ring refills are unconditional)
    chunks = sum(c[mm] // 48 for c in blocks if c[mm] % 48 == 0 and exps(c) == c[mm] // 3)
    assert len(bare) <= 1 and chunks >= 3, ([(c[mm], exps(c)) for c in blocks])


def test_mlp_eight_wave_option_does_not_spill():
    res = _resources("mlp_rows.hip", ["-DMLP_NW=8"])
    hits = {k: v for k, v in res.items() if "mlp_rows_kernelILi2ELb1ELi8E" in k}
    assert hits and max(hits.values()) == 0, hits


ABLATIONS = re.compile(r"\b(A2_NO[A-Z]+|MLP_NO[A-Z0-9]+|RG_NO[A-Z]+|GT_NO[A-Z]+|A2_S?PRIO)\b")


def test_product_sources_carry_no_ablation_switches():
    """Timing ablations (switches that drop exps, stores, fills or barriers and give wrong results) are
    not part of the product sources; A/B experiments live in local variant builds only."""
    for src in sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp")) + sorted(CSRC.glob("*.h")):
        hits = ABLATIONS.findall(src.read_text())
        assert not hits, (src.name, sorted(set(hits)))


def test_shipped_library_is_the_production_build():
    """Variant builds export ``mmpfn_variant_flags`` (tools/build_variant*.sh, make dbg) and the loader
    refuses them without MMPFN_DIAGNOSTICS=1; the in-tree library must not carry the marker."""
    lib = CSRC.parent / "libmmpfn_hip.so"
    if not lib.exists():
        pytest.skip("library not built")
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    syms = subprocess.run([nm, "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    assert "mmpfn_variant_flags" not in syms
    assert "mmpfn_forward" in syms


@pytest.mark.parametrize("src,extra", [("attention.hip", ["-fno-honor-nans"]), ("attention_pipe.hip", ["-fno-honor-nans"]),
                                       ("gemm.hip", []), ("mlp_rows.hip", []),
                                       ("rowgemm.hip", []), ("rowgemm3.hip", []), ("mlp.hip", [])])
def test_hot_kernels_use_no_scratch(src, extra):
    """No private (scratch) segment in the hot kernels: an out-of-line lambda once sent the parity-mode
    attention's tile state through scratch (16.8 ms instead of 0.72 ms per launch) with zero reported spills."""
    asm = _asm(src, extra)
    sizes = re.findall(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.private_segment_fixed_size: (\d+)", asm)
    assert sizes
    # the CAP tail (mixer, once per predict) spills row addresses once in its prologue (tests the limit above)
    bad = [(n, int(v)) for n, v in sizes if int(v) and "mlp_rows_kernelILi2ELb1ELi4ELb0ELb1E" not in n]
    assert not bad, bad


@pytest.mark.parametrize("src,extra", [("attention_pipe.hip", ["-fno-honor-nans"]), ("mlp_rows.hip", []),
                                       ("gemm.hip", []), ("modality.hip", []), ("featrow.hip", ["-fno-honor-nans"])])
def test_lds_dma_asm_owns_m0(src, extra):
    """The LDS-DMA issues write m0 in inline asm.  clang keeps m0 reserved, so the asm's "m0" clobber
    cannot stop the compiler from assuming a value of its own survives the asm; this checks that no such value
    exists: every m0 reference in the compiled kernels is one of the asm's own writes, each followed by its DMA."""
    lines = [ln.strip() for ln in _asm(src, extra).splitlines()]
    ours = 0
    for i, ln in enumerate(lines):
        if not re.search(r"\bm0\b", ln) or ln.startswith((";", ".", "//")):
            continue
        assert re.match(r"s_mov_b32 m0, s\d+$", ln), ln
        nxt = [x for x in lines[i + 1:i + 4] if x and not x.startswith(";")]
        assert nxt[0] == "s_nop 0" and nxt[1].startswith("global_load_lds_dwordx4"), (ln, nxt)
        ours += 1
    assert ours > 0


def test_mlp_f16_gelu_asm_spacing():
    """The fp16 MLP's GELU runs as two-pair asm blocks (common.h gelu_tanh_h2x2_f32): the high halves of the
    v_exp_f16 / v_rcp_f16 results are written in place by SDWA (no v_pack_b32_f16 left in the kernel), and the
    compiler cannot see inside the asm, so the block itself must keep gfx950's one wait state between a
    transcendental (or v_pk_fma_f16) and the next instruction that reads its result (a preserving SDWA write reads
    its destination), and must not end on a transcendental."""
    asm = _asm("mlp_rows.hip")
    checked = 0
    for variant in ("Lb1E", "Lb0E"):
        body = _function(asm, f"mlp_rows_kernelILi2E{variant}Li4ELb1ELb0E")
        assert "v_pack_b32_f16" not in body
        for blk in re.findall(r";;#ASMSTART\n(.*?);;#ASMEND", body, re.S):
            ins = [ln.strip() for ln in blk.splitlines() if ln.strip().startswith("v_")]
            if not any(i.startswith("v_exp_f16") for i in ins):
                continue
            checked += 1
            regs = [re.findall(r"\bv\d+\b", i) for i in ins]
            for k in range(1, len(ins)):
                prev = ins[k - 1]
                if not re.match(r"v_(exp|rcp)_f16|v_pk_fma_f16", prev):
                    continue
                written = regs[k - 1][0]
                reads = regs[k][1:] + (regs[k][:1] if "UNUSED_PRESERVE" in ins[k] else [])
                assert written not in reads, (prev, ins[k])
            assert not re.match(r"v_(exp|rcp)_f16", ins[-1]), ins[-1]
    assert checked >= 8, checked
