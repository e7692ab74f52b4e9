"""CPU tier: properties of the shipped gfx950 code (federated_multi_modal_amd/lib/libmapfed.so) that no numerical test
on a quiet GPU can see (DESIGN.md §6, r06 LayerNorm-backward finding).

* No packed fp32 VALU arithmetic (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32) in any kernel.  r06 traced the r05
  run-to-run different vision LayerNorm dgamma partials to the packed fp32 path: the r05 build of ln_bwd2_kernel
  gave partials its own inputs do not determine (private input copies, every memory operation waited to zero:
  still different) and was clean when the same source was compiled without packed fp32
  (tests/diagnostics/ln_bwd_snapshot.py); the library is now built with -packed-fp32-ops (csrc/Makefile).
* Every load a LayerNorm kernel issues is covered by an s_waitcnt vmcnt before the first instruction that reads or
  overwrites its registers, on every control-flow path (tests/isa_tools.py), so their results cannot depend on
  memory latency.
* No fp16-result mixed-precision FMA (v_fma_mixlo_f16 / v_fma_mixhi_f16) in the optimizer and logit / loss kernels:
  the compiler folds fp16(a * b) into one, which rounds the exact product to fp16 once, where the reference's fp16
  op rounds its fp32 product first (61 of the 61 094 finite fp16 inputs of f * 1.702f differ,
  tests/diagnostics/mixround/); those products go through mf_common.h mul32.  (The GEMMs' QuickGELU keeps the
  folded form, measured against the parity gates: mf_common.h.)
"""
import re
import shlex
import subprocess
from pathlib import Path

import pytest

import isa_tools as T

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "federated_multi_modal_amd" / "lib" / "libmapfed.so"
CSRC = ROOT / "federated_multi_modal_amd" / "csrc"
PACKED_F32 = re.compile(r"\bv_pk_(mul|add|fma)_f32\b")
MIX_F16 = re.compile(r"\bv_fma_mix(lo|hi)_f16\b")
# kernels whose fp16 results must follow the reference's two roundings of a product (the caption pool's products
# are of two fp16 values, exact in fp32, so a single rounding is the same there)
MIX_CHECKED = re.compile(r"sgd|logits_kernel|loss_kernel")


@pytest.fixture(scope="module")
def disasm():
    if not LIB.exists():
        pytest.skip("libmapfed.so not built")
    return T.device_disassembly(LIB)


def test_library_code_objects_cover_every_source(disasm):
    names = " ".join(disasm)
    for k in ("gemm8f_kernel", "ln_bwd2_kernel", "ln_fwd2_kernel", "attn_fwd4_kernel", "attn_bwd_fused_kernel",
              "sgd8_both", "aug_fused"):
        assert k in names, k


def test_no_packed_fp32_arithmetic_in_any_kernel(disasm):
    bad = {k: sum(1 for ln in body if PACKED_F32.search(ln)) for k, body in disasm.items()}
    bad = {k: n for k, n in bad.items() if n}
    assert not bad, f"{len(bad)} kernels use packed fp32 VALU ops, e.g. {sorted(bad.items())[:3]}"


def test_no_single_rounding_fp16_products(disasm):
    bad = {k: sum(1 for ln in body if MIX_F16.search(ln)) for k, body in disasm.items() if MIX_CHECKED.search(k)}
    bad = {k: n for k, n in bad.items() if n}
    assert not bad, f"{len(bad)} kernels round a product to fp16 in one step, e.g. {sorted(bad.items())[:3]}"


def _makefile_flags():
    text = (CSRC / "Makefile").read_text().replace("\\\n", " ")
    m = re.search(r"^FLAGS \?=(.*)$", text, re.M)
    return shlex.split(m.group(1).replace("$(ARCH)", "gfx950"))


def test_layernorm_loads_are_waited_for_on_every_path(tmp_path):
    out = tmp_path / "layernorm.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *_makefile_flags(), "--cuda-device-only", "-S", str(CSRC / "layernorm.hip"),
                    "-o", str(out)], check=True, capture_output=True)
    asm = out.read_text()
    kernels = T.kernel_names(asm, "ln_")
    assert len(kernels) >= 10
    assert not any(PACKED_F32.search(ln) for ln in asm.splitlines())
    for k in kernels:
        assert T.check_kernel(asm, k) == [], k
