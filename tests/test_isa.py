"""Static checks of the gfx950 code object (CPU only: hipcc cross-compiles).

The reference never fuses multiply-add, so the sign-hash kernels must contain
no v_fma*/v_fmac*/v_pk_fma*/v_mad_f32 at all, and the dot products of the merge kernels must use
separate v_mul/v_add.  sqrt and division must be the correctly rounded expansions (those use
FMA-based refinement internally, which is exact by construction).
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "kmerlsh_amd", "csrc")
ASMS = [os.path.join(ROOT, "kmerlsh_amd", "build", f) for f in ("klsh_kernels.s", "klsh_merge.s")]
FMA = re.compile(r"^\s+(v_fma\w*|v_fmac\w*|v_pk_fma\w*|v_mad_f32\w*|v_fmamk\w*|v_fmaak\w*)\b")


@pytest.fixture(scope="module")
def kernels():
    subprocess.run(["make", "-s", "-C", CSRC, "isa"], check=True)
    text = "".join(open(a).read() for a in ASMS)
    out = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.M | re.S):
        out[m.group(1)] = m.group(2)
    assert out, "no kernels found in the assembly"
    return out


def test_target_is_gfx950(kernels):
    for a in ASMS:
        assert "gfx950" in open(a).read()


def test_projection_has_no_fused_multiply_add(kernels):
    proj = {k: v for k, v in kernels.items() if "k_project" in k}
    # d = 8, 16, 32, 64: packed (8 chains, 1 row per lane); the packed wide-row kernel; the generic
    # kernel; the wide-row matrix-core screen (any d, and unrolled for d = 512) + its exact fix-up
    # kernel; the fp16-image screens (d = 16, 32, 64; their close calls settled in the same
    # kernel)
    assert len(proj) == 12, sorted(proj)
    for name, body in proj.items():
        bad = [ln.strip() for ln in body.splitlines() if FMA.match(ln)]
        assert not bad, (name, bad[:5])
        if "mfma" in name:  # fp16x3 MFMA screen + the exact unfused chain for the close calls
            assert "v_mfma_f32_32x32x16_f16" in body, name
            assert "v_mul_f32" in body and "v_add_f32" in body, name
        elif "h16" in name:  # fp16-image screen (x~ . (w_hi + w_lo)) + the exact unfused chain
            assert "v_mfma_f32_32x32x16_f16" in body, name
            assert "v_mul_f32" in body and "v_add_f32" in body, name
        elif "_pk" in name:  # packed kernels: every product a separately rounded v_pk_mul_f32
            assert body.count("v_pk_mul_f32") == body.count("v_pk_add_f32") > 0, name
        else:
            assert "v_mul_f32" in body or "v_pk_mul_f32" in body
            assert "v_add_f32" in body


def test_merge_dot_products_are_unfused(kernels):
    """In the merge kernels every FMA must belong to a sqrt/div expansion: their count per kernel
    is bounded by the number of sqrt/div sequences, while the dot products (d multiplies + adds
    per pair) appear as v_mul/v_add."""
    merge = {k: v for k, v in kernels.items() if "k_merge" in k}
    assert merge
    for name, body in merge.items():
        n_fma = sum(1 for ln in body.splitlines() if FMA.match(ln))
        n_div = body.count("v_div_fixup_f32")
        n_sqrt = body.count("v_sqrt_f32")
        # correctly rounded f32 division = 1 rcp + 5 fma-class ops + fmas + fixup; sqrt
        # refinement <= 4 fma-class ops
        assert n_fma <= 6 * n_div + 4 * n_sqrt, (name, n_fma, n_div, n_sqrt)
        assert n_div >= 1 and n_sqrt >= 1, name
        assert "v_add_f32" in body


def test_correctly_rounded_division_and_sqrt(kernels):
    body = kernels[next(k for k in kernels if "k_fp_selftest" in k)]
    assert "v_div_scale_f32" in body and "v_div_fixup_f32" in body
    assert "v_sqrt_f32" in body
