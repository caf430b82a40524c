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
ASMS = [os.path.join(ROOT, "kmerlsh_amd", "build", f)
        for f in ("klsh_kernels.s", "klsh_merge.s", "klsh_shard.s")]
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


def _ops(body):
    """The instruction lines of a kernel body (labels, comments and directives dropped)."""
    out = []
    for ln in body.splitlines():
        t = ln.strip()
        if t and not t.startswith((";", ".")) and not t.endswith(":"):
            out.append(t)
    return out


def _waited_loads(body, load=r"(global|buffer|flat)_load\w*"):
    """Vector loads followed at once by s_waitcnt vmcnt(0): each one a round trip of its own."""
    ops = _ops(body)
    pat = re.compile(load)
    return [ops[i] for i in range(len(ops) - 1)
            if pat.match(ops[i]) and ops[i + 1].startswith("s_waitcnt") and "vmcnt(0)" in ops[i + 1]]


def _kernel(kernels, *parts):
    names = [k for k in kernels if all(p in k for p in parts)]
    assert names, parts
    return names


def test_load_batches_stay_in_flight(kernels):
    """Regression guard for the load->wait chains the round-6 ISA audit removed:
    a per-lane index into a kernel-argument pointer array, a store under a bounds branch that lets
    the compiler sink its load into the branch, a load then a branch on its value."""
    # run listing: no pointer load per entry, no flat (generic) entry stores
    for name in _kernel(kernels, "k_tail_local") + _kernel(kernels, "k_runs_write"):
        body = kernels[name]
        assert not any(op.startswith("flat_") for op in _ops(body)), name
        # (one: the list-pointer table itself, read once per workgroup)
        assert len(_waited_loads(body, r"global_load_dwordx2")) <= 1, (name, _waited_loads(body)[:4])
    # big-run row staging (LDS rows at d = 16 / 32 / 64): no load -> wait -> LDS store triples
    for name in [k for k in kernels if "k_merge_bigIL" in k and "ELb1E" in k]:
        ops = _ops(kernels[name])
        triples = [i for i in range(len(ops) - 2)
                   if ops[i].startswith("global_load_dwordx4") and "vmcnt(0)" in ops[i + 1]
                   and ops[i + 2].startswith("ds_write_b128")]
        assert not triples, (name, len(triples))
    # k_project_fix's hyperplane staging and the wide group merges' chunk staging
    for name in _kernel(kernels, "k_project_fix") + _kernel(kernels, "k_merge_group_wide"):
        w = _waited_loads(kernels[name], r"global_load_dwordx4")
        assert len(w) <= 1, (name, len(w))
    # k_merge_long's row copy for the next step (global -> LDS, typed: not a flat chain)
    for name in _kernel(kernels, "long_mem_decide"):
        assert len(_waited_loads(kernels[name])) <= 2, name
    # the sharded loop's bin split
    for name in _kernel(kernels, "k_bin_split"):
        assert len(_waited_loads(kernels[name])) <= 2, name
