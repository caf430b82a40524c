"""The reference-signature adapter (include/klsh_cluster.hpp) compiles against a reference-like
Abundance type (CPU), and, on the GPU, reproduces the reference's Cluster() output."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden

SRC = os.path.join(ROOT, "tests", "cpp", "adapter_main.cpp")


REF_ABUNDANCE = "/root/reference/common/abundance.h"


def build(out, defines=()):
    subprocess.run(["g++", "-std=c++11", "-O2", *defines, "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", out, "-L", os.path.join(ROOT, "kmerlsh_amd", "lib"), "-lklsh",
                    "-Wl,-rpath," + os.path.join(ROOT, "kmerlsh_amd", "lib")], check=True)


def test_adapter_compiles(tmp_path):
    build(str(tmp_path / "adapter"))


@pytest.mark.skipif(not os.path.exists(REF_ABUNDANCE), reason="reference tree not present")
def test_adapter_compiles_against_reference_abundance(tmp_path):
    """The adapter instantiated with the reference's own Core::Abundance (common/abundance.h,
    read in place), as app/kmerLSH.cc would after INTEGRATION.md's change: compile and link."""
    build(str(tmp_path / "adapter_ref"), [f'-DKLSH_REF_ABUNDANCE="{REF_ABUNDANCE}"'])


@pytest.mark.gpu
def test_adapter_matches_reference(tmp_path):
    z = golden("cluster_d16.npz")
    exe = str(tmp_path / "adapter")
    build(exe)
    rows = z["rows"]
    rows.astype("<f4").tofile(tmp_path / "rows.f32")
    env = dict(os.environ, KLSH_SEED=str(int(z["seed"])))
    subprocess.run([exe, str(tmp_path / "rows.f32"), str(rows.shape[0]), str(rows.shape[1]),
                    repr(float(z["min_sim"])), str(int(z["iters"])), str(int(z["bthr"])),
                    str(tmp_path / "out.f32"), str(tmp_path / "out.clust")], check=True, env=env,
                   timeout=300)
    out = np.fromfile(tmp_path / "out.f32", dtype="<f4").reshape(-1, rows.shape[1])
    assert np.array_equal(out.view(np.uint32), z["out_rows"].view(np.uint32))
    sizes, ids = [], []
    for line in (tmp_path / "out.clust").read_text().splitlines():
        parts = [int(v) for v in line.split()]
        sizes.append(parts[0])
        ids.extend(parts[1:])
    assert np.array_equal(np.concatenate([[0], np.cumsum(sizes)]), z["out_off"].astype(np.int64))
    assert np.array_equal(np.array(ids), z["out_ids"].astype(np.int64))
