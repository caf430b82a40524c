"""The C-ABI engine library on CPU: it loads, exports every symbol include/klsh.h declares, its
host-side pieces (hyperplane draws, synthetic workload) are right, and without a gfx950 device it
fails loudly instead of falling back.  No compute kernel is launched here.
"""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden


def header_symbols():
    with open(os.path.join(ROOT, "include", "klsh.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(klsh_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from kmerlsh_amd import _native

    lib = _native.load_library()
    declared = header_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_native.EXPORTED)
    assert b"gfx950" in lib.klsh_version()


def test_host_hyperplanes_match_reference_tables():
    """The product's host RNG (libstdc++ instantiated in klsh_host_rng.cpp) reproduces the
    reference's generateHashTable bits (fixtures made by the reference, hash/lshash.cc:3-42)."""
    from kmerlsh_amd import _native

    z = golden("rng_tables.npz")
    for name in z.files:
        seed, h, d = (int(p[1:]) for p in name.split("_"))
        w, counter = _native.hyperplanes(seed, 0, h, d)
        assert counter == h
        assert np.array_equal(w.view(np.uint32), z[name].view(np.uint32)), name


def test_host_hyperplanes_counter(oracle):
    from kmerlsh_amd import _native

    for seed, k, h, d in [(12345, 0, 5, 64), (9, 77, 3, 512), (4294967295, 1 << 20, 2, 7)]:
        w, c = _native.hyperplanes(seed, k, h, d)
        w2, c2 = oracle.table(seed, k, h, d)
        assert c == c2 == k + h
        assert np.array_equal(w.view(np.uint32), w2.view(np.uint32))


def test_synth_is_deterministic_and_plausible():
    from kmerlsh_amd import _native

    a, ca = _native.synth_counts(20000, 8, seed=11, threads=4)
    b, cb = _native.synth_counts(20000, 8, seed=11, threads=1)
    assert a.shape == (8, 20000) and a.dtype == np.uint16
    assert np.array_equal(a, b) and np.array_equal(ca, cb)
    c, _ = _native.synth_counts(20000, 8, seed=12, threads=2)
    assert not np.array_equal(a, c)
    # coverage = sum of ln(count) over nonzero counts, ascending i, in double
    col = a[3].astype(np.float64)
    exp = 0.0
    for v in col[col > 0]:
        exp += np.log(v)
    assert abs(ca[3] - exp) <= 1e-9 * abs(exp)
    # rows of one genome (n/50 genomes) share a profile: means are far from uniform noise
    assert 1.0 < a.mean() < 60.0


def test_no_device_fails_loudly():
    """No CPU fallback: without a gfx950 device the engine refuses to start."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible here")
    from kmerlsh_amd import _native

    with pytest.raises(_native.KlshError, match="KLSH_E_NODEVICE"):
        _native.Engine(0)


def test_python_mirror_interface():
    import kmerlsh_amd

    a = kmerlsh_amd.Abundance([1.0, 2.0], [7])
    assert a._values.dtype == np.float32 and a._ids == [7]
    s = kmerlsh_amd.SeedStream(5)
    assert s.counter == 0


def test_io_roundtrip(tmp_path):
    from kmerlsh_amd import io as kio

    rows = np.arange(24, dtype=np.float32).reshape(4, 6)
    off = np.array([0, 6, 13, 14, 20], dtype=np.uint64)
    ids = np.arange(20, dtype=np.uint64)[::-1].copy()
    kio.save_result(str(tmp_path / "r.txt.clust"), off, ids, 5)
    kio.save_binary(str(tmp_path / "r.txt"), rows, off, 5)
    text = (tmp_path / "r.txt.clust").read_text()
    assert text.splitlines()[0] == "6\t19\t18\t17\t16\t15\t14"
    assert len(text.splitlines()) == 3  # the 1-member cluster is dropped (n > 5)
    r2, o2, i2 = kio.read_cluster_all(str(tmp_path / "r.txt"), 6)
    assert np.array_equal(r2, rows[[0, 1, 3]])
    assert list(np.diff(o2)) == [6, 7, 6]


@pytest.mark.gpu
def test_stats_struct_size_is_checked(tmp_path):
    """A caller built against another klsh.h (a statistics struct of another size) is refused with
    KLSH_E_ARG before anything is written into its struct: klsh_cluster, klsh_extract_fastq and
    klsh_build_khtable (include/klsh.h, ABI v2+ struct_size)."""
    import ctypes

    from kmerlsh_amd import _native

    lib = _native.load_library()
    with _native.Engine(0) as eng:
        rows = np.random.default_rng(3).random((256, 16), dtype=np.float32)
        eng.load_rows(rows)
        for cls, call in [
            (_native.KlshStats,
             lambda st: lib.klsh_cluster(eng._ctx, ctypes.c_float(0.9), 2, 1000, 12345,
                                         ctypes.byref(ctypes.c_uint64(0)), None, ctypes.byref(st))),
            (_native.KlshKhtableStats,
             lambda st: lib.klsh_build_khtable(eng._ctx, (ctypes.c_char_p * 1)(b"missing"), 1, 31,
                                               str(tmp_path).encode(), ctypes.byref(st))),
        ]:
            st = cls()
            st.struct_size = ctypes.sizeof(st) - 8
            assert call(st) == -1, cls.__name__  # KLSH_E_ARG
            assert st.struct_size == ctypes.sizeof(st) - 8  # untouched
        ks = _native.KmerSet(eng, np.arange(1, 9, dtype=np.uint64))
        try:
            st = _native.KlshExtractStats()
            st.struct_size = ctypes.sizeof(st) - 8
            fq = tmp_path / "r.fq"
            fq.write_bytes(b"@r\nACGT\n+\nIIII\n")
            rc = lib.klsh_extract_fastq(eng._ctx, ks._set, str(fq).encode(),
                                        str(tmp_path / "o.fq").encode(), 3, ctypes.c_float(0.5),
                                        ctypes.byref(st))
            assert rc == -1
        finally:
            ks.close()
