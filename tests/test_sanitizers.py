"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; SURVEY.md §5 "race
detection / sanitizers").

`make -C kmerlsh_amd/csrc asan` builds the engine library with ASan + UBSan on its HOST code
(device code untouched) and tests/cpp/asan_host, a driver over the host entry points that read
untrusted input or whose arithmetic the GPU path depends on: the FASTQ reader (the reference's
kseq rules, plain and gzip) on the mode-E fixtures and on truncated / byte-flipped copies and
random streams, the KMC prefix-file parse on the mode-B databases and 300 corruptions of each (8 of a >1 MB one),
ALGLIB's t-test restatement and AB::WRS on random and degenerate groups, the libcuckoo replay
(k = 1..32, table growth), the hyperplane draw and the synthetic workload.  The plain-C oracle's
mode-C CLI runs the KAT pipeline under the same sanitizers.  Any report aborts: exit 0 = clean.
"""
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT

sys.path.insert(0, GOLDEN)
import kat_inputs  # noqa: E402
import kmc_inputs  # noqa: E402
import mode_e_inputs  # noqa: E402

DRIVER = os.path.join(ROOT, "kmerlsh_amd", "build_asan", "asan_host")
ORACLE = os.path.join(ROOT, "oracle", "klsh_oracle_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def driver():
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "kmerlsh_amd", "csrc"), "asan"],
                   check=True, capture_output=True, timeout=1200)
    return DRIVER


def run(args, cwd=None):
    p = subprocess.run(args, cwd=cwd, env=ENV, capture_output=True, text=True, timeout=600)
    report = "AddressSanitizer" in p.stderr or "runtime error" in p.stderr or "LeakSanitizer" in p.stderr
    assert p.returncode == 0 and not report, p.stdout[-2000:] + p.stderr[-4000:]
    return p.stdout


def test_fastq_reader_sanitized(driver, tmp_path):
    files = []
    for case in sorted(mode_e_inputs.CASES):
        d = tmp_path / case
        d.mkdir()
        info = mode_e_inputs.write_case(str(d), case)
        files += [str(d / nm) for nm in info["samples1"] + info["samples2"]]
    assert "fastq ok" in run([driver, "fastq", str(tmp_path)] + files)


def test_kmc_prefix_parse_sanitized(driver, tmp_path):
    names = []
    for case in sorted(kmc_inputs.CASES):
        d = tmp_path / case
        d.mkdir()
        info = kmc_inputs.write_case(str(d), case)
        names += [str(d / nm) for nm in info["names"]]
    out = run([driver, "kmc"] + names)
    assert "kmc ok" in out


@pytest.mark.parametrize("what", ["ttest", "cuckoo", "rng"])
def test_host_arithmetic_sanitized(driver, what):
    assert f"{what} ok" in run([driver, what])


def test_oracle_cli_sanitized(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True,
                   capture_output=True, timeout=600)
    kat_inputs.write_kat("katF", str(tmp_path))
    run([ORACLE, "-a", "a.txt", "-b", "b.txt", "-I", "10", "-T", "2", "-M", "C", "--only",
         "--seed", "12345"], cwd=tmp_path)
    assert os.path.getsize(tmp_path / "clustering_result.txt") > 0
