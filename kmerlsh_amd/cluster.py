"""Host-side mirror of the reference's clustering interface, driving the gfx950 engine.

Reference interface mirrored (same names, argument meaning and in-place behaviour):
  Core::Abundance {vector<float> _values; vector<uint64_t> _ids;}   common/abundance.h:18-36
  void Cluster(vector<Abundance*>* unknown_abundance_ptr, float min_similarity,
               int cluster_iteration, unsigned threads_to_use, int dim,
               int bucket_size_threshold, bool verbose)               function/cluster.h:42
  void p_cluster(vector<Abundance*>* part_ab, vector<Abundance*>* candidates, float threshold)
                                                                       function/cluster.h:38

`threads_to_use` is accepted and ignored: results equal the reference at -T 1 for every value.
The reference seeds every hyperplane from std::random_device; here draws follow the seeding
convention of SURVEY.md §8(c) through a process-wide `SeedStream` (the counter carries across
calls, like the reference's stream of rd() calls: init pass, then main loop).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _native


class Abundance:
    """A row: abundance values over samples and the k-mer ids merged into it."""

    __slots__ = ("_values", "_ids")

    def __init__(self, values=None, ids=None):
        self._values = np.asarray(values if values is not None else [], dtype=np.float32)
        self._ids = list(ids) if ids is not None else []

    def __repr__(self) -> str:
        return f"Abundance(ids={self._ids!r}, values={self._values.tolist()!r})"


@dataclass
class SeedStream:
    """KLSH_SEED base and the number of hyperplanes drawn so far."""

    base: int = 12345
    counter: int = 0


DEFAULT_STREAM = SeedStream()
_engines: dict[int, _native.Engine] = {}


def engine(device: int = 0) -> _native.Engine:
    if device not in _engines:
        _engines[device] = _native.Engine(device)
    return _engines[device]


def _to_arrays(rows: list[Abundance], dim: int):
    n = len(rows)
    x = np.zeros((n, dim), dtype=np.float32)
    off = np.zeros(n + 1, dtype=np.uint64)
    for i, a in enumerate(rows):
        x[i] = a._values
        off[i + 1] = off[i] + len(a._ids)
    ids = np.fromiter((v for a in rows for v in a._ids), dtype=np.uint64, count=int(off[-1]))
    return x, off, ids


def _from_engine(eng: _native.Engine) -> list[Abundance]:
    x, off, ids = eng.result()
    out = []
    for i in range(x.shape[0]):
        out.append(Abundance(x[i].copy(), ids[off[i]: off[i + 1]].tolist()))
    return out


def Cluster(unknown_abundance: list[Abundance], min_similarity: float, cluster_iteration: int,
            threads_to_use: int, dim: int, bucket_size_threshold: int, verbose: bool = False,
            *, stream: SeedStream | None = None, device: int = 0) -> dict:
    """reference function/cluster.cc:181-340, in place on `unknown_abundance`.

    Returns {"trace": N_t per iteration, "stats": engine statistics}.
    """
    del threads_to_use
    stream = stream or DEFAULT_STREAM
    eng = engine(device)
    x, off, ids = _to_arrays(unknown_abundance, dim)
    eng.load_rows(x, off, ids)
    trace, stream.counter, stats = eng.cluster(np.float32(min_similarity), cluster_iteration,
                                               bucket_size_threshold, stream.base,
                                               stream.counter)
    if verbose:
        for t, n in enumerate(trace.tolist()):
            print(f"Iteration:\t{t + 1}")
            print(f"Size of profilings : {n}")
        print(f"kmerLSH algorithm hash+cluster takes (secs): {stats['wall_ms'] / 1000.0}")
    unknown_abundance[:] = _from_engine(eng)
    return {"trace": trace, "stats": stats}


def p_cluster(part_ab: list[Abundance], candidates: list[Abundance], threshold: float,
              *, device: int = 0) -> None:
    """reference function/cluster.cc:56-87: greedy merge of one bucket, survivors appended."""
    if not candidates:
        return
    dim = len(candidates[0]._values)
    eng = engine(device)
    x, off, ids = _to_arrays(candidates, dim)
    eng.load_rows(x, off, ids)
    eng.pcluster(np.float32(threshold))
    part_ab.extend(_from_engine(eng))
