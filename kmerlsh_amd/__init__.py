"""kmerlsh_amd — MI355X (gfx950) engine for the kmerLSH LSH k-mer clustering loop.

The hot path (reference function/cluster.cc:181-340 and the functions it calls) runs as
hand-written CDNA4 HIP kernels behind the C ABI in include/klsh.h (lib/libklsh.so).  This package
is the Python side: a ctypes binding (`_native`), a mirror of the reference's Cluster()/p_cluster
interface (`cluster`) and the mode-C file formats (`io`).
"""
from ._native import Engine, KlshError, hyperplanes, load_library, synth_counts  # noqa: F401
from .cluster import Abundance, Cluster, SeedStream, p_cluster  # noqa: F401

__all__ = ["Engine", "KlshError", "hyperplanes", "load_library", "synth_counts", "Abundance",
           "Cluster", "SeedStream", "p_cluster"]
