"""ctypes binding of the C-ABI engine library (include/klsh.h -> kmerlsh_amd/lib/libklsh.so).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C kmerlsh_amd/csrc``).
There is no fallback: if the library is missing, or no gfx950 device is visible, every entry point
raises.  Loading the library itself needs no GPU (the symbol checks in tests/ run on CPU).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KLSH_LIB overrides the library path (A/B runs of engine builds; the default is the in-tree build)
LIB_PATH = os.environ.get("KLSH_LIB") or os.path.join(_HERE, "lib", "libklsh.so")
CLI_PATH = os.path.join(_HERE, "bin", "kmerLSH")

KLSH_OK = 0
ERRORS = {
    -1: "KLSH_E_ARG",
    -2: "KLSH_E_HIP",
    -3: "KLSH_E_NOMEM",
    -4: "KLSH_E_STATE",
    -5: "KLSH_E_NODEVICE",
    -6: "KLSH_E_RANGE",
}

# Every symbol include/klsh.h declares (tests/test_native_lib.py checks the .so exports them).
EXPORTED = (
    "klsh_create", "klsh_destroy", "klsh_last_error", "klsh_version", "klsh_abi_version",
    "klsh_load_rows",
    "klsh_load_counts", "klsh_snapshot", "klsh_restore", "klsh_cluster", "klsh_count",
    "klsh_result", "klsh_hash_keys", "klsh_bucket_sort", "klsh_pcluster", "klsh_hyperplanes", "klsh_fp_selftest",
    "klsh_synth_counts", "klsh_comm_unique_id", "klsh_comm_init", "klsh_comm_init_local",
    "klsh_comm_info", "klsh_set_option", "klsh_get_option", "klsh_wrs", "klsh_ttest2", "klsh_fastq_open",
    "klsh_fastq_next", "klsh_fastq_close", "klsh_kset_create", "klsh_kset_destroy",
    "klsh_check_reads", "klsh_extract_fastq", "klsh_build_khtable", "klsh_cuckoo_order",
    "klsh_kmc_info", "klsh_bucket_runs",
)


# include/klsh.h KLSH_ABI_VERSION (the structs below mirror that header)
ABI_VERSION = 3
# klsh_stats.kern indices (include/klsh.h KLSH_K_*); "merge" is a phase (KLSH_K_MERGE)
KERNEL_CLASSES = ("project", "sort", "runs", "small", "big128", "big192", "big384", "big896",
                  "huge", "tail", "compact", "screen", "merge")
KCLASSES = 13


class KlshKstat(ctypes.Structure):
    _fields_ = [
        ("ms", ctypes.c_double),
        ("launches", ctypes.c_uint64),
        ("rows", ctypes.c_uint64),
        ("runs", ctypes.c_uint64),
    ]


class _Sized(ctypes.Structure):
    """A statistics struct whose leading struct_size field the caller fills in."""

    def __init__(self):
        super().__init__()
        self.struct_size = ctypes.sizeof(self)

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "struct_size"}


class KlshStats(_Sized):
    _fields_ = [
        ("struct_size", ctypes.c_uint64),
        ("iterations", ctypes.c_uint64),
        ("sum_rows", ctypes.c_uint64),
        ("sum_merges", ctypes.c_uint64),
        ("sum_proj_bits", ctypes.c_uint64),
        ("nested_calls", ctypes.c_uint64),
        ("hyperplanes", ctypes.c_uint64),
        ("n_final", ctypes.c_uint64),
        ("project_launches", ctypes.c_uint64),
        ("project_timed_launches", ctypes.c_uint64),
        ("wall_ms", ctypes.c_double),
        ("project_ms", ctypes.c_double),
        ("sort_ms", ctypes.c_double),
        ("merge_ms", ctypes.c_double),
        ("compact_ms", ctypes.c_double),
        ("host_ms", ctypes.c_double),
        ("comm_ms", ctypes.c_double),
        ("world", ctypes.c_uint64),
        ("small_ms", ctypes.c_double),
        ("small_launches", ctypes.c_uint64),
        ("small_rows", ctypes.c_uint64),
        ("small_iter_merges", ctypes.c_uint64),
        ("kern", KlshKstat * KCLASSES),
        ("proj_fix_pairs", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("kern", "struct_size")}
        d["kern"] = {name: {f: getattr(self.kern[i], f) for f, _ in KlshKstat._fields_}
                     for i, name in enumerate(KERNEL_CLASSES)}
        return d


class KlshExtractStats(_Sized):
    _fields_ = [
        ("struct_size", ctypes.c_uint64),
        ("reads", ctypes.c_uint64),
        ("bases", ctypes.c_uint64),
        ("reads_tested", ctypes.c_uint64),
        ("kmers_checked", ctypes.c_uint64),
        ("reads_extracted", ctypes.c_uint64),
        ("abnormal", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("parse_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
    ]


class KlshKhtableStats(_Sized):
    _fields_ = [
        ("struct_size", ctypes.c_uint64),
        ("kmap_size", ctypes.c_uint64),
        ("records", ctypes.c_uint64),
        ("records_listed", ctypes.c_uint64),
        ("io_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("order_ms", ctypes.c_double),
    ]


class KlshError(RuntimeError):
    pass


_lib = None

_P = ctypes.c_void_p
_u64p = ctypes.POINTER(ctypes.c_uint64)


def load_library() -> ctypes.CDLL:
    """Load libklsh.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KlshError(
            f"{LIB_PATH} is missing: the gfx950 engine has no CPU fallback; "
            "build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "klsh_create": (_P, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "klsh_destroy": (None, [_P]),
        "klsh_last_error": (ctypes.c_char_p, []),
        "klsh_version": (ctypes.c_char_p, []),
        "klsh_abi_version": (ctypes.c_int, []),
        "klsh_load_rows": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, _P, _P]),
        "klsh_load_counts": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_int, _P]),
        "klsh_snapshot": (ctypes.c_int, [_P]),
        "klsh_restore": (ctypes.c_int, [_P]),
        "klsh_cluster": (ctypes.c_int, [_P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint32, _u64p, _P, _P]),
        "klsh_count": (ctypes.c_int, [_P, _u64p, _u64p]),
        "klsh_result": (ctypes.c_int, [_P, _P, _P, _P]),
        "klsh_hash_keys": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, _P,
                                          ctypes.c_int, _P]),
        "klsh_bucket_sort": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, _P, _P]),
        "klsh_pcluster": (ctypes.c_int, [_P, ctypes.c_float]),
        "klsh_bucket_runs": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, _u64p, _P, _P,
                                            _P]),
        "klsh_hyperplanes": (ctypes.c_int, [ctypes.c_uint32, _u64p, ctypes.c_int,
                                            ctypes.c_int, _P]),
        "klsh_fp_selftest": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, _P, _P]),
        "klsh_synth_counts": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int, _P, _P]),
        "klsh_comm_unique_id": (ctypes.c_int, [_P]),
        "klsh_comm_init": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _P]),
        "klsh_comm_init_local": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
        "klsh_comm_info": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int)]),
        "klsh_set_option": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int64]),
        "klsh_get_option": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
        "klsh_wrs": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _P,
                                    ctypes.c_float, ctypes.c_int, _P]),
        "klsh_ttest2": (ctypes.c_int, [_P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P, _P]),
        "klsh_fastq_open": (_P, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
        "klsh_fastq_next": (ctypes.c_int64, [_P, ctypes.c_uint64] + [ctypes.POINTER(_P)] * 6),
        "klsh_fastq_close": (None, [_P]),
        "klsh_kset_create": (_P, [_P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]),
        "klsh_kset_destroy": (None, [_P]),
        "klsh_check_reads": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.c_float, _P, _P]),
        "klsh_extract_fastq": (ctypes.c_int, [_P, _P, ctypes.c_char_p, ctypes.c_char_p,
                                              ctypes.c_int, ctypes.c_float, _P]),
        "klsh_build_khtable": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                              ctypes.c_int, ctypes.c_char_p, _P]),
        "klsh_cuckoo_order": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_int, _P]),
        "klsh_kmc_info": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), _u64p, _u64p]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("KLSH_LIB") and not hasattr(lib, name):
            continue  # an A/B build of an older engine: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # every library is checked, the KLSH_LIB ones (diagnostics / A/B builds, the likeliest to be
    # stale) too; KLSH_ABI_ANY=1 turns the refusal into a warning for an older A/B build, whose
    # calls with statistics structs then fail on their struct_size check instead
    if hasattr(lib, "klsh_abi_version") and lib.klsh_abi_version() != ABI_VERSION:
        msg = (f"{os.environ.get('KLSH_LIB') or LIB_PATH}: ABI version {lib.klsh_abi_version()}, "
               f"this binding mirrors {ABI_VERSION}: rebuild the library")
        if os.environ.get("KLSH_ABI_ANY") != "1":
            raise KlshError(msg)
        import warnings

        warnings.warn(msg)
    _lib = lib
    return lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _check(rc: int, what: str) -> None:
    if rc != KLSH_OK:
        msg = load_library().klsh_last_error().decode(errors="replace")
        raise KlshError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")


def hyperplanes(seed: int, counter: int, h: int, d: int) -> tuple[np.ndarray, int]:
    """LSH::generateHashTable under the seeding convention (host; no GPU needed)."""
    lib = load_library()
    out = np.zeros((max(h, 0), d), dtype=np.float32)
    c = ctypes.c_uint64(counter)
    _check(lib.klsh_hyperplanes(seed, ctypes.byref(c), h, d, _ptr(out)), "klsh_hyperplanes")
    return out, c.value


def comm_unique_id() -> bytes:
    """128-byte RCCL id for klsh_comm_init (create on rank 0, ship to the others)."""
    lib = load_library()
    buf = (ctypes.c_uint8 * 128)()
    _check(lib.klsh_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)), "klsh_comm_unique_id")
    return bytes(buf)


def comm_init_local(engines) -> None:
    """Bind Engines into one in-process sharded group (each must then run on its own thread)."""
    lib = load_library()
    arr = (ctypes.c_void_p * len(engines))(*[e._ctx for e in engines])
    _check(lib.klsh_comm_init_local(arr, len(engines)), "klsh_comm_init_local")


def cuckoo_order(images: np.ndarray, k: int) -> tuple[np.ndarray, int]:
    """The reference's libcuckoo table order of distinct k-mer images inserted in the given order
    (host): (index of each table element in iteration order, final hash power)."""
    lib = load_library()
    im = np.ascontiguousarray(images, np.uint64)
    out = np.zeros(im.size, np.uint32)
    hp = lib.klsh_cuckoo_order(_ptr(im), im.size, k, _ptr(out))
    if hp < 0:
        _check(hp, "klsh_cuckoo_order")
    return out, int(hp)


def synth_counts(n: int, d: int, seed: int, genomes: int = 0, threads: int = 0):
    """klsh-synth v1 (host): sample-major (d, n) uint16 counts and per-sample coverage."""
    lib = load_library()
    counts = np.empty((d, n), dtype=np.uint16)
    cov = np.empty(d, dtype=np.float64)
    _check(lib.klsh_synth_counts(n, d, seed, genomes, threads, _ptr(counts), _ptr(cov)),
           "klsh_synth_counts")
    return counts, cov


def ttest2(x: np.ndarray, y: np.ndarray) -> tuple[float, float, float]:
    """alglib::studentttest2 as AB::WRS calls it (host restatement): (both, left, right) tails."""
    lib = load_library()
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros(3, np.float64)
    base = out.ctypes.data
    _check(lib.klsh_ttest2(_ptr(x), x.size, _ptr(y), y.size, base, base + 8, base + 16),
           "klsh_ttest2")
    return float(out[0]), float(out[1]), float(out[2])


def wrs(centroids: np.ndarray, member_counts: np.ndarray, n1: int, n2: int, pvalue_thresh: float,
        size_thresh: int) -> np.ndarray:
    """AB::WRS over every cluster (host): uint8 group per cluster, 1 = group A, 2 = group B."""
    lib = load_library()
    c = np.ascontiguousarray(centroids, np.float32).reshape(-1, n1 + n2) if n1 + n2 else \
        np.zeros((len(member_counts), 0), np.float32)
    mc = np.ascontiguousarray(member_counts, np.uint64)
    g = np.zeros(mc.size, np.uint8)
    _check(lib.klsh_wrs(_ptr(c), mc.size, n1, n2, _ptr(mc), ctypes.c_float(pvalue_thresh),
                        int(size_thresh), _ptr(g)), "klsh_wrs")
    return g


def fastq_records(path: str, batch: int = 1 << 16):
    """Every record of a FASTQ(.gz) as the reference's FastqFile/kseq reads it (host):
    a list of (name, seq, qual) byte strings."""
    lib = load_library()
    err = ctypes.c_int(0)
    f = lib.klsh_fastq_open(path.encode(), ctypes.byref(err))
    if not f:
        _check(err.value or -1, "klsh_fastq_open")
    out = []
    try:
        while True:
            ptrs = [_P() for _ in range(6)]
            n = lib.klsh_fastq_next(f, batch, *[ctypes.byref(p) for p in ptrs])
            if n < 0:
                _check(int(n), "klsh_fastq_next")
            if n == 0:
                break
            offs = [np.ctypeslib.as_array(ctypes.cast(ptrs[i], ctypes.POINTER(ctypes.c_uint64)),
                                          shape=(n + 1,)).copy() for i in (1, 3, 5)]
            blobs = [ctypes.string_at(ptrs[i], int(o[-1])) if o[-1] else b""
                     for i, o in zip((0, 2, 4), offs)]
            so, no, qo = offs
            sb, nb, qb = blobs
            for r in range(n):
                out.append((nb[no[r]:no[r + 1]], sb[so[r]:so[r + 1]], qb[qo[r]:qo[r + 1]]))
    finally:
        lib.klsh_fastq_close(f)
    return out


class KmerSet:
    """A differential k-mer set on an Engine's device (``klsh_kset``)."""

    def __init__(self, engine: "Engine", kmers: np.ndarray):
        self._lib = engine._lib
        self.engine = engine
        k = np.ascontiguousarray(kmers, np.uint64)
        err = ctypes.c_int(0)
        self._set = self._lib.klsh_kset_create(engine._ctx, _ptr(k), k.size, ctypes.byref(err))
        if not self._set:
            _check(err.value or -2, "klsh_kset_create")
        self.size = k.size

    def close(self) -> None:
        if getattr(self, "_set", None):
            self._lib.klsh_kset_destroy(self._set)
            self._set = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check_reads(self, seqs, k: int, kmer_vote: float):
        """IOFQ::CheckRead on the GPU: (hits uint32, flags uint8) per read (bytes sequences)."""
        blob = b"".join(seqs)
        off = np.zeros(len(seqs) + 1, np.uint64)
        off[1:] = np.cumsum([len(s) for s in seqs], dtype=np.uint64)
        buf = np.frombuffer(blob + b"\0", np.uint8)
        hits = np.zeros(len(seqs), np.uint32)
        flags = np.zeros(len(seqs), np.uint8)
        _check(self._lib.klsh_check_reads(self.engine._ctx, self._set, _ptr(buf), _ptr(off),
                                          len(seqs), k, ctypes.c_float(kmer_vote), _ptr(hits),
                                          _ptr(flags)), "klsh_check_reads")
        return hits, flags

    def extract_fastq(self, in_path: str, out_path: str, k: int, kmer_vote: float) -> dict:
        """IOFQ::ReadExtract for one sample (host parse + GPU vote + writer)."""
        st = KlshExtractStats()
        _check(self._lib.klsh_extract_fastq(self.engine._ctx, self._set, in_path.encode(),
                                            out_path.encode(), k, ctypes.c_float(kmer_vote),
                                            ctypes.byref(st)), "klsh_extract_fastq")
        return st.as_dict()


class Engine:
    """One device context (``klsh_ctx``)."""

    def __init__(self, device: int = 0):
        lib = load_library()
        err = ctypes.c_int(0)
        self._ctx = lib.klsh_create(device, ctypes.byref(err))
        if not self._ctx:
            _check(err.value or -2, "klsh_create")
        self._lib = lib
        self.d = 0

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.klsh_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- loading
    def load_rows(self, rows: np.ndarray, member_offsets: np.ndarray | None = None,
                  member_ids: np.ndarray | None = None) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.float32)
        n, d = rows.shape
        mo = None if member_offsets is None else np.ascontiguousarray(member_offsets, np.uint64)
        mi = None if member_ids is None else np.ascontiguousarray(member_ids, np.uint64)
        _check(self._lib.klsh_load_rows(self._ctx, _ptr(rows), n, d, _ptr(mo), _ptr(mi)),
               "klsh_load_rows")
        self.d = d

    def load_counts(self, counts: np.ndarray, v_kmers: np.ndarray, batch_offset: int = 0,
                    batch_size: int | None = None) -> None:
        counts = np.ascontiguousarray(counts, dtype=np.uint16)
        d, n_total = counts.shape
        if batch_size is None:
            batch_size = n_total - batch_offset
        vk = np.ascontiguousarray(v_kmers, dtype=np.float32)
        _check(self._lib.klsh_load_counts(self._ctx, _ptr(counts), n_total, batch_offset,
                                          batch_size, d, _ptr(vk)), "klsh_load_counts")
        self.d = d

    def comm_init(self, rank: int, world: int, uid: bytes) -> None:
        """Join the RCCL group `uid` as `rank` of `world` (one process per GPU)."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        _check(self._lib.klsh_comm_init(self._ctx, rank, world, ctypes.cast(buf, ctypes.c_void_p)),
               "klsh_comm_init")

    def set_option(self, name: str, value: int) -> None:
        _check(self._lib.klsh_set_option(self._ctx, name.encode(), int(value)), "klsh_set_option")

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64(0)
        _check(self._lib.klsh_get_option(self._ctx, name.encode(), ctypes.byref(v)),
               "klsh_get_option")
        return v.value

    def comm_info(self) -> tuple[int, int]:
        r = ctypes.c_int(0)
        w = ctypes.c_int(1)
        _check(self._lib.klsh_comm_info(self._ctx, ctypes.byref(r), ctypes.byref(w)),
               "klsh_comm_info")
        return r.value, w.value

    def snapshot(self) -> None:
        _check(self._lib.klsh_snapshot(self._ctx), "klsh_snapshot")

    def restore(self) -> None:
        _check(self._lib.klsh_restore(self._ctx), "klsh_restore")

    # ---- hot path
    def cluster(self, min_similarity: float, iterations: int, bucket_size_threshold: int,
                seed: int = 12345, counter: int = 0):
        """Returns (trace of N_t, new rng counter, stats dict)."""
        c = ctypes.c_uint64(counter)
        trace = np.zeros(max(iterations, 1), dtype=np.uint64)
        st = KlshStats()
        _check(self._lib.klsh_cluster(self._ctx, ctypes.c_float(min_similarity), iterations,
                                      bucket_size_threshold, seed, ctypes.byref(c), _ptr(trace),
                                      ctypes.byref(st)), "klsh_cluster")
        return trace[: st.iterations], c.value, st.as_dict()

    def build_khtable(self, kmc_names, k: int, out_dir: str = "") -> dict:
        """Mode B: kmer_set.hex / kmer_count.bin / kmer_count.log from KMC databases."""
        arr = (ctypes.c_char_p * len(kmc_names))(*[n.encode() for n in kmc_names])
        st = KlshKhtableStats()
        _check(self._lib.klsh_build_khtable(self._ctx, arr, len(kmc_names), k, out_dir.encode(),
                                            ctypes.byref(st)), "klsh_build_khtable")
        return st.as_dict()

    def pcluster(self, thr: float) -> None:
        _check(self._lib.klsh_pcluster(self._ctx, ctypes.c_float(thr)), "klsh_pcluster")

    def hash_keys(self, rows: np.ndarray, table: np.ndarray) -> np.ndarray:
        rows = np.ascontiguousarray(rows, dtype=np.float32)
        table = np.ascontiguousarray(table, dtype=np.float32)
        n, d = rows.shape
        h = table.shape[0]
        keys = np.zeros(n, dtype=np.uint32)
        _check(self._lib.klsh_hash_keys(self._ctx, _ptr(rows), n, d, _ptr(table), h,
                                        _ptr(keys)), "klsh_hash_keys")
        return keys

    def bucket_sort(self, keys: np.ndarray, bits: int):
        """merge_hashtable's stable bucket order on the GPU: (sorted keys, permutation)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        out = np.zeros_like(keys)
        perm = np.zeros_like(keys)
        _check(self._lib.klsh_bucket_sort(self._ctx, _ptr(keys), keys.size, bits, _ptr(out),
                                          _ptr(perm)), "klsh_bucket_sort")
        return out, perm

    def bucket_runs(self, sorted_keys: np.ndarray, bucket_thr: int):
        """The merge step's runs of equal sorted keys: (starts, lengths, lists), start order."""
        k = np.ascontiguousarray(sorted_keys, dtype=np.uint32)
        cap = k.size // 2 + 1
        st = np.zeros(cap, np.uint32)
        ln = np.zeros(cap, np.uint32)
        li = np.zeros(cap, np.int32)
        nr = ctypes.c_uint64(cap)
        _check(self._lib.klsh_bucket_runs(self._ctx, _ptr(k), k.size, int(bucket_thr),
                                          ctypes.byref(nr), _ptr(st), _ptr(ln), _ptr(li)),
               "klsh_bucket_runs")
        m = nr.value
        return st[:m], ln[:m], li[:m]

    def fp_selftest(self, a: np.ndarray, b: np.ndarray):
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        s = np.zeros_like(a)
        q = np.zeros_like(a)
        _check(self._lib.klsh_fp_selftest(self._ctx, _ptr(a), _ptr(b), a.size, _ptr(s), _ptr(q)),
               "klsh_fp_selftest")
        return s, q

    # ---- results
    def count(self) -> tuple[int, int]:
        n = ctypes.c_uint64(0)
        m = ctypes.c_uint64(0)
        _check(self._lib.klsh_count(self._ctx, ctypes.byref(n), ctypes.byref(m)), "klsh_count")
        return n.value, m.value

    def result(self):
        """(rows (n, d) float32, member_offsets (n+1,) uint64, member_ids (m,) uint64)."""
        n, m = self.count()
        rows = np.zeros((n, self.d), dtype=np.float32)
        off = np.zeros(n + 1, dtype=np.uint64)
        ids = np.zeros(m, dtype=np.uint64)
        _check(self._lib.klsh_result(self._ctx, _ptr(rows), _ptr(off), _ptr(ids)),
               "klsh_result")
        return rows, off, ids
