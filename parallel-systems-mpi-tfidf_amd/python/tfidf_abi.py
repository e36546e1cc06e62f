"""ctypes binding of include/tfidf.h (libtfidf_hip.so).

Plumbing for tests and bench.py: every compute call goes through the C-ABI into the
gfx950 HIP kernels.  Loading fails loudly when the library has not been built; there is
no Python or CPU fallback for any stage.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TFIDF_LIB=<variant> selects a diagnostic build lib/libtfidf_hip_<variant>.so (K1 phase
# stamps, K1 ablations); never used for benches or tests
_VARIANT = os.environ.get("TFIDF_LIB", "")
LIB_PATH = os.path.join(PKG_DIR, "lib", "libtfidf_hip_%s.so" % _VARIANT if _VARIANT else "libtfidf_hip.so")
CLI_PATH = os.path.join(PKG_DIR, "bin", "tfidf")

TFIDF_CORPUS_DEVICE = 1
UNIQUE_ID_BYTES = 128
RUN_K1_VS = 2   # tfidf_run_info.flags (include/tfidf.h): slot-keyed K1 ...
RUN_K1_ST = 4   # retired (round 3's k_tokcount_st, removed in round 5): never set
RUN_K1_SL = 8   # ... run as k_tokcount_sl (the default up to 32M vocabulary slots; else k_tokcount_vs)
RUN_XCHG_DENSE = 16  # multi-rank: the DF exchange used the dense all-reduce form
ABI_VERSION = 2  # TFIDF_ABI_VERSION of include/tfidf.h this binding is written for

# exported symbols declared by include/tfidf.h
EXPORTS = [
    "tfidf_open", "tfidf_close", "tfidf_strerror", "tfidf_abi_version", "tfidf_comm_unique_id",
    "tfidf_comm_init", "tfidf_run", "tfidf_fetch", "tfidf_result_free", "tfidf_last_run_info", "tfidf_alloc_stats",
    "tfidf_stage_name", "tfidf_set_timing", "tfidf_write_output", "tfidf_print_jobs",
    "tfidf_ingest_dir", "tfidf_free", "tfidf_synth_host", "tfidf_synth_device",
    "tfidf_format", "tfidf_copy_text", "tfidf_write_output_gpu", "tfidf_format_f64",
    "tfidf_ingest_dir_device", "tfidf_hbm_probe", "tfidf_group_open", "tfidf_group_size", "tfidf_group_ctx",
    "tfidf_group_run", "tfidf_group_write_output", "tfidf_group_close", "tfidf_plan_dir", "tfidf_plan_free",
    "tfidf_ingest_shard_device", "tfidf_doc_name_order", "tfidf_shard_split", "tfidf_device_count",
    "tfidf_last_output_info", "tfidf_run_totals_get",
]
TFIDF_GROUP_LOCAL = 1
E_PEER = -11


class Corpus(C.Structure):
    _fields_ = [
        ("bytes", C.c_void_p), ("nbytes", C.c_uint64), ("doc_off", C.c_void_p), ("doc_ids", C.c_void_p),
        ("ndocs", C.c_uint32), ("flags", C.c_uint32), ("ndocs_total", C.c_uint64),
    ]


class Result(C.Structure):
    _fields_ = [
        ("npairs", C.c_uint64), ("ndocs", C.c_uint32), ("nterms", C.c_uint32), ("ndocs_total", C.c_uint64),
        ("pair_doc", C.POINTER(C.c_uint32)), ("pair_term", C.POINTER(C.c_uint32)),
        ("pair_count", C.POINTER(C.c_uint32)), ("pair_docsize", C.POINTER(C.c_uint32)),
        ("pair_df", C.POINTER(C.c_uint32)), ("pair_score", C.POINTER(C.c_double)),
        ("doc_id", C.POINTER(C.c_uint32)), ("doc_size", C.POINTER(C.c_uint32)),
        ("term_off", C.POINTER(C.c_uint64)), ("term_bytes", C.POINTER(C.c_uint8)),
        ("term_df", C.POINTER(C.c_uint32)),
    ]


class RunInfo(C.Structure):
    _fields_ = [
        ("size", C.c_uint64), ("nbytes", C.c_uint64), ("ntokens", C.c_uint64), ("npairs", C.c_uint64), ("nterms", C.c_uint32),
        ("nterms_global", C.c_uint32), ("nchunks", C.c_uint64), ("partial_records", C.c_uint64),
        ("ndocs", C.c_uint32), ("vocab_capacity", C.c_uint32), ("ms_total", C.c_double),
        ("ms_tokcount", C.c_double), ("ms_stage", C.c_double * 16), ("nstages", C.c_uint32), ("flags", C.c_uint32),
        ("device_allocs", C.c_uint64), ("device_alloc_bytes", C.c_uint64),
        ("idf_logs", C.c_uint64), ("ms_idf_host", C.c_double), ("ms_idf_wait", C.c_double),
    ]


class RunTotals(C.Structure):
    _fields_ = [("runs", C.c_uint64), ("ms_tokcount", C.c_double), ("ms_total", C.c_double),
                ("idf_logs", C.c_uint64), ("ms_idf_host", C.c_double), ("ms_idf_wait", C.c_double)]


class OutputInfo(C.Structure):
    _fields_ = [
        ("size", C.c_uint64), ("text_bytes", C.c_uint64), ("writers", C.c_uint32), ("formatted", C.c_uint32),
        ("ms_prepare", C.c_double), ("ms_d2h_busy", C.c_double), ("ms_write", C.c_double), ("ms_total", C.c_double),
    ]


class DirPlan(C.Structure):
    _fields_ = [
        ("ndocs", C.c_uint32), ("nshards", C.c_uint32), ("doc_ids", C.POINTER(C.c_uint32)),
        ("doc_bytes", C.POINTER(C.c_uint64)), ("shard_first", C.POINTER(C.c_uint32)),
        ("shard_bytes", C.POINTER(C.c_uint64)),
    ]


class IngestInfo(C.Structure):
    _fields_ = [
        ("nbytes", C.c_uint64), ("segments", C.c_uint64), ("ndocs", C.c_uint32), ("threads", C.c_uint32),
        ("ms_scan", C.c_double), ("ms_read", C.c_double), ("ms_total", C.c_double),
    ]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libtfidf_hip.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        L.tfidf_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.tfidf_close.argtypes = [C.c_void_p]
        L.tfidf_close.restype = None
        L.tfidf_strerror.restype = C.c_char_p
        L.tfidf_run.argtypes = [C.c_void_p, C.POINTER(Corpus)]
        L.tfidf_fetch.argtypes = [C.c_void_p, C.POINTER(Result)]
        L.tfidf_result_free.argtypes = [C.POINTER(Result)]
        L.tfidf_result_free.restype = None
        L.tfidf_last_run_info.argtypes = [C.c_void_p, C.POINTER(RunInfo)]
        L.tfidf_run_totals_get.argtypes = [C.c_void_p, C.POINTER(RunTotals), C.c_int]
        L.tfidf_alloc_stats.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.tfidf_stage_name.restype = C.c_char_p
        L.tfidf_set_timing.argtypes = [C.c_void_p, C.c_int]
        L.tfidf_comm_unique_id.argtypes = [C.c_void_p]
        L.tfidf_comm_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.tfidf_write_output.argtypes = [C.POINTER(Result), C.c_char_p]
        L.tfidf_format.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.tfidf_copy_text.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        L.tfidf_write_output_gpu.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.tfidf_last_output_info.argtypes = [C.c_void_p, C.POINTER(OutputInfo)]
        L.tfidf_format_f64.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.tfidf_synth_host.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint32, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]
        L.tfidf_synth_device.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_uint32, C.c_uint64, C.POINTER(Corpus)]
        L.tfidf_ingest_dir_device.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.POINTER(Corpus),
                                              C.POINTER(C.c_uint32), C.POINTER(IngestInfo)]
        L.tfidf_hbm_probe.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.tfidf_group_open.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]
        L.tfidf_group_size.argtypes = [C.c_void_p]
        L.tfidf_group_ctx.argtypes = [C.c_void_p, C.c_int]
        L.tfidf_group_ctx.restype = C.c_void_p
        L.tfidf_group_run.argtypes = [C.c_void_p, C.c_void_p]
        L.tfidf_group_write_output.argtypes = [C.c_void_p, C.c_char_p]
        L.tfidf_group_close.argtypes = [C.c_void_p]
        L.tfidf_group_close.restype = None
        L.tfidf_plan_dir.argtypes = [C.c_char_p, C.c_uint32, C.c_int, C.POINTER(DirPlan), C.POINTER(C.c_uint32)]
        L.tfidf_plan_free.argtypes = [C.POINTER(DirPlan)]
        L.tfidf_plan_free.restype = None
        L.tfidf_ingest_shard_device.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(DirPlan), C.c_uint32, C.c_int,
                                                C.POINTER(Corpus), C.POINTER(C.c_uint32), C.POINTER(IngestInfo)]
        L.tfidf_doc_name_order.argtypes = [C.c_uint32, C.c_void_p]
        L.tfidf_shard_split.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        if L.tfidf_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH}: ABI version {L.tfidf_abi_version()}, binding expects {ABI_VERSION} "
                               f"(stale build: rebuild with __graft_entry__.build())")
        _lib = L
    return _lib


class TfidfError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what}: {lib().tfidf_strerror(rc).decode()} ({rc})")
        self.rc = rc


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise TfidfError(rc, what)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def synth_host(seed: int, V: int, mode: int, cdf, doc_ids, ntok):
    """Host generation (csrc/synth.h).  Returns (bytes uint8, doc_off uint64)."""
    ntok = np.ascontiguousarray(ntok, dtype=np.uint64)
    ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint32)
    cdf = None if cdf is None else np.ascontiguousarray(cdf, dtype=np.float64)
    n = C.c_uint64(0)
    _chk(lib().tfidf_synth_host(seed, V, mode, _ptr(cdf), _ptr(ids), _ptr(ntok), len(ntok), None, C.byref(n), None),
         "synth size")
    buf = np.empty(max(int(n.value), 1), dtype=np.uint8)
    off = np.empty(len(ntok) + 1, dtype=np.uint64)
    _chk(lib().tfidf_synth_host(seed, V, mode, _ptr(cdf), _ptr(ids), _ptr(ntok), len(ntok), _ptr(buf), C.byref(n),
                                _ptr(off)), "synth")
    return buf[: int(n.value)], off


class Engine:
    """One GPU context (one HIP stream; optional RCCL communicator)."""

    def __init__(self, device: int = 0, handle=None):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _chk(lib().tfidf_open(device, C.byref(h)), "tfidf_open")
            handle = h
        self.h = handle if isinstance(handle, C.c_void_p) else C.c_void_p(handle)
        self._keep = None

    def close(self):
        if self.h and self._owned:
            lib().tfidf_close(self.h)
        self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_timing(self, on):
        """True / 1: every stage; 2: K1 and the whole run only; False / 0: none"""
        lvl = 2 if (on == 2 and on is not True) else (1 if on else 0)
        _chk(lib().tfidf_set_timing(self.h, lvl), "set_timing")

    def comm_init(self, uid: bytes, rank: int, nranks: int):
        buf = (C.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(uid)
        _chk(lib().tfidf_comm_init(self.h, buf, rank, nranks), "tfidf_comm_init")

    def run_host(self, data: np.ndarray, doc_off: np.ndarray, doc_ids=None, ndocs_total: int = 0):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint32)
        c = Corpus()
        c.bytes = data.ctypes.data if len(data) else None
        c.nbytes = len(data)
        c.doc_off = doc_off.ctypes.data
        c.doc_ids = None if ids is None else ids.ctypes.data
        c.ndocs = len(doc_off) - 1
        c.flags = 0
        c.ndocs_total = ndocs_total
        self._keep = (data, doc_off, ids)
        _chk(lib().tfidf_run(self.h, C.byref(c)), "tfidf_run")

    def run_corpus(self, c: Corpus):
        _chk(lib().tfidf_run(self.h, C.byref(c)), "tfidf_run")

    def synth_device(self, seed, V, mode, cdf, doc_ids, ntok, ndocs_total=0) -> Corpus:
        ntok = np.ascontiguousarray(ntok, dtype=np.uint64)
        ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint32)
        cdf = None if cdf is None else np.ascontiguousarray(cdf, dtype=np.float64)
        c = Corpus()
        _chk(lib().tfidf_synth_device(self.h, seed, V, mode, _ptr(cdf), _ptr(ids), _ptr(ntok), len(ntok),
                                      ndocs_total, C.byref(c)), "tfidf_synth_device")
        return c

    def ingest_dir(self, path: str, threads: int = 0):
        """input/doc1..N streamed into HBM (tfidf_ingest_dir_device).  Returns (Corpus, info);
        raises TfidfError (rc -6 / -7, `bad_doc` attribute set for -7) like the reference."""
        c, bad, ii = Corpus(), C.c_uint32(0), IngestInfo()
        rc = lib().tfidf_ingest_dir_device(self.h, path.encode(), threads, C.byref(c), C.byref(bad), C.byref(ii))
        if rc:
            e = TfidfError(rc, "tfidf_ingest_dir_device")
            e.bad_doc, e.ndocs = bad.value, c.ndocs
            raise e
        return c, {k: getattr(ii, k) for k, _ in IngestInfo._fields_}

    def hbm_probe(self, nbytes: int = 2 << 30, iters: int = 10) -> dict:
        """Measured streaming read / copy GB/s of this device (tfidf_hbm_probe)."""
        r, c = C.c_double(0), C.c_double(0)
        _chk(lib().tfidf_hbm_probe(self.h, nbytes, iters, C.byref(r), C.byref(c)), "tfidf_hbm_probe")
        return {"read_GBps": r.value, "copy_GBps": c.value}

    def corpus_bytes(self, c: Corpus) -> np.ndarray:
        """Device corpus bytes copied back to the host (test plumbing)."""
        out = np.empty(c.nbytes, dtype=np.uint8)
        hip = C.CDLL("libamdhip64.so.7")
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        if c.nbytes and hip.hipMemcpy(out.ctypes.data, c.bytes, c.nbytes, 2) != 0:
            raise RuntimeError("hipMemcpy D2H failed")
        off = np.empty(c.ndocs + 1, dtype=np.uint64)
        if hip.hipMemcpy(off.ctypes.data, c.doc_off, off.nbytes, 2) != 0:
            raise RuntimeError("hipMemcpy D2H failed")
        return out, off

    def alloc_counters(self):
        """(device allocations, bytes) the library has made in this process so far."""
        a, b = C.c_uint64(), C.c_uint64()
        _chk(lib().tfidf_alloc_stats(C.byref(a), C.byref(b)), "tfidf_alloc_stats")
        return int(a.value), int(b.value)

    def totals(self, reset: bool = False) -> dict:
        """sums over the successful runs since the last reset (tfidf_run_totals_get)"""
        t = RunTotals()
        _chk(lib().tfidf_run_totals_get(self.h, C.byref(t), 1 if reset else 0), "tfidf_run_totals_get")
        return {k: getattr(t, k) for k, _ in RunTotals._fields_}

    def info(self) -> dict:
        r = RunInfo()
        r.size = C.sizeof(RunInfo)
        _chk(lib().tfidf_last_run_info(self.h, C.byref(r)), "tfidf_last_run_info")
        d = {k: getattr(r, k) for k, _ in RunInfo._fields_ if k not in ("ms_stage", "size")}
        d["stages"] = {lib().tfidf_stage_name(i).decode(): r.ms_stage[i] for i in range(r.nstages)}
        return d

    def format_bytes(self) -> int:
        """Formats the last run's lines on the GPU; returns the text size."""
        n = C.c_uint64(0)
        _chk(lib().tfidf_format(self.h, C.byref(n)), "tfidf_format")
        return int(n.value)

    def text(self) -> bytes:
        """output.txt bytes formatted on the GPU (tfidf_format + tfidf_copy_text)."""
        n = C.c_uint64(0)
        _chk(lib().tfidf_format(self.h, C.byref(n)), "tfidf_format")
        buf = np.empty(int(n.value), dtype=np.uint8)
        if n.value:
            _chk(lib().tfidf_copy_text(self.h, 0, buf.ctypes.data, n.value), "tfidf_copy_text")
        return buf.tobytes()

    def write_output(self, path: str, append: bool = False):
        _chk(lib().tfidf_write_output_gpu(self.h, path.encode(), 1 if append else 0), "tfidf_write_output_gpu")

    def output_info(self) -> dict:
        """Timings of the last write_output (tfidf_last_output_info)."""
        o = OutputInfo()
        o.size = C.sizeof(OutputInfo)
        _chk(lib().tfidf_last_output_info(self.h, C.byref(o)), "tfidf_last_output_info")
        return {k: getattr(o, k) for k, _ in OutputInfo._fields_ if k != "size"}

    def format_f64(self, vals) -> list:
        """The device %.16f formatter on host doubles (tests)."""
        v = np.ascontiguousarray(vals, dtype=np.float64)
        out = np.zeros(v.size * 32, dtype=np.uint8)
        _chk(lib().tfidf_format_f64(self.h, v.ctypes.data, v.size, out.ctypes.data), "tfidf_format_f64")
        return [bytes(out[i * 32:(i + 1) * 32]).rstrip(b"\0") for i in range(v.size)]

    @contextlib.contextmanager
    def fetched(self):
        """The last run's result as numpy views of the library's host arrays (tfidf_fetch
        without copies and without the text; valid inside the with block): for full-size
        runs whose pairs do not fit twice in host memory."""
        r = Result()
        _chk(lib().tfidf_fetch(self.h, C.byref(r)), "tfidf_fetch")
        try:
            P, N, V = int(r.npairs), int(r.ndocs), int(r.nterms)

            def view(p, n):
                return np.ctypeslib.as_array(p, shape=(n,)) if n else np.zeros(0, dtype=np.uint8)

            yield {
                "npairs": P, "ndocs": N, "nterms": V, "ndocs_total": int(r.ndocs_total),
                "doc": view(r.pair_doc, P), "term": view(r.pair_term, P), "count": view(r.pair_count, P),
                "docsize": view(r.pair_docsize, P), "df": view(r.pair_df, P), "score": view(r.pair_score, P),
                "doc_id": view(r.doc_id, N), "doc_size": view(r.doc_size, N), "term_df": view(r.term_df, V),
                "term_off": view(r.term_off, V + 1),
                "term_bytes": view(r.term_bytes, int(r.term_off[V]) if V else 0),
            }
        finally:
            lib().tfidf_result_free(C.byref(r))

    def fetch(self) -> dict:
        r = Result()
        _chk(lib().tfidf_fetch(self.h, C.byref(r)), "tfidf_fetch")
        try:
            P, N, V = int(r.npairs), int(r.ndocs), int(r.nterms)

            def arr(p, n, dt):
                if n == 0:
                    return np.zeros(0, dtype=dt)
                return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)

            out = {
                "npairs": P, "ndocs": N, "nterms": V, "ndocs_total": int(r.ndocs_total),
                "doc": arr(r.pair_doc, P, np.uint32), "term": arr(r.pair_term, P, np.uint32),
                "count": arr(r.pair_count, P, np.uint32), "docsize": arr(r.pair_docsize, P, np.uint32),
                "df": arr(r.pair_df, P, np.uint32), "score": arr(r.pair_score, P, np.float64),
                "doc_id": arr(r.doc_id, N, np.uint32), "doc_size": arr(r.doc_size, N, np.uint32),
                "term_df": arr(r.term_df, V, np.uint32),
            }
            toff = arr(r.term_off, V + 1, np.uint64)
            tb = bytes(arr(r.term_bytes, int(toff[-1]) if V else 0, np.uint8))
            out["terms"] = [tb[int(toff[i]):int(toff[i + 1])] for i in range(V)]
            out["output_txt"] = format_lines(out)
            return out
        finally:
            lib().tfidf_result_free(C.byref(r))


class Group:
    """Several shards in this process (tfidf_group_*): rank r on devices[r]; RCCL when
    every rank has its own GPU, the in-process transport when a device is shared (or
    local=True).  Every run is collective over all ranks."""

    def __init__(self, nranks: int, devices=None, local: bool = False):
        dev = None if devices is None else (C.c_int * nranks)(*devices)
        h = C.c_void_p()
        _chk(lib().tfidf_group_open(nranks, dev, TFIDF_GROUP_LOCAL if local else 0, C.byref(h)), "tfidf_group_open")
        self.h = h
        self.n = nranks
        self.ranks = [Engine(handle=lib().tfidf_group_ctx(h, r)) for r in range(nranks)]
        self._keep = None

    def close(self):
        if self.h:
            lib().tfidf_group_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def run(self, shards):
        """shards: list of Corpus (one per rank)."""
        arr = (Corpus * self.n)(*shards)
        _chk(lib().tfidf_group_run(self.h, arr), "tfidf_group_run")

    def run_host(self, shards):
        """shards: list of (data, doc_off, doc_ids, ndocs_total) host arrays, one per rank."""
        cs, keep = [], []
        for data, off, ids, nt in shards:
            data = np.ascontiguousarray(data, dtype=np.uint8)
            off = np.ascontiguousarray(off, dtype=np.uint64)
            ids = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
            c = Corpus()
            c.bytes = data.ctypes.data if len(data) else None
            c.nbytes = len(data)
            c.doc_off = off.ctypes.data
            c.doc_ids = None if ids is None else ids.ctypes.data
            c.ndocs = len(off) - 1
            c.flags = 0
            c.ndocs_total = nt
            cs.append(c)
            keep.append((data, off, ids))
        self._keep = keep
        self.run(cs)

    def write_output(self, path: str):
        _chk(lib().tfidf_group_write_output(self.h, path.encode()), "tfidf_group_write_output")


def plan_dir(path: str, nshards: int, threads: int = 0) -> dict:
    """tfidf_plan_dir: byte-balanced "docN@"-ordered shards of an input directory."""
    p, bad = DirPlan(), C.c_uint32(0)
    rc = lib().tfidf_plan_dir(path.encode(), nshards, threads, C.byref(p), C.byref(bad))
    if rc:
        e = TfidfError(rc, "tfidf_plan_dir")
        e.bad_doc, e.ndocs = bad.value, p.ndocs
        raise e
    try:
        N = int(p.ndocs)
        ids = np.ctypeslib.as_array(p.doc_ids, shape=(N,)).copy() if N else np.zeros(0, np.uint32)
        nb = np.ctypeslib.as_array(p.doc_bytes, shape=(N,)).copy() if N else np.zeros(0, np.uint64)
        first = np.ctypeslib.as_array(p.shard_first, shape=(nshards + 1,)).copy()
        sb = np.ctypeslib.as_array(p.shard_bytes, shape=(nshards,)).copy()
        return {"ndocs": N, "doc_ids": ids, "doc_bytes": nb, "shard_first": first, "shard_bytes": sb}
    finally:
        lib().tfidf_plan_free(C.byref(p))


def doc_name_order(n: int) -> np.ndarray:
    out = np.zeros(max(n, 1), dtype=np.uint32)
    _chk(lib().tfidf_doc_name_order(n, out.ctypes.data), "tfidf_doc_name_order")
    return out[:n]


def shard_split(sizes, nshards: int) -> np.ndarray:
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    first = np.zeros(nshards + 1, dtype=np.uint32)
    _chk(lib().tfidf_shard_split(sizes.ctypes.data if len(sizes) else None, len(sizes), nshards, first.ctypes.data),
         "tfidf_shard_split")
    return first


def format_lines(res: dict) -> bytes:
    """output.txt bytes ("docN@word\\t%.16f\\n", TFIDF.c:245,281) from a fetched result."""
    terms = res["terms"]
    parts = []
    for d, t, s in zip(res["doc"].tolist(), res["term"].tolist(), res["score"].tolist()):
        parts.append(b"doc%d@" % d + terms[t] + b"\t%.16f\n" % s)
    return b"".join(parts)


def device_count() -> int:
    """Visible HIP devices (tfidf_device_count; 0 without a GPU)."""
    return int(lib().tfidf_device_count())


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * UNIQUE_ID_BYTES)()
    _chk(lib().tfidf_comm_unique_id(buf), "tfidf_comm_unique_id")
    return bytes(buf)
