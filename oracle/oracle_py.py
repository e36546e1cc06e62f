"""ctypes binding of the oracle restatement (oracle/tfidf_oracle.c -> _build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker or the CPU baseline, never by the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
CLI = os.path.join(HERE, "_build", "tfidf_oracle")


class OracleOut(C.Structure):
    _fields_ = [
        ("npairs", C.c_uint64), ("nterms", C.c_uint32), ("ndocs", C.c_uint32),
        ("doc_id", C.POINTER(C.c_uint32)), ("term", C.POINTER(C.c_uint32)), ("count", C.POINTER(C.c_uint32)),
        ("docsize", C.POINTER(C.c_uint32)), ("df", C.POINTER(C.c_uint32)), ("score", C.POINTER(C.c_double)),
        ("term_off", C.POINTER(C.c_uint64)), ("term_pool", C.POINTER(C.c_char)),
        ("lines", C.POINTER(C.c_char)), ("lines_len", C.c_uint64),
        ("tf_jobs", C.POINTER(C.c_char)), ("tf_len", C.c_uint64),
        ("idf_jobs", C.POINTER(C.c_char)), ("idf_len", C.c_uint64),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(OracleOut)]
        L.oracle_free.argtypes = [C.POINTER(OracleOut)]
        L.oracle_free.restype = None
        L.oracle_run_sharded.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64)]
        L.oracle_free_text.argtypes = [C.c_void_p]
        L.oracle_free_text.restype = None
        _lib = L
    return _lib


def run(data: np.ndarray, doc_off: np.ndarray, doc_ids=None, n_total: int = 0, arrays: bool = True) -> dict:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint32)
    o = OracleOut()
    lib().oracle_run(data.ctypes.data if len(data) else None, doc_off.ctypes.data, len(doc_off) - 1,
                     None if ids is None else ids.ctypes.data, n_total, C.byref(o))
    try:
        P, V = int(o.npairs), int(o.nterms)
        res = {"npairs": P, "nterms": V, "output_txt": C.string_at(o.lines, o.lines_len),
               "tf_jobs": C.string_at(o.tf_jobs, o.tf_len), "idf_jobs": C.string_at(o.idf_jobs, o.idf_len)}
        if arrays:
            def arr(p, n, dt):
                return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dt)
            res.update(doc=arr(o.doc_id, P, np.uint32), term=arr(o.term, P, np.uint32),
                       count=arr(o.count, P, np.uint32), docsize=arr(o.docsize, P, np.uint32),
                       df=arr(o.df, P, np.uint32), score=arr(o.score, P, np.float64))
            toff = arr(o.term_off, V + 1, np.uint64)
            pool = C.string_at(o.term_pool, int(toff[-1])) if V else b""
            res["terms"] = [pool[int(toff[i]):int(toff[i + 1])] for i in range(V)]
        return res
    finally:
        lib().oracle_free(C.byref(o))


def run_sharded(data: np.ndarray, doc_off: np.ndarray, doc_ids, n_total: int, order: np.ndarray,
                first: np.ndarray) -> tuple:
    """The CPU baseline of the multi-worker path (oracle_run_sharded): one host thread per
    shard (documents order[first[s]:first[s+1]]), DF combine, per-shard sort, shard-order
    concatenation.  Returns (output.txt bytes, pairs)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint32)
    order = np.ascontiguousarray(order, dtype=np.uint32)
    first = np.ascontiguousarray(first, dtype=np.uint32)
    txt, n, npairs = C.c_void_p(), C.c_uint64(), C.c_uint64()
    lib().oracle_run_sharded(data.ctypes.data if len(data) else None, doc_off.ctypes.data,
                             None if ids is None else ids.ctypes.data, n_total, order.ctypes.data,
                             first.ctypes.data, len(first) - 1, C.byref(txt), C.byref(n), C.byref(npairs))
    try:
        return C.string_at(txt, n.value), int(npairs.value)
    finally:
        lib().oracle_free_text(txt)
