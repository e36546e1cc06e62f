"""Debug aid: small crafted corpora through two K1 kernels; prints terms per document."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"), os.path.join(REPO, "tests")]
import tfidf_abi  # noqa: E402
from helpers import docs_to_arrays  # noqa: E402

CASES = [
    [b"a\x01 a a\n", b"\xc2\xa0x x\n", b"ab cd ab zz\n", b"", b"a\x01 zz\n"],
    [b"a\x01 a a\n", b"\xc2\xa0x x\n", b"ab\x00cd ab zz\n", b"a\x01 zz\n"],
    [b"a\x01 a a\n", b"\xc2\xa0x x\n", b"ab\x00cd ab zz\n", b"", b"a\x01 zz\n"],
    [b"ab\x00cd zz\n", b"zz\n"],
    [b"aa bb\n", b"", b"cc dd\n"],
    [b"q w e r t y\n", b"q w\n"],
]


def run(mode, data, off):
    os.environ["TFIDF_K1"] = mode
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off)
        r = e.fetch()
    by = {}
    for d, t, c in zip(r["doc"].tolist(), r["term"].tolist(), r["count"].tolist()):
        by.setdefault(d, []).append((r["terms"][t], c))
    return by, r["doc_size"].tolist()


for i, docs in enumerate(CASES):
    data, off = docs_to_arrays(docs)
    a = run("st", data, off)
    b = run("sl", data, off)
    print(i, "SAME" if a == b else "DIFF")
    if a != b:
        print("   st", a)
        print("   sl", b)
