"""Ad-hoc GPU diagnostics (not collected by pytest): python tests/debug_gpu.py <what>"""
import sys
import os

sys.path[:0] = [os.path.join(os.path.dirname(__file__), d) for d in
                ("../parallel-systems-mpi-tfidf_amd/python", "../oracle", ".")]
import numpy as np  # noqa: E402

import oracle_py  # noqa: E402
import tfidf_abi  # noqa: E402
import tfidf_configs  # noqa: E402


def dup_report(res, tag):
    terms = res["terms"]
    seen = {}
    dups = [t for t in terms if t in seen or seen.setdefault(t, 0)]
    print(tag, "nterms", len(terms), "distinct strings", len(set(terms)), "dup examples", dups[:5])
    d, t = res["doc"], res["term"]
    same = np.flatnonzero((d[1:] == d[:-1]) & (t[1:] == t[:-1]))
    print(tag, "adjacent duplicate (doc,term) records:", len(same), same[:5])


def c2_small():
    p = tfidf_configs.plan("c2", scale=0.003)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        print(e.info())
        res = e.fetch()
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    dup_report(res, "gpu")
    print("oracle pairs", ora["npairs"], "gpu pairs", res["npairs"], "oracle nterms", ora["nterms"])
    # per-doc count sums vs docsize
    for name, r in (("gpu", res), ("ora", ora)):
        starts = np.flatnonzero(np.r_[True, r["doc"][1:] != r["doc"][:-1]])
        sums = np.add.reduceat(r["count"].astype(np.int64), starts)
        bad = np.flatnonzero(sums != r["docsize"][starts])
        print(name, "docs with count-sum != docsize:", [(int(r["doc"][starts[b]]), int(sums[b]),
                                                         int(r["docsize"][starts[b]])) for b in bad[:5]])
    # where are the 'aagt' records of doc106
    for name, r in (("gpu", res), ("ora", ora)):
        idx = [i for i in np.flatnonzero(r["doc"] == 106) if r["terms"][r["term"][i]] == b"aagt"]
        print(name, "doc106 aagt records", [(int(i), int(r["term"][i]), int(r["count"][i])) for i in idx])


def rccl1():
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        e.comm_init(tfidf_abi.comm_unique_id(), 0, 1)
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        print(e.info())
        res = e.fetch()
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    print("rccl1 equal:", res["output_txt"] == ora["output_txt"])


if __name__ == "__main__":
    globals()[sys.argv[1]]()
