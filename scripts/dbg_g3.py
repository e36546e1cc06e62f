"""Debug aid: one golden case through two K1 kernels, per-pair results side by side."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"), os.path.join(REPO, "tests")]
import tfidf_abi  # noqa: E402
from helpers import load_golden  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "g3_bytes"
g = load_golden(case)
for mode in ("st", "sl"):
    os.environ["TFIDF_K1"] = mode
    with tfidf_abi.Engine(0) as e:
        e.run_host(g["data"], g["off"])
        r = e.fetch()
        print(mode, "flags", e.info()["flags"], "V", r["nterms"], "P", r["npairs"], "ok", r["output_txt"] == g["output"])
        print("  terms", r["terms"], "term_df", r["term_df"].tolist())
        print("  doc_size", r["doc_size"].tolist())
        for d, t, c, df, s in zip(r["doc"].tolist(), r["term"].tolist(), r["count"].tolist(), r["df"].tolist(),
                                  r["score"].tolist()):
            print("   ", d, r["terms"][t], c, df, s)
