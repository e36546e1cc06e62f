"""K1 phase cycles (diagnostic build lib/libtfidf_hip_stamps.so, tokcount_sl.hip SL_STAMPS):
per-wave average s_memtime cycles per phase, summed over three runs of one config.
Usage (GPU box): TFIDF_LIB=stamps TFIDF_STAMPS=1 python scripts/k1_stamps.py [config]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"))
import tfidf_abi  # noqa: E402
import tfidf_configs  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
p = tfidf_configs.plan(cfg)
L = tfidf_abi.lib()
L.tfidf_debug_k1_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
with tfidf_abi.Engine(0) as e:
    c = e.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
    for _ in range(3):
        e.run_corpus(c)
    info = e.info()
    buf = (C.c_uint64 * 32)()
    n = L.tfidf_debug_k1_stamps(e.h, buf, 32)
    v = list(buf)[:n]
names = ["chunk setup", "walk", "token list", "round build", "round finish", "last rounds", "chunk end",
         "flush wait", "flush writes", "flush counts", "flush alloc", "finish: load wait"]
NPH = len(names)
waves = v[NPH + 1] or 1
tot = sum(v[:NPH])
print(cfg, "K1 ms", round(info["ms_tokcount"], 4), "waves", waves, "chunk visits/wave", round(v[NPH] / waves, 1))
for k, nm in enumerate(names):
    print("  %-12s %10.0f cycles/wave  %5.1f %%" % (nm, v[k] / waves, 100.0 * v[k] / max(tot, 1)))
cnt = v[NPH + 2:NPH + 10]
if len(cnt) == 8 and cnt[4]:
    print("  rounds %d (per wave %.0f): with a slow lane %.1f %%, slow lanes/round %.2f, lost claims/round %.2f,"
          " still slow after the inline retry %.1f %% (SL_RETRY builds)" %
          (cnt[4], cnt[4] / waves, 100.0 * cnt[0] / cnt[4], cnt[1] / cnt[4], cnt[2] / cnt[4], 100.0 * cnt[3] / cnt[4]))
    print("  lanes still slow per round: lost every retry %.3f, bucket full %.3f, overflow mode %.3f" %
          (cnt[5] / cnt[4], cnt[6] / cnt[4], cnt[7] / cnt[4]))
