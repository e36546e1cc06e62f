#!/usr/bin/env python3
"""bench.py — TF-IDF hot path throughput on MI355X (BASELINE.json metric: corpus GB/s and
TF-IDF pairs/s at 1/2/4/8 GPUs; % of HBM peak).

A step = one full pass of the hot path (tokenize -> per-document TF -> vocabulary -> DF
[RCCL all-gather + all-reduce across ranks] -> idf -> tf*idf -> output order) over one
batch: the config-2 corpus (1e5 synthetic Zipfian documents, V = 5e4, ~1 GB) resident in
HBM.  Multi-GPU is weak scaling: every rank owns one config-2-sized shard of a corpus of
N x 1e5 documents (contiguous "docN" strcmp ranges; idf uses the global N).

    python bench.py [--gpus N --steps K --warmup W]      (N > 1: one process, N GPUs, tfidf_group)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one process per GPU)

Rank 0 prints one JSON line.  `roofline` is priced on the dominant kernel (K1
tokenize+count), algorithmic bytes per launch = C + 12*P, divided by K1's
average duration measured with HIP events on the engine's stream inside the timed steps.
`roofline.measured_read_peak` / `measured_copy_peak` are this device's streaming read and
copy rates (tfidf_hbm_probe, 2 GiB, outside the timed region).
`cpu_baseline` (N = 1 only) times the oracle restatement on the host cores (one thread per document
shard, OMP_NUM_THREADS = 16 threads on the GPU box) on a bounded sample, with a
single-thread leg alongside.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"))

import numpy as np  # noqa: E402

import tfidf_abi  # noqa: E402  (loads libtfidf_hip.so before torch: one HIP runtime)
import tfidf_configs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)


def hip_device_sync():
    hip = C.CDLL("libamdhip64.so.7")
    if hip.hipDeviceSynchronize() != 0:
        raise RuntimeError("hipDeviceSynchronize failed")


K1_SOURCES = {"k_tokcount_sl": "tokcount_sl.hip", "k_tokcount_vs": "tokcount_vs.hip",
              "k_tokcount": "tokcount.hip"}


def k1_kernel(flags: int) -> str:
    """The tokenize+count kernel the last run used (tfidf_run_info.flags)."""
    if flags & tfidf_abi.RUN_K1_SL:
        return "k_tokcount_sl"
    return "k_tokcount_vs" if flags & tfidf_abi.RUN_K1_VS else "k_tokcount"


def k1_source_sha(kernel: str) -> str:
    """Digest of the K1 source: a committed PMC figure is valid only for the kernel it was
    measured on."""
    import hashlib
    with open(os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "csrc", K1_SOURCES[kernel]), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(cfg: str, strong: bool, ngpu: int, kernel: str):
    """HBM bytes per K1 launch from the committed rocprofv3 PMC passes of THIS config, THIS
    K1 kernel and THIS source (profiles/k1_pmc_traffic.json, written by
    scripts/traffic_k1.py), or None: never another config's or kernel's figure."""
    p = os.path.join(REPO, "profiles", "k1_pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        tab = json.load(f)
    key = f"{cfg}{'_strong' if strong else ''}_g{ngpu}" if ngpu > 1 else cfg
    e = tab.get(key) if isinstance(tab, dict) else None
    if not isinstance(e, dict) or e.get("kernel") != kernel or e.get("k1_source_sha") != k1_source_sha(kernel):
        return None, None
    return e.get("hbm_bytes_per_launch"), e.get("source")


def host_cpu_info() -> dict:
    """What the CPU baseline ran on: the CPU model, nproc, this process's affinity and the
    cgroup CPU quota (the box's share of a larger machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": aff, "cgroup_cpus": quota}


def cpu_baseline(cfg: str, ndocs_sample: int, threads: int, info: dict):
    """The oracle restatement (C, oracle/tfidf_oracle.c) timed on the host cores.

    Multi-core leg (the reported value): the reference's worker structure
    on `threads` host threads — the sample's documents in "docN@" order cut into one
    byte-balanced shard per thread; each thread tokenizes and counts its shard, the DF
    tables are combined (CustomReduce + Bcast), each thread scores, formats and sorts its
    lines, and the texts are concatenated in shard order (the gather).  All of it is in
    the timed region (oracle_run_sharded).  Single-thread leg: oracle_run over a sixteenth
    of the sample."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py  # oracle: CPU baseline only (never the measured GPU path)
    p = tfidf_configs.plan(cfg)
    n = min(ndocs_sample, len(p["doc_ids"]))
    ids, ntok = p["doc_ids"][:n], p["ntok"][:n]
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], ids, ntok)
    order = np.argsort(tfidf_configs.doc_name_key(ids), kind="stable").astype(np.uint32)
    first = tfidf_configs.shard_cuts(np.diff(off.astype(np.int64))[order], threads)
    oracle_py.lib()
    t0 = time.perf_counter()
    _, pairs = oracle_py.run_sharded(data, off, ids, p["ndocs_total"], order, first)
    dt = time.perf_counter() - t0
    n1 = max(1, n // 16)
    o1 = off[: n1 + 1]
    d1 = data[: int(o1[-1])]
    t1 = time.perf_counter()
    p1 = oracle_py.run(d1, o1, ids[:n1], p["ndocs_total"], arrays=False)["npairs"]
    dt1 = time.perf_counter() - t1
    out = {"value": round(len(data) / dt / 1e9, 6), "unit": "GB/s", "cores": threads, "kind": "port",
           "sample": f"oracle/tfidf_oracle.c (C restatement of TFIDF.c) on the first {n} documents of {cfg} "
                     f"({len(data) / 1e6:.1f} MB, {pairs} pairs): {threads} host threads, one byte-balanced "
                     f"docN@-ordered shard each; tokenize+count, DF combine, score+format+sort, shard-order "
                     f"concatenation all timed; {dt:.2f} s wall",
           "pairs_per_s": round(pairs / dt, 1),
           "single_thread": {"value": round(len(d1) / dt1 / 1e9, 6), "unit": "GB/s", "cores": 1,
                             "sample": f"first {n1} documents ({len(d1) / 1e6:.1f} MB, {p1} pairs); {dt1:.2f} s",
                             "pairs_per_s": round(p1 / dt1, 1)}}
    out.update(info)
    return out


def main_shards(args):
    """K shards of one config on one GPU through tfidf_group (LocalXport): the exchange
    stage (key all-gather by device copies, union sort, DF all-reduce) at K ranks."""
    K = args.shards
    g = tfidf_abi.Group(K, devices=[0] * K)
    corpora, plans = [], []
    for r in range(K):
        p = tfidf_configs.plan(args.config, scale=args.scale, rank=r, nranks=K, weak=False)
        plans.append(p)
        corpora.append(g.ranks[r].synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"],
                                               p["ndocs_total"]))
        g.ranks[r].set_timing(True)
    hip_device_sync()
    tc = time.perf_counter()
    g.run(corpora)
    hip_device_sync()
    cold_ms = (time.perf_counter() - tc) * 1e3
    for _ in range(max(0, args.warmup - 1)):
        g.run(corpora)
    hip_device_sync()
    a0 = g.ranks[0].alloc_counters()
    steps = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.run(corpora)
        steps.append([e.info() for e in g.ranks])
    hip_device_sync()
    elapsed = time.perf_counter() - t0
    a1 = g.ranks[0].alloc_counters()
    infos = steps[-1]
    C_all = sum(i["nbytes"] for i in infos)
    P_all = sum(i["npairs"] for i in infos)
    stage_names = list(infos[0]["stages"].keys())
    # per step: the slowest rank's time of each stage (the ranks meet in the exchange)
    st_max = {k: float(np.mean([max(i["stages"][k] for i in st) for st in steps])) for k in stage_names}
    # the rank that reaches the exchange last waits least in it: its exchange stage is the
    # exchange's own work (collectives, owner aggregation) without the stragglers' wait
    xmin = float(np.mean([min(i["stages"].get("exchange", 0.0) for i in st) for st in steps]))
    line = {
        "metric": "corpus GB/s (TF-IDF hot path, K shards on one GPU: multi-rank path incl. the DF exchange)",
        "value": round(C_all * args.steps / elapsed / 1e9, 4),
        "unit": "GB/s",
        "n_gpus": 1,
        "shards": K,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "data": "synthetic (device-generated Zipfian corpus), resident in HBM",
        "config": {"workload": f"{args.config} x{args.scale}: {sum(len(p['doc_ids']) for p in plans)} docs in {K} "
                               f"shards, V={plans[0]['V']}, {C_all / 1e9:.3f} GB, {P_all} pairs",
                   "parallelism": f"{K} ranks on 1 GPU (in-process transport: the key all-gather and DF "
                                  f"all-reduce are device copies; xGMI time excluded)"},
        "stage_ms_max_over_ranks_mean": {k: round(v, 4) for k, v in st_max.items()},
        "exchange_ms": round(st_max.get("exchange", 0.0), 4),
        "exchange_ms_min_over_ranks": round(xmin, 4),
        "exchange_frac_of_step": round(st_max.get("exchange", 0.0) / (elapsed / args.steps * 1e3), 4),
        "exchange_mode": "dense all-reduce" if infos[0]["flags"] & tfidf_abi.RUN_XCHG_DENSE else "hash-owner all-to-all",
        "nterms_global": int(infos[0]["nterms_global"]),
        "nterms_per_rank": [int(i["nterms"]) for i in infos],
        "device_allocs_in_timed_steps": a1[0] - a0[0],
        "cold_run_ms": round(cold_ms, 3),
        "note": "ranks run concurrently on one GPU (host thread each); a rank's stage times include waiting "
                "for its peers at the exchange (exchange_ms: the slowest rank's, i.e. with the wait for the last "
                "rank's local stages; exchange_ms_min_over_ranks: the last-arriving rank's)",
    }
    print(json.dumps(line), flush=True)
    g.close()


def main_group(args):
    """`--gpus N` without a launcher: ONE process drives N GPUs through tfidf_group (rank r
    on device r, one host thread per rank, the RCCL clique of ncclCommInitAll over xGMI;
    group.cpp).  The same engine path as one process per GPU under torch.distributed.run;
    exits non-zero when fewer than N GPUs are visible instead of measuring fewer."""
    N = args.gpus
    have = tfidf_abi.device_count()
    if have < N:
        print(f"bench.py: --gpus {N} needs {N} visible GPUs, found {have}", file=sys.stderr)
        sys.exit(2)
    g = tfidf_abi.Group(N, devices=list(range(N)))
    plans, corpora = [], []
    for r in range(N):
        p = tfidf_configs.plan(args.config, scale=args.scale, rank=r, nranks=N, weak=not args.strong,
                               vocab=args.vocab)
        plans.append(p)
        corpora.append(g.ranks[r].synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"],
                                               p["ndocs_total"]))
        g.ranks[r].set_timing(True)
    hip_device_sync_all(N)
    a0 = g.ranks[0].alloc_counters()
    tc = time.perf_counter()
    g.run(corpora)
    hip_device_sync_all(N)
    cold_ms = (time.perf_counter() - tc) * 1e3
    for _ in range(max(0, args.warmup - 1)):
        g.run(corpora)
    hip_device_sync_all(N)
    a1 = g.ranks[0].alloc_counters()
    steps = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.run(corpora)   # returns when every rank's run is done (one host thread per rank, joined)
        steps.append([e.info() for e in g.ranks])
    hip_device_sync_all(N)
    elapsed = time.perf_counter() - t0
    a2 = g.ranks[0].alloc_counters()
    infos = steps[-1]
    C_all = float(sum(i["nbytes"] for i in infos))
    P_all = float(sum(i["npairs"] for i in infos))
    T_all = float(sum(i["ntokens"] for i in infos))
    names = list(infos[0]["stages"].keys())
    st_max = {k: float(np.mean([max(i["stages"][k] for i in st) for st in steps])) for k in names}
    xmin = float(np.mean([min(i["stages"].get("exchange", 0.0) for i in st) for st in steps]))
    k1 = [i["ms_tokcount"] for st in steps for i in st]
    i0 = infos[0]
    kern = k1_kernel(int(i0["flags"]))
    alg0 = i0["nbytes"] + 12.0 * i0["npairs"]
    k1_r0 = float(np.mean([st[0]["ms_tokcount"] for st in steps]))
    achieved = alg0 / (k1_r0 * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.config, args.strong, N, kern)
    ms_step = elapsed / args.steps * 1e3
    line = {
        "metric": "corpus GB/s (TF-IDF hot path: tokenize->TF->DF->tf*idf->ordered output)",
        "value": round(C_all * args.steps / elapsed / 1e9, 4),
        "unit": "GB/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 (f64 score)",
        "data": "synthetic (device-generated Zipfian corpus, csrc/synth.h), resident in HBM",
        "config": {"workload": f"{args.config}: {sum(len(p['doc_ids']) for p in plans)} docs over {N} GPUs, "
                               f"V={plans[0]['V']}, {C_all / 1e9:.3f} GB, {int(P_all)} pairs",
                   "docs_total": int(plans[0]["ndocs_total"]), "corpus_bytes_total": int(C_all),
                   "parallelism": f"doc-shard x{N}, one process (tfidf_group: RCCL clique, DF exchange over "
                                  f"xGMI)"},
        "pairs_per_s": round(P_all * args.steps / elapsed, 1),
        "tokens_per_s": round(T_all * args.steps / elapsed, 1),
        "launcher": "in-process group (tfidf_group_open -> ncclCommInitAll)",
        "stage_ms_max_over_ranks_mean": {k: round(v, 4) for k, v in st_max.items()},
        "exchange_ms": round(st_max.get("exchange", 0.0), 4),
        "exchange_ms_min_over_ranks": round(xmin, 4),
        "exchange_mode": "dense all-reduce" if i0["flags"] & tfidf_abi.RUN_XCHG_DENSE else "hash-owner all-to-all",
        "k1_ms_mean_over_ranks": round(float(np.mean(k1)), 4),
        "roofline": {"bound": "hbm", "kernel": f"{kern} (K1, rank 0)", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "alg_bytes_per_launch": int(alg0),
                     "k1_avg_ms": round(k1_r0, 4)},
        "cpu_baseline": None,
        "device_allocs_in_timed_steps": a2[0] - a1[0],
        "cold_run_ms": round(cold_ms, 3),
        "cold_run": {"ms": round(cold_ms, 3), "device_allocs": a1[0] - a0[0]},
    }
    if want_c3(args):
        try:
            c3 = []
            for r in range(N):
                p = tfidf_configs.plan("c3", rank=r, nranks=N, weak=False)
                c3.append(g.ranks[r].synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"],
                                                  p["ndocs_total"]))
            g.run(c3)   # cold run of the new shard sizes
            hip_device_sync_all(N)
            nb = float(sum(e.info()["nbytes"] for e in g.ranks))

            def steps_fn(k):
                for _ in range(k):
                    g.run(c3)
            line["c3_strong"] = c3_strong_measure(steps_fn, lambda: g.ranks[0].info(), nb, N,
                                                  lambda: hip_device_sync_all(N))
        except Exception as ex:   # reported, never silently dropped
            line["c3_strong"] = {"error": repr(ex)}
    print(json.dumps(line), flush=True)
    g.close()


def want_c3(args) -> bool:
    return args.gpus >= 2 and args.config == "c2" and not args.strong and not args.no_c3 and args.scale == 1.0


def hip_device_sync_all(n: int):
    """hipDeviceSynchronize on devices 0..n-1 (the group's ranks)."""
    hip = C.CDLL("libamdhip64.so.7")
    for d in range(n):
        if hip.hipSetDevice(d) != 0 or hip.hipDeviceSynchronize() != 0:
            raise RuntimeError("hipDeviceSynchronize failed on device %d" % d)


def plan_summary(cfg: str, ngpu: int, strong: bool, scale: float = 1.0) -> dict:
    """What a run would measure (no GPU touched): per-rank shards of `cfg` over `ngpu` ranks."""
    shards = []
    for r in range(ngpu):
        p = tfidf_configs.plan(cfg, scale=scale, rank=r, nranks=ngpu, weak=not strong)
        est = float(np.sum(p["ntok"])) * tfidf_configs.bytes_per_token(p["V"])
        shards.append({"rank": r, "docs": int(len(p["doc_ids"])), "est_bytes": int(est)})
    return {"config": cfg, "n_gpus": ngpu, "scaling": "strong" if strong else "weak",
            "docs_total": int(tfidf_configs.plan(cfg, scale=scale, rank=0, nranks=ngpu,
                                                 weak=not strong)["ndocs_total"]),
            "docs_in_shards": int(sum(x["docs"] for x in shards)),
            "est_bytes_total": int(sum(x["est_bytes"] for x in shards)), "shards": shards}


# BASELINE.json config 3 ("10M docs, ~40 GB Zipfian corpus sharded over 8 MI355X"): a --gpus N
# run (N >= 2) of the default c2 line measures it too, after the headline steps, so the
# driver's scaling runs carry it unattended (not in `value`; --no-c3 skips it)
C3_STRONG_STEPS, C3_STRONG_WARMUP = 3, 1


def c3_strong_measure(run_steps, info_of, corpora_bytes, ngpu, sync, barrier=lambda: None, max_over=lambda x: x):
    """Times C3_STRONG_STEPS collective runs of the c3 strong split; run_steps(k) runs k steps on
    every rank, info_of() is this process's rank-0 info; returns the nested line."""
    run_steps(C3_STRONG_WARMUP)
    barrier()
    sync()
    t0 = time.perf_counter()
    run_steps(C3_STRONG_STEPS)
    sync()
    barrier()
    el = max_over(time.perf_counter() - t0)
    i = info_of()
    alg = i["nbytes"] + 12.0 * i["npairs"]
    return {"workload": f"c3 strong: 10M docs / ~40 GB split over {ngpu} GPUs (BASELINE config 3)",
            "value": round(corpora_bytes * C3_STRONG_STEPS / el / 1e9, 4), "unit": "GB/s",
            "ms_per_step": round(el / C3_STRONG_STEPS * 1e3, 4), "steps": C3_STRONG_STEPS,
            "warmup": C3_STRONG_WARMUP, "corpus_bytes_total": int(corpora_bytes),
            "k1_ms_rank0": round(i["ms_tokcount"], 4),
            "k1_frac_rank0": round(alg / (i["ms_tokcount"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "exchange_ms_rank0": round(i["stages"].get("exchange", 0.0), 4),
            "exchange_mode": "dense all-reduce" if i["flags"] & tfidf_abi.RUN_XCHG_DENSE else "hash-owner all-to-all",
            "command": f"python -m torch.distributed.run --nproc-per-node {ngpu} bench.py --gpus {ngpu} "
                       f"--config c3 --strong (the same measurement as a headline line)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--cpu-sample-docs", type=int, default=48000)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: the CPUs this process may use (affinity, capped by the cgroup quota)")
    ap.add_argument("--strong", action="store_true",
                    help="split the config's corpus over the GPUs (c3 at --gpus 8: BASELINE's 10M docs / 40 GB "
                         "over 8 MI355X) instead of one config-sized shard per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the measured HBM read/copy peak probe")
    ap.add_argument("--no-emit", action="store_true", help="skip the (untimed) output-emission measurement")
    ap.add_argument("--stage-steps", type=int, default=3,
                    help="untimed steps after the timed ones with per-stage HIP events (stage_ms_*)")
    ap.add_argument("--vocab", type=int, default=0, help="diagnostics only: override the config's vocabulary size")
    ap.add_argument("--plan-only", action="store_true",
                    help="print what would be measured (shards per rank, and the c3 strong follow-up of a "
                         "multi-GPU c2 run) as JSON and exit, without touching a GPU")
    ap.add_argument("--shard-of", default="",
                    help="R/N: diagnostics only (K1 PMC traffic of a multi-GPU plan, scripts/r05_final.sh): run rank R's "
                         "shard of the N-GPU plan alone on one GPU, no exchange (idf over the global N)")
    ap.add_argument("--no-c3", action="store_true",
                    help="--gpus N >= 2: skip the c3 strong (BASELINE config 3) measurement after the c2 line")
    ap.add_argument("--shards", type=int, default=0,
                    help="K >= 2: the config's corpus cut into K byte-balanced shards run by K contexts on ONE "
                         "GPU (tfidf_group, in-process transport): measures the multi-rank path and the DF "
                         "exchange (xGMI time excluded); not the headline line")
    args = ap.parse_args()
    if args.shards >= 2:
        return main_shards(args)

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.plan_only:
        out = plan_summary(args.config, args.gpus, args.strong, args.scale)
        if want_c3(args):
            out["c3_strong"] = plan_summary("c3", args.gpus, True)
        print(json.dumps(out))
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return main_group(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # rendezvous, barriers and max-reduce over gloo (CPU)
        dist.init_process_group("gloo", init_method="env://")
    ngpu = world

    eng = tfidf_abi.Engine(local)
    if world > 1:
        import torch
        uid = torch.zeros(tfidf_abi.UNIQUE_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            uid[:] = torch.frombuffer(bytearray(tfidf_abi.comm_unique_id()), dtype=torch.uint8)
        dist.broadcast(uid, 0)
        eng.comm_init(bytes(uid.numpy().tobytes()), rank, world)

    if args.shard_of and world == 1:
        sr, sn = (int(x) for x in args.shard_of.split("/"))
        p = tfidf_configs.plan(args.config, scale=args.scale, rank=sr, nranks=sn, weak=not args.strong,
                               vocab=args.vocab)
    else:
        p = tfidf_configs.plan(args.config, scale=args.scale, rank=rank, nranks=world, weak=not args.strong,
                               vocab=args.vocab)
    corpus = eng.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
    # the timed steps record HIP events around K1 and the whole run only (the roofline's K1
    # time, device_ms_per_step); the per-stage breakdown comes from --stage-steps extra steps
    # after the timed region (each event record costs the stream ~5 us: ten of them are ~2 %
    # of a c2 step)
    eng.set_timing(2)

    # cold run: the first tfidf_run of this fresh context (table growth retries, the idf LUT
    # of this N, every first device allocation), timed on its own and reported beside the
    # steady-state value; it is warmup step 1
    allocs0 = eng.alloc_counters()
    hip_device_sync()
    tc = time.perf_counter()
    eng.run_corpus(corpus)
    hip_device_sync()
    cold_ms = (time.perf_counter() - tc) * 1e3
    allocs1 = eng.alloc_counters()
    for _ in range(max(0, args.warmup - 1)):
        eng.run_corpus(corpus)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    hip_device_sync()
    alloc_t0 = eng.alloc_counters()
    eng.totals(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):   # nothing but the runs: their K1 / run / idf times are summed by the engine
        eng.run_corpus(corpus)
    hip_device_sync()
    barrier()
    elapsed = time.perf_counter() - t0
    alloc_t1 = eng.alloc_counters()
    tt = eng.totals(reset=True)
    nrun = max(1, int(tt["runs"]))
    k1_ms = [tt["ms_tokcount"] / nrun]
    tot_ms = [tt["ms_total"] / nrun]
    idf_steps = [(tt["idf_logs"] / nrun, tt["ms_idf_host"] / nrun, tt["ms_idf_wait"] / nrun)]
    info = eng.info()
    C_bytes, P_pairs, T_tok = info["nbytes"], info["npairs"], info["ntokens"]
    # the stage breakdown, after the timed region: every stage's events
    eng.set_timing(True)
    stage_steps = []
    for _ in range(max(1, args.stage_steps)):
        eng.run_corpus(corpus)
        stage_steps.append(eng.info()["stages"])
    info = eng.info()

    # output emission, outside the timed region and not in `value`:
    # GPU %.16f formatting of the last step's lines, then the pinned D2H + write path
    emit = None
    if not args.no_emit:
        # 1) the CLI's path: formatting in document groups overlapped with the pinned D2H
        #    (first call: also pins the context's staging ring); 2) the text again (already
        #    formatted, ring warm): the D2H rate alone
        t1 = time.perf_counter()
        eng.write_output("/dev/null")
        t_fw = time.perf_counter() - t1
        oi1 = eng.output_info()
        n = eng.format_bytes()
        t2 = time.perf_counter()
        eng.write_output("/dev/null")
        t_wr = time.perf_counter() - t2
        oi2 = eng.output_info()
        emit = {"text_bytes": int(n), "format_d2h_overlapped_ms": round(t_fw * 1e3, 3),
                "d2h_devnull_ms": round(t_wr * 1e3, 3),
                "d2h_GBps": round(n / t_wr / 1e9, 2) if t_wr > 0 else None,
                "first_call": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in oi1.items()},
                "second_call": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in oi2.items()},
                "note": "GPU %.16f formatting in 8 document groups overlapped with the D2H through a "
                        "8 x 16 MB pinned ring (first call, incl. pinning the ring), then the D2H alone; "
                        "written to /dev/null; not in value"}

    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([C_bytes, P_pairs, T_tok], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        C_all, P_all, T_all = (float(x) for x in tot.tolist())
    else:
        C_all, P_all, T_all = float(C_bytes), float(P_pairs), float(T_tok)

    # measured streaming peaks, outside the timed region, rank 0 only
    probe = eng.hbm_probe(2 << 30, 10) if (rank == 0 and not args.no_probe) else None

    c3_line = None
    if want_c3(args) and world > 1:   # BASELINE config 3 after the headline steps (not in value)
        import torch
        try:
            p3 = tfidf_configs.plan("c3", rank=rank, nranks=world, weak=False)
            c3c = eng.synth_device(p3["seed"], p3["V"], p3["mode"], p3["cdf"], p3["doc_ids"], p3["ntok"],
                                   p3["ndocs_total"])
            eng.run_corpus(c3c)   # cold run of the new shard size
            hip_device_sync()
            nb = torch.tensor([float(eng.info()["nbytes"])], dtype=torch.float64)
            dist.all_reduce(nb, op=dist.ReduceOp.SUM)

            def steps_fn(k):
                for _ in range(k):
                    eng.run_corpus(c3c)

            def max_over(x):
                t = torch.tensor([x], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                return float(t.item())
            c3_line = c3_strong_measure(steps_fn, eng.info, float(nb.item()), world, hip_device_sync, barrier, max_over)
        except Exception as ex:   # reported, never silently dropped
            c3_line = {"error": repr(ex)}

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        k1_avg_ms = float(np.mean(k1_ms))
        alg_bytes = C_bytes + 12.0 * P_pairs  # per K1 launch on this rank
        achieved = alg_bytes / (k1_avg_ms * 1e-3) / 1e9
        kern = k1_kernel(int(info["flags"]))
        traffic, traffic_src = load_traffic(args.config, args.strong, ngpu, kern)
        line = {
            "metric": "corpus GB/s (TF-IDF hot path: tokenize->TF->DF->tf*idf->ordered output)",
            "value": round(C_all * args.steps / elapsed / 1e9, 4),
            "unit": "GB/s",
            "n_gpus": ngpu,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8/u32 (f64 score)",
            "data": "synthetic (device-generated Zipfian corpus, csrc/synth.h), resident in HBM",
            "config": {"workload": f"{args.config}: {len(p['doc_ids'])} docs/GPU, V={p['V']}, "
                                   f"{C_bytes / 1e9:.3f} GB/GPU, {P_pairs} pairs/GPU",
                       "docs_total": int(p["ndocs_total"]), "corpus_bytes_total": int(C_all),
                       "parallelism": f"doc-shard x{ngpu} + RCCL DF all-reduce" if ngpu > 1 else "1 GPU"},
            "pairs_per_s": round(P_all * args.steps / elapsed, 1),
            "tokens_per_s": round(T_all * args.steps / elapsed, 1),
            "device_ms_per_step": round(float(np.mean(tot_ms)), 4),
            "stage_ms": {k: round(v, 4) for k, v in info["stages"].items()},
            "stage_ms_mean": {k: round(float(np.mean([st[k] for st in stage_steps])), 4) for k in info["stages"]},
            "stage_ms_max": {k: round(float(np.max([st[k] for st in stage_steps])), 4) for k in info["stages"]},
            "stage_ms_source": f"{len(stage_steps)} untimed steps after the timed ones, with per-stage HIP events "
                               f"(the timed steps record K1's and the whole run's events only)",
            # the idf table (log(N/df) on the host's libm, TFIDF.c:243) is rebuilt inside every
            # timed step on host threads beside the device stages (no cache across runs)
            "idf": {"idf_cached": False,
                    "logs_per_step": int(np.mean([x[0] for x in idf_steps])),
                    "lut_host_ms_mean": round(float(np.mean([x[1] for x in idf_steps])), 4),
                    "wait_ms_mean": round(float(np.mean([x[2] for x in idf_steps])), 4)},
            "k1_work": {"chunks": int(info["nchunks"]), "partial_records": int(info["partial_records"]),
                        "vocab_capacity": int(info["vocab_capacity"]), "terms": int(info["nterms"])},
            "roofline": {"bound": "hbm", "kernel": f"{kern} (K1)", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "alg_bytes_per_launch": int(alg_bytes),
                         "k1_avg_ms": round(k1_avg_ms, 4),
                         "measured_read_peak": round(probe["read_GBps"], 1) if probe else None,
                         "measured_copy_peak": round(probe["copy_GBps"], 1) if probe else None,
                         "frac_of_measured_read": round(achieved / probe["read_GBps"], 4) if probe else None},
            "cpu_baseline": None,
            "emit": emit,
            # device (re)allocations between the first and the last timed step (hipMalloc
            # counted inside the library): 0 = every buffer was sized before timing began
            "device_allocs_in_timed_steps": alloc_t1[0] - alloc_t0[0],
            "device_alloc_bytes_in_timed_steps": alloc_t1[1] - alloc_t0[1],
            "cold_run_ms": round(cold_ms, 3),
            "cold_run": {"ms": round(cold_ms, 3), "device_allocs": allocs1[0] - allocs0[0],
                         "device_alloc_bytes": allocs1[1] - allocs0[1],
                         "note": "first tfidf_run of a fresh context (warmup step 1): vocabulary/record "
                                 "capacity retries, the idf table of this N, first allocations; not in value"},
        }
        if c3_line is not None:
            line["c3_strong"] = c3_line
        if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
            hi = host_cpu_info()
            thr = args.cpu_threads or hi["affinity"]
            if hi["cgroup_cpus"]:
                thr = min(thr, max(1, int(hi["cgroup_cpus"])))
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_sample_docs, max(1, thr), hi)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
