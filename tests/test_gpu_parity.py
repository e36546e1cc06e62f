"""GPU parity tests: the HIP path (through the C-ABI) against the reference goldens and
the oracle restatement.  TF counts, docSize and DF are compared bit-exactly; scores are
compared bit-exactly too (host-libm idf LUT), the north-star tolerance being 1e-12
relative.  Edge cases follow SURVEY §8c / Appendix A."""
import ctypes as C
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_py
import tfidf_abi
import tfidf_configs
from conftest import golden_cases, GOLDEN
from helpers import assert_same_result, check_full_properties, docs_to_arrays, jobs_from_result, load_golden

pytestmark = pytest.mark.gpu


def check_vs_oracle(engine, data, off, ids=None, n_total=0):
    engine.run_host(data, off, ids, n_total)
    res = engine.fetch()
    ora = oracle_py.run(data, off, ids, n_total)
    assert_same_result(res, ora)
    assert res["output_txt"] == ora["output_txt"]
    # the GPU-formatted text (emit.hip) is the same bytes
    assert engine.text() == ora["output_txt"]
    return res


@pytest.mark.parametrize("case", golden_cases())
def test_golden_output_txt(engine, case):
    g = load_golden(case)
    engine.run_host(g["data"], g["off"])
    res = engine.fetch()
    assert res["output_txt"] == g["output"]
    tf, idf = jobs_from_result(res)
    assert tf == g["tf_jobs"]
    assert idf == g["idf_jobs"]


@pytest.mark.parametrize("cfg,scale", [("c1", 1.0), ("c2", 0.003), ("c3", 0.00005), ("c4", 0.002), ("c5", 0.0005)])
def test_synthetic_configs_vs_oracle(engine, cfg, scale):
    p = tfidf_configs.plan(cfg, scale=scale)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    res = check_vs_oracle(engine, data, off, p["doc_ids"], p["ndocs_total"])
    assert res["npairs"] > 0


def test_document_boundaries_split_tokens(engine):
    data, off = docs_to_arrays([b"ab", b"cd", b"ab", b"", b"ab cd"])
    res = check_vs_oracle(engine, data, off)
    assert res["output_txt"].count(b"\n") == 5


def test_empty_corpus_and_blank_docs(engine):
    data, off = docs_to_arrays([b"", b"  \n\t", b"\r\n", b"x"])
    res = check_vs_oracle(engine, data, off)
    assert res["npairs"] == 1


def test_nul_and_control_bytes(engine):
    docs = [b"ab\x00cd ab \x00zz \x01\x02 a\x01 a\x7f a\xff\xfe",
            b"\x00 \x00\x00 ab\x00 ab\x00\x00x",
            b"a\x08 a\x09a a\x0ea"]
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_long_tokens_and_shared_prefixes(engine):
    rng = np.random.default_rng(7)
    base = b"abcdefghijklmnop"  # 16 bytes
    words = [base, base + b"q", base + b"\x01", base + b"qr" * 40, b"x" * 15, b"x" * 16, b"x" * 17,
             base[:15], base[:15] + b"\x00tail", bytes(rng.integers(33, 127, 5000, dtype=np.uint8)),
             b"y" * 70000]
    docs = []
    for i in range(6):
        pick = rng.choice(len(words), size=12)
        docs.append(b" ".join(words[j] for j in pick) + b"\n")
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_tokens_across_windows_and_chunks(engine):
    # one big document (> BIG_DOC, split across chunks) whose tokens straddle the 4 KiB
    # windows and chunk boundaries (24 KiB for tokcount_sl, 12 KiB for the other K1
    # kernels) at every offset
    rng = np.random.default_rng(3)
    parts = []
    n = 0
    while n < 300_000:
        L = int(rng.integers(1, 40))
        w = bytes(rng.integers(97, 100, L, dtype=np.uint8))
        sep = b" " if rng.random() < 0.9 else b"\n\t "
        parts.append(w + sep)
        n += L + len(sep)
    docs = [b"".join(parts), b"aa bb", b"".join(parts[:5000])]
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_many_tiny_documents(engine):
    rng = np.random.default_rng(11)
    docs = []
    for i in range(20000):
        k = int(rng.integers(0, 4))
        docs.append(b"" if k == 0 else b" ".join(b"w%d" % rng.integers(0, 50) for _ in range(k)))
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_doc_ids_and_ndocs_total(engine):
    p = tfidf_configs.plan("c2", scale=0.002, rank=1, nranks=3)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    check_vs_oracle(engine, data, off, p["doc_ids"], p["ndocs_total"])


def _hip_d2h(dst: np.ndarray, src_ptr: int):
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(dst.ctypes.data, C.c_void_p(src_ptr), dst.nbytes, 2) == 0


def test_device_generator_matches_host(engine):
    p = tfidf_configs.plan("c5", scale=0.0002)
    h, hoff = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    c = engine.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
    assert c.nbytes == len(h)
    d = np.empty(len(h), dtype=np.uint8)
    _hip_d2h(d, c.bytes)
    doff = np.empty(len(hoff), dtype=np.uint64)
    _hip_d2h(doff, c.doc_off)
    assert np.array_equal(d, h) and np.array_equal(doff, hoff)
    engine.run_corpus(c)
    res = engine.fetch()
    ora = oracle_py.run(h, hoff, p["doc_ids"], p["ndocs_total"])
    assert_same_result(res, ora)


def test_repeat_runs_identical(engine):
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    outs = []
    for _ in range(3):
        engine.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        outs.append(engine.fetch()["output_txt"])
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.parametrize("case", golden_cases())
def test_cli_drop_in(case):
    """`tfidf` with no arguments in the fixture directory writes the reference output.txt;
    with --debug-jobs its stdout, split into the TF Job / IDF Job blocks and sorted, is the
    reference's tf_jobs.txt / idf_jobs.txt (TFIDF.c:199-205,236-239)."""
    from test_gpu_multirank import split_jobs
    g = load_golden(case)
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(os.path.join(GOLDEN, case, "input"), os.path.join(td, "input"))
        p = subprocess.run([tfidf_abi.CLI_PATH], cwd=td, capture_output=True, timeout=120)
        assert p.returncode == 0, p.stderr
        with open(os.path.join(td, "output.txt"), "rb") as f:
            assert f.read() == g["output"]
        p = subprocess.run([tfidf_abi.CLI_PATH, "--debug-jobs"], cwd=td, capture_output=True, timeout=120)
        assert p.returncode == 0, p.stderr
    tf, idf = split_jobs(p.stdout)
    assert tf == g["tf_jobs"] and idf == g["idf_jobs"]


def test_cli_error_contract():
    with tempfile.TemporaryDirectory() as td:
        # no input/ (TFIDF.c:100-103)
        p = subprocess.run([tfidf_abi.CLI_PATH], cwd=td, capture_output=True, timeout=60)
        assert p.returncode == 1 and p.stdout == b"Directory failed to open\n"
        # empty input/: N = 0 < workers (TFIDF.c:120-123), no output.txt
        os.makedirs(os.path.join(td, "input"))
        for args in ([], ["--shards", "2"]):
            p = subprocess.run([tfidf_abi.CLI_PATH] + args, cwd=td, capture_output=True, timeout=60)
            assert p.returncode == 0 and p.stdout == b"More workers than input files! Exiting.\n"
            assert not os.path.exists(os.path.join(td, "output.txt"))
        # a missing document (TFIDF.c:134-138)
        with open(os.path.join(td, "input", "doc2"), "wb") as f:
            f.write(b"x")
        for args in ([], ["--shards", "2"]):
            p = subprocess.run([tfidf_abi.CLI_PATH] + args, cwd=td, capture_output=True, timeout=60)
            assert p.returncode == 0 and p.stdout.startswith(b"Error Opening File: input/doc1"), p.stdout
        # output.txt cannot be written (TFIDF.c:274-278): a directory in its place
        with open(os.path.join(td, "input", "doc1"), "wb") as f:
            f.write(b"a b a\n")
        os.makedirs(os.path.join(td, "output.txt"))
        for args in ([], ["--shards", "2"]):
            p = subprocess.run([tfidf_abi.CLI_PATH] + args, cwd=td, capture_output=True, timeout=60)
            assert p.returncode == 0 and p.stdout == b"Error Opening File: output.txt\n", (p.stdout, p.stderr)


@pytest.mark.parametrize("cfg", ["c2", "c4", "c5", "c3"])
def test_full_config_properties(cfg):
    """BASELINE configs at full size on one GPU, device-generated: c2 (1e5 docs, ~1 GB), c4
    (V = 1e7: ~1e7 distinct terms, vocabulary-table growth, radix-sorted vocabulary), c5
    (four 100 MB documents among 1e6 ~600 B ones), c3 (1e7 documents, ~40 GB, ~2.9e9 pairs:
    the whole 8-GPU workload on one GPU).  Size-independent properties
    (helpers.check_full_properties) — sum of counts = tokens, per-document sums = docSize,
    DF = pairs per term, strict output order, scores recomputed (<= 1e-12 relative) — on
    views of the fetched arrays, in chunks."""
    p = tfidf_configs.plan(cfg)
    with tfidf_abi.Engine(0) as e:
        c = e.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
        e.run_corpus(c)
        info = e.info()
        assert info["ntokens"] == int(p["ntok"].sum())
        with e.fetched() as r:
            assert r["npairs"] == info["npairs"] and r["npairs"] > 1_000_000
            assert r["ndocs"] == len(p["ntok"]) and r["ndocs_total"] == (p["ndocs_total"] or len(p["ntok"]))
            check_full_properties(r, info["ntokens"])


@pytest.mark.parametrize("cfg,scale", [("c2", 0.002), ("c5", 0.0005), ("c4", 0.001)])
def test_k1_variants_agree(cfg, scale):
    """The default K1 (k_tokcount_sl up to 32M vocabulary slots, k_tokcount_vs beyond), the
    round-1 slot-keyed K1 (TFIDF_K1=vs) and the general K1 (unaligned corpora) give identical
    results, equal to the oracle."""
    p = tfidf_configs.plan(cfg, scale=scale)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    outs = []
    modes = [("auto", 2), ("sl", 2), ("vs", 2), ("general", 0)]
    for mode, flag in modes:
        os.environ["TFIDF_K1"] = mode
        try:
            with tfidf_abi.Engine(0) as e:
                e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
                f = e.info()["flags"]
                assert (f & 3) == flag
                if mode in ("auto", "sl"):
                    assert f & tfidf_abi.RUN_K1_SL
                outs.append(e.fetch())
        finally:
            os.environ.pop("TFIDF_K1", None)
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    for o in outs:
        assert_same_result(o, ora)


def _distinct_words(n, rng, lo=2, hi=12):
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    words = set()
    while len(words) < n:
        L = int(rng.integers(lo, hi + 1))
        words.add(bytes(alpha[rng.integers(0, 26, L)]))
    return sorted(words)


def test_doc_with_more_pairs_than_lds_table(engine):
    """One ~60 KB document (a single chunk) with ~7000 distinct terms: the open document
    overflows the LDS table (partial flushes) and exceeds K5's in-LDS sort size."""
    rng = np.random.default_rng(11)
    words = _distinct_words(7000, rng)
    toks = [words[i] for i in rng.permutation(len(words))] + [words[i] for i in rng.integers(0, 300, 1500)]
    docs = [b"x y z\n", b" ".join(toks)[:63000] + b"\n", b"x q\n"]
    check_vs_oracle(engine, *docs_to_arrays(docs))


@pytest.mark.parametrize("V", [65535, 65536, 65537])
def test_df_histogram_vocabulary_boundary(engine, V):
    """Vocabularies at the LDS histogram's limit (finalize.hip DFH_MAXV): at V = 65536 the
    u16 bins (128 KB) and the slot -> rank cache (32 KB) fill the 160 KB of LDS exactly;
    V = 65537 takes the partitioned global-atomic path.  Every term occurs at least once and
    16 frequent terms occur in every document (the cache's hits)."""
    rng = np.random.default_rng(V)
    words = _distinct_words(V, rng)
    hot = [words[i] for i in rng.choice(V, 16, replace=False)]
    docs = []
    for part in np.array_split(rng.permutation(V), 1500):
        toks = [words[i] for i in part] + hot + [words[i] for i in rng.integers(0, V, 8)]
        rng.shuffle(toks)
        docs.append(b" ".join(toks) + b"\n")
    res = check_vs_oracle(engine, *docs_to_arrays(docs))
    assert engine.info()["nterms"] == V
    assert int(np.max(res["df"])) == len(docs)


def test_complete_doc_over_k5_limit(engine):
    """~2500 distinct terms in a 25 KB document: complete inside one chunk but larger than
    K5's in-LDS sort, so it is routed through the partial merge."""
    rng = np.random.default_rng(12)
    words = _distinct_words(2500, rng, 3, 8)
    docs = [b" ".join(words[i] for i in rng.permutation(len(words))) + b"\n", b"a b\n"]
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_many_tiny_docs_without_separators(engine):
    """Thousands of 0-6 byte documents, most with no trailing whitespace: document starts
    are token boundaries, more documents per chunk than one LDS document group."""
    rng = np.random.default_rng(13)
    pool = [b"a", b"b", b"ab", b"ba", b"abc", b" ", b"", b"c\t", b"\nd", b"ee ee"]
    docs = [pool[i] for i in rng.integers(0, len(pool), 5000)]
    check_vs_oracle(engine, *docs_to_arrays(docs))


def test_big_docs_split_across_chunks(engine):
    """Documents far above BIG_DOC are split across work units mid-token; their partial
    counts are merged."""
    rng = np.random.default_rng(14)
    words = _distinct_words(3000, rng, 1, 20)
    z = rng.zipf(1.3, 60000) % len(words)
    big = b" ".join(words[i] for i in z)
    docs = [big, b"tail words here", big[:200000], b"", big[5:] + b"\n"]
    check_vs_oracle(engine, *docs_to_arrays(docs))


@pytest.mark.parametrize("cap,load", [("1024", "50"), ("4096", "12")])
def test_vocabulary_table_growth(monkeypatch, cap, load):
    """A vocabulary table that starts too small: K1 flags the overflow (or the load check
    fires) and the run repeats with a larger table — results unchanged."""
    monkeypatch.setenv("TFIDF_VCAP", cap)
    monkeypatch.setenv("TFIDF_VLOAD", load)
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        res = check_vs_oracle(e, data, off, p["doc_ids"], p["ndocs_total"])
        info = e.info()
    assert info["vocab_capacity"] > int(cap)
    assert res["nterms"] * 100 <= info["vocab_capacity"] * int(load)


@pytest.mark.parametrize("split", ["1", "0"])
@pytest.mark.parametrize("cfg,scale", [("c2", 0.002), ("c5", 0.002), ("c4", 0.002)])
def test_df_split_pass(monkeypatch, split, cfg, scale):
    """With partial records to merge, the main records' DF pass runs on the side stream beside
    the merge stage and the merged records are added after it (engine.cpp run_local; the LDS
    histogram for V <= 65536, the sliced pass above: c4); TFIDF_DF_SPLIT=0 keeps one pass
    after the merge.  Both agree with the oracle."""
    monkeypatch.setenv("TFIDF_DF_SPLIT", split)
    p = tfidf_configs.plan(cfg, scale=scale)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        check_vs_oracle(e, data, off, p["doc_ids"], p["ndocs_total"])
        info = e.info()
    if cfg == "c5":   # its long documents always span chunks
        assert info["partial_records"] > 0


def _py_fixed16(vals):
    return [b"%.16f" % v for v in vals]


def test_gpu_format_f64_matches_printf(engine):
    """Device %.16f against Python's (correctly rounded, ties to even = glibc printf):
    exact ties k/2^17, powers of two, tiny and subnormal values, values just
    around the 17th-decimal rounding boundary, and a random sweep over score ranges."""
    rng = np.random.default_rng(11)
    vals = [0.0, 1.0, 0.5, 22.999999999999996, 10.0, 9.999999999999998, 5e-324, 2.2250738585072014e-308,
            1e-17, 5e-17, 4.9999999999999996e-17, 1.5e-16, 0.1, 0.2, 0.3, 1 / 3, 2 / 3]
    vals += [k / 2 ** 17 for k in range(1, 200)]
    vals += [k / 2 ** 20 for k in range(1, 64)]
    vals += [2.0 ** -e for e in range(0, 80)]
    vals += [(k + 0.5) * 1e-16 for k in range(0, 50)]
    vals += list(rng.random(20000) * 23.0)
    vals += list(np.exp(rng.uniform(np.log(1e-12), np.log(23.0), 20000)))
    got = engine.format_f64(vals)
    want = _py_fixed16(vals)
    bad = [(v, g, w) for v, g, w in zip(vals, got, want) if g != w]
    assert not bad, bad[:5]


def test_gpu_output_file_matches_golden(engine, tmp_path):
    """tfidf_write_output_gpu (pinned double-buffered D2H + fwrite) writes the golden
    output.txt bytes; append mode concatenates."""
    for case in golden_cases()[:3]:
        g = load_golden(case)
        engine.run_host(g["data"], g["off"])
        path = str(tmp_path / (case + ".txt"))
        engine.write_output(path)
        assert open(path, "rb").read() == g["output"]
        engine.write_output(path, append=True)
        assert open(path, "rb").read() == g["output"] * 2


def test_gpu_text_c2_slice_vs_oracle(engine):
    """A c2 slice through the whole path: GPU text == oracle output.txt."""
    p = tfidf_configs.plan("c2", scale=0.004)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    engine.run_host(data, off, p["doc_ids"], p["ndocs_total"])
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    assert engine.text() == ora["output_txt"]


def test_gpu_output_file_grouped_format(engine, tmp_path):
    """tfidf_write_output_gpu on an unformatted result formats in document groups whose
    copies overlap the next group's formatting (groups share 16-byte chunks at their
    boundaries): the file equals the oracle's output.txt, several 16 MB staging blocks
    deep, and a second write of the now formatted text equals it too."""
    p = tfidf_configs.plan("c2", scale=0.02)          # ~19 MB corpus -> ~45 MB of text
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    engine.run_host(data, off, p["doc_ids"], p["ndocs_total"])
    path = str(tmp_path / "out.txt")
    engine.write_output(path)
    got = open(path, "rb").read()
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    assert len(got) > (32 << 20)
    assert got == ora["output_txt"]
    engine.write_output(path)
    assert open(path, "rb").read() == got


def test_dense_merge_long_documents(engine):
    """Documents longer than DENSE_DOC (4 MiB) take the dense merge (partial records summed
    per document over term ranks, emitted in rank order); a 180 KB document (split across
    chunks, below DENSE_DOC) still takes the sorted merge in the same run.  Against the
    oracle, bit-exact."""
    p = tfidf_configs.plan("c5", scale=0.05)        # four ~5 MB documents among 50k small ones
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    sizes = np.diff(off.astype(np.int64))
    assert (sizes > (4 << 20)).sum() >= 2
    mid = bytes(data[int(off[0]):int(off[300])])      # ~180 KB: split, but sorted-merged
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(len(off) - 1)] + [mid]
    d2, o2 = docs_to_arrays(docs)
    check_vs_oracle(engine, d2, o2)


def test_many_long_terms_sharing_prefixes(engine):
    """~1e5 distinct long terms tied on their first 16 (and 32, 48, ...) bytes: URL-like
    runs, terms that are prefixes of others, a byte < TAB after a shared prefix, and a
    few terms sharing 200 bytes.  Their order (strcmp of "w\\t") comes from the iterated
    segmented sort (vocab_long_fixup); against the oracle, bit-exact."""
    rng = np.random.default_rng(21)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789_/", dtype=np.uint8)
    words = set()
    for pre in (b"https://en.wikipedia.org/wiki/", b"/usr/local/lib/python3/site-packages/", b"x" * 40):
        while len(words) < 30000 * (1 + [b"https://en.wikipedia.org/wiki/", b"/usr/local/lib/python3/site-packages/",
                                          b"x" * 40].index(pre)):
            L = int(rng.integers(0, 12))
            words.add(pre + bytes(alpha[rng.integers(0, len(alpha), L)]))
    base = b"q" * 200
    extra = [base, base + b"a", base + b"\x01", base + b"ab", base[:150] + b"z", b"abcdefghijklmnopq",
             b"abcdefghijklmnop\x05", b"abcdefghijklmnopqr"]
    words = sorted(words) + extra
    order = rng.permutation(len(words))
    docs, cur = [], []
    for k, i in enumerate(order):
        cur.append(words[i])
        if len(cur) == 700 or k == len(order) - 1:
            cur += [words[j] for j in rng.integers(0, len(words), 50)]
            docs.append(b" ".join(cur) + b"\n")
            cur = []
    check_vs_oracle(engine, *docs_to_arrays(docs))


@pytest.mark.parametrize("wgs", [None, "16"])
def test_df_histogram_bin_overflow(wgs, monkeypatch):
    """17 M one-word documents: every record is the same term, the case where a u16 LDS bin
    of the DF histogram would wrap.  Default split: 65535 records or fewer per workgroup.
    TFIDF_DF_WGS=16: 1.06 M records per workgroup, the wide form (k_df_hist_lds<true>, the
    one c3 runs), whose counter moves 0x8000 to the global df at each crossing — 32 per
    workgroup here, all on one LDS word.  df is N for every pair, each score log(N/N) = 0
    (TFIDF.c:243-244)."""
    if wgs:
        monkeypatch.setenv("TFIDF_DF_WGS", wgs)
    N = 17_000_000
    data = np.frombuffer(b"a\n" * N, dtype=np.uint8).copy()
    off = (np.arange(N + 1, dtype=np.uint64) * 2)
    with tfidf_abi.Engine(0) as engine:
        engine.run_host(data, off)
        info = engine.info()
        assert info["npairs"] == N and info["nterms"] == 1
        with engine.fetched() as r:
            assert np.all(r["df"] == N) and np.all(r["count"] == 1) and np.all(r["docsize"] == 1)
            assert np.all(r["score"] == 0.0)


@pytest.mark.parametrize("split", ["1", "0"])
def test_df_wide_form_vs_oracle(split, monkeypatch):
    """The wide DF form (TFIDF_DF_WGS=3: ~100 K records per workgroup) against the oracle on
    300 K short documents over a 40-term Zipf-like vocabulary plus rare terms — the frequent
    terms' u16 counters cross 0x8000 in every workgroup, the rare ones never — with the DF
    pass split beside the merge and not (TFIDF_DF_SPLIT)."""
    monkeypatch.setenv("TFIDF_DF_WGS", "3")
    monkeypatch.setenv("TFIDF_DF_SPLIT", split)
    rng = np.random.default_rng(5)
    vocab = np.array([b"f%02d" % i for i in range(40)] + [b"rare%05d" % i for i in range(20000)], dtype=object)
    p = np.r_[1.0 / np.arange(1, 41), np.full(20000, 0.0005)]
    n = 300_000
    lens = rng.integers(1, 6, size=n)
    toks = vocab[rng.choice(len(vocab), size=int(lens.sum()), p=p / p.sum())]
    cut = np.r_[0, np.cumsum(lens)]
    docs = [b" ".join(toks[cut[i]:cut[i + 1]]) for i in range(n)]
    data, off = docs_to_arrays(docs)
    ora = oracle_py.run(data, off)
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off)
        assert e.info()["npairs"] > 3 * 65535
        res = e.fetch()
    assert_same_result(res, ora)
    assert res["output_txt"] == ora["output_txt"]


def _doc_with_terms(rng, n, vocab):
    """a document holding exactly n distinct terms of `vocab`, each 1-3 times, shuffled"""
    ids = rng.choice(len(vocab), size=n, replace=False)
    toks = np.repeat(ids, rng.integers(1, 4, size=n))
    rng.shuffle(toks)
    return b" ".join(vocab[i] for i in toks)


def test_score_document_classes_vs_oracle(engine):
    """K5's document classes at their boundaries (finalize.hip k5_class): <= 128 pairs
    (k_score_small), <= 64 / <= 1024 (wave kernel: bitonic, counting, bucket paths), > 1024
    (k_score_large, both instances), and one > 4 MiB document (dense merge: a presorted run
    over 4096 pairs, emitted by k_emit_split's chunk tasks), among many small documents."""
    rng = np.random.default_rng(11)
    vocab = [b"t%05d" % i for i in range(30000)]
    sizes = [1, 2, 63, 64, 65, 127, 128, 129, 511, 512, 513, 1023, 1024, 1025, 2047, 2048, 2049, 4096, 4097, 9000]
    docs = [_doc_with_terms(rng, n, vocab) for n in sizes]
    docs += [_doc_with_terms(rng, int(n), vocab) for n in rng.integers(1, 200, size=300)]
    big = []
    total = 0
    while total < (4 << 20) + 65536:   # > 4 MiB: the dense merge's presorted run
        d = _doc_with_terms(rng, 20000, vocab)
        big.append(d)
        total += len(d) + 1
    docs.append(b" ".join(big))
    order = rng.permutation(len(docs))
    docs = [docs[i] for i in order]
    data, off = docs_to_arrays(docs)
    res = check_vs_oracle(engine, data, off)
    assert res["npairs"] > 20000


def test_term_of_16_mib_is_a_capacity_error(engine):
    """A token of 16 MiB or more (one document without whitespace) is legal input for the
    reference; here its vocabulary entry cannot hold the length (24 bits), and the run
    fails cleanly with TFIDF_E_CAPACITY (include/tfidf.h) instead of emitting a truncated
    term.  The same engine then runs a normal corpus."""
    big = np.full((16 << 20) + 7, ord("a"), dtype=np.uint8)
    data = np.concatenate([np.frombuffer(b"x y\n", dtype=np.uint8), big])
    off = np.array([0, 4, len(data)], dtype=np.uint64)
    with pytest.raises(tfidf_abi.TfidfError) as ei:
        engine.run_host(data, off)
    assert ei.value.rc == -9
    g = load_golden("g1_whitespace")
    engine.run_host(g["data"], g["off"])
    assert engine.fetch()["output_txt"] == g["output"]


def _long_term_corpus(nterms, ndocs, seed):
    """documents of distinct terms of 18-30 bytes (long keys: 120-bit hashes), each term in
    several documents, with a few short words between them"""
    rng = np.random.default_rng(seed)
    terms = sorted({bytes(rng.integers(97, 123, int(rng.integers(18, 31)), dtype=np.uint8)) for _ in range(nterms)})
    docs = []
    for d in range(ndocs):
        pick = rng.choice(len(terms), size=min(len(terms), 40))
        docs.append(b" ".join(terms[j] + b" w%d" % (j % 7) for j in pick) + b"\n")
    return docs_to_arrays(docs)


_LONGTAG_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]); sys.path.insert(0, sys.argv[3])
import numpy as np, tfidf_abi, test_gpu_parity as t, oracle_py
from helpers import assert_same_result
with tfidf_abi.Engine(0) as e:
    # few distinct long terms: no 16-bit collision among them, each repeated in many
    # documents at different offsets -> the byte verification must accept every match
    data, off = t._long_term_corpus(4, 300, 5)
    e.run_host(data, off)
    ora = oracle_py.run(data, off)
    assert_same_result(e.fetch(), ora)
    print("RESULT few ok")
    # thousands of distinct long terms: ~70 pairs share a 16-bit key
    data, off = t._long_term_corpus(3000, 400, 6)
    try:
        e.run_host(data, off)
        print("RESULT many merged")
    except tfidf_abi.TfidfError as ex:
        print("RESULT many rc=%d" % ex.rc)
"""


def test_long_term_hash_collisions_are_reported():
    """Identity of terms of >= 16 bytes is exact (dev_vocab.h): their 120-bit key only picks the
    vocabulary slot; every match is verified byte by byte against the incumbent's first
    occurrence, as TFIDF.c:152,172's strcmp would.  The test library lib/libtfidf_hip_longtag16.so
    truncates the key to 16 bits so distinct long terms DO collide: a corpus of a few long terms
    (no collision) still matches the oracle exactly, and one of 3000 long terms fails with
    TFIDF_E_CAPACITY instead of merging counts.  The product library runs the 3000-term corpus
    against the oracle."""
    here = os.path.dirname(os.path.abspath(__file__))
    pydir = os.path.join(os.path.dirname(here), "parallel-systems-mpi-tfidf_amd", "python")
    env = dict(os.environ, TFIDF_LIB="longtag16")
    import sys
    r = subprocess.run([sys.executable, "-c", _LONGTAG_CHILD, pydir, here, os.path.join(os.path.dirname(here), "oracle")],
                       env=env,
                       capture_output=True, text=True, timeout=240, cwd=here)
    out = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    assert out == ["RESULT few ok", "RESULT many rc=-9"], r.stdout + r.stderr[-3000:]
    assert "share their 120-bit identity key" in r.stderr


def test_many_distinct_long_terms_vs_oracle(engine):
    check_vs_oracle(engine, *_long_term_corpus(3000, 400, 6))
