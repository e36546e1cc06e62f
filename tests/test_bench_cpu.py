"""bench.py's rank plumbing on the CPU (no GPU needed): `--gpus N` is never silently run on
fewer GPUs.  Without a launcher, N > 1 is one process driving N GPUs through tfidf_group
(the RCCL clique); with fewer visible GPUs it exits non-zero with a message.  Under a
launcher, --gpus must match WORLD_SIZE."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env, cwd=REPO)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="needs a host without visible GPUs")
def test_gpus_more_than_visible_fails_loudly():
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "1"])
    assert p.returncode == 2
    assert "needs 2 visible GPUs" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_gpus_must_match_launcher_world():
    p = _bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "launcher started 2 ranks" in p.stderr


def test_gpus_zero_rejected():
    p = _bench(["--gpus", "0"])
    assert p.returncode != 0


def test_plan_c3_strong_two_way_split():
    """`--gpus 2 --config c3 --strong` plans BASELINE's config 3 (10M documents, ~40 GB) as a
    2-way byte-balanced split, n_gpus 2, before any GPU call (--plan-only touches no GPU)."""
    import json
    p = _bench(["--gpus", "2", "--config", "c3", "--strong", "--plan-only"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and len(d["shards"]) == 2
    assert d["docs_total"] == 10_000_000 and d["docs_in_shards"] == 10_000_000
    assert 35e9 < d["est_bytes_total"] < 45e9
    a, b = (x["est_bytes"] for x in d["shards"])
    assert abs(a - b) < 0.01 * (a + b)          # balanced by bytes
    assert "c3_strong" not in d


def test_plan_multi_gpu_c2_carries_c3_followup():
    """A `--gpus N` (N >= 2) weak c2 run also measures the c3 strong split afterwards (nested
    `c3_strong` object, not in `value`), so the driver's scaling runs carry config 3."""
    import json
    p = _bench(["--gpus", "4", "--plan-only"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["config"] == "c2" and d["scaling"] == "weak" and d["docs_total"] == 400_000
    assert d["c3_strong"]["n_gpus"] == 4 and d["c3_strong"]["docs_in_shards"] == 10_000_000
    p1 = _bench(["--gpus", "1", "--plan-only"])
    assert "c3_strong" not in json.loads(p1.stdout.strip().splitlines()[-1])
