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
