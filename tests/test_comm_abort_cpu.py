"""CPU test of the RCCL ranks' abort protocol (csrc/comm_rank.h): a fake clique whose
collectives complete only when every rank issued them, so a rank that waits for a failed
peer is released only by the protocol itself.  Replaces the reference's exit()-and-let-
mpirun-kill behaviour (TFIDF.c:122,137).  Also the communicator init with a deadline
(csrc/comm_init.h): an init that never completes returns at its deadline, a process keeps at
most one blocked helper thread, and a late init's communicator is aborted.  No GPU: the C++
state machines are compiled with g++."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "csrc")


def test_comm_abort_state_machine(tmp_path):
    exe = str(tmp_path / "comm_abort_test")
    src = os.path.join(REPO, "tests", "native", "comm_abort_test.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-Wall", "-Werror", "-I", CSRC, src, "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
    assert r.stdout.count("ok  ") == 11
