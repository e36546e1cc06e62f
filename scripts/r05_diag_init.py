"""Round 5 diagnostic: where a 2-rank tfidf_comm_init whose peer never joins spends its time
(progress lines with timestamps on stderr).  Run under `timeout`."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "parallel-systems-mpi-tfidf_amd", "python"))
import tfidf_abi  # noqa: E402

t0 = time.time()


def say(m):
    print("%6.2f %s" % (time.time() - t0, m), file=sys.stderr, flush=True)


say("open")
e = tfidf_abi.Engine(0)
say("uid")
u = tfidf_abi.comm_unique_id()
say("comm_init(rank 0 of 2)")
try:
    e.comm_init(u, 0, 2)
    say("joined?!")
except tfidf_abi.TfidfError as ex:
    say("rc=%d" % ex.rc)
say("close")
e.close()
say("done")
