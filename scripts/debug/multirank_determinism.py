"""Run-to-run spread of the 2-rank (gloo, one GPU) graph-replayed DKD training
of tests/test_gpu_multirank.py: split vs split, events vs events, and events
vs split, all at one bucket size -- is the events-vs-split difference larger
than the path's own run-to-run spread (fp64 atomics in the BN regions make
the sums' rounding order-dependent)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
os.environ.setdefault("MDA_TEST_BUCKET_MB", "1.0")

import test_gpu_multirank as T  # noqa: E402


def rel(a, b):
    return float((a["flat"] - b["flat"]).norm() / b["flat"].norm())


if __name__ == "__main__":
    s1, s2 = T._spawn("dkd"), T._spawn("dkd")
    e1, e2 = T._spawn("dkd_events"), T._spawn("dkd_events")
    print(f"split vs split   {rel(s1[0], s2[0]):.3g}", flush=True)
    print(f"events vs events {rel(e1[0], e2[0]):.3g}", flush=True)
    print(f"events vs split  {rel(e1[0], s1[0]):.3g}", flush=True)
