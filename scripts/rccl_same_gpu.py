"""Probe: the RCCL halo + second round with two ranks on the box's ONE GPU
(NCCL-style libraries normally refuse duplicate devices; this records what
RCCL does here).  usage (on the box): python3 scripts/rccl_same_gpu.py"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    from oracle.oracle import Oracle
    from tests.test_gpu_slab import _run_two_ranks

    for hs in (1.0, 0.1):
        with tempfile.TemporaryDirectory() as d:
            _run_two_ranks(d, Oracle(), rccl=True, hscale=hs, same_gpu=True)
            print(f"two ranks on one GPU over RCCL, halo scale {hs}: rows equal the single tree",
                  flush=True)
