"""One rank of tests/test_gpu_multiproc.py: runs a contiguous cell shard of the
SURVEY.md §8(d) batch through the library on device 0 and saves its trajectories."""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--total", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import bench
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    soc0, tc = bench.batch_inputs(a.total)
    lo, hi = bench.shard_range(a.total, a.world, a.rank)
    out = M.runMPC(P.make_synth_rom(), soc0[lo:hi], tc[lo:hi], a.steps, device=0)
    np.savez(a.out, lo=lo, hi=hi, **{k: out[k] for k in ("u", "v", "soc", "phise", "nexec", "status")})
    print(f"rank {a.rank}: cells [{lo}, {hi}) done", flush=True)


if __name__ == "__main__":
    main()
