#!/usr/bin/env python3
"""Converts tools/hild_problems.npz (captured from the numpy oracle) into the
binary problem records hild_micro.hip reads, and builds the micro-benchmark."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
z = np.load(os.path.join(HERE, "..", "hild_problems.npz"))
recs = []
i = 0
while f"E{i}" in z:
    M, g = z[f"M{i}"], z[f"g{i}"]
    Hv, He, Hs = M[8:13, 0], -M[13:18, 0], M[18:23, 0]
    assert np.array_equal(M[9:13, 1], Hv[:4]) and np.array_equal(M[19:23, 1], Hs[:4])
    recs.append(np.concatenate([Hv, He, Hs, g, z[f"E{i}"].ravel(), z[f"F{i}"], z[f"l0{i}"]]))
    print(f"problem {i}: oracle nexec {int(z[f'ne{i}'])}")
    i += 1
np.array(recs).astype(np.float64).tofile(os.path.join(HERE, "hild_problems.bin"))
if "--build" in sys.argv:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                    "-Wno-unused-result", "-Wno-unused-value", "-mllvm", "-pragma-unroll-threshold=200000",
                    *os.environ.get("MICRO_FLAGS", "").split(),
                    os.path.join(HERE, "hild_micro.hip"), "-o",
                    os.path.join(HERE, os.environ.get("MICRO_OUT", "hild_micro"))], check=True)
