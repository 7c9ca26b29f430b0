"""Builds libmpcekf.so in-tree with hipcc for gfx950 (no JIT cache, no CPU fallback).

Flags: ``-ffp-contract=off`` (no FMA contraction: the kernels reproduce the
oracle's defined evaluation order) and never ``-ffast-math`` (IEEE NaN/inf
semantics are part of the reference behaviour, SURVEY.md §7 hard part 3).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libmpcekf.so")
ARCH = os.environ.get("MPCEKF_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -pragma-unroll-threshold: the Hildreth sweep (23 x 23 guarded terms) must unroll
# fully so the per-lane arrays stay in registers instead of scratch.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-Wno-unused-result", "-mllvm", "-pragma-unroll-threshold=200000"]
SOURCES = ["mpcekf_kernels.hip", "mpcekf_wide.hip", "mpcekf_io.hip", "mpcekf_host.cpp"]
DEPS = ["mpcekf_kernels.hpp", "mpcekf_mpc.hpp", "mpcekf_eig.hpp", os.path.join("..", "..", "include", "mpcekf.h")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _stale(obj, src):
    # the host embeds the source hash and includes the public header; the kernel files
    # include only the csrc headers
    if os.path.basename(src) == "mpcekf_host.cpp":
        deps = DEPS + SOURCES
    else:
        deps = [d for d in DEPS if not d.endswith("mpcekf.h")]
    newest = max([_mtime(src)] + [_mtime(os.path.join(SRC, d)) for d in deps])
    return _mtime(obj) < newest


def source_hash():
    """sha256 (16 hex) over the kernel/host sources and headers: the library reports it
    (mpcekf_build_id) and profiles/pmc_traffic.json records the one it was measured on."""
    h = hashlib.sha256()
    for f in sorted(SOURCES + DEPS):
        with open(os.path.join(SRC, f), "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def build(force=False, verbose=False, variant="", defines=(), flags=()):
    """variant "stamps": profiling build _build/libmpcekf_stamps.so (-DMPCEKF_STAMPS);
    any other variant name with ``defines`` (["NAME=VAL", ..]) builds an A/B library
    _build/libmpcekf_<variant>.so that bench.py loads through MPCEKF_LIB; ``flags`` are extra
    hipcc arguments for such a variant (e.g. ["-mllvm", "-amdgpu-sched-strategy=max-ilp"])."""
    os.makedirs(OUT, exist_ok=True)
    jobs = []
    objs = []
    sfx = f"_{variant}" if variant else ""
    extra = ["-DMPCEKF_STAMPS"] if variant == "stamps" else []
    extra += [f"-D{d}" for d in defines] + list(flags)
    extra.append(f'-DMPCEKF_SRC_HASH="{source_hash()}"')
    lib = os.path.join(OUT, f"libmpcekf{sfx}.so")
    for s in SOURCES:
        src = os.path.join(SRC, s)
        obj = os.path.join(OUT, os.path.splitext(s)[0] + sfx + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            jobs.append([HIPCC, *CFLAGS, *extra, "-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")

    if jobs:
        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            list(ex.map(run, jobs))
    if jobs or force or not os.path.exists(lib) or any(_mtime(o) > _mtime(lib) for o in objs):
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs])
    return lib


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="extra hipcc argument (variants)")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, variant="stamps" if a.stamps else a.variant, defines=a.defines,
                flags=a.flags))
