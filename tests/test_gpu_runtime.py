"""One HIP runtime per GPU process (round-3 finding: torch's bundled libamdhip64 /
libhsa-runtime64 mapped next to the ROCm ones libmpcekf links, with torch-allocated
device pointers handed to the library's kernels).  The GPU session, bench.py's rank
processes and smoke() use library-allocated device buffers (mpcekf_dev_alloc) and never
import torch; bench.py's timing collectives run over gloo in a coordinator child."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one_runtime(rt, where):
    assert len(rt["hip"]) == 1 and len(rt["hsa"]) == 1, f"{where}: HIP runtimes mapped {rt}"
    assert "torch" not in rt["hip"][0] and "torch" not in rt["hsa"][0], f"{where}: {rt}"


def test_session_maps_exactly_one_hip_runtime(rom, M):
    """After a context has run (and a library device buffer held outputs), this process maps
    exactly one libamdhip64 and one libhsa-runtime64, the ones libmpcekf links; torch was
    never imported by the GPU suite."""
    n, steps = 256, 4
    soc0 = np.linspace(8, 25, n)
    tc = np.full(n, 25.0)
    with M.DeviceBuffer((steps, n), np.float64) as u, M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        ctx.step_device(steps, u)
        ctx.sync()
        dev = u.to_host()
    ref = M.runMPC(rom, soc0, tc, steps)["u"]
    np.testing.assert_array_equal(dev, ref)     # device-buffer outputs == host-output path
    _one_runtime(M.hip_runtimes(), "pytest session")
    assert "torch" not in sys.modules


def test_device_buffer_copies(M):
    """mpcekf_dev_copy / _copy2d round trips, including the sampled-column read."""
    a = np.arange(6 * 64, dtype=np.float64).reshape(6, 64)
    with M.DeviceBuffer(a.shape) as b:
        b.from_host(a)
        np.testing.assert_array_equal(b.to_host(), a)
        np.testing.assert_array_equal(b.to_host(4), a[:4])
        np.testing.assert_array_equal(b.sampled(5, 16), a[:5, ::16])
    with M.DeviceBuffer((3, 32), np.int32) as b:
        x = np.arange(96, dtype=np.int32).reshape(3, 32)
        b.from_host(x)
        np.testing.assert_array_equal(b.sampled(3, 8), x[:, ::8])


def test_bench_ranks_map_one_runtime():
    """bench.py with the gloo coordinator (world size 1, --force-dist): the rank process
    reports one HIP and one HSA runtime, the library's."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist", "--cells-per-gpu", "2048",
                        "--steps", "20", "--warmup", "2", "--no-cpu"], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["config"]["timing_collectives"] == "gloo"
    _one_runtime(line["checks"]["hip_runtime"], "bench.py rank")
