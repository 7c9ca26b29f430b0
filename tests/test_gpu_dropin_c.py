"""GPU: the drop-in stage route driven from C (tools/dropin_loop.c, built by
__graft_entry__.build into _build/libdropin_loop.so) -- the sequence a MEX host runs each
step (get_scalars, plant_step, ekf_step, get_scalars, linearize kept on the device,
lin_fields, mpc_diag, mpc_step_ex), with every output array a fresh malloc as MATLAB's
mxArrays (or reused), synchronous and through the _async twins with the device hand-offs
(Vcell, zk(end)) and one synchronisation per step.  Each mode's last command equals the
fused step's bit for bit (include/mpcekf.h)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import batch_inputs

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "mpc-ekf4fastcharge_amd", "_build", "libdropin_loop.so")


@pytest.mark.parametrize("mode", [0, 1, 2, 3], ids=["sync", "async", "sync-reuse", "async-reuse"])
@pytest.mark.parametrize("n", [64, 1000])
def test_c_driven_stage_route_equals_the_fused_step(M, mode, n):
    import importlib
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    assert os.path.exists(SO), "libdropin_loop.so missing: run __graft_entry__.build()"
    lib = C.CDLL(SO)
    lib.dropin_loop.restype = C.c_int
    rom = P.make_synth_rom()
    soc0, tc = batch_inputs(n, seed=91)
    sc = M.Context.SCALARS
    sa = np.array([sc.index(k) for k in ("SOCnAvg", "SOCpAvg")], dtype=np.int32)
    sb = np.array([sc.index(k) for k in ("x0", "SigmaX0", "priorI")], dtype=np.int32)
    fields = np.array(list(range(20, 27)) + [28] + list(range(29, 35)), dtype=np.int32)
    uk = np.zeros(n)
    ms = np.zeros(7)
    tot, byt = C.c_double(), C.c_double()
    ip = lambda x: x.ctypes.data_as(C.POINTER(C.c_int32))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
    steps, warm = 12, 3
    with M.Context(rom, n, M.make_config(bounds=True)) as ctx:
        ctx.init_cells(soc0, tc)
        rc = lib.dropin_loop(ctx.h, C.c_int64(n), C.c_int32(ctx.nz), C.c_int32(steps), C.c_int32(warm),
                             C.c_int32(mode), dp(tc), ip(sa), len(sa), ip(sb), len(sb), ip(fields), len(fields),
                             dp(uk), dp(ms), C.byref(tot), C.byref(byt))
        assert rc == 0, M._lib.load().mpcekf_last_error().decode()
        st = ctx.get_state()
    ref = M.runMPC(rom, soc0, tc, warm + steps)["u"][-1]
    np.testing.assert_array_equal(uk, ref)
    assert (st["status"] == 0).all()
    assert byt.value == (928 if mode & 1 == 0 else 912)   # host bytes per cell-step (nz = 26)
