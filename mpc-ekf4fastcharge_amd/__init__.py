"""MI355X batched MPC+EKF fast-charge control step (drop-in for the
per-timestep loop of Rodrigops27/MPC-EKF4FastCharge, runMPC.m:83-112).

Import as ``importlib.import_module("mpc-ekf4fastcharge_amd")``.  The compute
path is libmpcekf.so (HIP, gfx950) behind include/mpcekf.h; this package is the
host-side mirror of the reference's MATLAB function interface.
"""
from .rom import ROM, make_synth_rom  # noqa: F401

__all__ = ["ROM", "make_synth_rom", "mpcekf"]


def __getattr__(name):
    # the ctypes layer loads libmpcekf.so lazily so that `import` works before build()
    if name in ("mpcekf", "Context", "runMPC", "predMat", "hildreth", "constraintsMPC", "make_config"):
        from . import mpcekf as _m
        return _m if name == "mpcekf" else getattr(_m, name)
    raise AttributeError(name)
