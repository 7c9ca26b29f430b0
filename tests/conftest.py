"""Shared test setup.  GPU tests are marked ``gpu`` and run only on the MI355X box."""
import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pkg():
    return importlib.import_module("mpc-ekf4fastcharge_amd")


@pytest.fixture(scope="session")
def P():
    return pkg()


@pytest.fixture(scope="session")
def rom(P):
    return P.make_synth_rom()


@pytest.fixture(scope="session")
def oc():
    import oracle_c
    oracle_c.build()
    return oracle_c


def batch_inputs(n, seed=0x5EED):
    """SURVEY.md §8(d) config 2/3 inputs: SOC0 ~ U[5,30] %, TC ~ U[20,30] degC, PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(5, 30, n), rng.uniform(20, 30, n)


@pytest.fixture(scope="session")
def M(P):
    return importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
