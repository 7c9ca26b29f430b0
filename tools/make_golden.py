#!/usr/bin/env python3
"""Generates tests/golden/*.npz with the numpy oracle (oracle/oracle_np.py).

The reference itself cannot run here (MATLAB, missing ROM), so
these vectors come from the MATLAB-faithful numpy restatement on the synthetic
ROM.  They pin the C oracle and the kernels to that restatement (parity with the
MATLAB reference stays unpinned).  Re-run only when the oracle or ROM generator
changes:  python tools/make_golden.py
"""
import hashlib
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_np as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def rom_hash(rom):
    h = hashlib.sha256()
    for k, v in sorted(rom.to_npz_dict().items()):
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def run_cells(rom, soc0, tc, steps, cfg=None, tc_traj=None):
    outs = [O.run_cell(rom, s, t, steps, cfg, tc_traj=None if tc_traj is None else tc_traj[:, i])
            for i, (s, t) in enumerate(zip(soc0, tc))]
    res = {k: np.stack([o[k] for o in outs], axis=1) for k in ("u", "v", "soc", "phise", "nexec")}
    res["status"] = np.array([o["status"][-1] for o in outs])
    res["zk_last"] = np.stack([o["zk"][-1] for o in outs])
    res["zbk_last"] = np.stack([o["zbk"][-1] for o in outs])
    return res


def make_mb(rom, hsh):
    """Model-blend ('MB') EKF trajectories (iterEKF.m:90-102 and the MB branches): the fixture
    the C oracle and the kernel's MB variant will be checked against."""
    rng = np.random.Generator(np.random.PCG64(0x5EED))
    soc0, tc = rng.uniform(5, 30, 4), rng.uniform(20, 30, 4)
    r = run_cells(rom, soc0, tc, 200, {"method": "MB"})
    np.savez_compressed(os.path.join(OUT, "mb_batch4_200.npz"), rom_hash=hsh, soc0=soc0, tc=tc, **r)


def tprofile(steps):
    k = np.arange(steps)[:, None]
    base = np.array([[20.0, 25.0, 10.0, 30.0]])
    slope = np.array([[0.02, -0.01, 0.15, 0.05]])
    ripple = np.array([[1.0, 2.5, 0.5, 0.0]])
    return base + slope * k + ripple * np.sin(k / 17.0)


def make_tprofile(rom, hsh):
    soc0 = np.array([10.0, 35.0, 20.0, 60.0])
    steps = 300
    tct = tprofile(steps)
    r = run_cells(rom, soc0, tct[0], steps, tc_traj=tct)
    np.savez_compressed(os.path.join(OUT, "tprofile4_300.npz"), rom_hash=hsh, soc0=soc0, tc=tct[0], tc_traj=tct, **r)


def _wide_cell(args):
    soc0, tc, steps = args
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    o = O.run_cell(P.make_synth_rom(), soc0, tc, steps, {"Np": 20, "Nc": 10})
    return o


def make_wide(rom, hsh):
    """configs[4]'s horizons (Np = 20 / Nc = 10) on the MATLAB-faithful restatement (dense
    H = M*(E\\M'), hildreth.m:28-42): 8 cells of the batched workload x 400 steps, and 4
    near-limit cells (88-95 % SOC, the voltage / eta rows active, Hildreth into maxIter)
    x 200 steps.  The GPU and the C oracle evaluate the rank-10 defined arithmetic
    (DESIGN.md §3); this fixture holds them to the dense form within north_star's 1e-6."""
    from multiprocessing import Pool
    rng = np.random.Generator(np.random.PCG64(0x5EED))
    soc0, tc = rng.uniform(5, 30, 8), rng.uniform(20, 30, 8)
    soc0n, tcn = np.array([88.0, 90.5, 93.0, 95.0]), np.array([25.0, 21.0, 29.0, 24.0])
    jobs = [(s, t, 400) for s, t in zip(soc0, tc)] + [(s, t, 200) for s, t in zip(soc0n, tcn)]
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        outs = pool.map(_wide_cell, jobs)
    for name, sl, s0, t0 in (("wide_batch8_400.npz", slice(0, 8), soc0, tc), ("wide_near4_200.npz", slice(8, 12), soc0n, tcn)):
        o = outs[sl]
        r = {k: np.stack([x[k] for x in o], axis=1) for k in ("u", "v", "soc", "phise", "nexec")}
        r["status"] = np.array([x["status"][-1] for x in o])
        np.savez_compressed(os.path.join(OUT, name), rom_hash=hsh, soc0=s0, tc=t0, Np=20, Nc=10, **r)


def main():
    os.makedirs(OUT, exist_ok=True)
    if "--wide-only" in sys.argv:
        P = importlib.import_module("mpc-ekf4fastcharge_amd")
        rom = P.make_synth_rom()
        t0 = time.time()
        make_wide(rom, rom_hash(rom))
        print(f"wide fixtures written in {time.time() - t0:.0f} s")
        return
    if "--tprofile-only" in sys.argv:
        P = importlib.import_module("mpc-ekf4fastcharge_amd")
        rom = P.make_synth_rom()
        make_tprofile(rom, rom_hash(rom))
        return
    if "--mb-only" in sys.argv:
        P = importlib.import_module("mpc-ekf4fastcharge_amd")
        rom = P.make_synth_rom()
        make_mb(rom, rom_hash(rom))
        return
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    rom = P.make_synth_rom()
    hsh = rom_hash(rom)
    t0 = time.time()
    # 1. the runMPC.m cell: SOC0 = 10 %, TC = 25 degC, 3001 steps (runMPC.m:8-13)
    r = run_cells(rom, [10.0], [25.0], 3001)
    np.savez_compressed(os.path.join(OUT, "runmpc_soc10_tc25.npz"), rom_hash=hsh, soc0=[10.0], tc=[25.0], **r)
    # 2. eight cells of the batched workload, 200 steps
    rng = np.random.Generator(np.random.PCG64(0x5EED))
    soc0, tc = rng.uniform(5, 30, 8), rng.uniform(20, 30, 8)
    r = run_cells(rom, soc0, tc, 200)
    np.savez_compressed(os.path.join(OUT, "batch8_200.npz"), rom_hash=hsh, soc0=soc0, tc=tc, **r)
    # 3. edge cells: thetae < 0 error (SOC0 130 %), EKF lock-out (SOC0 -15 %: warnCount > 10),
    #    near target (88 %: voltage limit + Hildreth maxIter), exact set-point temperatures
    #    (15 / 35 degC) and a set-point SOC (25 %)
    soc0 = np.array([130.0, 88.0, 25.0, 60.0, 5.0, -15.0])
    tc = np.array([25.0, 30.0, 15.0, 35.0, 25.0, 25.0])
    r = run_cells(rom, soc0, tc, 400)
    np.savez_compressed(os.path.join(OUT, "edge_cells_400.npz"), rom_hash=hsh, soc0=soc0, tc=tc, **r)
    # 4. single-temperature ROM (nT = 1: the single-setpoint branches of getXind/OB_step)
    rom1 = P.make_synth_rom(T_degC=(25.0,))
    r = run_cells(rom1, [12.0, 40.0], [25.0, 22.0], 200)
    np.savez_compressed(os.path.join(OUT, "rom_nt1_200.npz"), rom_hash=rom_hash(rom1), soc0=[12.0, 40.0],
                        tc=[25.0, 22.0], **r)
    # 5. model-blend EKF variant
    make_mb(rom, hsh)
    # 5b. a temperature profile per step (OB_step / iterEKF / EKFmatsHandler take Tc every
    #     call): warming ramps with a ripple, one profile crossing a set-point and the table
    #     grid ends (0 and 50 degC, clamped), 300 steps
    make_tprofile(rom, hsh)
    # 5c. the wide horizons (configs[4]: Np = 20 / Nc = 10)
    make_wide(rom, hsh)
    # 6. per-function vectors: predMat and hildreth (incl. the zero row of G_soc)
    rng = np.random.default_rng(11)
    n = 24
    a = np.concatenate([rng.uniform(0.2, 0.999, (n, 5)), np.ones((n, 1))], 1)
    Cr = np.concatenate([rng.normal(0, 1e-3, (n, 5)), rng.normal(0, 1e-5, (n, 1))], 1)
    D = rng.normal(0, 1e-3, n)
    Phi = np.zeros((n, 5, 7))
    G = np.zeros((n, 5, 2))
    for i in range(n):
        Phi[i], G[i] = O.pred_mat(a[i], Cr[i], D[i], 5, 2)
    E = np.zeros((n, 2, 2))
    F = rng.normal(0, 1, (n, 2))
    M = rng.normal(0, 1, (n, 23, 2))
    gam = rng.normal(0.5, 1.0, (n, 23))
    M[:, 18, :] = 0.0                           # G_soc row 1 is identically zero
    gam[: n // 2, 18] = np.abs(gam[: n // 2, 18]) + 0.1   # gamma > 0: lambda stays 0
    gam[n // 2:, 18] = -np.abs(gam[n // 2:, 18]) - 0.1    # gamma < 0: inf/NaN period-2 pattern
    lam0 = np.abs(rng.normal(0, 0.1, (n, 23)))
    DU = np.zeros((n, 2))
    lam = np.zeros((n, 23))
    nexec = np.zeros(n, dtype=np.int64)
    with np.errstate(all="ignore"):
        for i in range(n):
            A = rng.normal(0, 1, (2, 2))
            E[i] = A @ A.T + 0.5 * np.eye(2)
            E[i] = (E[i] + E[i].T) / 2
            DU[i], lam[i], nexec[i] = O.hildreth(E[i], F[i], M[i], gam[i], lam0[i].copy(), 100)
    np.savez_compressed(os.path.join(OUT, "functions.npz"), a=a, C=Cr, D=D, Phi=Phi, G=G, E=E, F=F, M=M,
                        gamma=gam, lam0=lam0, DU=DU, lam=lam, nexec=nexec)
    print(f"golden fixtures written to {OUT} in {time.time() - t0:.0f} s (rom {hsh[:12]})")


if __name__ == "__main__":
    main()
