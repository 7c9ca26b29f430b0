#!/usr/bin/env python3
"""Error of the electrode tables' linear-in-T interpolation against an Arrhenius handle
k(T) = k_ref exp(Ea/R (1/T_ref - 1/T)) (the usual form of the ROM's k0 and of any
Arrhenius-scaled Rf / Cdleff; the reference's .mat is not in the repository, so Ea is a
parameter).  The library is exact at table temperatures (the lookup's weight is 0) and
linear between them (include/mpcekf.h mpcekf_electrode, ETab::f).

    python tools/k0_interp_error.py            -> DESIGN.md 3's table"""
import numpy as np

R = 8.314462618


def worst_rel_error(Ea, grid_C):
    T = np.asarray(grid_C, float) + 273.15
    worst = 0.0
    for a, b in zip(T[:-1], T[1:]):
        t = np.linspace(a, b, 2001)
        k = np.exp(-Ea / R / t)
        lin = np.exp(-Ea / R / a) + (t - a) / (b - a) * (np.exp(-Ea / R / b) - np.exp(-Ea / R / a))
        worst = max(worst, float(np.max(np.abs(lin / k - 1))))
    return worst


def r03_default(setpoints, TC=(25.0,)):
    """matlab/mpcekf_rom_struct.m's default grid: set-points, TC, guards, widest split."""
    g = sorted(set(setpoints) | set(TC))
    if len(g) + 2 <= 8:
        g = [g[0] - 10] + g + [g[-1] + 10]
    while len(g) < 8:
        k = int(np.argmax(np.diff(g)))
        g = g[:k + 1] + [(g[k] + g[k + 1]) / 2] + g[k + 1:]
    return g


grids = {"r02 default, ROM at 15/25/35 degC: linspace(5, 45, 6), h = 8 K, 25 degC off-grid": np.linspace(5, 45, 6),
         "r03 default, same ROM: " + ", ".join(f"{t:g}" for t in r03_default([15, 25, 35])): r03_default([15, 25, 35]),
         "h = 5 K (15..35)": np.arange(15, 35.1, 5),
         "h = 2.5 K (15..35)": np.arange(15, 35.1, 2.5)}
print("| grid | Ea = 30 kJ/mol | Ea = 50 kJ/mol | Ea = 70 kJ/mol |")
print("|---|---|---|---|")
for name, g in grids.items():
    print(f"| {name} | " + " | ".join(f"{100 * worst_rel_error(Ea, g):.2f} %" for Ea in (30e3, 50e3, 70e3)) + " |")
