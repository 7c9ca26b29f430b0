"""Ulp-ensemble envelopes of the chaotic tails (tests/golden/env_*.npz, written by
tools/make_golden.py make_envelopes from the MATLAB-faithful numpy restatement).

Where hildreth.m runs into maxIter on infeasible QPs every step -- the last ~100 steps of
the runMPC.m charge, steps ~25-200 of the Np = 20 near-limit cells -- one trajectory
cannot be followed to 1e-6 by any implementation (a 1-ulp change of SOC0 moves it by
O(1)).  The envelope is the per-step [min, max] of the restatement over an ensemble of
indistinguishable runs: SOC0 moved by a few ulps, and the command moved by a random
-1..1 ulp every step (ulp-level implementation differences).  A trajectory is held to
lie inside it, widened by north_star's 1e-6 relative."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("u", "v", "soc", "phise")
RTOL = 1e-6
RUN_TAIL = (2800, 3001)    # the runMPC cell: the numpy fixture test holds steps < ~2,900
NEAR_TAIL = (25, 200)      # the Np = 20 near-limit cells: the fixture test holds steps < 25


def load(name):
    return np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))


# Window statistics (check_near, check_tail_stats) are held to the members' range widened by
# this fraction of its width on each side.  One more trajectory drawn like the N members
# lands outside their raw [min, max] with probability 2 / (N + 1) per statistic, and the
# checks make 12 per cell (48 for the near-limit cells): at N = 73 a fair sample fails some
# raw range most of the time.  A quarter of the range still separates another attractor or a
# biased implementation (the cells' statistics differ between cells by several ranges).
STAT_MARGIN = 0.25


def outside(x, lo, hi, rtol=RTOL, margin=0.0):
    """Boolean mask of entries of x outside [lo, hi] widened by rtol * max(|lo|, |hi|) and
    by margin * (hi - lo)."""
    tol = rtol * np.maximum(np.abs(lo), np.abs(hi)) + margin * (hi - lo)
    return (x < lo - tol) | (x > hi + tol)


def check_run(out, e, window=RUN_TAIL):
    """The runMPC cell's trajectories [3001] (or [3001, 1]) against env_runmpc_3001."""
    a, b = window
    for k in KEYS:
        x = np.asarray(out[k]).reshape(-1)[a:b]
        bad = outside(x, e[k + "_min"][a:b], e[k + "_max"][a:b])
        assert not bad.any(), f"{k}: {int(bad.sum())} steps outside the envelope, first at {a + int(np.argmax(bad))}"
    soc = np.asarray(out["soc"]).reshape(-1)
    t90 = int(np.argmax(soc >= 0.90)) if (soc >= 0.90).any() else -1
    assert e["t90"].min() <= t90 <= e["t90"].max(), (t90, e["t90"].min(), e["t90"].max())


def check_near(out, e, window=NEAR_TAIL):
    """The 4 near-limit cells' trajectories [200, 4] against env_wide_near4_200.

    These closed loops are chaotic at Np = 20: within a few dozen steps the ensemble's
    members range over the whole attractor (u anywhere between the current limits at a
    given step), so no per-step band from a finite ensemble holds an independent
    trajectory.  What is held is the trajectory's distribution over the window: its mean,
    10th and 90th percentile of u, v, soc and phise, and its final SOC, each inside the
    range the members' own statistics span (widened by 1e-6 relative and STAT_MARGIN)."""
    a, b = window
    stats = {"wmean": lambda x: x.mean(0), "wlo": lambda x: np.percentile(x, 10, axis=0),
             "whi": lambda x: np.percentile(x, 90, axis=0)}
    for k in KEYS:
        x = np.asarray(out[k])[a:b]
        for nm, f in stats.items():
            m = e[f"{k}_{nm}"]                      # [4 cells, members]
            bad = outside(f(x), m.min(1), m.max(1), margin=STAT_MARGIN)
            assert not bad.any(), (f"{k} {nm}: cells {np.nonzero(bad)[0].tolist()} outside the members' range: "
                                   f"{f(x)[bad]} vs [{m.min(1)[bad]}, {m.max(1)[bad]}]")
    end = np.asarray(out["soc"])[-1]
    bad = outside(end, e["soc_end"].min(1), e["soc_end"].max(1), margin=STAT_MARGIN)
    assert not bad.any(), f"final SOC of cells {np.nonzero(bad)[0].tolist()} outside the members' range"


def check_tail_stats(out, e):
    """One cell's trajectories [steps] (or [steps, 1]) over its chaotic tail [tail0, end)
    against the members of a ulp ensemble (tests/golden/handles_runmpc_3001): the window
    mean, 10th and 90th percentile of u, v, soc and phise each inside the range the
    members' own statistics span (widened by 1e-6 relative and STAT_MARGIN), and the step to 90 % SOC
    one of the members' (check_near's rule for a single cell)."""
    a = int(e["tail0"])
    stats = {"wmean": lambda x: x.mean(), "wlo": lambda x: np.percentile(x, 10), "whi": lambda x: np.percentile(x, 90)}
    for k in KEYS:
        x = np.asarray(out[k]).reshape(-1)[a:]
        for nm, f in stats.items():
            m = e[f"{k}_{nm}"]
            assert not outside(np.array([f(x)]), m.min(), m.max(), margin=STAT_MARGIN).any(), \
                f"{k} {nm} over steps {a}-: {f(x)!r} outside the members' [{m.min()!r}, {m.max()!r}]"
    soc = np.asarray(out["soc"]).reshape(-1)
    t90 = int(np.argmax(soc >= 0.90)) if (soc >= 0.90).any() else -1
    assert e["t90"].min() <= t90 <= e["t90"].max(), (t90, e["t90"].min(), e["t90"].max())
