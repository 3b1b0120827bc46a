"""Census for the north-star K1 bound-pruning idea: how many pixels would
still need the exact Shi-Tomasi response if every pixel first had the cheap bounds
lambda_max in [lo, hi] = [max(a, c), a + c] (a = Sxx/9, c = Syy/9; the tensor is positive semidefinite,
so sqrt((a - c)^2 + 4 b^2) lies in [|a - c|, a + c]).

A pixel p with gate a + c > thr (the reference's precheck, feature_point_shi_tomas_detector.cpp:96) is
  * decided "not a candidate" if hi(p) <= max(thr, max over its 4 neighbours n of lo(n));
  * decided "candidate" if lo(p) > thr and lo(p) > max over n of hi(n);
  * undecided otherwise (its exact value matters to its own decision).
A decided pixel may still need its exact value as a neighbour of an undecided one; that count is given
too ("needed"). Pure numpy on the CPU oracle's exact integer tensor sums (oracle.tensor_sums); the
reference's float rounding is ignored (bounds are compared in float64), so the counts are the idea's
ceiling, not an exact kernel plan. Run: python tools/k1_bounds_census.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

THR = 40.0


def census(img):
    sxx, syy, sxy = (x.astype(np.float64) for x in O.tensor_sums(img))
    a, c = sxx / 9.0, syy / 9.0
    R, C = img.shape
    valid = np.zeros((R, C), bool)
    valid[2:R - 2, 2:C - 2] = True  # responses live in rows/cols [2, R-3] (the reference's loop bounds)
    gate = (a + c > THR) & valid
    lo = np.where(gate, np.maximum(a, c), 0.0)
    hi = np.where(gate, a + c, 0.0)
    pad = lambda m: np.pad(m, 1)
    lp, hp = pad(lo), pad(hi)
    nb_lo = np.maximum.reduce([lp[:-2, 1:-1], lp[2:, 1:-1], lp[1:-1, :-2], lp[1:-1, 2:]])
    nb_hi = np.maximum.reduce([hp[:-2, 1:-1], hp[2:, 1:-1], hp[1:-1, :-2], hp[1:-1, 2:]])
    no = gate & (hi <= np.maximum(THR, nb_lo))
    yes = gate & (lo > THR) & (lo > nb_hi)
    und = gate & ~no & ~yes
    up = pad(und)
    nb_und = up[:-2, 1:-1] | up[2:, 1:-1] | up[1:-1, :-2] | up[1:-1, 2:]
    needed = gate & (und | nb_und)
    n = valid.sum()
    return {"pixels": int(n), "gate": gate.sum() / n, "undecided": und.sum() / n, "needed_exact": needed.sum() / n,
            "decided_no": no.sum() / n, "decided_yes": yes.sum() / n}


for pat in ("noise", "checker"):
    for seed in (1234, 99):
        img = O.make_frame(pat, seed, 1080, 1920, 64 if pat == "checker" else 16)
        r = census(img)
        print(f"{pat:7s} seed {seed}: " + ", ".join(f"{k} {v:.4f}" if isinstance(v, float) else f"{k} {v}" for k, v in r.items()))
