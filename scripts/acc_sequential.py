"""Group-sequential correction of the accuracy-protocol equivalence test.

The from-scratch TOST of round 4 was evaluated after every batch of paired seeds and the pairs were added until
it passed, so its nominal 90 % interval (two one-sided 5 % tests) does not hold its error rate.  This script
prices those interim looks: for looks after n_1 < ... < n_K pairs it finds the one-sided critical value c of a
Pocock boundary (the same c at every look) and of an O'Brien-Fleming boundary (c * sqrt(n_K / n_k) at look k)
such that, under the null, the probability that the standardised running mean difference crosses the boundary
at ANY look is alpha = 0.05 — by Monte Carlo of the partial sums of iid N(0, 1) increments (independent
increments, the canonical joint law of sequential z statistics).  The corrected interval at the final look is
mean +- c * se, with c scaled by t_{0.95, n-1} / z_{0.95} for the estimated variance; equivalence within +-0.2 pp
holds when that interval lies inside (-0.2, +0.2).

    python scripts/acc_sequential.py profiles/r4_accuracy_parity.json --looks 33,42,52,62,74,86,98 \
        [--looks-alt 12,21,33,42,52,62,74,86,98] > profiles/r5_accuracy_parity_sequential.json
"""
from __future__ import annotations

import argparse
import json

import numpy as np
from scipy import stats

ALPHA = 0.05
MARGIN = 0.2


def crossing_prob(looks, c_of_k, sims, rng):
    n = np.asarray(looks, dtype=np.int64)
    inc = np.diff(np.concatenate([[0], n]))
    hit = np.zeros(sims, dtype=bool)
    s = np.zeros(sims)
    for k, dn in enumerate(inc):
        s += rng.standard_normal(sims) * np.sqrt(dn)
        hit |= s / np.sqrt(n[k]) > c_of_k(k)
    return hit.mean()


def solve(looks, shape, sims=400_000, seed=0):
    """Critical value c of the boundary family `shape` ('pocock' | 'obf') with P(cross at any look) = ALPHA."""
    n = np.asarray(looks, dtype=np.float64)
    lo, hi = stats.norm.ppf(1 - ALPHA), 4.0
    for _ in range(30):
        mid = 0.5 * (lo + hi)
        rng = np.random.default_rng(seed)  # common random numbers: monotone in c
        if shape == "pocock":
            p = crossing_prob(looks, lambda k: mid, sims, rng)
        else:
            p = crossing_prob(looks, lambda k: mid * np.sqrt(n[-1] / n[k]), sims, rng)
        lo, hi = (mid, hi) if p > ALPHA else (lo, mid)
    return 0.5 * (lo + hi)


def interval(d, c):
    m, sd = float(d.mean()), float(d.std(ddof=1))
    se = sd / np.sqrt(len(d))
    scale = stats.t.ppf(1 - ALPHA, len(d) - 1) / stats.norm.ppf(1 - ALPHA)
    h = c * scale * se
    return [round(m - h, 3), round(m + h, 3)], bool(m - h > -MARGIN and m + h < MARGIN)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("parity_json")
    ap.add_argument("--looks", required=True, help="pairs at each interim look, ascending; the last = all pairs")
    ap.add_argument("--looks-alt", default=None, help="a second look schedule (sensitivity)")
    a = ap.parse_args()
    doc = json.load(open(a.parity_json))
    r = np.asarray(doc["test_accuracy_ai"]["reference"])
    o = np.asarray(doc["test_accuracy_ai"]["ours"])
    d = 100 * (o - r)
    out = {"what": __doc__.split("\n\n")[0], "source": a.parity_json, "paired_runs": int(len(d)),
           "endpoint": doc.get("endpoint"), "margin_pp": MARGIN, "alpha_one_sided": ALPHA,
           "naive": {"ci90_pp": doc["test_accuracy_ai"]["paired"]["ci90_pp"],
                     "equivalent": doc["test_accuracy_ai"]["paired"]["equivalent_at_0.2pp"]},
           "delta_pp": round(float(d.mean()), 3), "paired_sd_pp": round(float(d.std(ddof=1)), 3)}
    for name, spec in (("looks", a.looks), ("looks_alt", a.looks_alt)):
        if not spec:
            continue
        looks = [int(x) for x in spec.split(",")]
        if looks[-1] != len(d):
            raise SystemExit(f"last look {looks[-1]} != {len(d)} pairs")
        res = {"looks": looks}
        for shape in ("pocock", "obf"):
            c = solve(looks, shape)
            ci, eq = interval(d, c)
            res[shape] = {"critical_z_final_look": round(c, 4), "ci_pp": ci, "equivalent": eq}
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
