"""Where the conv family's HBM bytes come from, per step: compulsory operand bytes
versus the split-K slab bytes the tuned tile configurations add.

For every conv launch of the batch-128 step (the tuned table's entries with their per-step counts; the
engine's selection in engine.py:set_algos — the fused dgrad+wgrad launch where the table holds a `bwd`
pair, the stem's weight gradient alone) it sums
  * compulsory bytes: forward x + w + y, backward dy + x + w + dx + dw (fp32, every operand once);
  * slab bytes: the launch's split-K workspace (tspm_conv_*_workspace), written once and read once.
The workspace query is host arithmetic in libtspm.so (no GPU needed).  Compare the total with the PMC
figure (profiles/r3_v1_pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE over the conv kernels).

  python scripts/conv_traffic_budget.py [--table tuned/mi355x_b128.json] [--json out.json]
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from tspm_amd import _lib as L  # noqa: E402


def main() -> None:
    path = os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "tuned", "mi355x_b128.json")
    if "--table" in sys.argv:
        path = sys.argv[sys.argv.index("--table") + 1]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    lib = L.lib()
    tab = json.load(open(path))["entries"]
    pairs = {tuple(e["shape"]): e for e in tab if e["kind"] == "bwd"}
    rows, tot = [], {"compulsory": 0, "slabs": 0}
    for e in tab:
        if e["kind"] not in ("fwd", "wgrad"):
            continue
        n, h, w, c, k, r, s, st, pad = e["shape"]
        p, q = (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1
        shp = L.ConvShape(n, h, w, c, k, r, s, st, pad, p, q)
        x, y, wt = 4 * n * h * w * c, 4 * n * p * q * k, 4 * k * r * s * c
        if e["kind"] == "fwd":
            a = L.ConvAlgo(*e["algo"][:6])
            comp, slab = x + wt + y, 2 * lib.tspm_conv_fwd_workspace(ctypes.byref(shp), ctypes.byref(a))
            kind = "fwd"
        elif tuple(e["shape"]) in pairs:
            pa = pairs[tuple(e["shape"])]["algo"]
            ad, aw = L.ConvAlgo(*pa[:6]), L.ConvAlgo(*pa[6:12])
            comp = y + x + wt + x + wt  # dy, x, w read; dx, dw written
            slab = 2 * (lib.tspm_conv_dgrad_workspace(ctypes.byref(shp), ctypes.byref(ad))
                        + lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(aw)))
            kind = "bwd"
        else:  # the stem: weight gradient only (no input gradient)
            a = L.ConvAlgo(*e["algo"][:6])
            comp, slab = y + x + wt, 2 * lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(a))
            kind = "wgrad"
        cnt = e["count"]
        rows.append({"kind": kind, "shape": e["shape"], "count": cnt, "compulsory_mb": round(comp * cnt / 1e6, 2),
                     "slab_mb": round(slab * cnt / 1e6, 2)})
        tot["compulsory"] += comp * cnt
        tot["slabs"] += slab * cnt
    rows.sort(key=lambda r: -r["slab_mb"])
    doc = {"table": os.path.relpath(path, REPO), "launches": sum(r["count"] for r in rows),
           "compulsory_gb": round(tot["compulsory"] / 1e9, 3), "slab_gb": round(tot["slabs"] / 1e9, 3),
           "by_kind": {k: {"compulsory_gb": round(sum(r["compulsory_mb"] for r in rows if r["kind"] == k) / 1e3, 3),
                           "slab_gb": round(sum(r["slab_mb"] for r in rows if r["kind"] == k) / 1e3, 3)}
                       for k in ("fwd", "bwd", "wgrad")},
           "top_slab_launches": rows[:10]}
    print(json.dumps(doc, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
