"""Write a merged tuned table (every tuned/*.json entry) with the variant-4 twins of scripts/split_ab.py --json
switched in where they were faster in isolation (v4_us <= THRESHOLD * v1_us), for a TSPM_TUNED_FILE A/B.
Fused dgrad + wgrad ("bwd") entries switch when both twins exist and their sum is faster.
    python scripts/twin_table.py AB_JSON OUT [THRESHOLD]"""
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ab, out = sys.argv[1], sys.argv[2]
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.97
entries = {}
for p in sorted(glob.glob(os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "tuned", "*.json"))):
    for e in json.load(open(p)).get("entries", []):
        entries[(e["kind"],) + tuple(e["shape"][:8])] = e
twin = {(r["kind"],) + tuple(r["shape"][:8]): r for r in json.load(open(ab))["rows"]}
changed = []
for k, e in entries.items():
    if k[0] in ("fwd", "dgrad", "wgrad") and k in twin and twin[k]["v4_us"] <= thr * twin[k]["v1_us"]:
        if list(e["algo"]) == list(twin[k]["v1_algo"]):
            changed.append({"kind": k[0], "shape": list(k[1:]), "algo": twin[k]["v4_algo"]})
    elif k[0] == "bwd":
        kd, kw = ("dgrad",) + k[1:], ("wgrad",) + k[1:]
        if kd in twin and kw in twin:
            d, w = twin[kd], twin[kw]
            if d["v4_us"] + w["v4_us"] <= thr * (d["v1_us"] + w["v1_us"]):
                ad, aw = list(e["algo"][:6]), list(e["algo"][6:12])
                if ad[5] in (1, 2) and aw[5] == ad[5] and ad[3] <= 2 and aw[3] <= 2:
                    changed.append({"kind": "bwd", "shape": list(k[1:]), "algo": ad[:5] + [4] + aw[:5] + [4]})
for c in changed:
    entries[(c["kind"],) + tuple(c["shape"][:8])] = dict(entries[(c["kind"],) + tuple(c["shape"][:8])], algo=c["algo"])
json.dump({"entries": list(entries.values()), "changed": changed}, open(out, "w"), indent=1)
print(f"{len(changed)} entries switched to their variant-4 twins -> {out}")
