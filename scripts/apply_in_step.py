"""Apply the configurations an in-step tuning pass accepted (scripts/tune_in_step.py --out X.json: its "changed"
entries) to a tuned table, keeping each entry's previous algo for the record.
    python scripts/apply_in_step.py X.json task-specific-pretraining-multimodal_amd/tuned/mi355x_b128.json NOTE"""
import json
import sys

src, dst, note = sys.argv[1], sys.argv[2], sys.argv[3]
t = json.load(open(dst))
idx = {(e["kind"], tuple(e["shape"][:8])): e for e in t["entries"]}
n = 0
for c in json.load(open(src))["changed"]:
    k = (c["kind"], tuple(c["shape"][:8]))
    e = idx.get(k)
    if e is None:
        e = {"kind": c["kind"], "shape": list(c["shape"]), "algo": c["algo"]}
        t["entries"].append(e)
        idx[k] = e
    elif list(e["algo"]) != list(c["algo"]):
        e.setdefault("algo_before_r5", e["algo"])
    e["algo"] = list(c["algo"])
    e["note_r5"] = note
    n += 1
json.dump(t, open(dst, "w"), indent=1)
print(f"{n} entries updated in {dst}")
