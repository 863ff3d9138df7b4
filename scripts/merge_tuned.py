"""Merge tuned tables for an A/B run: every tuned/*.json entry (the engine's default set), optionally
overridden by the entries of a new partial table.  usage: merge_tuned.py OUT [NEW_PARTIAL]"""
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
entries = {}
for p in sorted(glob.glob(os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "tuned", "*.json"))):
    for e in json.load(open(p)).get("entries", []):
        entries[(e["kind"],) + tuple(e["shape"][:8])] = e
n_new = 0
if len(sys.argv) > 2:
    for e in json.load(open(sys.argv[2])).get("entries", []):
        k = (e["kind"],) + tuple(e["shape"][:8])
        if k not in entries or tuple(entries[k]["algo"]) != tuple(e["algo"]):
            n_new += 1
        entries[k] = e
json.dump({"entries": list(entries.values())}, open(sys.argv[1], "w"), indent=1)
print(f"{len(entries)} entries, {n_new} changed")
