"""scripts/conv_traffic_budget.py (the conv family's HBM byte budget): host-only queries of
libtspm.so, no GPU.  The step's 112 conv launches, and compulsory bytes equal to the operand sizes."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_budget_counts_launches_and_operand_bytes(tmp_path):
    out = tmp_path / "b.json"
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "conv_traffic_budget.py"), "--json", str(out)],
                   check=True, capture_output=True, timeout=120)
    d = json.loads(out.read_text())
    assert d["launches"] == 112  # 56 forward + 54 fused backward + 2 stem weight gradients
    tab = json.load(open(os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "tuned", "mi355x_b128.json")))
    comp = 0
    for e in tab["entries"]:
        if e["kind"] != "fwd":
            continue
        n, h, w, c, k, r, s, st, pad = e["shape"]
        p, q = (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1
        comp += 4 * (n * h * w * c + k * r * s * c + n * p * q * k) * e["count"]
    assert abs(d["by_kind"]["fwd"]["compulsory_gb"] - comp / 1e9) < 1e-3
    assert d["slab_gb"] > 0 and all(r["slab_mb"] >= 0 for r in d["top_slab_launches"])
