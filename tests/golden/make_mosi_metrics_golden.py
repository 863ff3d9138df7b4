"""Generate tests/golden/mosi_metrics.json by running the REAL reference epoch bookkeeping for the MOSI
UTT-Fusion config: ``MetricRecorder`` (MML_Suite/experiment_utils/metric_recorder.py) built from the metric
block of configs/mosi/centralised/utt_fusion_base_training.yaml (``MSA: metrics.msa_binary_classification``,
``ConfusionMatrix: sklearn.metrics.confusion_matrix(labels=[0, 1, 2])``), fed pattern-grouped validation
batches through ``update_group_all`` as UttFusionModel.validation_step does (utt_fusion.py:231-244), then
``calculate_all_groups`` + ``flatten_dict`` as _train_loop does.  Predictions are seeded numpy draws over the
seven missing-modality patterns of the YAML's validation split (stored in the fixture); one pattern has no
neutral sample, one no non-neutral sample (the reference's per-metric error path).

    python tests/golden/make_mosi_metrics_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/MML_Suite"
sys.path.insert(0, HERE)
from make_data_golden import _write_stubs  # noqa: E402

PATTERNS = ["atv", "a", "v", "t", "av", "at", "tv"]  # utt_fusion_base_training.yaml:99
BATCHES = [32, 32, 32, 32, 17]


def main() -> None:
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import yaml
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from config.metric_config import MetricConfig
    from experiment_utils.metric_recorder import MetricRecorder
    from experiment_utils.utils import flatten_dict

    with open(os.path.join(REF, "configs/mosi/centralised/utt_fusion_base_training.yaml")) as f:
        text = f.read()
    block = text[text.index("\nmetrics:\n") + 1:text.index("\nlogging:")]
    mcfg_dict = yaml.safe_load(block)["metrics"]
    rec = MetricRecorder(MetricConfig.from_dict(mcfg_dict))

    rng = np.random.default_rng(2025)
    out = {"metric_config": mcfg_dict, "patterns": PATTERNS, "batches": []}
    for n in BATCHES:
        m_types = rng.choice(PATTERNS, size=n)
        targets = rng.integers(0, 3, size=n)
        targets[m_types == "a"] = 1       # pattern "a": neutral only (no non-neutral sample)
        targets[m_types == "v"] = np.where(targets[m_types == "v"] == 1, 2, targets[m_types == "v"])  # no neutral
        preds = np.where(rng.random(n) < 0.6, targets, rng.integers(0, 3, size=n))
        # the pattern-grouped eval collate (data/mosi.py:236-251): one validation_step per group
        for p in dict.fromkeys(m_types.tolist()):
            sel = m_types == p
            rec.update_group_all("classification", predictions=preds[sel], targets=targets[sel], m_types=m_types[sel])
        out["batches"].append({"targets": targets.tolist(), "preds": preds.tolist(), "m_types": m_types.tolist()})
    res = flatten_dict(rec.calculate_all_groups(epoch=1, loss=0.5))
    out["results"] = {k: (np.asarray(v).tolist() if isinstance(v, np.ndarray) else float(v)) for k, v in res.items()}
    dst = os.path.join(HERE, "mosi_metrics.json")
    with open(dst, "w") as f:
        json.dump(out, f)
    print("wrote", dst, len(out["results"]), "result keys")


if __name__ == "__main__":
    main()
