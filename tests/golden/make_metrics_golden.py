"""Generate tests/golden/avmnist_metrics.json by running the REAL reference epoch bookkeeping:
``MetricRecorder`` (MML_Suite/experiment_utils/metric_recorder.py) built from the AVMNIST YAML's
metric config (configs/avmnist/centralised/train_avmnist_resnet.yaml:105-166) fed batch by batch
through ``update_group_all`` as validation_step does, ``calculate_all_groups`` + ``flatten_dict``
as _train_loop does, and ``check_early_stopping`` (train_multimodal.py:329-377) over a loss
sequence.  Inputs are seeded numpy draws (stored in the fixture).

    python tests/golden/make_metrics_golden.py
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

BATCHES = [64, 64, 64, 37]
LOSSES = [2.30, 1.10, 0.80, 0.7995, 0.81, 0.79, 0.7891, 0.80, 0.83, 0.9, 0.7]
PATIENCE, MIN_DELTA = 3, 1e-3


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
    import train_multimodal as tm

    with open(os.path.join(REF, "configs/avmnist/centralised/train_avmnist_resnet.yaml")) as f:
        text = f.read()
    # only the plain `metrics:` mapping (no custom tags inside it)
    block = text[text.index("\nmetrics:\n") + 1:text.index("\nlogging:")]
    mcfg_dict = yaml.safe_load(block)["metrics"]
    mcfg = MetricConfig.from_dict(mcfg_dict)
    rec = MetricRecorder(mcfg)

    rng = np.random.default_rng(2024)
    out = {"metric_config": mcfg_dict, "batches": []}
    for n in BATCHES:
        targets = rng.integers(0, 10, size=n)
        # mostly-right predictions with a class that is never predicted in some batches
        preds = np.where(rng.random(n) < 0.7, targets, rng.integers(0, 9, size=n))
        m_types = rng.choice(["ai", "a", "i"], size=n, p=[0.5, 0.3, 0.2])
        rec.update_group_all("classification", predictions=preds, targets=targets, m_types=m_types)
        out["batches"].append({"targets": targets.tolist(), "preds": preds.tolist(), "m_types": m_types.tolist()})
    res = flatten_dict(rec.calculate_all_groups(epoch=1, loss=0.5))
    out["results_keys"] = list(res.keys())
    out["results"] = {k: (np.asarray(v).tolist() if isinstance(v, np.ndarray) else float(v)) for k, v in res.items()}

    es = []
    best, wait = None, 0
    for ep, loss in enumerate(LOSSES, 1):
        vm = {"loss": loss}
        is_best, cont, wait = tm.check_early_stopping(vm, best, PATIENCE, MIN_DELTA, wait, "minimize", "loss")
        if is_best:
            best = dict(vm)
        es.append({"epoch": ep, "loss": loss, "is_best": bool(is_best), "continue": bool(cont), "wait": wait})
    out["early_stopping"] = {"patience": PATIENCE, "min_delta": MIN_DELTA, "trace": es}
    dst = os.path.join(HERE, "avmnist_metrics.json")
    with open(dst, "w") as f:
        json.dump(out, f)
    print("wrote", dst, len(out["results_keys"]), "result keys")


if __name__ == "__main__":
    main()
