"""Epoch metrics from confusion counts against the REAL reference MetricRecorder's results
(tests/golden/avmnist_metrics.json, make_metrics_golden.py) and against raw-array sklearn calls;
early stopping against the reference's check_early_stopping trace.  CPU only."""
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytest.importorskip("sklearn")


@pytest.fixture(scope="module")
def mgold():
    with open(os.path.join(REPO, "tests", "golden", "avmnist_metrics.json")) as f:
        return json.load(f)


def confusion_by_pattern(batches, patterns=("ai", "a", "i"), k=10):
    conf = np.zeros((len(patterns), k, k), dtype=np.int64)
    for b in batches:
        for t, p, m in zip(b["targets"], b["preds"], b["m_types"]):
            conf[patterns.index(m), t, p] += 1
    return conf


class _Log:
    def __init__(self, conf, groups):
        self.conf, self.groups = conf, list(groups)

    def fetch(self):
        return self.conf, np.zeros(0, np.float32), int(self.conf.sum())

    def reset(self):
        pass


def test_recorder_matches_reference_metric_recorder(mgold):
    from tspm_amd.metrics import DeviceMetricRecorder
    groups = ("ai", "a", "i")
    rec = DeviceMetricRecorder(mgold["metric_config"], _Log(confusion_by_pattern(mgold["batches"], groups), groups))
    res = rec.calculate_all_groups(epoch=1, loss=0.5)["classification"]
    assert list(res.keys()) == mgold["results_keys"]
    for k, v in mgold["results"].items():
        got = res[k]
        if isinstance(v, list):
            assert np.array_equal(np.asarray(got), np.asarray(v)), k
        else:
            assert float(got) == v, (k, got, v)  # bit-exact


@pytest.mark.parametrize("seed", range(12))
def test_compressed_evaluation_is_bit_exact_vs_raw_sklearn(seed):
    from tspm_amd.metrics import evaluate
    import sklearn.metrics as skm
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    k = 10
    t = rng.integers(0, k, size=n)
    p = np.where(rng.random(n) < rng.random(), t, rng.integers(0, k - int(rng.integers(0, 4)), size=n))
    if seed % 3 == 0:  # some classes absent entirely
        keep = t % 3 != 1
        t, p = t[keep], np.where(p[keep] % 3 == 1, 0, p[keep])
        if t.size == 0:
            t, p = np.array([0]), np.array([0])
    conf = np.zeros((k, k), np.int64)
    np.add.at(conf, (t, p), 1)
    cases = [("sklearn.metrics.accuracy_score", {}), ("sklearn.metrics.balanced_accuracy_score", {}),
             ("sklearn.metrics.confusion_matrix", {"labels": list(range(10))}),
             ("sklearn.metrics.confusion_matrix", {}), ("sklearn.metrics.cohen_kappa_score", {}),
             ("sklearn.metrics.matthews_corrcoef", {})]
    for avg in ("macro", "micro", "weighted"):
        for f in ("f1_score", "precision_score", "recall_score"):
            cases.append((f"sklearn.metrics.{f}", {"average": avg, "zero_division": 0}))
    for path, kw in cases:
        want = getattr(skm, path.rsplit(".", 1)[1])(t, p, **kw)
        got = evaluate(path, kw, conf)
        if isinstance(want, np.ndarray):
            assert np.array_equal(got, want) and got.dtype == want.dtype, path
        else:
            assert float(got) == float(want), (path, kw, got, want)


def test_early_stopping_matches_reference_trace(mgold):
    from tspm_amd.harness import check_early_stopping
    es = mgold["early_stopping"]
    best, wait = None, 0
    for row in es["trace"]:
        vm = {"loss": row["loss"]}
        is_best, cont, wait = check_early_stopping(vm, best, es["patience"], es["min_delta"], wait, "minimize", "loss")
        if is_best:
            best = dict(vm)
        assert (is_best, cont, wait) == (row["is_best"], row["continue"], row["wait"]), row


def test_mean_loss_is_numpy_mean_of_python_floats():
    from tspm_amd.metrics import ClassificationLog
    xs = np.random.default_rng(0).random(1000).astype(np.float32)
    assert ClassificationLog.mean_loss(xs) == np.mean([float(x) for x in xs])


def test_mosi_recorder_matches_reference_metric_recorder():
    """MOSI's YAML metrics (MSA = metrics.msa_binary_classification restated in tspm_amd.msa_metrics, and the
    3-class confusion matrix) over the seven missing-modality patterns, from per-pattern confusion counts, against
    the REAL reference MetricRecorder fed the pattern-grouped batches (tests/golden/make_mosi_metrics_golden.py)
    — bit-exact, NaN where the reference gives NaN (a pattern with no non-neutral sample)."""
    import math
    from tspm_amd.metrics import DeviceMetricRecorder
    with open(os.path.join(REPO, "tests", "golden", "mosi_metrics.json")) as f:
        g = json.load(f)
    pats = tuple(g["patterns"])
    rec = DeviceMetricRecorder(g["metric_config"], _Log(confusion_by_pattern(g["batches"], pats, k=3), pats))
    res = rec.calculate_all_groups(epoch=1, loss=0.5)["classification"]
    assert set(res.keys()) == set(g["results"].keys())
    for k, v in g["results"].items():
        got = res[k]
        if isinstance(v, list):
            assert np.array_equal(np.asarray(got), np.asarray(v)), k
        elif isinstance(v, float) and math.isnan(v):
            assert math.isnan(float(got)), k
        else:
            assert float(got) == v, (k, got, v)


def test_msa_metric_equals_reference_formula_on_raw_arrays():
    """msa_binary_classification from expanded confusion counts equals the call on the raw (unsorted) arrays."""
    from tspm_amd.metrics import evaluate
    from tspm_amd.msa_metrics import msa_binary_classification
    rng = np.random.default_rng(7)
    for _ in range(8):
        n = int(rng.integers(5, 300))
        t, p = rng.integers(0, 3, size=n), rng.integers(0, 3, size=n)
        conf = np.zeros((3, 3), np.int64)
        np.add.at(conf, (t, p), 1)
        assert evaluate("metrics.msa_binary_classification", {}, conf) == msa_binary_classification(t, p)
