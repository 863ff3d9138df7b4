"""MMIMDb late-fusion path (BASELINE configs[3]) — CPU side: the oracle against the golden vectors
captured from the REAL reference modules (tests/golden/make_mmimdb_golden.py), the drop-in classes'
seeded init / state_dict against the same vectors, YAML tag + resolver registration, and the
f1 metric reduction against sklearn."""
import hashlib
import os

import numpy as np
import pytest
import torch

import tspm_amd
from oracle import mmimdb_ref as orc
from oracle.avmnist_ref import OracleAdam
from tspm_amd import mmimdb as M

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def mg():
    return dict(np.load(os.path.join(HERE, "golden", "mmimdb_step_b4.npz"), allow_pickle=False))


def _sha(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].contiguous().numpy().tobytes())
    return h.hexdigest()


def dropin(seed=0, pooling=None):
    torch.manual_seed(seed)
    ie, te = M.MMIMDbModalityEncoder(4096, 512), M.MMIMDbModalityEncoder(300, 512)
    if pooling is not None:  # YAML order of configs/mmimdb/centralised/pooling/*.yaml: no GMU
        c = M.MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
        return M.MMIMDb(ie, te, multimodal_pooling=dict(pooling), classifier=c)
    g = M.GatedBiModalNetwork(input_one_dim=512, output_one_dim=512, input_two_dim=512, output_two_dim=512)
    c = M.MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
    return M.MMIMDb(ie, te, gated_bimodal_network=g, classifier=c)


POOL_KINDS = ["max", "avg", "sum", "attention", "gated"]
POOL_GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mmimdb_pool_b4.npz")


def pool_cfg(kind):
    return {"pooling_type": kind, "hidden_dim": 512, "dropout": 0.1}


@pytest.mark.parametrize("kind", POOL_KINDS)
def test_pooling_oracle_and_dropin_match_reference(kind):
    """multimodal_pooling (models/pooling.py): the oracle replays the REAL reference's 2 train steps
    bitwise (its own dropout masks; tests/golden/make_mmimdb_pooling_golden.py), and the drop-in builds
    the same state_dict (keys and seeded values) and parameter order."""
    from oracle.avmnist_ref import OracleAdam
    g = dict(np.load(POOL_GOLDEN, allow_pickle=False))
    I, T, y = (torch.from_numpy(g[k]) for k in ("image", "text", "labels"))
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        model = orc.build_oracle_mmimdb(0, pooling=pool_cfg(kind))
        ours = dropin(0, pool_cfg(kind))
        assert list(model.state_dict()) == list(ours.state_dict()) == list(g[f"{kind}/state_dict_keys"])
        for k, v in ours.state_dict().items():
            assert torch.equal(v, model.state_dict()[k]), k
        assert [n for n, _ in ours.named_parameters()] == list(g[f"{kind}/param_names"])
        opt = OracleAdam(list(model.parameters()), lr=1e-5, weight_decay=1e-3)
        for s in range(2):
            kp = torch.from_numpy(g[f"{kind}/keep_pool"][s])
            r = orc.train_step(model, opt, I, T, y, torch.from_numpy(g[f"{kind}/keep1"][s]),
                               torch.from_numpy(g[f"{kind}/keep2"][s]), keep_pool=(kp[0], kp[1]))
            assert r["loss"].item() == g[f"{kind}/losses"][s]
            assert torch.equal(r["logits"], torch.from_numpy(g[f"{kind}/logits"][s]))
            if s == 0:
                gn = np.array([p.grad.double().norm().item() for p in model.parameters()])
                np.testing.assert_array_equal(gn, g[f"{kind}/grad_norm_step1"])
            ps = np.array([p.detach().double().sum().item() for p in model.parameters()])
            np.testing.assert_array_equal(ps, g[f"{kind}/param_sums"][s])
    finally:
        torch.set_num_threads(nt)


def test_oracle_init_matches_reference(mg):
    sd = orc.build_oracle_mmimdb(0).state_dict()
    assert list(sd) == list(mg["state_dict_keys"])
    assert _sha(sd) == str(mg["state_dict_sha256"])


def test_dropin_init_and_keys_match_reference(mg):
    m = dropin(0)
    assert list(m.state_dict()) == list(mg["state_dict_keys"])
    assert _sha(m.state_dict()) == str(mg["state_dict_sha256"])
    assert [n for n, _ in m.named_parameters()] == list(mg["param_names"])


def test_oracle_three_steps_bit_exact(mg):
    torch.set_num_threads(4)
    model = orc.build_oracle_mmimdb(0)
    opt = OracleAdam(list(model.parameters()), lr=1e-5, weight_decay=1e-3)
    I, T, y = (torch.from_numpy(mg[k]) for k in ("image", "text", "labels"))
    for s in range(3):
        r = orc.train_step(model, opt, I, T, y, torch.from_numpy(mg["keep1"][s]), torch.from_numpy(mg["keep2"][s]))
        assert r["loss"].item() == float(mg["losses"][s])
        assert torch.equal(r["logits"], torch.from_numpy(mg["logits"][s]))
        if s == 0:
            gn = np.array([p.grad.double().norm().item() for p in model.parameters()])
            np.testing.assert_allclose(gn, mg["grad_norm_step1"], rtol=1e-12)
        np.testing.assert_allclose([p.detach().double().sum().item() for p in model.parameters()],
                                   mg["param_sums"][s], rtol=1e-12)
    assert torch.equal(orc.eval_forward(model, I, T), torch.from_numpy(mg["eval_logits"]))


def test_synthetic_batch_shapes():
    I, T, y = orc.synthetic_batch(16, seed=5)
    assert I.shape == (16, 4096) and T.shape == (16, 300) and y.shape == (16, 23)
    assert (I >= 0).all() and (y.sum(1) >= 1).all()


def test_f1_metrics_match_sklearn():
    from sklearn.metrics import f1_score
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(200, 23, generator=g)
    labels = (torch.rand(200, 23, generator=g) < 0.2).float()
    counts = orc.f1_counts(logits, labels)
    stats = torch.tensor([0.0, 200.0] + counts, dtype=torch.float64)
    got = M.f1_metrics(stats, 23)
    pred = (torch.sigmoid(logits) > 0.5).int().numpy()
    yt = labels.int().numpy()
    for avg in ("samples", "macro", "weighted", "micro"):
        assert got[f"f1_{avg}"] == pytest.approx(f1_score(yt, pred, average=avg, zero_division=0), abs=1e-12)


def test_yaml_tags_and_resolver():
    import yaml
    tspm_amd.plugin.register_yaml()
    doc = """
image_encoder: !MMIMDbModalityEncoder {input_dim: 4096, output_dim: 512}
gmu: !GatedBiModalNetwork {input_one_dim: 512, output_one_dim: 512, input_two_dim: 512, output_two_dim: 512}
clf: !MLPGenreClassifier {input_size: 512, hidden_size: 512, output_size: 23}
"""
    d = yaml.safe_load(doc)
    assert isinstance(d["image_encoder"], M.MMIMDbModalityEncoder)
    assert isinstance(d["gmu"], M.GatedBiModalNetwork) and isinstance(d["clf"], M.MLPGenreClassifier)
    assert tspm_amd.plugin.MODELS["mmimdb"] is M.MMIMDb


def test_rejects_unsupported_configs():
    with pytest.raises(ValueError):  # models/pooling.py raises on an unknown pooling type
        M.MMIMDb(M.MMIMDbModalityEncoder(8, 8), M.MMIMDbModalityEncoder(8, 8),
                 multimodal_pooling={"pooling_type": "median"}, classifier=M.MLPGenreClassifier(8, 2, 8))
    with pytest.raises(ValueError):
        M.MMIMDb(M.MMIMDbModalityEncoder(8, 8), M.MMIMDbModalityEncoder(8, 8), classifier=M.MLPGenreClassifier(8, 2, 8))


def test_bce_weight_checks_the_loss_group():
    class Term:
        def __init__(self, fn, w):
            self.loss_fn, self.weight = fn, w

    class Group(dict):
        pass

    assert M._bce_weight(Group(bce=Term(torch.nn.BCEWithLogitsLoss(), 2.0))) == 2.0
    with pytest.raises(tspm_amd.TspmError):
        M._bce_weight(Group(ce=Term(torch.nn.CrossEntropyLoss(), 1.0)))


def test_early_stopping_epoch_pinned_on_a_loss_sequence():
    """fit_mmimdb stops through harness.check_early_stopping with min_delta 1e-3
    (TrainingConfig.early_stopping_min_delta, config/multimodal_training_config.py:48): improvements
    smaller than 1e-3 count as no improvement (train_multimodal.py:329-377)."""
    from tspm_amd.harness import check_early_stopping
    losses = [0.50, 0.40, 0.3995, 0.3991, 0.3992, 0.3989, 0.30]
    best, wait, stopped = None, 0, None
    for ep, v in enumerate(losses, 1):
        is_best, cont, wait = check_early_stopping({"loss": v}, best, 3, 1e-3, wait)
        if is_best:
            best = {"loss": v}
        if not cont:
            stopped = ep
            break
    assert stopped == 5 and best == {"loss": 0.40}
