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


def dropin(seed=0):
    torch.manual_seed(seed)
    ie, te = M.MMIMDbModalityEncoder(4096, 512), M.MMIMDbModalityEncoder(300, 512)
    g = M.GatedBiModalNetwork(input_one_dim=512, output_one_dim=512, input_two_dim=512, output_two_dim=512)
    c = M.MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
    return M.MMIMDb(ie, te, gated_bimodal_network=g, classifier=c)


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
    with pytest.raises(NotImplementedError):
        M.MMIMDb(M.MMIMDbModalityEncoder(8, 8), M.MMIMDbModalityEncoder(8, 8), multimodal_pooling={"x": 1},
                 classifier=M.MLPGenreClassifier(8, 2, 8))


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
