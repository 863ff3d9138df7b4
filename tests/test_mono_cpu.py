"""Monomodal pre-training path (MML_Suite/train_monomodal.py, BASELINE.json configs[1]) without a GPU:
the oracle against the golden vectors captured from the REAL reference (tests/golden/
make_mono_golden.py — bit-exact), the drop-in module's seeded init / state_dict keys, the
reference's batch-key choice, plugin registration, FLOP accounting and loud failure off-GPU."""
import hashlib
import os
import sys
import types
from enum import Enum

import numpy as np
import pytest
import torch

import tspm_amd
from oracle import avmnist_ref as orc
from oracle import monomodal_ref as mref
from tspm_amd.monomodal import modality_of_experiment, select_modality_key

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "avmnist_mono_b4.npz")


@pytest.fixture(scope="module")
def mono_golden():
    return dict(np.load(GOLD, allow_pickle=False))


def _sha(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].contiguous().numpy().tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("which", ["audio", "image"])
def test_oracle_bit_exact_vs_reference(mono_golden, which):
    torch.set_num_threads(4)
    g = mono_golden
    m = mref.build_oracle_monomodal(which, 0)
    assert list(m.state_dict()) == list(g[f"{which}_state_dict_keys"])
    assert _sha(m.state_dict()) == str(g[f"{which}_state_dict_sha256"])
    opt = orc.OracleAdam(list(m.parameters()), lr=5e-4, weight_decay=1e-4)
    x, labels = torch.from_numpy(g[f"{which}_x"]), torch.from_numpy(g["labels"])
    for s in range(3):
        r = mref.train_step(m, opt, x, labels)
        assert r["loss"].item() == float(g[f"{which}_losses"][s])
        assert np.array_equal(r["logits"].numpy(), g[f"{which}_logits"][s])
        assert r["accuracy"].item() == float(g[f"{which}_accuracy"][s])
        assert np.array_equal(r["preds"].numpy(), g[f"{which}_preds"][s])
        if s == 0:
            gn = np.array([p.grad.double().norm().item() for p in m.parameters()])
            assert np.array_equal(gn, g[f"{which}_grad_norm_step1"])
    psum = np.array([p.detach().double().sum().item() for p in m.parameters()])
    assert np.array_equal(psum, g[f"{which}_param_sum_final"])
    ev = mref.validation_step(m, x, labels)
    assert np.array_equal(ev["logits"].numpy(), g[f"{which}_eval_logits"])
    assert ev["loss"].item() == float(g[f"{which}_eval_loss"])
    assert np.array_equal(ev["preds"].numpy(), g[f"{which}_preds"][3])


@pytest.mark.parametrize("which", ["audio", "image"])
def test_dropin_seeded_init_and_state_dict(mono_golden, which):
    torch.manual_seed(0)
    enc = tspm_amd.ResNet18(1, 64) if which == "audio" else tspm_amd.ResNet34(1, 128)
    m = tspm_amd.MonomodalEncoder(enc, 64 if which == "audio" else 128, 10)
    sd, rsd = m.state_dict(), mref.build_oracle_monomodal(which, 0).state_dict()
    assert list(sd) == list(rsd) == list(mono_golden[f"{which}_state_dict_keys"])
    for k in sd:
        assert torch.equal(sd[k], rsd[k]), k
    assert m.get_encoder() is enc
    assert [n for n, _ in m.named_parameters()] == list(mono_golden[f"{which}_param_names"])


def test_select_modality_key_follows_reference():
    class Modality(Enum):
        AUDIO = "audio"
        IMAGE = "image"

        def __str__(self):
            return f"Modality.{self.name}"

    b = {"labels": 0, "pattern_name": 0, "missing_masks": {}, Modality.AUDIO: 1, Modality.IMAGE: 2, "pattern_ids": 3}
    assert select_modality_key(b, "AVMNIST_Audio_Encoder_Resnet_Pretrain") is Modality.AUDIO
    assert select_modality_key(b, "AVMNIST_Image_Encoder_Resnet_Pretrain") is Modality.IMAGE
    # no name match: the LAST non-bookkeeping key (train_monomodal.py:122-125)
    assert select_modality_key(b, "MMIMDb_Text_Encoder") is Modality.IMAGE
    assert select_modality_key({"audio": 1, "labels": 0}, "AVMNIST_Audio_Encoder") == "audio"
    with pytest.raises(ValueError):
        select_modality_key({"labels": 0, "sample_idx": 1}, "AVMNIST_Audio_Encoder")


def test_modality_of_experiment_name():
    assert modality_of_experiment("AVMNIST_Audio_Encoder_Resnet_Pretrain") == "audio"
    assert modality_of_experiment("AVMNIST_Image_Encoder_Resnet_Pretrain") == "image"
    assert modality_of_experiment("MMIMDb_Text_Encoder_Pretrain") == "text"
    assert modality_of_experiment("x") == "unknown"


def test_plugin_rebinds_the_script_class():
    fake = types.ModuleType("train_monomodal")

    class RefMonomodalEncoder:
        pass

    fake.MonomodalEncoder = RefMonomodalEncoder
    sys.modules["train_monomodal"] = fake
    try:
        assert tspm_amd.plugin.register_monomodal()
        assert fake.MonomodalEncoder is tspm_amd.MonomodalEncoder
    finally:
        del sys.modules["train_monomodal"]


def test_mono_flop_accounting():
    from tspm_amd.roofline import conv_macs, encoder_convs, mono_flops_per_sample
    nom, val = mono_flops_per_sample()
    fwd = sum(conv_macs(1, *shp)[0] for _, shp in encoder_convs((2, 2, 2, 2), 32, 94))
    stem = conv_macs(1, *next(iter(encoder_convs((2, 2, 2, 2), 32, 94)))[1])[0]
    assert nom == 2 * (3 * fwd - stem) + 6 * (512 * 64 + 64 * 10)
    assert 0.55 < val / nom < 0.7


def test_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    m = tspm_amd.MonomodalEncoder(tspm_amd.ResNet18(1, 64), 64, 10)
    with pytest.raises(tspm_amd.TspmError):
        m(torch.randn(2, 32, 94))
    with pytest.raises(tspm_amd.TspmError):
        tspm_amd.FusedAdam(m.parameters(), lr=5e-4)
