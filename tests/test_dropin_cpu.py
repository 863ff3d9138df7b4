"""Drop-in API checks that need no GPU: constructor signatures, seeded init and state_dict
layout identical to the reference, YAML tag / resolver registration, and loud failure off-GPU."""
import os
import sys
import types

import pytest
import torch
import yaml

import tspm_amd
from oracle import avmnist_ref as orc


def test_state_dict_and_seeded_init_identical_to_reference(golden):
    torch.manual_seed(0)
    m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5)
    ref = orc.build_oracle_avmnist(0)
    sd, rsd = m.state_dict(), ref.state_dict()
    assert list(sd) == list(rsd) == list(golden["state_dict_keys"])
    for k in sd:
        assert sd[k].shape == rsd[k].shape and torch.equal(sd[k], rsd[k]), k


def test_encoder_api_surface():
    e = tspm_amd.ResNet18(in_channels=1, hidden_dim=64)
    assert e.hidden_dim == 64 and e.get_embedding_size() == 64
    assert sum(p.numel() for p in e.parameters()) == 11_203_072
    e34 = tspm_amd.ResNet34(1, 128)
    assert sum(p.numel() for p in e34.parameters()) == 21_344_064
    enc = tspm_amd.ResNetEncoder(block="basic", layers=[2, 2, 2, 2], in_channels=1, hidden_dim=32)
    assert enc.fc.out_features == 32
    with pytest.raises(NotImplementedError):
        tspm_amd.ResNetEncoder(block=type("Bottleneck", (), {"expansion": 4}), layers=[3, 4, 6, 3])


def test_avmnist_api_surface():
    a, i = tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128)
    m = tspm_amd.AVMNIST(a, i, 128, dropout=0.5, fusion_fn="concat")
    assert m.get_encoder("audio") is a and m.get_encoder("image") is i
    assert [k for k, _ in m.net.named_children()] == ["0", "1", "2", "3", "4", "5"]
    with pytest.raises(ValueError):
        tspm_amd.AVMNIST(a, i, 128, fusion_fn="sum")
    assert sum(p.numel() for p in m.net.parameters()) == 33_610


def test_conv_weights_become_ohwi_without_changing_values():
    e = tspm_amd.ResNet18(1, 64)
    before = {n: p.detach().clone() for n, p in e.named_parameters()}
    tspm_amd.prepare_encoder_layout(e)
    for n, p in e.named_parameters():
        assert torch.equal(p, before[n])
        if p.dim() == 4:
            assert p.is_contiguous(memory_format=torch.channels_last)
    sd = e.state_dict()
    assert tuple(sd["conv1.weight"].shape) == (64, 1, 7, 7)


def test_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    e = tspm_amd.ResNet18(1, 64)
    with pytest.raises(tspm_amd.TspmError):
        e(torch.randn(2, 32, 94))
    with pytest.raises(tspm_amd.TspmError):
        tspm_amd.FusedAdam(e.parameters(), lr=5e-4)


def test_yaml_tags_build_hip_modules():
    loader = type("L", (yaml.SafeLoader,), {})
    tspm_amd.plugin.register_yaml(loader)
    doc = """
audio_encoder: !ResNet18
  in_channels: 1
  hidden_dim: 64
image_encoder: !ResNet34
  in_channels: 1
  hidden_dim: 128
"""
    cfg = yaml.load(doc, Loader=loader)
    assert isinstance(cfg["audio_encoder"], tspm_amd.ResNetEncoder)
    assert cfg["audio_encoder"].hidden_dim == 64 and cfg["image_encoder"].hidden_dim == 128


def test_resolver_rebinding_falls_through():
    mod = types.ModuleType("config.resolvers_fake")
    mod.resolve_model_name = lambda name: ("orig", name)
    mod.resolve_encoder = lambda name: ("orig", name)
    mod.resolve_optimizer = lambda name: ("orig", name)
    mod.resolve_dataset_name = lambda name: ("orig", name)
    user = types.ModuleType("fake_user")
    user.resolve_optimizer = mod.resolve_optimizer
    sys.modules["fake_user"] = user
    try:
        assert tspm_amd.plugin.register_resolvers(mod)
        assert mod.resolve_model_name("AVMNIST") is tspm_amd.AVMNIST
        assert mod.resolve_encoder("ResNet34") is tspm_amd.ResNet34
        assert mod.resolve_optimizer("Adam") is tspm_amd.FusedAdam
        assert mod.resolve_optimizer("sgd") == ("orig", "sgd")
        assert mod.resolve_dataset_name("AVMNIST") is tspm_amd.data.AVMNIST
        assert mod.resolve_dataset_name("MOSI") is tspm_amd.mosi_data.MOSI
        assert mod.resolve_dataset_name("iemocap") == ("orig", "iemocap")
        assert user.resolve_optimizer is mod.resolve_optimizer  # imported-by-name copies rebound too
        tspm_amd.plugin.register_resolvers(mod)  # idempotent
        assert mod.resolve_model_name("mosi") == ("orig", "mosi")
    finally:
        del sys.modules["fake_user"]


def test_modality_key_lookup():
    from enum import Enum

    class Modality(Enum):
        AUDIO = "audio"
        IMAGE = "image"

    b = {Modality.AUDIO: 1, Modality.IMAGE: 2, "labels": 3}
    assert tspm_amd.modality_key(b, "audio") is Modality.AUDIO
    assert tspm_amd.modality_key({"image": 1}, "image") == "image"
    with pytest.raises(KeyError):
        tspm_amd.modality_key({"labels": 1}, "audio")


def test_roofline_accounting_matches_survey():
    from tspm_amd.roofline import step_flops_per_sample
    nominal, valid = step_flops_per_sample()
    assert nominal == 1_049_740_032
    assert 0.6 < valid / nominal < 0.62


def test_reference_config_resolution_fixture(golden):
    """tests/golden/plugin_resolution.json was produced by the REAL reference (make_plugin_golden.py):
    both AVMNIST configs — including the pretrained one, whose optimizer comes from
    getattr(torch.optim, "Adam")(param_groups) at train_multimodal.py:216-304, not from
    resolve_optimizer — resolve to this package's modules and FusedAdam once plugin.register() ran."""
    import json
    path = os.path.join(os.path.dirname(__file__), "golden", "plugin_resolution.json")
    with open(path) as f:
        fx = json.load(f)
    assert fx["script_torch_is_proxy"] == "_TorchProxy"
    cfgs = fx["configs"]
    assert set(cfgs) == {"configs/avmnist/centralised/train_avmnist_resnet.yaml",
                         "configs/avmnist/centralised/train_avmnist_resnet_pretrained.yaml"}
    assert cfgs["configs/avmnist/centralised/train_avmnist_resnet_pretrained.yaml"]["optimizer_branch"].startswith(
        "param_groups")
    keys = list(golden["state_dict_keys"])
    for name, d in cfgs.items():
        assert d["model"] == "tspm_amd.modules.AVMNIST", name
        assert d["audio_encoder"] == d["image_encoder"] == "tspm_amd.modules.ResNetEncoder", name
        assert d["optimizer"] == "tspm_amd.optim.FusedAdam", name
        assert d["state_dict_keys"] == keys, name
        assert d["model_parameters"] == 178 and sum(g["params"] for g in d["param_groups"]) == 178, name
        assert d["loss_terms"] == ["cross_entropy"], name
        # one group over the whole model at the base optimizer's settings (the AVMNIST model has no
        # image_model / audio_model attributes, so the encoder group of the pretrained branch is empty)
        assert [(g["lr"], g["weight_decay"]) for g in d["param_groups"]] == [(5e-4, 1e-4)], name


def test_script_optimizer_seam_is_scoped_to_the_script():
    from tspm_amd import plugin
    script = types.ModuleType("train_multimodal_fake")
    script.torch = torch
    script.setup_model_components = lambda *a: None
    assert plugin.register_script_optimizer(script)
    assert getattr(script.torch.optim, "Adam") is tspm_amd.FusedAdam
    assert script.torch.optim.SGD is torch.optim.SGD and script.torch.nn is torch.nn
    assert script.torch.no_grad is torch.no_grad
    assert torch.optim.Adam is not tspm_amd.FusedAdam  # the real torch is untouched
    assert plugin.register_script_optimizer(script)  # idempotent
