"""Plugin registration: rebind the reference's extension seams to the HIP implementations.

The reference builds models through two seams:
  1. YAML tags on ``yaml.SafeLoader`` — ``register_constructor(tag, cls, deep=True)`` runs
     ``cls(**mapping)`` while the config is parsed (MML_Suite/config/yaml_constructors.py:37-43,
     159-178: ``!ResNet18``, ``!ResNet34``, ``!ResNetEncoder``).
  2. Name resolvers — ``resolve_model_name("AVMNIST")`` (config/resolvers.py:18-23),
     ``resolve_encoder`` (:93-122), ``resolve_optimizer("Adam")`` (:125-156) and
     ``resolve_dataset_name("AVMNIST")`` (:192-220, called by config/data_config.py:134).

``register()`` overrides the tags on the given loader (default ``yaml.SafeLoader``) and, when the
reference's ``config.resolvers`` module is importable in the process, wraps the resolvers so the
names above return this package's classes (other names fall through to the originals).  After that,
``train_multimodal.py`` / ``train_monomodal.py`` and the YAML configs run unchanged on the HIP path.

A third seam: with ``training.encoder_optimizer`` set and ``pretrained_encoders`` given (the
pretrained late-fusion config, configs/avmnist/centralised/train_avmnist_resnet_pretrained.yaml:36),
``setup_model_components`` bypasses ``resolve_optimizer`` and builds
``getattr(torch.optim, config.training.optimizer.name)(param_groups)`` (train_multimodal.py:216-304).
``register_script_optimizer`` makes that lookup return ``FusedAdam`` for "Adam" — inside the script
module only (its global ``torch`` becomes a proxy whose ``optim.Adam`` is ``FusedAdam``; every other
attribute is torch's own), so nothing else in the process is affected.
"""
from __future__ import annotations

import sys
from typing import Dict, Optional

from . import data
from .modules import AVMNIST, ResNet18, ResNet34, ResNetEncoder
from .optim import FusedAdam
from . import mmimdb as _mm
from . import mosi as _mosi
from . import mosi_data as _mosi_data

TAGS = {"!ResNet18": ResNet18, "!ResNet34": ResNet34, "!ResNetEncoder": ResNetEncoder,
        # MMIMDb late-fusion path (config/yaml_constructors.py:126-142)
        "!MMIMDbModalityEncoder": _mm.MMIMDbModalityEncoder, "!MaxOut": _mm.MaxOut,
        "!GatedBiModalNetwork": _mm.GatedBiModalNetwork, "!MMIMDb": _mm.MMIMDb,
        "!MLPGenreClassifier": _mm.MLPGenreClassifier,
        # MOSI UTT-Fusion path (config/yaml_constructors.py:99-110)
        "!LSTMEncoder": _mosi.LSTMEncoder, "!TextCNN": _mosi.TextCNN, "!FcClassifier": _mosi.FcClassifier}
MODELS = {"avmnist": AVMNIST, "mmimdb": _mm.MMIMDb, "mmimdbmodalityencoder": _mm.MMIMDbModalityEncoder,
          "utt-fusion": _mosi.UttFusionModel}  # config/resolvers.py:28-31
ENCODERS = {"resnet18": ResNet18, "resnet34": ResNet34, "resnetencoder": ResNetEncoder,
            "lstmencoder": _mosi.LSTMEncoder, "textcnn": _mosi.TextCNN}
OPTIMIZERS = {"adam": FusedAdam}
DATASETS = {"avmnist": data.AVMNIST, "mosi": _mosi_data.MOSI, "mosei": _mosi_data.MOSEI}


def _ctor(cls):
    def constructor(loader, node):
        data = loader.construct_mapping(node, deep=True)
        return cls(**data)
    return constructor


def register_yaml(loader=None) -> None:
    import yaml
    loader = loader or yaml.SafeLoader
    for tag, cls in TAGS.items():
        loader.add_constructor(tag, _ctor(cls))


def _wrap(orig, table: Dict[str, object]):
    if getattr(orig, "__tspm_wrapped__", False):
        return orig

    def resolver(name: str, *a, **k):
        hit = table.get(str(name).lower())
        return hit if hit is not None else orig(name, *a, **k)

    resolver.__tspm_wrapped__ = True
    resolver.__wrapped__ = orig
    resolver.__name__ = getattr(orig, "__name__", "resolver")
    return resolver


def register_resolvers(resolvers_module: Optional[object] = None, rebind_everywhere: bool = True) -> bool:
    """Wrap resolve_model_name / resolve_encoder / resolve_optimizer / resolve_dataset_name of the reference's
    ``config.resolvers`` (if loaded) and every module that imported them by name."""
    mod = resolvers_module or sys.modules.get("config.resolvers")
    if mod is None:
        return False
    pairs = [("resolve_model_name", MODELS), ("resolve_encoder", ENCODERS), ("resolve_optimizer", OPTIMIZERS),
             ("resolve_dataset_name", DATASETS)]
    for name, table in pairs:
        orig = getattr(mod, name, None)
        if orig is None:
            continue
        new = _wrap(orig, table)
        setattr(mod, name, new)
        if rebind_everywhere:
            for m in list(sys.modules.values()):
                # the module's own namespace only: getattr would trigger lazy-import hooks
                # (e.g. transformers' _LazyModule) in unrelated packages
                d = getattr(m, "__dict__", None) if m is not None else None
                if isinstance(d, dict) and m is not mod and d.get(name) is orig:
                    setattr(m, name, new)
    return True


def register_monomodal(module: Optional[object] = None) -> bool:
    """``train_monomodal.py`` defines ``MonomodalEncoder`` in the script itself and ``setup_experiment``
    looks the name up when it runs (MML_Suite/train_monomodal.py:64,525-529): rebind it in the loaded
    script module (imported as ``train_monomodal``, or ``__main__`` when the script is the program)."""
    from .monomodal import MonomodalEncoder
    cands = [module] if module is not None else [sys.modules.get("train_monomodal"), sys.modules.get("__main__")]
    done = False
    for m in cands:
        if m is None or not hasattr(m, "MonomodalEncoder"):
            continue
        if m is sys.modules.get("train_monomodal") or module is not None or hasattr(m, "train_monomodal"):
            setattr(m, "MonomodalEncoder", MonomodalEncoder)
            done = True
    return done


class _OptimProxy:
    """``torch.optim`` as the training script sees it: ``Adam`` is FusedAdam, the rest is torch's."""

    def __init__(self, optim):
        self._optim = optim

    def __getattr__(self, name):
        hit = OPTIMIZERS.get(name.lower())
        return hit if hit is not None else getattr(self._optim, name)


class _TorchProxy:
    """The script module's global ``torch``: torch itself except for ``torch.optim`` (_OptimProxy)."""

    def __init__(self, torch_mod):
        self._torch = torch_mod
        self.optim = _OptimProxy(torch_mod.optim)

    def __getattr__(self, name):
        return getattr(self._torch, name)


def register_script_optimizer(module: Optional[object] = None) -> bool:
    """Route ``getattr(torch.optim, "Adam")`` in ``train_multimodal`` (imported, or running as
    ``__main__``) to FusedAdam: the script's own module global ``torch`` is replaced by a proxy."""
    import torch
    cands = [module] if module is not None else [sys.modules.get("train_multimodal"), sys.modules.get("__main__")]
    done = False
    for m in cands:
        if m is None or not hasattr(m, "setup_model_components"):
            continue
        cur = getattr(m, "torch", None)
        if isinstance(cur, _TorchProxy):
            done = True
            continue
        if cur is torch:
            m.torch = _TorchProxy(torch)
            done = True
    return done


def register(loader=None, resolvers_module=None) -> None:
    """Install the HIP implementations behind the reference's YAML tags, resolvers, the monomodal
    script's model class and the multimodal script's param-group optimizer lookup."""
    register_yaml(loader)
    register_resolvers(resolvers_module)
    register_monomodal()
    register_script_optimizer()
