"""MI355X-native AVMNIST late-fusion training path (gfx950 HIP kernels behind a C ABI).

Importable as ``tspm_amd`` (root shim ``tspm_amd.py`` maps the hyphenated directory name).

    import tspm_amd
    tspm_amd.plugin.register()          # rebind !ResNet18 / !ResNet34 / "AVMNIST" / "Adam"
    enc = tspm_amd.ResNet18(1, 64).cuda()

The HIP library ``libtspm.so`` is built in-tree (``__graft_entry__.build()``); every op raises if it
is missing — there is no CPU or ATen fallback on the product path.
"""
import torch  # noqa: F401  (load torch's HIP runtime before libtspm.so binds to it)

from . import _lib
from ._lib import TspmError, TspmLibraryError
from .engine import EncoderEngine, prepare_encoder_layout
from .modules import AVMNIST, BasicBlock, ResNet18, ResNet34, ResNetEncoder, modality_key
from .optim import FusedAdam
from .step import FusedTrainStep
from .monomodal import FusedMonoStep, MonomodalEncoder
from . import plugin, ddp, data, monomodal, mmimdb
from .mmimdb import MMIMDb, FusedMMIMDbStep

__all__ = ["AVMNIST", "BasicBlock", "ResNet18", "ResNet34", "ResNetEncoder", "FusedAdam", "FusedTrainStep",
           "EncoderEngine", "prepare_encoder_layout", "TspmError", "TspmLibraryError", "plugin", "ddp", "data",
           "modality_key", "MonomodalEncoder", "FusedMonoStep", "monomodal", "mmimdb", "MMIMDb", "FusedMMIMDbStep"]
__version__ = "0.1.0"
