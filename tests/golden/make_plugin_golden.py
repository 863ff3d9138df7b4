"""Record how the REAL reference resolves the AVMNIST configs with the plugin registered (run HERE, in
the build container only — the reference does not travel to the GPU box).

With throw-away stubs for the reference's absent imports (make_golden._write_stubs) it imports
``config.multimodal_training_config`` and ``train_multimodal`` from ``/root/reference/MML_Suite``,
calls ``tspm_amd.plugin.register()``, then for
``configs/avmnist/centralised/train_avmnist_resnet.yaml`` and ``..._pretrained.yaml``:

* ``train_multimodal.setup_experiment`` = ``StandardMultimodalConfig.load`` (YAML tags → encoder
  objects) + the script's logger,
* ``train_multimodal.setup_model_components(config)`` — the reference's own model / optimizer /
  scheduler construction: ``resolve_model_name`` → model class, and either ``config.get_optimizer``
  (scratch config) or the param-group branch ``getattr(torch.optim, name)(param_groups)``
  (pretrained config, train_multimodal.py:216-304),

and records the classes that came out, the optimizer's param groups (lr, weight decay, parameter
count) and the model's state_dict keys in ``plugin_resolution.json``.  There is no GPU here, so
FusedAdam's device buffers are not built: its constructor is wrapped to record its arguments and set
up only torch.optim.Optimizer's bookkeeping.  tests/test_dropin_cpu.py checks the fixture.

Usage:  python tests/golden/make_plugin_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MML_Suite"
CONFIGS = ["configs/avmnist/centralised/train_avmnist_resnet.yaml",
           "configs/avmnist/centralised/train_avmnist_resnet_pretrained.yaml"]


def main() -> None:
    sys.path.insert(0, HERE)
    from make_golden import _write_stubs
    stubdir = tempfile.mkdtemp(prefix="tspm_stubs_")
    _write_stubs(stubdir)
    exp = tempfile.mkdtemp(prefix="tspm_exp_")
    os.environ["EXP_PATH"] = exp
    os.makedirs(os.path.join(exp, "DATA", "avmnist"), exist_ok=True)
    for split in ("train", "validation", "test"):
        with open(os.path.join(exp, "DATA", "avmnist", f"{split}_subset.csv"), "w") as f:
            f.write("audio,image,label\n")
    sys.path[:0] = [stubdir, REF, REPO]
    cwd = os.getcwd()
    os.chdir(exp)  # the reference writes logs relative to the working directory
    import torch
    import config.multimodal_training_config as mtc  # noqa: F401  (import order: train_multimodal.py:14)
    import train_multimodal
    import tspm_amd
    from tspm_amd import optim as topt

    created = []
    orig_init = topt.FusedAdam.__init__

    def recording_init(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, **kw):
        torch.optim.Optimizer.__init__(self, params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                                          weight_decay=weight_decay, amsgrad=False))
        self.grad_scale, self._flat = 1.0, []
        created.append(self)

    topt.FusedAdam.__init__ = recording_init
    tspm_amd.plugin.register()
    out = {"reference": "MML_Suite @ /root/reference (real modules, build container)",
           "script_torch_is_proxy": type(train_multimodal.torch).__name__, "configs": {}}
    try:
        for rel in CONFIGS:
            # the script's own entry: StandardMultimodalConfig.load + its logger (train_multimodal.py:75-97)
            cfg = train_multimodal.setup_experiment(os.path.join(REF, rel), 1)
            kw = cfg.model.kwargs
            created.clear()
            model, opt, crit, sched, device, rec = train_multimodal.setup_model_components(cfg)
            q = lambda o: f"{type(o).__module__}.{type(o).__qualname__}"  # noqa: E731
            ids = {id(p): n for n, p in model.named_parameters()}
            out["configs"][rel] = {
                "audio_encoder": q(kw["audio_encoder"]), "image_encoder": q(kw["image_encoder"]),
                "model": q(model), "optimizer": q(opt),
                "optimizer_branch": "param_groups (train_multimodal.py:216-304)"
                if getattr(cfg.training, "encoder_optimizer", None) is not None and cfg.model.pretrained_encoders
                else "config.get_optimizer",
                "param_groups": [{"lr": g["lr"], "weight_decay": g["weight_decay"], "params": len(g["params"]),
                                  "first": ids.get(id(g["params"][0])), "last": ids.get(id(g["params"][-1]))}
                                 for g in opt.param_groups],
                "model_parameters": len(ids),
                "state_dict_keys": list(model.state_dict().keys()),
                "loss_terms": list(crit.keys()) if hasattr(crit, "keys") else None,
                "scheduler": q(sched) if sched is not None else None,
            }
    finally:
        topt.FusedAdam.__init__ = orig_init
        os.chdir(cwd)
        import shutil
        shutil.rmtree(exp, ignore_errors=True)
        shutil.rmtree(stubdir, ignore_errors=True)
    path = os.path.join(HERE, "plugin_resolution.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for rel, d in out["configs"].items():
        print(rel, d["model"], d["optimizer"], d["optimizer_branch"], [(g["lr"], g["params"]) for g in d["param_groups"]],
              len(d["state_dict_keys"]))


if __name__ == "__main__":
    main()
