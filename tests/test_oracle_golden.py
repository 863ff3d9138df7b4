"""The oracle (CPU fp32 restatement) against the golden vectors captured from the REAL reference
modules (tests/golden/make_golden.py).  On CPU the restatement is bit-exact; these checks pin it."""
import hashlib

import numpy as np
import torch

from oracle import avmnist_ref as orc


def test_seeded_init_matches_reference(golden):
    model = orc.build_oracle_avmnist(seed=0)
    sd = model.state_dict()
    assert list(sd.keys()) == list(golden["state_dict_keys"])
    assert len(sd) == 346
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].contiguous().numpy().tobytes())
    assert h.hexdigest() == str(golden["state_dict_sha256"])
    names = [n for n, _ in model.named_parameters()]
    assert names == list(golden["param_names"])
    for i, n in enumerate(names):
        p = sd[n].reshape(-1)
        k = min(8, p.numel())
        assert np.array_equal(p[:k].numpy(), golden["w_sample_first8"][i][:k])


def test_three_train_steps_bit_exact(golden):
    torch.set_num_threads(4)
    model = orc.build_oracle_avmnist(seed=0)
    opt = orc.OracleAdam(list(model.parameters()), lr=5e-4, weight_decay=1e-4)
    audio = torch.from_numpy(golden["audio"])
    image = torch.from_numpy(golden["image"])
    labels = torch.from_numpy(golden["labels"])
    params = dict(model.named_parameters())
    names = list(golden["param_names"])
    for s in range(3):
        r = orc.train_step(model, opt, audio, image, labels, torch.from_numpy(golden["keep_masks"][s]))
        assert r["loss"].item() == float(golden["losses"][s])
        assert np.array_equal(r["logits"].numpy(), golden["logits"][s])
        if s == 0:
            gn = np.array([params[n].grad.double().norm().item() for n in names])
            assert np.array_equal(gn, golden["grad_norm_step1"])
            g8 = np.stack([np.pad(params[n].grad.reshape(-1)[:8].numpy(), (0, max(0, 8 - params[n].numel())))
                           for n in names])
            assert np.array_equal(g8, golden["grad_first8_step1"])
    psum = np.array([params[n].detach().double().sum().item() for n in names])
    assert np.array_equal(psum, golden["param_sum_final"])
    model.eval()
    with torch.no_grad():
        ev, _, _ = orc.avmnist_forward(model, audio, image, False)
    assert np.array_equal(ev.numpy(), golden["eval_logits"])


def test_synthetic_batch_matches_fixture(golden, lut):
    audio, image, labels, u8 = orc.synthetic_batch(4, seed=1234, lut=lut.long())
    assert np.array_equal(audio.numpy(), golden["audio"])
    assert np.array_equal(image.numpy(), golden["image"])
    assert np.array_equal(labels.numpy(), golden["labels"])
    assert 2.2e-9 * 0.999 <= audio.min().item() and audio.max().item() <= 1.52e7 * 1.001


def test_lut_fixture_shape_and_endpoints(lut):
    # MML_Suite/data/avmnist.py:186-191: gist_earth → RGBA*255 → PIL "L"; LUT[0]=0, LUT[255]=251
    assert lut.numel() == 256
    assert int(lut[0]) == 0 and int(lut[255]) == 251
