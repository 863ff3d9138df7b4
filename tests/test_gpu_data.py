"""Input stage on the GPU: ``tspm_avmnist_gather`` through the drop-in dataset / DataLoader path and the
epoch DeviceLoader, bit-exact against the golden batches of the REAL reference dataset and against the
numpy oracle at full corpus size; edge cases (partial last batch, masks, audio-/image-only targets,
out-of-range indices, unaligned element counts)."""
import hashlib
import os

import numpy as np
import pytest
import torch

from oracle import avmnist_data_ref as dref
from oracle import avmnist_ref as orc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("train", "multimodal", ["ai"]), ("valid", "multimodal", ["ai", "a", "i"]), ("test", "image", ["i", "ai"])]


@pytest.fixture(scope="module")
def dgold():
    return dict(np.load(os.path.join(REPO, "tests", "golden", "avmnist_data.npz"), allow_pickle=False))


def lut_np():
    with open(os.path.join(REPO, "tests", "golden", "lut_gist_earth_L.bin"), "rb") as f:
        return np.frombuffer(f.read(), dtype=np.uint8).copy()


def sha(t) -> str:
    a = t.detach().cpu().contiguous().numpy() if isinstance(t, torch.Tensor) else np.ascontiguousarray(t)
    return hashlib.sha256(a.tobytes()).hexdigest()


def corpus(n, seed):
    from tspm_amd.data import AVMNISTCorpus
    audio, _, labels, u8 = orc.synthetic_batch(n, seed=seed)
    return AVMNISTCorpus(audio.numpy(), u8.numpy(), labels.numpy())


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_dataloader_dropin_matches_reference_batches(gpu, dgold, ci):
    from tspm_amd.data import AVMNIST
    split, target, sel = CASES[ci]
    ds = AVMNIST(None, split, target, selected_patterns=sel, corpus=corpus(int(dgold["n"]), int(dgold["seed"])),
                 device=gpu)
    dl = torch.utils.data.DataLoader(ds, batch_size=int(dgold["batch"]), shuffle=False, collate_fn=ds.collate_fn)
    batches = list(dl)
    assert len(batches) == int(dgold[f"c{ci}_batches"])
    for bi, b in enumerate(batches):
        key = f"c{ci}_b{bi}"
        assert b["labels"].is_cuda and b["labels"].dtype == torch.int64
        assert np.array_equal(b["labels"].cpu().numpy(), dgold[key + "_labels"])
        assert b["pattern_name"] == list(dgold[key + "_pattern"])
        assert b["missing_masks"] == {}
        if target == "multimodal":
            a = b[ds.keys["audio"]]
            assert list(a.shape) == list(dgold[key + "_audio_shape"])
            assert sha(a) == str(dgold[key + "_audio_sha256"])
        else:
            assert ds.keys["audio"] not in b
        im = b[ds.keys["image"]]
        assert np.array_equal(im.cpu().numpy(), dgold[key + "_image"])


def test_getitem_and_list_collate(gpu, dgold):
    from tspm_amd.data import AVMNIST
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"],
                 corpus=corpus(int(dgold["n"]), int(dgold["seed"])), device=gpu)
    items = [ds[i] for i in range(4, 8)]  # crosses the ai → a boundary
    b = ds.collate_fn(items)
    assert sha(b[ds.keys["audio"]]) == str(dgold["c1_b1_audio_sha256"])
    assert np.array_equal(b[ds.keys["image"]].cpu().numpy(), dgold["c1_b1_image"])
    assert items[2]["sample_idx"] == 0 and items[2]["pattern_name"] == "a"


def test_pattern_batches(gpu, dgold):
    from tspm_amd.data import AVMNIST
    c = corpus(int(dgold["n"]), int(dgold["seed"]))
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"], corpus=c, device=gpu)
    loaders = ds.get_pattern_batches(4)
    assert list(loaders) == ["ai", "a", "i"]
    for p, dl in loaders.items():
        got = list(dl)
        assert [len(b["labels"]) for b in got] == [4, 2]
        for b in got:
            assert set(b["pattern_name"]) == {p}
        a = torch.cat([b[ds.keys["audio"]] for b in got]).cpu().numpy()
        im = torch.cat([b[ds.keys["image"]] for b in got]).cpu().numpy()
        assert (a == 0).all() == (p == "i") and (im == 0).all() == (p == "a")
        if p != "i":
            assert np.array_equal(a, c.audio)


@pytest.mark.parametrize("batch", [128, 100])
def test_full_corpus_gather_bit_exact(gpu, batch):
    # AVMNIST-size corpus (60,000 samples ≈ 0.77 GB in HBM), shuffled epoch order, 3 patterns mixed
    from tspm_amd.data import AVMNIST, AVMNISTCorpus
    n = 60000
    rng = np.random.default_rng(7)
    audio = rng.standard_normal((n, 32, 94), dtype=np.float32)
    u8 = rng.integers(0, 256, size=(n, 28, 28), dtype=np.uint8)
    labels = rng.integers(0, 10, size=n)
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"],
                 corpus=AVMNISTCorpus(audio, u8, labels), device=gpu)
    g = torch.Generator().manual_seed(3)
    dl = ds.device_loader(batch, shuffle=True, generator=g)
    state = g.get_state()
    order = dl.items()  # the order the next epoch will draw
    g.set_state(state)
    lut = lut_np()
    nb = len(dl)
    check = {0, 1, nb // 2, nb - 1}
    for bi, b in enumerate(dl):
        if bi not in check:
            continue
        items = order[bi * batch:(bi + 1) * batch]
        ref = dref.collate(audio, u8, labels, lut, items, "valid", ["ai", "a", "i"])
        assert np.array_equal(b["labels"].cpu().numpy(), ref["labels"])
        assert b["pattern_name"] == ref["pattern_name"]
        assert np.array_equal(b[ds.keys["audio"]].cpu().numpy(), ref["audio"])
        assert np.array_equal(b[ds.keys["image"]].cpu().numpy(), ref["image"])
    assert bi == nb - 1 == -(-3 * n // batch) - 1


def test_device_loader_equals_dataloader(gpu):
    from tspm_amd.data import AVMNIST
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"], corpus=corpus(40, 11), device=gpu)
    dl = torch.utils.data.DataLoader(ds, batch_size=16, shuffle=True, collate_fn=ds.collate_fn,
                                     generator=torch.Generator().manual_seed(5))
    dv = ds.device_loader(16, shuffle=True, generator=torch.Generator().manual_seed(5))
    n = 0
    for a, b in zip(dl, dv):
        n += 1
        assert a["pattern_name"] == b["pattern_name"]
        for k in ("labels", ds.keys["audio"], ds.keys["image"]):
            assert torch.equal(a[k], b[k])
    assert n == len(dv) == 8


def test_distributed_device_loader_shards(gpu):
    from tspm_amd.data import AVMNIST
    c = corpus(37, 12)
    ds = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=c, device=gpu)
    seen = []
    for rank in range(4):
        dl = ds.device_loader(4, shuffle=True, rank=rank, world_size=4, seed=1)
        dl.set_epoch(2)
        for b in dl:
            seen.extend(b["labels"].cpu().tolist())
        assert sum(len(b["labels"]) for b in dl) == 10
    idx = np.concatenate([dref.distributed_indices(37, 4, r, True, 1, 2) for r in range(4)])
    assert seen == c.labels[idx].tolist()


def test_out_of_range_index_is_nan_not_a_fault(gpu):
    from tspm_amd.data import DeviceCorpus
    c = corpus(8, 3)
    dc = DeviceCorpus(c, gpu)
    idx = torch.tensor([0, 8, -1, 7], dtype=torch.int64, device=gpu)
    a, im, lab = dc.gather(idx)
    torch.cuda.synchronize()
    assert lab.cpu().tolist() == [int(c.labels[0]), -1, -1, int(c.labels[7])]
    assert torch.isnan(a[1]).all() and torch.isnan(im[2]).all()
    assert torch.equal(a[0].cpu(), torch.from_numpy(c.audio[0]))
    # tspm_cross_entropy turns label -1 into NaN instead of reading out of bounds
    from tspm_amd import _lib as L
    logits = torch.zeros(4, 10, device=gpu)
    loss = torch.empty(1, device=gpu)
    L.check(L.lib().tspm_cross_entropy(4, 10, logits.data_ptr(), lab.data_ptr(), loss.data_ptr(), None, 1.0, None,
                                       L.stream_handle()), "ce")
    assert torch.isnan(loss).all()


def test_unaligned_shapes_use_scalar_path(gpu):
    from tspm_amd.data import AVMNISTCorpus, DeviceCorpus
    rng = np.random.default_rng(1)
    audio = rng.standard_normal((9, 3, 5), dtype=np.float32)
    u8 = rng.integers(0, 256, size=(9, 3, 3), dtype=np.uint8)
    labels = rng.integers(0, 10, size=9)
    dc = DeviceCorpus(AVMNISTCorpus(audio, u8, labels), gpu)
    idx = torch.tensor([8, 0, 4, 4, 2], dtype=torch.int64, device=gpu)
    am = torch.tensor([1, 0, 1, 1, 0], dtype=torch.float32, device=gpu)
    a, im, lab = dc.gather(idx, audio_mask=am)
    i = idx.cpu().numpy()
    assert np.array_equal(a.cpu().numpy(), audio[i] * am.cpu().numpy()[:, None, None])
    assert np.array_equal(im.cpu().numpy()[:, 0], lut_np()[u8[i]].astype(np.float32) * np.float32(1 / 255))
    assert np.array_equal(lab.cpu().numpy(), labels[i])


def test_train_step_from_device_batches(gpu):
    # the fused train step consumes the device batches directly (no host round trip)
    import tspm_amd
    from tspm_amd.data import AVMNIST
    from tspm_amd.step import FusedTrainStep
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    ds = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=corpus(96, 5), device=gpu)
    dl = torch.utils.data.DataLoader(ds, batch_size=32, shuffle=True, collate_fn=ds.collate_fn)
    losses = [model.train_step(b, opt, None, gpu, None)["loss"] for b in dl]
    assert len(losses) == 3 and all(np.isfinite(losses))
    assert isinstance(model._fused_step, FusedTrainStep)
