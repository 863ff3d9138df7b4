"""Input stage, CPU side: the data-stage oracle against the golden batches the REAL reference dataset
produced (tests/golden/make_data_golden.py), corpus file formats, sampler semantics, the dataset's
host logic, and the gather entry point's argument validation (no GPU: nothing is launched)."""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest
import torch

from oracle import avmnist_data_ref as dref
from oracle import avmnist_ref as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("train", "multimodal", ["ai"]), ("valid", "multimodal", ["ai", "a", "i"]), ("test", "image", ["i", "ai"])]


@pytest.fixture(scope="module")
def dgold():
    return dict(np.load(os.path.join(REPO, "tests", "golden", "avmnist_data.npz"), allow_pickle=False))


@pytest.fixture(scope="module")
def small_corpus(dgold):
    audio, _, labels, u8 = orc.synthetic_batch(int(dgold["n"]), seed=int(dgold["seed"]))
    return audio.numpy(), u8.numpy(), labels.numpy()


def lut_np():
    with open(os.path.join(REPO, "tests", "golden", "lut_gist_earth_L.bin"), "rb") as f:
        return np.frombuffer(f.read(), dtype=np.uint8).copy()


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_package_lut_is_the_golden_lut():
    from tspm_amd import data
    assert np.array_equal(data.default_lut(), lut_np())


def test_lut_matches_matplotlib_pil_pipeline():
    # data/avmnist.py:188-189 for every integer input value
    cm = pytest.importorskip("matplotlib.cm")
    Image = pytest.importorskip("PIL.Image")
    idx = np.arange(256, dtype=np.uint8).reshape(16, 16)
    img = Image.fromarray(np.uint8(cm.gist_earth(idx) * 255)).convert("L")
    assert np.array_equal(np.array(img, dtype=np.uint8).reshape(256), lut_np())


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_oracle_collate_matches_reference_batches(dgold, small_corpus, ci):
    audio, u8, labels = small_corpus
    split, target, sel = CASES[ci]
    n = audio.shape[0]
    assert dref.dataset_len(split, n, sel) == int(dgold[f"c{ci}_len"])
    B = int(dgold["batch"])
    L = int(dgold[f"c{ci}_len"])
    nb = int(dgold[f"c{ci}_batches"])
    assert nb == -(-L // B)
    for bi in range(nb):
        items = list(range(bi * B, min(L, (bi + 1) * B)))
        out = dref.collate(audio, u8, labels, lut_np(), items, split, sel, target=target)
        key = f"c{ci}_b{bi}"
        assert np.array_equal(out["labels"], dgold[key + "_labels"])
        assert out["pattern_name"] == list(dgold[key + "_pattern"])
        assert len(out["missing_masks"]) == int(dgold[key + "_mask_keys"]) == 0
        if target in ("multimodal", "audio"):
            assert list(out["audio"].shape) == list(dgold[key + "_audio_shape"])
            assert sha(out["audio"]) == str(dgold[key + "_audio_sha256"])
        else:
            assert key + "_audio_sha256" not in dgold
        assert np.array_equal(out["image"], dgold[key + "_image"])
        assert sha(out["image"]) == str(dgold[key + "_image_sha256"])


def test_pattern_names_and_defaults():
    assert dref.all_patterns() == ["a", "ai", "i"]
    from tspm_amd.data import AVMNIST
    assert AVMNIST.get_all_possible_patterns() == ["a", "ai", "i"]
    assert AVMNIST.get_full_modality() == "ai"


@pytest.mark.parametrize("n,world,drop,shuffle", [(10, 4, False, True), (10, 4, True, True), (12, 3, False, False),
                                                  (3, 8, False, True), (1000, 8, True, True), (7, 2, False, False)])
def test_distributed_indices_match_torch_sampler(n, world, drop, shuffle):
    for rank in range(world):
        s = torch.utils.data.DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=5,
                                                drop_last=drop)
        s.set_epoch(3)
        assert list(s) == dref.distributed_indices(n, world, rank, shuffle, 5, 3, drop).tolist()


# -- corpus file formats -----------------------------------------------------------------------------------
def write_reference_corpus(root, audio, u8, labels):
    rows = ["audio,image,label"]
    for i in range(audio.shape[0]):
        ap, ip = os.path.join(root, f"a{i}.pt"), os.path.join(root, f"i{i}.pt")
        torch.save(torch.from_numpy(audio[i].copy()), ap)
        torch.save(u8[i].copy(), ip)  # the reference's images are pickled numpy arrays
        rows.append(f"{os.path.basename(ap)},{os.path.basename(ip)},{int(labels[i])}")
    p = os.path.join(root, "c.csv")
    open(p, "w").write("\n".join(rows) + "\n")
    return p


def test_corpus_from_reference_csv_and_packed_roundtrip(tmp_path, small_corpus):
    from tspm_amd.data import AVMNISTCorpus, pack
    audio, u8, labels = small_corpus
    csv = write_reference_corpus(str(tmp_path), audio, u8, labels)
    c = AVMNISTCorpus.from_csv(csv)
    assert np.array_equal(c.audio, audio) and np.array_equal(c.image, u8) and np.array_equal(c.labels, labels)
    sub = AVMNISTCorpus.from_csv(csv, split_indices=[4, 1])
    assert np.array_equal(sub.labels, labels[[4, 1]]) and np.array_equal(sub.image, u8[[4, 1]])
    out = str(tmp_path / "packed")
    pack(csv, out)
    d = AVMNISTCorpus.load(out)
    assert np.array_equal(d.audio, audio) and np.array_equal(d.image, u8) and np.array_equal(d.labels, labels)
    assert np.array_equal(AVMNISTCorpus.open(out, [2]).audio, audio[[2]])


def test_corpus_csv_missing_columns_and_float_images(tmp_path, small_corpus):
    from tspm_amd.data import AVMNISTCorpus
    audio, u8, labels = small_corpus
    p = tmp_path / "bad.csv"
    p.write_text("audio,img,label\nx,y,1\n")
    with pytest.raises(ValueError, match="Missing required columns"):
        AVMNISTCorpus.from_csv(str(p))
    torch.save(torch.zeros(28, 28), str(tmp_path / "f.pt"))
    torch.save(torch.from_numpy(audio[0].copy()), str(tmp_path / "a.pt"))
    q = tmp_path / "f.csv"
    q.write_text("audio,image,label\na.pt,f.pt,3\n")
    with pytest.raises(ValueError, match="integer colormap indices"):
        AVMNISTCorpus.from_csv(str(q))


# -- dataset host logic ------------------------------------------------------------------------------------
def make_ds(small_corpus, split, target, sel, **kw):
    from tspm_amd.data import AVMNIST, AVMNISTCorpus
    audio, u8, labels = small_corpus
    return AVMNIST(None, split, target, selected_patterns=sel, corpus=AVMNISTCorpus(audio, u8, labels), **kw)


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_dataset_resolution_matches_oracle(small_corpus, ci):
    split, target, sel = CASES[ci]
    ds = make_ds(small_corpus, split, target, sel)
    n = small_corpus[0].shape[0]
    assert len(ds) == dref.dataset_len(split, n, sel)
    items = list(range(len(ds)))[::-1]
    samples, names, am, im = ds._resolve(items)
    masks = dref.missing_masks(dref.default_missing_patterns(), len(ds))
    for k, it in enumerate(items):
        p, s = dref.pattern_and_sample(it, split, n, sel, random.Random(0))
        assert names[k] == p and samples[k] == s
        assert am[k] == masks[p]["audio"][s] and im[k] == masks[p]["image"][s]


def test_train_pattern_draw_consumes_python_random_like_reference(small_corpus):
    # base_dataset.py:87 — one random.choice per item from the global `random` module
    ds = make_ds(small_corpus, "train", "multimodal", ["ai", "a"])
    random.seed(11)
    _, names, _, _ = ds._resolve(range(6))
    random.seed(11)
    assert names == [random.choice(["ai", "a"]) for _ in range(6)]


def test_dataset_validation_errors(small_corpus):
    from tspm_amd.data import AVMNIST
    with pytest.raises(ValueError, match="Invalid patterns"):
        make_ds(small_corpus, "valid", "multimodal", ["ia"])
    with pytest.raises(AssertionError):
        make_ds(small_corpus, "dev", "multimodal", ["ai"])
    with pytest.raises(AssertionError):
        make_ds(small_corpus, "valid", "text", ["ai"])
    with pytest.raises(FileNotFoundError):
        AVMNIST("/nonexistent/corpus.csv", "train")
    ds = make_ds(small_corpus, "valid", "multimodal", ["ai"])
    with pytest.raises(ValueError, match="only available for validation"):
        make_ds(small_corpus, "train", "multimodal", ["ai"]).get_pattern_batches(2)
    with pytest.raises(IndexError):
        ds._resolve([len(ds)])


def test_fractional_presence_masks_are_bernoulli(small_corpus):
    # fractional missing rates: parity unpinned (un-vendored create_missing_mask); only the rate is checked
    from tspm_amd.data import AVMNIST, AVMNISTCorpus
    audio, u8, labels = small_corpus
    big = AVMNISTCorpus(np.repeat(audio, 500, 0), np.repeat(u8, 500, 0), np.repeat(labels, 500))
    ds = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=big,
                 missing_patterns={"ai": {"audio": 0.7, "image": 1.0}})
    m = ds.masks["ai"]["audio"]
    assert set(np.unique(m)) <= {0.0, 1.0} and abs(m.mean() - 0.7) < 0.03
    assert (ds.masks["ai"]["image"] == 1.0).all()


def test_no_cpu_path_without_gpu(small_corpus):
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    from tspm_amd import TspmError
    ds = make_ds(small_corpus, "train", "multimodal", ["ai"])
    with pytest.raises(TspmError):
        ds[0]
    dl = torch.utils.data.DataLoader(ds, batch_size=2, collate_fn=ds.collate_fn)
    with pytest.raises(TspmError):
        next(iter(dl))


@pytest.mark.parametrize("shuffle,drop,world,gen", [(False, False, 1, True), (True, False, 1, True),
                                                    (True, True, 1, False), (True, False, 2, True),
                                                    (False, True, 4, False), (True, False, 1, False)])
def test_device_loader_order_matches_dataloader(small_corpus, shuffle, drop, world, gen):
    # the item order of iter(DataLoader(...)) including its RNG draws (base seed, then the sampler)
    ds = make_ds(small_corpus, "valid", "multimodal", ["ai", "a", "i"])
    for rank in range(world):
        torch.manual_seed(123)
        g = torch.Generator().manual_seed(9) if gen else None
        dl = ds.device_loader(4, shuffle=shuffle, drop_last=drop, generator=g, rank=rank, world_size=world, seed=2)
        dl.set_epoch(1)
        got = dl.items()
        after = torch.randint(0, 1 << 30, (1,)).item()
        torch.manual_seed(123)
        g = torch.Generator().manual_seed(9) if gen else None
        if world > 1:
            s = torch.utils.data.DistributedSampler(range(len(ds)), num_replicas=world, rank=rank, shuffle=shuffle,
                                                    seed=2, drop_last=drop)
            s.set_epoch(1)
            ref_dl = torch.utils.data.DataLoader(range(len(ds)), batch_size=4, sampler=s, drop_last=drop,
                                                 generator=g, collate_fn=list)
        else:
            ref_dl = torch.utils.data.DataLoader(range(len(ds)), batch_size=4, shuffle=shuffle, drop_last=drop,
                                                 generator=g, collate_fn=list)
        ref = [i for b in ref_dl for i in b]
        assert got[:len(ref)].tolist() == ref
        assert len(dl) == len(ref_dl)
        assert torch.randint(0, 1 << 30, (1,)).item() == after  # same global-RNG consumption


def test_pattern_view_offsets(small_corpus):
    from tspm_amd.data import PatternView
    ds = make_ds(small_corpus, "valid", "multimodal", ["ai", "a", "i"])
    v = PatternView(ds, "a")
    assert len(v) == 6 and list(v.__getitems__([0, 5])) == [6, 11]


# -- C ABI argument validation (returns before any HIP call) ------------------------------------------------
def test_gather_rejects_bad_arguments():
    from tspm_amd import _lib as L
    lib = L.load()
    f = lib.tspm_avmnist_gather
    dummy = ctypes.c_void_p(16)
    assert f(0, None, 0, None, 0, None, 0, None, None, None, None, None, None, None, None) == 0  # empty batch
    assert f(-1, dummy, 4, dummy, 4, dummy, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1
    assert f(4, None, 4, dummy, 4, dummy, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1  # no index
    assert f(4, dummy, 0, dummy, 4, dummy, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1  # empty corpus
    assert f(4, dummy, 4, None, 4, dummy, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1  # audio src
    assert f(4, dummy, 4, dummy, 4, None, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1  # image src
    assert f(4, dummy, 4, dummy, 4, dummy, 4, None, None, None, None, dummy, dummy, dummy, None) == 1  # labels src
    assert f(4, dummy, 4, dummy, 0, dummy, 4, dummy, None, None, None, dummy, dummy, dummy, None) == 1  # 0 elems


def test_package_synthetic_corpus_equals_oracle_generator():
    from tspm_amd.data import synthetic_corpus
    c = synthetic_corpus(5, seed=77)
    audio, _, labels, u8 = orc.synthetic_batch(5, seed=77)
    assert np.array_equal(c.audio, audio.numpy()) and np.array_equal(c.image, u8.numpy())
    assert np.array_equal(c.labels, labels.numpy())


def test_reference_host_pipeline_matches_reference_batches(tmp_path, dgold, small_corpus):
    # the CPU-baseline restatement (cm.gist_earth + PIL per sample, stack) reproduces the golden batches
    pytest.importorskip("matplotlib")
    audio, u8, labels = small_corpus
    csv = dref.write_reference_files(str(tmp_path), audio, u8, labels)
    got = list(dref.reference_host_batches(csv, int(dgold["batch"])))
    assert len(got) == int(dgold["c0_batches"])
    for bi, b in enumerate(got):
        assert sha(b["audio"].numpy()) == str(dgold[f"c0_b{bi}_audio_sha256"])
        assert np.array_equal(b["image"].numpy(), dgold[f"c0_b{bi}_image"])
        assert np.array_equal(b["labels"].numpy(), dgold[f"c0_b{bi}_labels"])


def test_reference_sample_files_load_weights_only():
    """Two of the reference's own per-sample files (MML_Suite/AVMNIST/dataset, copied as fixtures):
    the image is a numpy-1.x pickle, which the weights-only unpickler takes only with the allow-list
    entry under the old module name numpy.core.multiarray._reconstruct (data._np_safe_globals)."""
    import os
    import numpy as np
    import torch
    from tspm_amd.data import _np_safe_globals, load_sample_file
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with torch.serialization.safe_globals(_np_safe_globals()):
        img = load_sample_file(os.path.join(g, "ref_image_10000_10000_3.pt"))
        spec = load_sample_file(os.path.join(g, "ref_spectrogram_0_01_0.pt"))
    img = np.asarray(img)
    assert img.shape == (28, 28) and np.issubdtype(img.dtype, np.integer) and 0 <= img.min() and img.max() <= 255
    assert spec.shape == (32, 94) and spec.dtype == np.float32 and np.isfinite(spec).all() and spec.min() >= 0
