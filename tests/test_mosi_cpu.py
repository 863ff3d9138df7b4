"""MOSI UTT-Fusion (BASELINE configs[4]) checks that need no GPU: the CPU oracle against the vectors
captured from the REAL reference (tests/golden/make_mosi_golden.py → mosi_step_b4.npz, bit-exact),
and the drop-in modules' constructor signatures, seeded initialisation and state_dict layout."""
import os

import numpy as np
import pytest
import torch

import tspm_amd
from oracle import mosi_ref as orc
from tspm_amd import mosi as M

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mosi_step_b4.npz")
GOLDEN_MOSEI = os.path.join(os.path.dirname(__file__), "golden", "mosei_step_b4.npz")


@pytest.fixture(scope="module")
def mg():
    return dict(np.load(GOLDEN, allow_pickle=False))


@pytest.fixture(scope="module")
def meg():
    return dict(np.load(GOLDEN_MOSEI, allow_pickle=False))


def _dropin(seed=0, clip=None, cfg=orc.MOSI):
    torch.manual_seed(seed)
    a = M.LSTMEncoder(input_size=cfg.audio_dim, hidden_size=64, embd_method=cfg.embd_method)
    v = M.LSTMEncoder(input_size=cfg.video_dim, hidden_size=64, embd_method=cfg.embd_method)
    t = M.TextCNN(input_size=768, embd_size=64, dropout=cfg.text_dropout, in_channels=1, out_channels=128,
                  kernel_heights=[3, 4, 5])
    c = M.FcClassifier(input_dim=192, layers=list(cfg.cls_layers), output_dim=3, dropout=cfg.cls_dropout,
                       use_bn=cfg.use_bn)
    return M.UttFusionModel(a, v, t, c, clip=cfg.clip if clip is None else clip)


def test_oracle_reproduces_reference_train_steps_bitwise(mg):
    """3 train steps of oracle/mosi_ref.py equal the real UttFusionModel.train_step bit for bit (same
    seed-0 weights, inputs with zero padding, the reference's own dropout masks): logits, losses, the
    clip_grad_norm_ totals, step-1 gradients (after the clip) and the parameters after every step.
    (4 intra-op threads, as when the vectors were made: ATen's CPU reductions depend on the split.)"""
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        _replay(mg)
    finally:
        torch.set_num_threads(nt)


def test_oracle_reproduces_reference_mosei_train_steps_bitwise(meg):
    """The MOSEI config (configs/mosei/centralised/utt_fusion_train_mosei.yaml: "maxpool" LSTM embeddings,
    FcClassifier with BatchNorm1d, clip 0.5): 3 oracle train steps equal the real reference bit for bit,
    incl. the BatchNorm1d running statistics and num_batches_tracked after every step."""
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        _replay(meg, orc.MOSEI)
    finally:
        torch.set_num_threads(nt)


def _replay(mg, cfg=orc.MOSI):
    model = orc.build_oracle_utt(0, cfg=cfg)
    assert list(model.state_dict()) == list(mg["state_dict_keys"])
    opt = orc.OracleAdam(list(model.parameters()), lr=cfg.lr, weight_decay=cfg.weight_decay)
    A, V, T, y = (torch.from_numpy(mg[k]) for k in ("audio", "video", "text", "labels"))
    names = ["text"] + [f"cls{j}" for j in range(len(cfg.cls_layers))]
    bns = [m for m in model.netC.module if isinstance(m, torch.nn.BatchNorm1d)]
    for s in range(3):
        keeps = {k: torch.from_numpy(mg[f"keep_{k}"][s]) for k in names}
        r = orc.train_step(model, opt, A, V, T, y, keeps)
        assert torch.equal(r["logits"], torch.from_numpy(mg["logits"][s])), s
        assert r["loss"].item() == mg["losses"][s], s
        assert float(r["total_norm"]) == mg["total_norms"][s], s
        if s == 0:
            gn = np.array([p.grad.double().norm().item() for p in model.parameters()])
            np.testing.assert_array_equal(gn, mg["grad_norm_step1"])
        ps = np.array([p.detach().double().sum().item() for p in model.parameters()])
        np.testing.assert_array_equal(ps, mg["param_sums"][s])
        if bns:
            st = [float(t.double().sum()) for bn in bns for t in (bn.running_mean, bn.running_var)]
            st += [int(bn.num_batches_tracked) for bn in bns]
            np.testing.assert_array_equal(np.array(st), mg["bn_stat_sums"][s])
    model.eval()
    with torch.no_grad():
        ev = orc.forward(model, A, V, T, False)
    assert torch.equal(ev, torch.from_numpy(mg["eval_logits"]))


def test_dropin_state_dict_and_seeded_init_equal_reference(mg, meg):
    for cfg, g in ((orc.MOSI, mg), (orc.MOSEI, meg)):
        ours, ref = _dropin(0, cfg=cfg), orc.build_oracle_utt(0, cfg=cfg)
        sd, rsd = ours.state_dict(), ref.state_dict()
        assert list(sd) == list(rsd) == list(g["state_dict_keys"])
        for k in sd:
            assert torch.equal(sd[k], rsd[k]), k
        assert [n for n, _ in ours.named_parameters()] == list(g["param_names"])


def test_dropin_api_surface():
    m = _dropin(0)
    assert m.get_encoder("audio") is m.netA and m.get_encoder("video") is m.netV and m.get_encoder("text") is m.netT
    assert m.netA.hidden_size == 64 and m.netT.hidden_size == 64 and m.clip == 1.0
    with pytest.raises(NotImplementedError):
        M.LSTMEncoder(5, 64, embd_method="attention")
    assert M.LSTMEncoder(74, 64, embd_method="maxpool").embd_method == "maxpool"
    assert len(M.FcClassifier(192, [96, 48], 3, use_bn=True).bns()) == 2
    m.flatten_parameters()
    with pytest.raises(tspm_amd._lib.TspmError):  # no CPU fallback
        m.eval()
        m(torch.zeros(2, 8, 5), torch.zeros(2, 8, 20), torch.zeros(2, 8, 768))


def test_yaml_tags_build_dropins():
    import yaml
    tspm_amd.plugin.register_yaml()
    doc = yaml.safe_load("""
netA: !LSTMEncoder {input_size: 5, hidden_size: 64, embd_method: "last"}
netT: !TextCNN {input_size: 768, embd_size: 64, dropout: 0.5, in_channels: 1, out_channels: 128,
                kernel_heights: [3, 4, 5]}
netC: !FcClassifier {input_dim: 192, layers: [192, 64, 32], output_dim: 3, dropout: 0.5}
""")
    assert isinstance(doc["netA"], M.LSTMEncoder) and isinstance(doc["netT"], M.TextCNN)
    assert isinstance(doc["netC"], M.FcClassifier)
    assert tspm_amd.plugin.MODELS["utt-fusion"] is M.UttFusionModel


def test_mosi_corpus_packing_and_padded_length():
    """mosi_data: ragged rows packed per modality (offsets/lengths), pad length = the batch maximum
    (pad_sequence), an unaligned batch is refused unless pad_to covers it, pattern semantics."""
    from tspm_amd import mosi_data as D
    g = np.random.default_rng(0)
    lens = [3, 7, 5]
    seqs = {"audio": [g.standard_normal((l, 5), dtype=np.float32) for l in lens],
            "video": [g.standard_normal((l, 20), dtype=np.float32) for l in lens],
            "text": [g.standard_normal((l, 8), dtype=np.float32) for l in [3, 7, 6]]}
    c = D.MosiCorpus(seqs, np.array([0, 2, 1]))
    assert list(c.offsets["audio"]) == [0, 3, 10] and list(c.lengths["text"]) == [3, 7, 6]
    np.testing.assert_array_equal(c.data["video"][3:10], seqs["video"][1])

    class _Dc(D.DeviceMosiCorpus):  # host-side length logic only (no upload)
        def __init__(self, corpus):
            self.host_lengths = corpus.lengths
    dc = _Dc(c)
    assert dc.steps_for(np.array([0, 1])) == 7
    with pytest.raises(tspm_amd._lib.TspmError):
        dc.steps_for(np.array([2]))  # audio 5 vs text 6: pad_sequence would pad them differently
    assert dc.steps_for(np.array([2]), pad_to=50) == 50
    assert D.pattern_keep("at") == {"audio": 1.0, "video": 0.0, "text": 1.0}
    split = {"audio": np.zeros((2, 4, 5)), "vision": np.zeros((2, 4, 20)), "text": np.zeros((2, 4, 8)),
             "classification_labels": np.array([[1], [2]])}
    c2 = D.MosiCorpus.from_split(split)
    assert len(c2) == 2 and c2.labels.dtype == np.int64 and list(c2.lengths["text"]) == [4, 4]


def test_mosi_dataset_loads_npz_and_refuses_pickles_by_default(tmp_path):
    from tspm_amd import mosi_data as D
    g = np.random.default_rng(1)
    arrs = {"train/audio": g.standard_normal((3, 6, 5)).astype(np.float32),
            "train/vision": g.standard_normal((3, 6, 20)).astype(np.float32),
            "train/text": g.standard_normal((3, 6, 768)).astype(np.float32),
            "train/classification_labels": np.array([0, 2, 1])}
    fp = tmp_path / "mosi.npz"
    np.savez(fp, **arrs)
    ds = D.MOSI(str(fp), "train", device="cpu", aligned=True, length=6)
    assert len(ds) == 3 and list(ds.corpus.lengths["video"]) == [6, 6, 6]
    np.testing.assert_array_equal(ds.corpus.data["text"][6:12], arrs["train/text"][1])
    pk = tmp_path / "mosi.pkl"
    pk.write_bytes(b"not read")
    with pytest.raises(ValueError):
        D.MOSI(str(pk), "train", device="cpu")


def test_build_utt_fusion_matches_both_yamls(mg, meg):
    """mosi.build_utt_fusion("mosi" / "mosei"): the YAML's modules in the YAML's order — state_dict keys and
    seeded weights equal to the real reference's (the golden files' state_dict sha256)."""
    import hashlib
    for name, g in (("mosi", mg), ("mosei", meg)):
        torch.manual_seed(0)
        sd = M.build_utt_fusion(name).state_dict()
        h = hashlib.sha256()
        for k in sorted(sd):
            h.update(k.encode())
            h.update(sd[k].contiguous().numpy().tobytes())
        assert list(sd) == list(g["state_dict_keys"]) and h.hexdigest() == str(g["state_dict_sha256"]), name
