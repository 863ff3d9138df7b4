"""MOSI UTT-Fusion step (BASELINE configs[4]) on the HIP path against the CPU oracle (oracle/mosi_ref.py,
pinned bit-exact to the real reference by tests/golden/make_mosi_golden.py / tests/test_mosi_cpu.py).

Criterion as tests/test_gpu_model.py (tests/parity.py): the oracle in fp64 with our decisions forced
into it — the TextCNN time-max argmax and the ReLU at it, the embedding and classifier ReLU masks, the
dropout masks — is the truth; every forced decision that differs from fp64's own must be a near-tie
(and rare); logits / loss rel-L2 <= 1e-4, every gradient rel-L2 <= 1e-3 and cosine >= 0.9999 and within
4x the fp32 reference's error on the same decisions; no relaxed branch.  The clip coefficient
(clip_grad_norm_ total) is checked against the fp64 gradients; Adam exactly (fp64 Adam applied to our
clipped gradient and moments).  Every step is checked from our own state.
"""
import numpy as np
import pytest
import torch

import tspm_amd
from oracle import mosi_ref as orc
from parity import (MAX_FLIP_FRAC, NEAR, Tally, check_adam, check_grad, check_out, pair_from, rel_l2, snapshot)
from test_mosi_cpu import _dropin
from tspm_amd import _lib as L
from tspm_amd import mosi as M

pytestmark = pytest.mark.gpu
LR, WD = 1e-3, 1e-3


def _decisions(eng):
    C, d = eng.C, {}
    for i in range(3):
        d[f"text.pool{i}"] = eng.argmax[:, i * C:(i + 1) * C].long().cpu()
        d[f"text.relu{i}"] = (eng.pooled[:, i * C:(i + 1) * C] > 0).cpu()
    col = eng.m.netA.hidden_size + eng.m.netV.hidden_size
    d["text.embd"] = (eng.fused[:, col:] > 0).cpu()
    for j, h in enumerate(eng.r if eng.use_bn else eng.h):  # with use_bn: the ReLU output before the BN
        d[f"cls.relu{j}"] = (h > 0).cpu()
    for name in ("a", "v"):  # "maxpool" LSTM embeddings: the time index of every unit's maximum
        if eng.lstm[name]["arg"] is not None:
            d[f"lstm.{name}.pool"] = eng.lstm[name]["arg"].long().cpu()
    return d


def _flips(t64, forced, keeps, use_bn=False):
    rep = {}
    for site, f in forced.items():
        if site.startswith("lstm."):
            r_out = t64.pre[site].double()  # [B, T, H]
            nat = t64.idx[site]
            flip = f != nat
            dist = (r_out.gather(1, f.unsqueeze(1)) - r_out.gather(1, nat.unsqueeze(1))).squeeze(1).abs()[flip]
            x = r_out
        elif site.startswith("text.pool"):
            conv = t64.pre[site].double().relu()
            nat = t64.idx[site]
            flip = f != nat
            dist = (conv.gather(2, f.unsqueeze(2)) - conv.gather(2, nat.unsqueeze(2))).squeeze(2).abs()[flip]
            x = conv
        else:
            x = t64.pre[site].double()
            flip = f != (x > 0)
            if site.startswith("cls.relu") and not use_bn:  # dropped after the ReLU: the decision is moot
                flip &= keeps[f"cls{site[-1]}"].bool()
            dist = x.abs()[flip]
        rms = x.pow(2).mean().sqrt().item() or 1.0
        nf = int(flip.sum())
        worst = dist.max().item() / rms if nf else 0.0
        assert worst <= NEAR, f"{site}: a flipped decision is {worst:.2e} x rms from its threshold / tie"
        assert nf <= max(1, MAX_FLIP_FRAC * f.numel()), f"{site}: {nf} of {f.numel()} decisions flipped"
        rep[site] = nf
    return {k: v for k, v in rep.items() if v}


def _forced(o32, o64, A, V, T, y, keeps, forced):
    o32.clip = o64.clip = None  # raw gradients; the clip is checked through the total norm
    t32, t64 = orc.MosiTrace(forced), orc.MosiTrace(forced)
    r32 = orc.train_step(o32, None, A, V, T, y, keeps, t32)
    r64 = orc.train_step(o64, None, A.double(), V.double(), T.double(), y, keeps, t64)
    return r32, r64, t64


def _check_step(ours, st, o32, o64, A, V, T, y, keeps, out, tally, ref32_logits=None, ref32_loss=None):
    eng = st.eng
    forced = _decisions(eng)
    r32, r64, t64 = _forced(o32, o64, A, V, T, y, keeps, forced)
    rep = _flips(t64, forced, keeps, eng.use_bn)
    check_out("logits", out["logits"], r32["logits"] if ref32_logits is None else ref32_logits, r64["logits"], tally)
    check_out("loss", out["loss"], (r32["loss"] if ref32_loss is None else ref32_loss).reshape(1),
              r64["loss"].reshape(1), tally)
    p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
    for n, p in ours.named_parameters():
        check_grad(f"grad {n}", p.grad, p32[n].grad, p64[n].grad, tally)
    norm64 = torch.sqrt(sum((q.grad.double() ** 2).sum() for q in o64.parameters()))
    norm32 = torch.sqrt(sum((q.grad.double() ** 2).sum() for q in o32.parameters()))
    check_out("total grad norm", eng.total_norm, norm32.reshape(1), norm64.reshape(1), tally)
    if eng.use_bn:  # the classifier BatchNorm1d running statistics and num_batches_tracked after the step
        b32, b64 = dict(o32.named_buffers()), dict(o64.named_buffers())
        for n, b in ours.named_buffers():
            if n.endswith("num_batches_tracked"):
                assert int(b) == int(b64[n]), n
            else:
                check_out(n, b, b32[n], b64[n], tally)
    return rep


def _check_adam(ours, opt, before, step, coef, cfg=orc.MOSI):
    check_adam(ours, opt, *before, step, lr=cfg.lr, wd=cfg.weight_decay, coef=coef)


def _run_steps(gpu, batch, steps, clip, n_steps=3, seed=3, lengths=None, golden=None, cfg=orc.MOSI):
    ours = _dropin(seed, clip=clip, cfg=cfg).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    if golden is not None:
        A, V, T, y = (torch.from_numpy(golden[k]) for k in ("audio", "video", "text", "labels"))
    else:
        A, V, T, y = orc.synthetic_batch(batch, steps, seed=1234 + batch, lengths=lengths, cfg=cfg)
    names = ["text"] + [f"cls{j}" for j in range(len(cfg.cls_layers))]
    st = M.FusedMosiStep(ours, opt, None, batch, steps)
    tally, coefs = Tally(), []
    for s in range(n_steps):
        if golden is not None:
            keeps = {k: torch.from_numpy(golden[f"keep_{k}"][s]) for k in names}
        else:
            keeps = orc.keep_masks(batch, 50 + s, cfg=cfg)
        o32, o64 = pair_from(ours, lambda: orc.build_oracle_utt(seed, cfg=cfg))
        before = snapshot(ours, opt if s else None)
        st.keep_override = {k: v.to(gpu) for k, v in keeps.items()}
        out = st.step(A.to(gpu), V.to(gpu), T.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        if golden is not None and s == 0:
            rep = _check_step(ours, st, o32, o64, A, V, T, y, keeps, out, tally,
                              torch.from_numpy(golden["logits"][0]), torch.tensor(float(golden["losses"][0])))
            # the reference's clip total (its own fp32 gradients, un-forced decisions)
            assert abs(st.eng.total_norm.item() - golden["total_norms"][0]) <= 1e-4 * golden["total_norms"][0]
        else:
            rep = _check_step(ours, st, o32, o64, A, V, T, y, keeps, out, tally)
        coef = float(st.eng.clip_coef.item())
        if clip is not None:
            exp = min(1.0, clip / (st.eng.total_norm.item() + 1e-6))
            assert abs(coef - exp) <= 1e-6 * exp
        coefs.append(coef)
        _check_adam(ours, opt, before, s + 1, coef if clip is not None else 1.0, cfg)
        print(f"[B={batch} T={steps} step {s + 1}] flips {rep} clip coef {coef:.4f}")
    print(tally)
    return ours, st, coefs


def test_fused_step_vs_golden_reference(gpu):
    """Steps on the B=4 batch the real UttFusionModel.train_step ran (20 steps, two samples zero-padded
    past their length, the reference's dropout masks), clip 1.0 as in the YAML."""
    import os
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "mosi_step_b4.npz"), allow_pickle=False))
    _run_steps(gpu, 4, 20, 1.0, seed=0, golden=g)


def test_mosei_fused_step_vs_golden_reference(gpu):
    """The MOSEI config (utt_fusion_train_mosei.yaml: 74/35-d inputs, "maxpool" LSTM embeddings,
    FcClassifier with BatchNorm1d + dropout 0.66, clip 0.5) on the B=4 batch the real reference ran."""
    import os
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "mosei_step_b4.npz"), allow_pickle=False))
    _run_steps(gpu, 4, 20, 0.5, seed=0, golden=g, cfg=orc.MOSEI)


@pytest.mark.parametrize("batch,steps", [(64, 50), (256, 50), (32, 23)])
def test_mosei_fused_step_vs_oracle(gpu, batch, steps):
    """MOSEI at its YAML batch (256) and smaller / odd lengths; clip 0.5 (active at these gradient norms)."""
    lengths = [steps - (i * 7) % (steps // 2) for i in range(batch)]
    _run_steps(gpu, batch, steps, 0.5, lengths=lengths, cfg=orc.MOSEI)


def test_mosei_graph_replay_equals_eager_and_eval(gpu):
    """Graph replay = eager bitwise (BN running statistics and num_batches_tracked included); then the
    eval forward (running statistics, no dropout) against the fp64 oracle's validation_step."""
    res = []
    for use_graph in (False, True):
        ours = _dropin(7, cfg=orc.MOSEI).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=orc.MOSEI.lr, weight_decay=orc.MOSEI.weight_decay)
        st = M.FusedMosiStep(ours, opt, None, 64, 50, use_graph=use_graph)
        A, V, T, y = orc.synthetic_batch(64, 50, seed=5, cfg=orc.MOSEI)
        for s in range(4):
            st.keep_override = {k: v.to(gpu) for k, v in orc.keep_masks(64, 90 + s, cfg=orc.MOSEI).items()}
            st.step(A.to(gpu), V.to(gpu), T.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        res.append(torch.cat([t.detach().reshape(-1).double() for t in ours.state_dict().values()]).cpu())
    assert torch.equal(res[0], res[1])
    assert all(int(bn.num_batches_tracked) == 4 for bn in ours.netC.bns())
    o = orc.build_oracle_utt(7, cfg=orc.MOSEI)
    o.load_state_dict({k: v.cpu() for k, v in ours.state_dict().items()})
    batch = {"audio": A, "video": V, "text": T, "label": y, "pattern_name": ["atv"] * 64}
    v = ours.validation_step(batch, None, gpu, None)
    r = orc.validation_step(o.double(), A.double(), V.double(), T.double(), y)
    check_out("mosei eval logits", ours._engine(64, 50, gpu).logits, None, r["logits"])
    assert abs(v["loss"] - r["loss"].item()) <= 1e-4 * abs(r["loss"].item())
    emb = ours.netA(A.to(gpu))  # standalone "maxpool" encoder = the model's audio columns
    assert rel_l2(emb, ours._engine(64, 50, gpu).fused[:, :64]) < 1e-6


@pytest.mark.parametrize("batch,steps,clip", [(32, 50, 1.0), (128, 50, 1.0), (64, 37, 0.05)])
def test_fused_step_vs_oracle(gpu, batch, steps, clip):
    """Full-size steps (aligned_50 length; an odd length; clip 0.05 so the coefficient is < 1 and the clip
    acts), variable lengths zero-padded to the batch length as pad_sequence does."""
    lengths = [steps - (i * 7) % (steps // 2) for i in range(batch)]
    _, _, coefs = _run_steps(gpu, batch, steps, clip, lengths=lengths)
    if clip == 0.05:
        assert max(coefs) < 1.0


def test_graph_replay_equals_eager(gpu):
    res = []
    for use_graph in (False, True):
        ours = _dropin(7).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD)
        st = M.FusedMosiStep(ours, opt, None, 64, 50, use_graph=use_graph)
        A, V, T, y = orc.synthetic_batch(64, 50, seed=5)
        for s in range(4):
            st.keep_override = {k: v.to(gpu) for k, v in orc.keep_masks(64, 90 + s).items()}
            st.step(A.to(gpu), V.to(gpu), T.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()]).cpu())
    assert torch.equal(res[0], res[1])


def test_lstm_bias_gradients_identical(gpu):
    """b_ih.grad and b_hh.grad are the same column sums of the gate gradients (as in ATen): bitwise."""
    ours = _dropin(1).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD)
    st = M.FusedMosiStep(ours, opt, None, 32, 50)
    A, V, T, y = orc.synthetic_batch(32, 50, seed=9)
    st.step(A.to(gpu), V.to(gpu), T.to(gpu), y.to(gpu))
    torch.cuda.synchronize()
    for enc in (ours.netA, ours.netV):
        assert torch.equal(enc.rnn.bias_ih_l0.grad, enc.rnn.bias_hh_l0.grad)


@pytest.mark.parametrize("cfg_name", ["mosi", "mosei"])
def test_device_dropout_masks(gpu, cfg_name):
    """Without keep_override the step draws fresh masks on the device every step: the TextCNN slice at the
    TextCNN's rate (MOSI 0.5, MOSEI 0.7 → ~30 % kept), the classifier slices at the classifier's (0.5 /
    0.66 → ~34 % kept), the two draws independent."""
    torch.manual_seed(2)
    ours = M.build_utt_fusion(cfg_name).to(gpu)
    cfg = orc.MOSI if cfg_name == "mosi" else orc.MOSEI
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD)
    st = M.FusedMosiStep(ours, opt, None, 64, 20)
    A, V, T, y = orc.synthetic_batch(64, 20, seed=11, cfg=cfg)
    masks = []
    for _ in range(3):
        st.step(A.to(gpu), V.to(gpu), T.to(gpu), y.to(gpu))
        masks.append([k.clone() for k in st.eng.keeps])
    torch.cuda.synchronize()
    pt, pc = ours.netT.dropout.p, ours.netC.dropout_p
    for j in range(len(masks[0])):
        assert not torch.equal(masks[0][j], masks[1][j]) and not torch.equal(masks[1][j], masks[2][j])
    for m in masks:
        assert abs(m[0].float().mean().item() - (1 - pt)) < 0.02, "text slice rate"
        cls = torch.cat([k.reshape(-1) for k in m[1:]]).float()
        assert abs(cls.mean().item() - (1 - pc)) < 0.02, "classifier slice rate"
        # independent draws: the text slice does not repeat the classifier bits at the same index
        n = min(m[0].numel(), cls.numel())
        agree = (m[0].reshape(-1)[:n].float() == cls[:n]).float().mean().item()
        expect = (1 - pt) * (1 - pc) + pt * pc
        assert abs(agree - expect) < 0.03


def test_autograd_path_fresh_masks(gpu):
    """The autograd-node path (torch optimizer / non-CE loss) advances its own counter: two training forwards
    draw different masks (the host counter was never incremented)."""
    ours = _dropin(2).to(gpu)
    ours.train()
    A, V, T, _ = orc.synthetic_batch(16, 12, seed=5)
    A, V, T = (x.to(gpu) for x in (A, V, T))
    got = []
    for _ in range(2):
        out = ours(A, V, T)
        out.sum().backward()
        eng = ours._engine(16, 12, A.device)
        got.append([k.clone() for k in eng.keeps])
    torch.cuda.synchronize()
    for a, b in zip(*got):
        assert not torch.equal(a, b)


def test_train_step_api_fused_and_autograd(gpu):
    """UttFusionModel.train_step with the reference's call signature: FusedAdam → the fused step; the
    reference's own torch.optim.Adam + LossFunctionGroup → forward / backward / clip_grad_norm_ / step
    through the autograd node (dropout off for a deterministic comparison of the two)."""
    from types import SimpleNamespace

    class Group(dict):
        def __call__(self, x, y):
            return {"total_loss": 0.0 + 1.0 * torch.nn.functional.cross_entropy(x, y)}

    A, V, T, y = orc.synthetic_batch(16, 30, seed=21)
    batch = {"audio": A, "video": V, "text": T, "label": y, "pattern_name": ["atv"] * 16}
    res = {}
    for kind in ("fused", "autograd"):
        ours = _dropin(4).to(gpu)
        ours.netT.dropout.p = 0.0
        ours.netC.dropout_p = 0.0  # the property sets every classifier nn.Dropout
        assert all(mm.p == 0.0 for mm in ours.netC.module if isinstance(mm, torch.nn.Dropout))
        opt = (tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD) if kind == "fused"
               else torch.optim.Adam(ours.parameters(), lr=LR, weight_decay=WD))
        r = ours.train_step(batch, opt, None if kind == "fused" else Group(), gpu, None)
        assert set(r) == {"loss"}
        assert (kind == "fused") == bool(ours._steps)
        torch.cuda.synchronize()
        res[kind] = (r["loss"], torch.cat([p.detach().reshape(-1) for p in ours.parameters()]).cpu())
    assert abs(res["fused"][0] - res["autograd"][0]) <= 1e-6 * abs(res["fused"][0])
    assert rel_l2(res["fused"][1], res["autograd"][1]) < 1e-6
    o = orc.build_oracle_utt(4)
    o.netT.p = 0.0
    o.netC.p = 0.0
    ro = orc.train_step(o, orc.OracleAdam(list(o.parameters()), lr=LR, weight_decay=WD), A, V, T, y)
    assert abs(res["fused"][0] - ro["loss"].item()) <= 1e-4 * abs(ro["loss"].item())
    _ = SimpleNamespace


def test_validation_step_and_embeddings(gpu):
    ours = _dropin(6).to(gpu)
    o = orc.build_oracle_utt(6)
    A, V, T, y = orc.synthetic_batch(48, 50, seed=31)
    batch = {"audio": A, "video": V, "text": T, "label": y, "pattern_name": ["atv"] * 48}

    class Rec:
        calls = []

        def update_group_all(self, group, predictions, targets, m_types):
            self.calls.append((group, predictions, targets, m_types))
    rec = Rec()
    v = ours.validation_step(batch, None, gpu, rec, return_test_info=True)
    r = orc.validation_step(o, A, V, T, y)
    assert abs(v["loss"] - r["loss"].item()) <= 1e-4 * abs(r["loss"].item())
    eng = ours._engine(48, 50, gpu)
    check_out("eval logits", eng.logits, None, orc.validation_step(o.double(), A.double(), V.double(), T.double(),
                                                                   y)["logits"])
    assert rec.calls and rec.calls[0][0] == "classification"
    emb = ours.netA(A.to(gpu))  # the standalone encoder embedding equals the model's audio columns
    assert rel_l2(emb, eng.fused[:, :64]) < 1e-6


def test_seq_gather_pads_like_pad_sequence(gpu):
    """tspm_seq_gather: ragged corpus rows → a zero-padded time-major batch, masks and labels —
    pad_sequence(batch_first) semantics (data/mosi.py:225-230), transposed."""
    rng = np.random.default_rng(0)
    lens = rng.integers(3, 25, size=40).astype(np.int32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    data = rng.standard_normal((int(lens.sum()), 7)).astype(np.float32)
    labels = rng.integers(0, 3, size=40).astype(np.int64)
    idx = torch.tensor([5, 0, 39, 17, 5, 22], dtype=torch.int64)
    tpad = int(lens[idx.numpy()].max())
    mask = torch.tensor([1, 0, 1, 1, 0, 1], dtype=torch.float32)
    dd = [torch.from_numpy(a).to(gpu) for a in (idx.numpy(), data, offs, lens, mask.numpy(), labels)]  # kept alive
    out = torch.empty(tpad, 6, 7, device=gpu)
    lab = torch.empty(6, dtype=torch.int64, device=gpu)
    L.check(L.lib().tspm_seq_gather(6, dd[0].data_ptr(), 40, dd[1].data_ptr(), dd[2].data_ptr(), dd[3].data_ptr(), 7,
                                    tpad, out.data_ptr(), 6 * 7, 7, dd[4].data_ptr(), dd[5].data_ptr(), lab.data_ptr(),
                                    L.stream_handle()), "seq_gather")
    seqs = [torch.from_numpy(data[offs[i]:offs[i] + lens[i]]) for i in idx.numpy()]
    ref = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True) * mask[:, None, None]
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().transpose(0, 1), ref)
    assert torch.equal(lab.cpu(), torch.from_numpy(labels[idx.numpy()]))


def test_mosi_dataset_collate_and_step_loader(gpu):
    """mosi_data.MOSI: collate_fn = pad_sequence(batch_first) x pattern mask per modality (data/mosi.py:198-247)
    with labels, eval batches grouped by pattern; device_loader(step_for=...) gathers the same batch
    time-major into the step's inputs, and the step on it equals the step on the collated batch."""
    from tspm_amd.mosi_data import MOSI, PATTERNS, pattern_keep, synthetic_mosi_corpus
    corpus = synthetic_mosi_corpus(40, seed=3, steps=12, min_len=4)
    ev = MOSI(split="valid", corpus=corpus, device=gpu)
    assert len(ev) == 40 * len(PATTERNS)
    items = [3, 41, 85, 200, 279]  # several patterns (pattern-major indexing)
    out = ev.collate_fn(ev.__getitems__(items))
    for it in items:
        p, s = PATTERNS[it // 40], it % 40
        b = out[p]
        j = [i % 40 for i in items if PATTERNS[i // 40] == p].index(s)
        for k, m in enumerate(("audio", "video", "text")):
            seqs = [torch.from_numpy(corpus.data[m][corpus.offsets[m][i % 40]:corpus.offsets[m][i % 40] +
                                                    corpus.lengths[m][i % 40]]) for i in items if PATTERNS[i // 40] == p]
            ref = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True) * pattern_keep(p)[m]
            assert torch.equal(b[m].cpu(), ref), (p, m)
        assert b["label"][j].item() == corpus.labels[s]
    # train loader straight into a step's buffers == the collated batch through train_step's load
    tr = MOSI(split="train", corpus=synthetic_mosi_corpus(16, seed=4, steps=10), device=gpu, selected_patterns=["atv"])
    m1 = _dropin(0).to(gpu)
    opt = tspm_amd.FusedAdam(m1.parameters(), lr=LR, weight_decay=WD)
    seen = []
    for b in tr.device_loader(8, shuffle=False, step_for=lambda n, t: seen.append((n, t)) or m1.fused_step(opt, None, n, t)):
        st = m1.fused_step(opt, None, 8, 10)
        assert b["audio"] is st.eng.A and b["time_major"]
        ref = tr.collate_fn(tr.__getitems__(list(range(len(seen) * 8 - 8, len(seen) * 8))))
        for m, buf in (("audio", st.eng.A), ("video", st.eng.V), ("text", st.eng.X)):
            assert torch.equal(buf.transpose(0, 1).cpu(), ref[m].cpu()), m
        assert torch.equal(st.eng.labels.cpu(), ref["label"].cpu())
    assert seen == [(8, 10), (8, 10)]


@pytest.mark.parametrize("B,T", [(128, 50), (6, 9)])
def test_textcnn_wgrad_slab_equals_rows_kernel(gpu, B, T):
    """The feature-slab TextCNN weight-gradient kernel is bitwise the per-(conv, channel) kernel (same fmaf
    order over the batch), including zero gradients and the bias sums."""
    import ctypes
    import os
    g = torch.Generator().manual_seed(B)
    F, C, hs = 768, 128, [3, 4, 5]
    nc = 3 * C
    x = torch.randn(T * B * F, generator=g).to(gpu)
    dout = torch.randn(B, nc, generator=g).to(gpu)
    keep = (torch.rand(B, nc, generator=g) > 0.5).to(torch.uint8).to(gpu)
    pooled = torch.randn(B, nc, generator=g).relu().to(gpu)
    arg = torch.stack([torch.randint(0, T - h + 1, (B, C), generator=g) for h in hs], 1).reshape(B, nc)
    arg = arg.to(torch.uint8).to(gpu)
    work = torch.empty(B, nc, device=gpu)

    def run():
        dws = [torch.full((C, h, F), float("nan"), device=gpu) for h in hs]
        dbs = [torch.full((C,), float("nan"), device=gpu) for _ in hs]
        L.check(L.lib().tspm_textcnn_bwd(B, T, F, 3, (ctypes.c_int32 * 3)(*hs), C, x.data_ptr(), dout.data_ptr(), nc,
                                         keep.data_ptr(), 2.0, pooled.data_ptr(), arg.data_ptr(),
                                         (ctypes.c_void_p * 3)(*[d.data_ptr() for d in dws]),
                                         (ctypes.c_void_p * 3)(*[d.data_ptr() for d in dbs]), work.data_ptr(),
                                         L.stream_handle()), "textcnn_bwd")
        torch.cuda.synchronize()
        return [d.cpu() for d in dws + dbs]
    slab = run()
    assert all(torch.equal(a, b) for a, b in zip(slab, run()))  # deterministic
    # against a dense float64 restatement
    gw = (dout * keep.float() * 2.0 * (pooled > 0).float()).cpu().double()
    xx = x.cpu().double().view(T, B, F)
    for i, h in enumerate(hs):
        ref = torch.zeros(C, h, F, dtype=torch.float64)
        a = arg.cpu().long()[:, i * C:(i + 1) * C]
        for dt in range(h):
            rowsx = xx[a + dt, torch.arange(B)[:, None]]  # [B, C, F]
            ref[:, dt] += (gw[:, i * C:(i + 1) * C, None] * rowsx).sum(0)
        assert rel_l2(slab[i], ref) < 1e-6


# ------------------------------------------------------------------------------------------------
# BASELINE configs[4]: the seven missing-modality patterns (data/mosi.py:61-69; the YAML's validation / test
# splits select all seven, utt_fusion_base_training.yaml:99,118) through the HIP step and validation_step
# ------------------------------------------------------------------------------------------------
def _corpus_from(A, V, T, y):
    from tspm_amd.mosi_data import MosiCorpus
    return MosiCorpus({"audio": list(A.numpy()), "video": list(V.numpy()), "text": list(T.numpy())}, y.numpy())


def _masked(A, V, T, pattern):
    from tspm_amd.mosi_data import pattern_keep
    k = pattern_keep(pattern)
    return A * k["audio"], V * k["video"], T * k["text"]


@pytest.mark.parametrize("pattern", ["atv", "at", "av", "tv", "a", "t", "v"])
def test_missing_pattern_step_and_eval_vs_oracle(gpu, pattern):
    """One fused train step and one validation_step at the config's batch (128, aligned_50) with every row under
    ``pattern``: the batch is gathered on the device with the pattern's modality mask (tspm_seq_gather, straight
    into the step's inputs) and must equal the host-masked batch bitwise; the step is then held to the §8(c)
    criterion against the forced-decision fp64 oracle fed the same zeroed modalities (a zeroed text makes every
    TextCNN time-max an exact tie; a zeroed audio / video drives the LSTM by its biases alone) and Adam is checked
    exactly; the eval logits and loss of validation_step against the fp64 oracle's validation_step."""
    from tspm_amd.mosi_data import MOSI
    B, S = 128, 50
    A, V, T, y = orc.synthetic_batch(B, S, seed=777)
    Am, Vm, Tm = _masked(A, V, T, pattern)
    corpus = _corpus_from(A, V, T, y)
    ours = _dropin(3).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD)
    ds = MOSI(split="train", corpus=corpus, device=gpu, selected_patterns=[pattern])
    b = next(iter(ds.device_loader(B, shuffle=False, step_for=lambda n, t: ours.fused_step(opt, None, n, t))))
    st = ours.fused_step(opt, None, B, S)
    assert b["audio"] is st.eng.A and b["pattern_name"] == [pattern] * B
    for buf, ref in ((st.eng.A, Am), (st.eng.V, Vm), (st.eng.X, Tm)):
        assert torch.equal(buf.transpose(0, 1).cpu(), ref)
    keeps = orc.keep_masks(B, 61)
    o32, o64 = pair_from(ours, lambda: orc.build_oracle_utt(3))
    before = snapshot(ours)
    st.keep_override = {k: v.to(gpu) for k, v in keeps.items()}
    st.run()
    torch.cuda.synchronize()
    tally = Tally()
    rep = _check_step(ours, st, o32, o64, Am, Vm, Tm, y, keeps, {"loss": st.eng.loss, "logits": st.eng.logits}, tally)
    coef = float(st.eng.clip_coef.item())
    _check_adam(ours, opt, before, 1, coef)
    # validation_step on the pattern-grouped eval collate of the same rows
    ev = MOSI(split="valid", corpus=corpus, device=gpu, selected_patterns=[pattern])
    grouped = ev.collate_fn(ev.__getitems__(list(range(B))))
    assert list(grouped) == [pattern]
    v = ours.validation_step(grouped[pattern], None, gpu, None)
    o = orc.build_oracle_utt(3)
    o.load_state_dict({k: x.cpu() for k, x in ours.state_dict().items()})
    r = orc.validation_step(o.double(), Am.double(), Vm.double(), Tm.double(), y)
    check_out(f"eval logits [{pattern}]", ours._engine(B, S, gpu).logits, None, r["logits"], tally)
    assert abs(v["loss"] - r["loss"].item()) <= 1e-4 * abs(r["loss"].item())
    print(f"[pattern {pattern}] flips {rep} clip coef {coef:.4f}; {tally}")


def test_mixed_pattern_eval_batch_grouped(gpu):
    """A shuffled validation batch mixing all seven patterns: collate groups it by pattern (first-seen order,
    data/mosi.py:236-251); every group's validation_step logits match the fp64 oracle on its masked rows, and
    the device loader's grouped batches (gathered into FusedMosiEvalStep buffers) give the same logits."""
    from tspm_amd.mosi_data import MOSI, PATTERNS
    from tspm_amd.metrics import ClassificationLog
    n = 40
    A, V, T, y = orc.synthetic_batch(n, 30, seed=91)
    corpus = _corpus_from(A, V, T, y)
    ours = _dropin(5).to(gpu)
    o = orc.build_oracle_utt(5).double()
    ev = MOSI(split="valid", corpus=corpus, device=gpu)
    items = torch.randperm(len(ev), generator=torch.Generator().manual_seed(3))[:128].tolist()
    grouped = ev.collate_fn(ev.__getitems__(items))
    seen = [PATTERNS[i // n] for i in items]
    assert list(grouped) == list(dict.fromkeys(seen))
    ref_logits = {}
    for p, sub in grouped.items():
        rows = [i % n for i in items if PATTERNS[i // n] == p]
        Am, Vm, Tm = _masked(A[rows], V[rows], T[rows], p)
        ours.validation_step(sub, None, gpu, None)
        r = orc.validation_step(o, Am.double(), Vm.double(), Tm.double(), y[rows])
        check_out(f"grouped eval [{p}]", ours._engine(len(rows), 30, gpu).logits, None, r["logits"])
        ref_logits[p] = ours._engine(len(rows), 30, gpu).logits.clone()
    # the same batch through the device loader into the harness's eval steps
    from tspm_amd.harness import MosiEpochRunner
    runner = MosiEpochRunner(ours, None, None)
    order_ds = MOSI(split="valid", corpus=corpus, device=gpu)
    got = {}
    sub_items = items
    rows_all, pid = order_ds._resolve(np.asarray(sub_items))
    for p in dict.fromkeys(pid.tolist()):
        sel = pid == p
        st = runner.eval_step_for(int(sel.sum()), 30)
        b = order_ds._collate(rows_all[sel], pid[sel], st)
        runner._run(st, b)
        got[PATTERNS[p]] = st.eng.logits.clone()
    torch.cuda.synchronize()
    for p in ref_logits:
        assert torch.equal(got[p], ref_logits[p]), p
    assert isinstance(runner.log, ClassificationLog)


def test_odd_batch_step_vs_oracle(gpu):
    """Odd batch (the last workgroup of each LSTM kernel carries one ghost row) and a short odd length."""
    lengths = [17 - (i * 5) % 8 for i in range(33)]
    _run_steps(gpu, 33, 17, 1.0, n_steps=2, lengths=lengths)


def test_mosi_epoch_harness_per_pattern_metrics(gpu, tmp_path):
    """harness.fit on UttFusionModel: training batches drawn over all seven patterns, validation / test on the
    pattern-grouped eval loader (every group one FusedMosiEvalStep replay), metrics per pattern from device
    confusion counts with the YAML's MSA + confusion-matrix functions.  Checked against a host replay of the
    validation epoch through validation_step (per-group losses, softmax-argmax predictions): the epoch loss is
    the mean of the group losses and every per-pattern metric equals the metric functions on the raw arrays."""
    from tspm_amd import harness
    from tspm_amd.metrics import evaluate
    from tspm_amd.mosi_data import MOSI, PATTERNS, synthetic_mosi_corpus
    from tspm_amd.msa_metrics import msa_binary_classification
    from sklearn.metrics import confusion_matrix
    ours = _dropin(8).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=LR, weight_decay=WD)
    tr = MOSI(split="train", corpus=synthetic_mosi_corpus(192, seed=1, steps=20), device=gpu, seed=4)
    va = MOSI(split="valid", corpus=synthetic_mosi_corpus(36, seed=2, steps=20), device=gpu)
    loaders = {"train": tr.loader(32, shuffle=True, seed=1), "validation": va.loader(32, shuffle=True, seed=9),
               "test": va.loader(32)}
    hist = harness.fit(ours, opt, None, loaders, epochs=2, early_stopping=False, checkpoint_dir=tmp_path / "ck",
                       metrics_path=tmp_path / "m")
    vm = hist["validation"][-1]
    for p in PATTERNS:
        assert f"MSA_Has0_Accuracy_{p.upper()}" in vm and f"ConfusionMatrix_{p.upper()}" in vm, p
    assert np.isfinite(hist["train"][-1]["loss"]) and (tmp_path / "m" / "epoch_metrics.json").exists()
    # host replay of the test epoch (fit loads best.pth before it): validation_step per pattern group
    losses, preds, labels = [], {p: [] for p in PATTERNS}, {p: [] for p in PATTERNS}

    class Rec:
        def update_group_all(self, group, predictions, targets, m_types):
            for pr, t, m in zip(predictions, targets, m_types):
                preds[m].append(int(pr))
                labels[m].append(int(t))
    for b in va.device_loader(32):
        for p, sub in b.items():
            losses.append(ours.validation_step(sub, None, gpu, Rec())["loss"])
    te = hist["test"]
    assert abs(te["loss"] - float(np.mean(losses))) <= 1e-6 * abs(te["loss"])
    for p in PATTERNS:
        t, pr = np.asarray(labels[p]), np.asarray(preds[p])
        conf = confusion_matrix(t, pr, labels=[0, 1, 2])
        assert np.array_equal(np.asarray(te[f"ConfusionMatrix_{p.upper()}"]), conf), p
        for k, val in msa_binary_classification(t, pr).items():
            got = te[f"MSA_{k}_{p.upper()}"]
            assert (np.isnan(val) and np.isnan(got)) or got == val, (p, k, got, val)
        assert evaluate("metrics.msa_binary_classification", {}, conf) == msa_binary_classification(t, pr)
    print({p: te[f"MSA_Has0_Accuracy_{p.upper()}"] for p in PATTERNS})
