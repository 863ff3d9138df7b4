"""The data-parallel train step itself, two ranks on the one GPU of the test box.

Two processes share cuda:0 and a gloo process group (gloo all-reduces device tensors through host
copies; the driver's 8-GPU runs use RCCL with the same calls).  Each rank runs FusedTrainStep with
``ddp.PhasedGradAllReduce`` — the overlapped exchange path bench.py uses at N > 1: forward + backward as
one HIP graph whose external events release the phase-1 gradients to the exchange while phase 2
computes — on its half of a 64-sample batch, with FusedAdam(grad_scale = 1/2).  Checked:

* the summed gradient buffer equals g_0 + g_1 bitwise, where g_r is rank r's gradient from a plain
  (no exchange) fused step on the same half batch;
* fp64 Adam applied to the averaged gradient (g_0 + g_1) / 2 reproduces every rank's update;
* both ranks hold bitwise identical parameters and Adam moments after 1 and after 4 steps (eager
  first step, then the captured graphs);
* on each REPLAYED step too, the exchanged gradient equals the sum of both ranks' plain-step gradients
  for the same weights and half batches (the exchange read what this step's backward wrote).

The MOSI and MMIMDb data-parallel steps (bench.py --mosi / --mmimdb at N > 1: fused fwd/bwd graph, one
bucketed all-reduce of the flat gradient, Adam) get the same sum / Adam / identical-state checks.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.dirname(here), here]
        import torch.distributed as dist
        import tspm_amd
        from oracle import avmnist_ref as orc
        from parity import adam_fp64
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        full_a, full_i, full_l, _ = orc.synthetic_batch(64, seed=2024)
        half = slice(32 * rank, 32 * rank + 32)
        keep_full = (torch.rand(64, 128, generator=torch.Generator().manual_seed(77)) > 0.5).to(torch.uint8)

        def build():
            torch.manual_seed(0)
            m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
            return m
        # plain fused step on this rank's half: the local gradient g_r
        m_loc = build()
        o_loc = tspm_amd.FusedAdam(m_loc.parameters(), lr=5e-4, weight_decay=1e-4)
        s_loc = tspm_amd.FusedTrainStep(m_loc, o_loc, None, 32)
        s_loc.keep_override = keep_full[half].to(dev)
        s_loc.step(full_a[half].to(dev), full_i[half].to(dev), full_l[half].to(dev))
        torch.cuda.synchronize()
        g_loc = o_loc.flat_groups()[0].grad.clone()
        # the DP step
        m = build()
        opt = tspm_amd.FusedAdam(m.parameters(), lr=5e-4, weight_decay=1e-4, grad_scale=1.0 / world)
        st = tspm_amd.FusedTrainStep(m, opt, None, 32)
        st.allreduce = st.phased_allreduce()
        fg = opt.flat_groups()[0]
        p0 = fg.param.detach().cpu().double().clone()
        st.keep_override = keep_full[half].to(dev)
        st.step(full_a[half].to(dev), full_i[half].to(dev), full_l[half].to(dev))
        torch.cuda.synchronize()
        gs = [torch.empty_like(g_loc) for _ in range(world)]
        dist.all_gather(gs, g_loc)
        ok_sum = bool(torch.equal(fg.grad, gs[0] + gs[1]))
        exp, _, _ = adam_fp64(p0, (fg.grad.double().cpu()) / world, 1)
        got = fg.param.detach().cpu().double()
        ok_adam = bool(((got - exp).abs() <= 1e-6 * exp.abs() + 2e-9).all())
        state1 = torch.cat([fg.param, fg.exp_avg, fg.exp_avg_sq]).clone()
        fl = o_loc.flat_groups()[0]
        replay_sums = []
        for s in range(3):  # eager done; capture + replays of the step graph
            a, i, lab, _ = orc.synthetic_batch(64, seed=3000 + s)
            st.keep_override = keep_full[half].to(dev)
            p_before = fg.param.detach().clone()
            st.step(a[half].to(dev), i[half].to(dev), lab[half].to(dev))
            torch.cuda.synchronize()
            # the exchanged gradient of this REPLAYED step against the two ranks' local gradients of the same
            # weights and half batches (plain fused step): catches an exchange that ran before the graph's
            # backward had written the gradients it reads (the external events' ordering)
            with torch.no_grad():
                fl.param.copy_(p_before)
            s_loc.keep_override = keep_full[half].to(dev)
            s_loc.step(a[half].to(dev), i[half].to(dev), lab[half].to(dev))
            torch.cuda.synchronize()
            gs = [torch.empty_like(fl.grad) for _ in range(world)]
            dist.all_gather(gs, fl.grad.clone())
            replay_sums.append(bool(torch.equal(fg.grad, gs[0] + gs[1])))
        ok_sum = ok_sum and all(replay_sums)
        state4 = torch.cat([fg.param, fg.exp_avg, fg.exp_avg_sq]).clone()
        same = []
        for t in (state1, state4):
            other = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(other, t)
            same.append(bool(torch.equal(other[0], other[1])))
        had_graph = st.graph is not None
        st.close()  # streams idle, graph and step flags released before the process group goes away
        s_loc.close()
        q.put((rank, (ok_sum, replay_sums), ok_adam, same, had_graph))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None, None))


def test_two_rank_phased_dp_step_on_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, ok_sum, ok_adam, same, captured in res:
        assert isinstance(ok_sum, tuple) and ok_sum[0] is True, (rank, ok_sum)
        assert ok_adam is True, rank
        assert same == [True, True], (rank, same)
        assert captured, rank


def _mosi_worker(rank, world, port, q):
    """MOSI UTT-Fusion data-parallel step (bench.py --mosi at N > 1): fused fwd/bwd graph, bucketed
    all-reduce of the flat gradient, then the global-norm clip on the AVERAGED gradient and Adam
    (torch DDP + clip_grad_norm_ semantics)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.dirname(here), here]
        import torch.distributed as dist
        import tspm_amd
        from oracle import mosi_ref as orc
        from parity import adam_fp64, adam_tolerance
        from test_mosi_cpu import _dropin
        from tspm_amd import ddp
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        A, V, T, y = orc.synthetic_batch(64, 30, seed=99)
        half = slice(32 * rank, 32 * rank + 32)
        keeps = orc.keep_masks(64, seed=5)

        def run_local(clip):
            m = _dropin(0, clip=clip).to(dev)
            o = tspm_amd.FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-3)
            st = m.fused_step(o, None, 32, 30)
            st.keep_override = {k: v[half].to(dev) for k, v in keeps.items()}
            st.step(A[half].to(dev), V[half].to(dev), T[half].to(dev), y[half].to(dev))
            torch.cuda.synchronize()
            return o.flat_groups()[0].grad.clone()
        g_loc = run_local(None)  # this rank's gradient (no clip, no exchange)
        m = _dropin(0, clip=0.05).to(dev)  # a tight clip so the coefficient is active
        opt = tspm_amd.FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-3, grad_scale=1.0 / world)
        st = m.fused_step(opt, None, 32, 30)
        fg = opt.flat_groups()[0]
        st.allreduce = ddp.GradAllReduce([fg.grad])
        p0 = fg.param.detach().cpu().double().clone()
        st.keep_override = {k: v[half].to(dev) for k, v in keeps.items()}
        st.step(A[half].to(dev), V[half].to(dev), T[half].to(dev), y[half].to(dev))
        torch.cuda.synchronize()
        gs = [torch.empty_like(g_loc) for _ in range(world)]
        dist.all_gather(gs, g_loc)
        ok_sum = bool(torch.equal(fg.grad, gs[0] + gs[1]))
        avg = fg.grad.double().cpu() / world
        coef = min(1.0, 0.05 / (float(avg.norm()) + 1e-6))
        ok_coef = abs(float(st.eng.clip_coef.item()) - coef) <= 1e-5 * coef
        g = avg * float(st.eng.clip_coef.item())
        exp, _, v = adam_fp64(p0, g, 1, lr=1e-3, wd=1e-3)
        got = fg.param.detach().cpu().double()
        ok_adam = bool(((got - exp).abs() <= 1e-6 * exp.abs() + adam_tolerance(p0, g, 1, v, 1e-3, 1e-3)).all())
        for s in range(3):
            st.keep_override = {k: v_[half].to(dev) for k, v_ in orc.keep_masks(64, seed=50 + s).items()}
            st.step(A[half].to(dev), V[half].to(dev), T[half].to(dev), y[half].to(dev))
        torch.cuda.synchronize()
        state = torch.cat([fg.param, fg.exp_avg, fg.exp_avg_sq]).clone()
        other = [torch.empty_like(state) for _ in range(world)]
        dist.all_gather(other, state)
        q.put((rank, ok_sum, ok_coef and ok_adam, bool(torch.equal(other[0], other[1])), st.graph is not None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None, None))


def test_two_rank_mosi_dp_step_on_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mosi_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, ok_sum, ok_step, same, captured in res:
        assert ok_sum is True, (rank, ok_sum)
        assert ok_step is True, rank
        assert same is True, rank
        assert captured, rank


def _mmimdb_worker(rank, world, port, q):
    """MMIMDb GMU late-fusion data-parallel step (bench.py --mmimdb at N > 1): fused fwd/bwd graph, one
    all-reduce of the flat gradient buffer (ddp.GradAllReduce), Adam with grad_scale = 1/world.  BatchNorm1d
    statistics stay per rank (torch DDP without SyncBatchNorm, as the reference trains)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.dirname(here), here]
        import torch.distributed as dist
        import tspm_amd
        from oracle import mmimdb_ref as orc
        from parity import adam_fp64, adam_tolerance
        from test_mmimdb_cpu import dropin
        from tspm_amd import ddp
        from tspm_amd import mmimdb as M
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        lr, wd = 1e-5, 1e-3
        I, T, y = orc.synthetic_batch(64, seed=31)
        half = slice(32 * rank, 32 * rank + 32)

        def keep(seed):
            g = torch.Generator().manual_seed(seed)
            return (torch.rand(2, 64, 512, generator=g) >= 0.5).to(torch.uint8)[:, half].contiguous().to(dev)

        m_loc = dropin(3).to(dev)
        o_loc = tspm_amd.FusedAdam(m_loc.parameters(), lr=lr, weight_decay=wd)
        s_loc = M.FusedMMIMDbStep(m_loc, o_loc, None, 32)
        s_loc.keep_override = keep(9)
        s_loc.step(I[half].to(dev), T[half].to(dev), y[half].to(dev))
        torch.cuda.synchronize()
        g_loc = o_loc.flat_groups()[0].grad.clone()
        m = dropin(3).to(dev)
        opt = tspm_amd.FusedAdam(m.parameters(), lr=lr, weight_decay=wd, grad_scale=1.0 / world)
        fg = opt.flat_groups()[0]
        st = M.FusedMMIMDbStep(m, opt, None, 32, allreduce=ddp.GradAllReduce([g.grad for g in opt.flat_groups()]))
        p0 = fg.param.detach().cpu().double().clone()
        st.keep_override = keep(9)
        st.step(I[half].to(dev), T[half].to(dev), y[half].to(dev))
        torch.cuda.synchronize()
        gs = [torch.empty_like(g_loc) for _ in range(world)]
        dist.all_gather(gs, g_loc)
        ok_sum = bool(torch.equal(fg.grad, gs[0] + gs[1]))
        g = fg.grad.double().cpu() / world
        exp, _, v = adam_fp64(p0, g, 1, lr=lr, wd=wd)
        got = fg.param.detach().cpu().double()
        ok_adam = bool(((got - exp).abs() <= 1e-6 * exp.abs() + adam_tolerance(p0, g, 1, v, lr, wd)).all())
        for s in range(3):  # graph capture + replays
            a2, t2, y2 = orc.synthetic_batch(64, seed=400 + s)
            st.keep_override = keep(60 + s)
            st.step(a2[half].to(dev), t2[half].to(dev), y2[half].to(dev))
        torch.cuda.synchronize()
        state = torch.cat([torch.cat([f.param, f.exp_avg, f.exp_avg_sq]) for f in opt.flat_groups()]).clone()
        other = [torch.empty_like(state) for _ in range(world)]
        dist.all_gather(other, state)
        q.put((rank, ok_sum, ok_adam, bool(torch.equal(other[0], other[1])), st.graph is not None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None, None))


def test_two_rank_mmimdb_dp_step_on_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mmimdb_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, ok_sum, ok_adam, same, captured in res:
        assert ok_sum is True, (rank, ok_sum)
        assert ok_adam is True, rank
        assert same is True, rank
        assert captured, rank
