"""Time the encoder chains of the bench step separately and together (HIP graphs, batch 128):
audio alone, image alone, both on two streams, both on one stream, and the full fused step.

    python scripts/encoder_timing.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tspm_amd  # noqa: E402


def timeit(fn, iters=50):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B = 128
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    step = tspm_amd.FusedTrainStep(model, opt, None, B, use_graph=True)
    g = torch.Generator().manual_seed(1234)  # AVMNIST-shaped random batch (values do not affect timing)
    a = (10.0 ** (torch.randn(B, 32, 94, generator=g) * 2)).to(dev)
    im = torch.rand(B, 1, 28, 28, generator=g).to(dev)
    lab = torch.randint(0, 10, (B,), generator=g).to(dev)
    step.load_batch(a, im, lab)
    step.run()
    torch.cuda.synchronize()
    ea, ei = step.eng_a, step.eng_i
    F = step.F
    side = torch.cuda.Stream()

    def audio():
        ea.forward(step.A, step.fused, F, train=True, bump_batches_tracked=False)
        ea.backward(step.dfused, F)

    def image():
        ei.forward(step.I, step.fused[:, model.embd_size_A:], F, train=True, bump_batches_tracked=False)
        ei.backward(step.dfused[:, model.embd_size_A:], F)

    def both_serial():
        audio()
        image()

    def both_par():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            image()
        audio()
        main.wait_stream(side)

    res = {}
    for name, fn in [("audio", audio), ("image", image), ("both_serial", both_serial), ("both_2streams", both_par)]:
        res[name] = timeit(fn)
        print(f"{name:14s} {res[name]:8.1f} us", flush=True)
    # the same without a graph (eager launches from this thread)
    for name, fn in [("eager_audio", audio), ("eager_image", image), ("eager_2streams", both_par)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        print(f"{name:14s} {(time.perf_counter() - t0) / 20 * 1e6:8.1f} us", flush=True)
    step.run(); step.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        step.run()
    torch.cuda.synchronize()
    print(f"{'full_step':14s} {(time.perf_counter() - t0) / 50 * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
