"""Does a CU-masked stream (hipExtStreamCreateWithCUMask) keep its CU mask when its work is captured into a HIP graph
and replayed?  Times one large LDS conv launch eagerly and in a replayed graph, on an unmasked stream and on a
stream restricted to a quarter of the CUs: if the masked graph replay is as slow as the masked eager launch, the
mask survives capture.
    python scripts/cumask_probe.py"""
import ctypes
import os
import sys

import torch

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__))]
from tune_convs import Bufs, launcher  # noqa: E402
from conv_bench import step_ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so")
    ops = step_ops(128, dev, ("audio",))
    key = [k for k in ops if k[0] == "fwd" and k[2:5] == (8, 24, 64)][0]
    s, xs, stem, count, algo = ops[key]
    b = Bufs(s, stem, dev)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    res = {}
    for label, frac in (("all", 1.0), ("quarter", 0.25)):
        n = max(1, int(ncu * frac))
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for i in range(n):
            mask[i // 32] |= 1 << (i % 32)
        h = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask) == 0
        st = torch.cuda.ExternalStream(h.value, device=dev)
        with torch.cuda.stream(st):
            f, _ = launcher("fwd", s, xs, b, algo)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(50):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            eager = e0.elapsed_time(e1) * 1000 / 50
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
                f2, _ = launcher("fwd", s, xs, b, algo)
                for _ in range(50):
                    f2()
            g.replay()
            torch.cuda.synchronize()
            e0.record(st)
            g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            graph = e0.elapsed_time(e1) * 1000 / 50
        res[label] = {"cus": n, "eager_us": round(eager, 2), "graph_us": round(graph, 2)}
        print(label, res[label], flush=True)
    print(res)


if __name__ == "__main__":
    main()
