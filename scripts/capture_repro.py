"""Minimal HIP-graph capture patterns with forked streams (diagnostic; one pattern per process).

    python scripts/capture_repro.py VARIANT
"""
import sys

import torch

v = sys.argv[1]
dev = torch.device("cuda", 0)
x = torch.zeros(1 << 16, device=dev)
side, aux, aux2 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()


def fork_join(parent, child, n=1):
    child.wait_stream(parent)
    with torch.cuda.stream(child):
        for _ in range(n):
            x.add_(1)
    parent.wait_stream(child)


def body():
    main = torch.cuda.current_stream()
    if v == "simple":
        fork_join(main, aux)
        fork_join(main, aux)
    elif v == "nested":
        side.wait_stream(main)
        with torch.cuda.stream(side):
            fork_join(side, aux)
            x.add_(1)
        main.wait_stream(side)
    elif v == "nested_join_origin":  # grandchild joins the origin stream, never its parent
        side.wait_stream(main)
        aux.wait_stream(side)
        with torch.cuda.stream(aux):
            x.add_(1)
        with torch.cuda.stream(side):
            x.add_(1)
        main.wait_stream(aux)
        main.wait_stream(side)
    elif v == "nested_double_join":  # grandchild joins its parent and, right after, the origin
        side.wait_stream(main)
        aux.wait_stream(side)
        with torch.cuda.stream(aux):
            x.add_(1)
        side.wait_stream(aux)
        main.wait_stream(aux)
        with torch.cuda.stream(side):
            x.add_(1)
        main.wait_stream(side)
    elif v == "nested_event_origin":  # parent->grandchild dependency through an event, joins via origin
        side.wait_stream(main)
        with torch.cuda.stream(side):
            x.add_(1)
        ev = torch.cuda.Event()
        ev.record(side)
        aux.wait_event(ev)
        with torch.cuda.stream(aux):
            x.add_(1)
        ev2 = torch.cuda.Event()
        ev2.record(aux)
        side.wait_event(ev2)
        with torch.cuda.stream(side):
            x.add_(1)
        main.wait_stream(side)
        main.wait_stream(aux)
    elif v == "nested2":  # nested twice (forward + backward)
        for _ in range(2):
            side.wait_stream(main)
            with torch.cuda.stream(side):
                fork_join(side, aux)
                x.add_(1)
            main.wait_stream(side)
    elif v == "multi_wait":  # child waits on parent several times, joins once
        for _ in range(3):
            aux.wait_stream(main)
            with torch.cuda.stream(aux):
                x.add_(1)
            x.add_(1)
        main.wait_stream(aux)
    elif v == "nested_multi":  # backward pattern inside the side branch
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for _ in range(3):
                aux.wait_stream(side)
                with torch.cuda.stream(aux):
                    x.add_(1)
                x.add_(1)
            side.wait_stream(aux)
        main.wait_stream(side)
    elif v == "two_aux":
        side.wait_stream(main)
        with torch.cuda.stream(side):
            fork_join(side, aux)
        fork_join(main, aux2)
        main.wait_stream(side)
    elif v == "reuse_after_join":  # aux forked, joined, then forked again from a different parent
        fork_join(main, aux)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            fork_join(side, aux)
        main.wait_stream(side)
    torch.cuda.current_stream().wait_stream(torch.cuda.current_stream())


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
g.replay()
torch.cuda.synchronize()
print(v, "ok", float(x[0]))
