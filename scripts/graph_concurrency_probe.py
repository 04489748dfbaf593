#!/usr/bin/env python3
"""Probe: do independent branches of ONE captured hipGraph run concurrently on MI355X?

Captures (a) one stream with 2*N small latency-bound kernels and (b) the same kernels as two
N-long chains forked onto two streams inside the capture, then times graph replays.
If (b) is ~2x faster than (a), forked rollout chains inside the engine's graph overlap.
Prints one JSON line.
"""
from __future__ import annotations

import json

import torch


def main(n: int = 200, reps: int = 20):
    dev = "cuda:0"
    xa = torch.randn(64, 64, device=dev)
    xb = torch.randn(64, 64, device=dev)
    w = torch.randn(64, 64, device=dev) * 0.01

    def chain(x, k):
        for _ in range(k):
            x = torch.tanh(x @ w)
        return x

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain(xa, 3)
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        chain(xa, 2 * n)
    g2 = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(g2):
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            chain(xb, n)
        chain(xa, n)
        main_s.wait_stream(side)
    torch.cuda.synchronize()

    def t(g):
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    def eager2():
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            chain(xb, n)
        chain(xa, n)
        main_s.wait_stream(side)
    eager2()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        eager2()
    b.record()
    torch.cuda.synchronize()
    t_e2 = a.elapsed_time(b) / 5
    t1, t2 = t(g1), t(g2)
    print(json.dumps({"kernels": 4 * n, "graph_serial_ms": round(t1, 3), "graph_forked_ms": round(t2, 3),
                      "eager_two_stream_ms": round(t_e2, 3), "forked_speedup": round(t1 / t2, 2)}), flush=True)


def main_big(n: int = 10, reps: int = 5):
    """Same fork/join test with long, narrow kernels (few workgroups each, ~100 us)."""
    dev = "cuda:0"
    a1 = torch.randn(64, 65536, device=dev)
    b1 = torch.randn(65536, 64, device=dev)
    a2 = torch.randn(64, 65536, device=dev)
    b2 = torch.randn(65536, 64, device=dev)

    def chain(a, b, k):
        out = None
        for _ in range(k):
            out = a @ b
        return out

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain(a1, b1, 2)
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        chain(a1, b1, n)
        chain(a2, b2, n)
    side = torch.cuda.Stream()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        ms = torch.cuda.current_stream()
        side.wait_stream(ms)
        with torch.cuda.stream(side):
            chain(a2, b2, n)
        chain(a1, b1, n)
        ms.wait_stream(side)
    torch.cuda.synchronize()

    def t(fn):
        fn()
        torch.cuda.synchronize()
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x.record()
        for _ in range(reps):
            fn()
        y.record()
        torch.cuda.synchronize()
        return x.elapsed_time(y) / reps

    def eager2():
        ms = torch.cuda.current_stream()
        side.wait_stream(ms)
        with torch.cuda.stream(side):
            chain(a2, b2, n)
        chain(a1, b1, n)
        ms.wait_stream(side)
    t1, t2, t3 = t(g1.replay), t(g2.replay), t(eager2)
    print(json.dumps({"narrow_kernels": 2 * n, "graph_serial_ms": round(t1, 3), "graph_forked_ms": round(t2, 3),
                      "eager_two_stream_ms": round(t3, 3), "forked_speedup": round(t1 / t2, 2),
                      "eager_speedup": round(t1 / t3, 2)}), flush=True)


if __name__ == "__main__":
    main()
    main_big()
