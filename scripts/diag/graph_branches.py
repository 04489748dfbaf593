"""Do the parallel branches of a captured hipGraph run concurrently?  Two chains of N small latency-bound kernels
(a 1-workgroup elementwise op each), captured (a) on one stream back to back, (b) forked onto two streams and joined,
and (c) the same two-stream program eagerly.  Prints ms per replay."""
import torch, time, json

import sys
N = 100
dev = "cuda"
KIND = sys.argv[1] if len(sys.argv) > 1 else "tiny"
if KIND == "tiny":
    a = torch.ones(4096, device=dev)
    b = torch.ones(4096, device=dev)
else:      # a few workgroups each, ~10 us: a latency-bound kernel like the rollout's at small populations
    a = torch.randn(2, 256, 4096, device=dev) * 0.01
    b = torch.randn(2, 256, 4096, device=dev) * 0.01
    w = torch.randn(2, 4096, 256, device=dev) * 0.01
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()


def chain(x, n):
    for _ in range(n):
        if KIND == "tiny":
            x.mul_(1.0000001).add_(1e-9)
        else:
            y = torch.bmm(x[:, :, :256], w[:, :256, :256])
            x[:, :, :256].copy_(y)


def serial():
    chain(a, N)
    chain(b, N)


def forked():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        chain(a, N)
    with torch.cuda.stream(s2):
        chain(b, N)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


out = {}
for name, fn in (("serial", serial), ("forked", forked)):
    out[f"eager_{name}"] = timeit(fn)
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cs, capture_error_mode="thread_local"):
            fn()
    torch.cuda.synchronize()
    out[f"graph_{name}"] = timeit(g.replay)
print(KIND, json.dumps({k: round(v, 3) for k, v in out.items()}))
