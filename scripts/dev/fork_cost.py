"""Graph-replay cost of a fork / join (side stream by events) on this ROCm, against the same
kernels on one stream."""
import time
import torch

dev = "cuda"
x = torch.zeros(1 << 20, device=dev)
y = torch.zeros(1 << 20, device=dev)
side = torch.cuda.Stream()


def body(nfork, forked):
    main = torch.cuda.current_stream()
    for i in range(nfork):
        x.add_(1.0)
        if forked:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y.add_(1.0)
            ev = torch.cuda.Event()
            ev.record(side)
            x.add_(1.0)
            main.wait_event(ev)
        else:
            y.add_(1.0)
            x.add_(1.0)


def timed(forked, nfork=50, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(nfork, forked)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(nfork, forked)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps / nfork * 1e6


for _ in range(2):
    a, b = timed(False), timed(True)
    print(f"3 kernels per unit: one stream {a:.2f} us / unit, forked {b:.2f} us / unit")
