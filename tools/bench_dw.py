"""Micro-benchmark: weight-gradient GEMM dW = dY^T X of the PPO MLPs, plain vs split-K (bmm + sum)."""
import torch

torch.manual_seed(0)
dev = "cuda:0"
shapes = [(5120, 101, 512), (5120, 512, 256), (5120, 256, 128), (5120, 128, 28),
          (5376, 212, 512), (5376, 512, 256), (5376, 256, 128), (5376, 128, 1)]


def t(f, n=50):
    """GPU time per call: n calls captured in one HIP graph (no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for N, i, o in shapes:
    X, dY = torch.randn(N, i, device=dev), torch.randn(N, o, device=dev)
    base = t(lambda: dY.t().mm(X))
    res = [f"N={N} in={i} out={o}: plain {base:6.1f} us"]
    for S in (2, 4, 8, 16):
        if N % S:
            continue
        f = lambda: torch.bmm(dY.view(S, N // S, o).transpose(1, 2), X.view(S, N // S, i)).sum(0)
        ref = dY.t().mm(X)
        err = float((f() - ref).abs().max() / ref.abs().max())
        res.append(f"S={S} {t(f):6.1f} us (rel {err:.1e})")
    print("  ".join(res), flush=True)
