"""Per-launch time of the training step's forward products in a dependent chain (each
product reads the previous one's output and its tile statistics), as the A2 forward
runs them: fs_linear_f32_ex (one problem), fs_linear_f32_ex2 (the two passes' problems in
one launch), BatchNorm-in-load or plain, batch 256, H = 128; 92 launches per graph (the
46 ResidualBlock products of a pass), replayed.  Compare tools/probes/block_fuse (the same
product as a minimal kernel)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
from flowstate import _lib  # noqa: E402

M, K, N, CH = 256, 128, 128, 92


def graph_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps / CH * 1e6)
    return best


def main():
    L, p = _lib.load(), _lib.ptr
    torch.manual_seed(0)
    w = (torch.randn(N, K, device="cuda") * 0.1)
    b = torch.randn(N, device="cuda") * 0.1
    gam, bet = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")
    out = {}
    for two in (False, True):
        P = 2 if two else 1
        xs = [[torch.randn(M, K, device="cuda") for _ in range(CH + 1)] for _ in range(P)]
        sts = [[torch.zeros((M // 32, K, 2), device="cuda") for _ in range(CH + 1)] for _ in range(P)]
        aos = [[torch.empty(M, K, device="cuda") for _ in range(CH)] for _ in range(P)]
        for bn in (False, True):
            def run():
                for i in range(CH):
                    gs, bs = [], []
                    for q in range(P):
                        gs.append(_lib.GemmF32(M, N, K, p(xs[q][i]), K, 1, p(w), 1, K, p(b), None, N,
                                               p(xs[q][i + 1]), N, None))
                        bs.append(_lib.BnIn(p(sts[q][i]), M // 32, M, p(gam), p(bet), 1e-5, 0.1, None, None, None,
                                            None, None, p(aos[q][i]), None) if bn else None)
                    if two:
                        _lib.check(L.fs_linear_f32_ex2(gs[0], bs[0], p(sts[0][i + 1]), gs[1], bs[1], p(sts[1][i + 1]),
                                                       _lib.stream_ptr()))
                    else:
                        _lib.check(L.fs_linear_f32_ex(gs[0], bs[0], p(sts[0][i + 1]), _lib.stream_ptr()))
            out[f"{'two' if two else 'one'}_problem{'s' if two else ''}_{'bn_in_load' if bn else 'plain'}_us"] = \
                round(graph_us(run), 3)
    print(json.dumps({"tool": "train_lin_chain", "shape": f"{M}x{N}x{K}", "launches_per_graph": CH, **out}),
          flush=True)


if __name__ == "__main__":
    main()
