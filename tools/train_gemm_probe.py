"""Per-shape time of fs_linear_f32 (csrc/train_kernels.hip) on the A2 training shapes
(batch 256, H = 128, final layer 64 x 46 outputs), forward / input-gradient /
weight-gradient layouts, each replayed 200x in a HIP graph; hipBLASLt alongside."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
from flowstate import _lib  # noqa: E402


def timed(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    L = _lib.load()
    tiny = torch.zeros(64, device="cuda")
    out = {"graph_node_floor_us (fill of 64 floats)": round(timed(lambda: tiny.zero_()), 2)}
    for M, N, K in ((256, 128, 128), (256, 2944, 128)):
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        dy = torch.randn(M, N, device="cuda")
        y = torch.empty(M, N, device="cuda")
        gx = torch.empty(M, K, device="cuda")
        gw = torch.empty(N, K, device="cuda")
        gb = torch.empty(N, device="cuda")
        s = lambda: _lib.stream_ptr()  # noqa: E731
        r = {
            "fwd": timed(lambda: L.fs_linear_f32(M, N, K, _lib.ptr(x), K, 1, _lib.ptr(w), 1, K, _lib.ptr(b), None, N,
                                                 _lib.ptr(y), N, None, s())),
            "dx": timed(lambda: L.fs_linear_f32(M, K, N, _lib.ptr(dy), N, 1, _lib.ptr(w), K, 1, None, None, 0,
                                                _lib.ptr(gx), K, None, s())),
            "dw": timed(lambda: L.fs_linear_f32(N, K, M, _lib.ptr(dy), 1, N, _lib.ptr(x), K, 1, None, None, 0,
                                                _lib.ptr(gw), K, _lib.ptr(gb), s())),
            "hipblaslt_fwd": timed(lambda: torch.addmm(b, x, w.t())),
            "hipblaslt_dx": timed(lambda: torch.mm(dy, w)),
            "hipblaslt_dw": timed(lambda: torch.mm(dy.t(), x)),
        }
        out[f"{M}x{N}x{K}"] = {k: round(v, 2) for k, v in r.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
