"""Skinny f32 GEMMs of the A2 training step (batch 256, H = 128) under hipBLASLt and
rocBLAS, and the graphed training step under each library (tools/bench_train.py)."""
import json
import sys
import time

import torch


def gemm_us(lib, M, N, K, reps=200):
    torch.backends.cuda.preferred_blas_library(lib)
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    for _ in range(10):
        torch.addmm(b, a, w.t())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            torch.addmm(b, a, w.t())
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    out = {}
    for lib in ("cublaslt", "cublas"):
        out[lib] = {f"{M}x{N}x{K}": gemm_us(lib, M, N, K)
                    for M, N, K in ((256, 128, 64), (256, 128, 128), (256, 32 * 46, 128), (128, 128, 256))}
    print(json.dumps(out), flush=True)
    sys.path.insert(0, "tools")
    import bench_train
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        print(lib, flush=True)
        bench_train.main(steps=10, warmup=2)


if __name__ == "__main__":
    main()
