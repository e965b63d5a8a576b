"""A/B of the energy kernel builds: the default library ("v2") vs another build ("v1": argv[1],
default the FS_ENERGY_V1 variant, the pair loop with inline LJ terms), bit-for-bit on sparse
(bench-like), clustered and overlapping configurations, and per-launch time at the bench shape
(65536 chains, N=64, float32 and float64)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from flowstate import _lib  # noqa: E402
from flowstate.MCMC.energy_calculator import make_phys  # noqa: E402
from oracle import physics as OP  # noqa: E402

libs = {"v2": _lib.load(), "v1": _lib.load(sys.argv[1] if len(sys.argv) > 1 else
                                         os.path.join(REPO, "flow-state_amd/flowstate/lib/variants/ev1/libflowstate.so"))}
N, C = 64, 65536
L = float(np.sqrt(N / 0.03))
phys = make_phys(L, L)
rng = np.random.default_rng(0)
base = OP.fcc_lattice(N)
sparse = np.mod(base[None] + rng.normal(0, 0.35, (C, N, 2)), L)
g = np.stack(np.meshgrid(np.arange(8), np.arange(8), indexing="ij"), -1).reshape(-1, 2).astype(float)
dense = np.mod(g[None] * rng.uniform(0.7, 0.9, (C, 1, 1)) + rng.uniform(0, L, (C, 1, 2)), L)
unif = rng.random((C, N, 2)) * L
out = {}
for name, pos in (("sparse", sparse), ("dense", dense), ("uniform", unif)):
    for dt in (np.float32, np.float64):
        x = torch.from_numpy(pos.astype(dt)).cuda()
        res = {}
        for k, L_ in libs.items():
            E = torch.empty(C, dtype=torch.float64, device="cuda")
            W = torch.empty_like(E)
            ov = torch.empty(C, dtype=torch.uint8, device="cuda")
            nbr = torch.empty((C, N), dtype=torch.int64, device="cuda")
            f = lambda: _lib.check(L_.fs_energy_lj_dw(phys, _lib.ptr(x), int(dt == np.float32), C, N, _lib.ptr(E),
                                                       _lib.ptr(W), _lib.ptr(ov), _lib.ptr(nbr), _lib.stream_ptr()))
            f()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[k] = (E.cpu().numpy(), W.cpu().numpy(), ov.cpu().numpy(), nbr.cpu().numpy(), min(ts))
        a, b = res["v2"], res["v1"]
        same = all(np.array_equal(a[i], b[i], equal_nan=True) for i in range(4))
        out[f"{name}_{np.dtype(dt).name}"] = {"bit_identical": same, "ms_v2": a[4], "ms_v1": b[4],
                                             "finite": int(np.isfinite(a[0]).sum())}
print(json.dumps(out, indent=1))
