import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "flow-state_amd")
import numpy as np, torch
from flowstate.MCMC import BatchedMonteCarlo, Physics
from flowstate.models import flow_from_state_dict
from oracle import flow as OF
from oracle import physics as OP
f = np.load("tests/golden/local_trace.npz")
for N in (3,):
    moves, C = int(f[f"N{N}_moves"]), int(f[f"N{N}_chains"])
    L = float(np.sqrt(N / 0.03))
    keys = [f"N{N}_c{c}" for c in range(C)]
    init = np.stack([f[k + "_init"] for k in keys])
    seeds = np.array([int(f[k + "_seed"]) for k in keys], np.uint64)
    b = BatchedMonteCarlo(None, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    print("N", N, "E0", b.E_old.cpu().numpy(), "W0", b.W_old.cpu().numpy())
    xy, ew, log = b.local_moves(moves, adjust_every=50, sample_every=1, log_accepts=True)
    dims = OF.FlowDims(N=N, B=OF.half_box(N), L=1, H=32, nb=1, K=5)
    sd = OF.random_state_dict(dims, seed=77)
    b.set_model(flow_from_state_dict(sd, N, bound=dims.B, L=1, H=32, nb=1, K=5))
    cfgs = np.stack([f[k + "_bigcfg"] for k in keys])
    acc = b.nf_big_move(torch.from_numpy(cfgs))
    print("big acc", acc.cpu().numpy(), "E after big", b.E_old.cpu().numpy())
    for c in range(C):
        print("  oracle E(cfg)", OP.total_energy(cfgs[c], OP.make_phys(N))[:2])
    xy, ew, log = b.local_moves(moves, adjust_every=50, sample_every=1, log_accepts=True)
    ew = ew.cpu().numpy(); log = log.cpu().numpy()
    for c, k in enumerate(keys):
        E = ew[c, :, 0]; R = f[k + "_E"][moves:]
        W = ew[c, :, 1]; RW = f[k + "_W"][moves:]
        print("ref E at end of phase0", f[k + "_E"][moves-1], "first of phase1", R[0], E[0])
        d = np.abs(E - R); dw = np.abs(W - RW)
        bad = np.nonzero(d > 1e-12 * np.maximum(1, np.abs(R)))[0]
        badw = np.nonzero(dw > 1e-12 * np.maximum(1, np.abs(RW)))[0]
        print(k, "first E mismatch", bad[:5], "first W mismatch", badw[:5])
        if len(bad):
            t = bad[0]
            print("  t", t, "acc", log[c, max(0,t-2):t+2], "E gpu", E[max(0,t-2):t+2], "ref", R[max(0,t-2):t+2])
            dE_g = np.diff(E[max(0,t-3):t+1]); dE_r = np.diff(R[max(0,t-3):t+1])
            print("  dE gpu", dE_g, "ref", dE_r)

# dump phase-1 samples of the last case for offline analysis
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dbg_local.npz", xy=xy.cpu().numpy(), ew=ew, log=log)
