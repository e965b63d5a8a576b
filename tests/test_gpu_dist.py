"""Multi-rank paths on the GPU box (BASELINE config 4's contract, SURVEY §8(e);
main_algorithm_1.py:138-186 independent chains, utils.py:488-495 histogram).

* RCCL: a 1-rank "nccl" process group pushes flowstate.parallel.final_reduction's
  all-reduce and all-gather through RCCL; the results equal the no-dist reduction.
* Sharding: 2 ranks (gloo, both on the one GPU: RCCL needs a GPU per rank) each run
  BatchedMonteCarlo over their half of the chains (chain_offset, seeds 42 + global
  index); every chain's state, energies, NLL, counters and PCG64 state equal those of a
  1-rank run over all chains, and the reduced histogram / gathered table are the 1-rank
  ones.
Each rank is a fresh child process (spawned, not forked), joined with a time limit."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETUP = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [{repo!r}, os.path.join({repo!r}, "flow-state_amd")]
    import numpy as np, torch
    from flowstate import parallel
    from flowstate.MCMC import BatchedMonteCarlo, Physics
    from flowstate.models import flow_from_state_dict, half_box
    from oracle import flow as OF
    from oracle import physics as OP

    N, L_, H, nb, K = 16, 2, 64, 1, 8

    def engine(C, c0, dev):
        dims = OF.FlowDims(N=N, L=L_, H=H, nb=nb, K=K, B=half_box(N))
        sd = OF.random_state_dict(dims, seed=3)
        model = flow_from_state_dict(sd, N, L=L_, H=H, nb=nb, K=K, bound=dims.B, device=dev)
        box = float(np.sqrt(N / 0.03))
        init = np.stack([np.mod(OP.fcc_lattice(N) + np.random.default_rng(500 + c0 + c).normal(0, 0.05, (N, 2)), box)
                         for c in range(C)])
        c0s, seeds = parallel.shard(C, c0 // C if C else 0)
        return BatchedMonteCarlo(model, init, Physics(box), seeds, device=dev, chain_offset=c0)

    def run(bmc):
        bmc.local_moves(40, adjust_every=20)
        bmc.step()
        bmc.step(3)
        bmc.local_moves(10)
        bmc.step()
        torch.cuda.synchronize()
        bmc.check_errors()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_children(script, world, tmp_path, timeout=150):
    path = tmp_path / "rank.py"
    path.write_text(script)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(path), str(tmp_path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return outs


def test_rccl_one_rank_final_reduction(tmp_path):
    script = SETUP.format(repo=REPO) + textwrap.dedent("""
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        bmc = engine(256, 0, dev)
        run(bmc)
        h0, w0, t0 = (t.clone() for t in parallel.final_reduction(bmc))
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_backend() == "nccl" and parallel.world_size() == 1
        # world size 1 skips the collectives in the helpers: push them through RCCL here
        h, w = h0.clone(), w0.clone()
        dist.all_reduce(h)
        dist.all_reduce(w)
        outs = [torch.empty_like(t0)]
        dist.all_gather(outs, t0.contiguous())
        torch.cuda.synchronize()
        assert torch.equal(h, h0) and torch.equal(w, w0) and torch.equal(outs[0], t0)
        x = torch.arange(1000, dtype=torch.float64, device=dev)
        dist.all_reduce(x)
        assert torch.equal(x, torch.arange(1000, dtype=torch.float64, device=dev))
        h1, w1, t1 = parallel.final_reduction(bmc)
        assert torch.equal(h1, h0) and torch.equal(w1, w0) and torch.equal(t1, t0)
        assert int(h0.sum()) == 256 * N
        dist.destroy_process_group()
        print("rccl ok")
    """)
    outs = _run_children(script, 1, tmp_path)
    assert "rccl ok" in outs[0]


def test_two_rank_shards_match_one_rank(tmp_path):
    C = 128
    script = SETUP.format(repo=REPO) + textwrap.dedent(f"""
        import torch.distributed as dist
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo")
        C = {C}
        bmc = engine(C, rank * C, dev)
        run(bmc)
        hist, wells, table = parallel.final_reduction(bmc)
        per = torch.cat([bmc.state.reshape(C, -1), bmc.E_old[:, None], bmc.W_old[:, None], bmc.nll_old[:, None],
                         bmc.pcg.view(torch.float64), bmc.attempts[:, None].double(), bmc.accepted[:, None].double(),
                         bmc.max_disp[:, None]], 1).cpu()
        outs = [torch.empty_like(per) for _ in range(world)]
        dist.all_gather(outs, per)
        if rank == 0:
            np.savez(os.path.join(sys.argv[1], "dist.npz"), per=torch.cat(outs).numpy(), hist=hist.cpu().numpy(),
                     wells=wells.cpu().numpy(), table=table.cpu().numpy())
        dist.barrier()
        dist.destroy_process_group()
    """)
    _run_children(script, 2, tmp_path)
    got = np.load(tmp_path / "dist.npz")
    # the same chains in one process (this test process)
    ns = {}
    exec(SETUP.format(repo=REPO), ns)
    dev = torch.device("cuda", 0)
    bmc = ns["engine"](2 * C, 0, dev)
    ns["run"](bmc)
    from flowstate import parallel

    hist, wells, table = parallel.final_reduction(bmc)
    per = torch.cat([bmc.state.reshape(2 * C, -1), bmc.E_old[:, None], bmc.W_old[:, None], bmc.nll_old[:, None],
                     bmc.pcg.view(torch.float64), bmc.attempts[:, None].double(), bmc.accepted[:, None].double(),
                     bmc.max_disp[:, None]], 1).cpu().numpy()
    assert bmc.accepted.sum().item() > 0
    np.testing.assert_array_equal(got["per"].view(np.uint64), per.view(np.uint64))  # bit-exact per chain
    np.testing.assert_array_equal(got["hist"], hist.cpu().numpy())
    np.testing.assert_array_equal(got["wells"], wells.cpu().numpy())
    np.testing.assert_array_equal(got["table"], table.cpu().numpy())
