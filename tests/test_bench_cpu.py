"""bench.py's launch contract on the CPU: `--gpus N` never prints a single-rank line.
With WORLD_SIZE set by a launcher it must equal --gpus; without one, bench.py starts
the N rank processes itself (torch.distributed.run as a child) and exits with their
code.  Here there is no GPU, so the ranks fail and the exit code is non-zero, with no
JSON line on stdout."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra, drop=()):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240)


def test_algorithm1_regime_cpu_sample_is_bounded():
    """The regime leg's CPU sample (the reference's per-call numpy local moves,
    oracle.physics.NumpyLocalChain, + torch-CPU log_prob) runs at least one attempt, stops
    near its budget and reports itself as a port of the reference's loop."""
    import time
    import bench
    t0 = time.perf_counter()
    r = bench.algorithm1_regime_cpu(N=3, interval=50, budget_s=0.3)
    # (the A1 flow's construction and 64 untimed CPU proposals dominate: ~2 s alone, more
    # when the suite runs in parallel workers)
    assert time.perf_counter() - t0 < 120
    assert r["value"] > 0 and r["kind"] == "port" and r["unit"] == "big-move attempts/s"
    assert r["cores"] >= 1 and "attempts of one run" in r["sample"] and "numpy" in r["sample"]


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr
    assert '"metric"' not in r.stdout


def test_gpus_without_launcher_spawns_ranks():
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {},
               drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"))
    assert r.returncode != 0
    assert '"metric"' not in r.stdout
    # the ranks were started by torch.distributed.run (its own banner / error report)
    assert "torch.distributed" in r.stderr or "ChildFailedError" in r.stderr or "2 ranks need 2 GPUs" in r.stderr, \
        r.stderr[-2000:]
