"""Do the parallel branches of a captured HIP graph run concurrently on this stack?
Captures K spin kernels (torch.cuda._sleep) on one stream, and K + K split over a
forked second stream, and times the replays.  One JSON line per case."""
import json
import time

import torch


def capture(K, cycles, fork):
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        if fork:
            s.wait_stream(main)
            for _ in range(K // 2):
                torch.cuda._sleep(cycles)
            with torch.cuda.stream(s):
                for _ in range(K - K // 2):
                    torch.cuda._sleep(cycles)
            main.wait_stream(s)
        else:
            for _ in range(K):
                torch.cuda._sleep(cycles)
    return g


def time_graph(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for K, cyc in ((64, 2000), (64, 20000), (256, 2000)):
    a = time_graph(capture(K, cyc, False))
    b = time_graph(capture(K, cyc, True))
    print(json.dumps({"kernels": K, "sleep_cycles": cyc, "one_stream_us": a * 1e6, "two_branches_us": b * 1e6,
                      "ratio": b / a}), flush=True)
