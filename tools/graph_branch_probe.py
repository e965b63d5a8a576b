"""Do independent branches of a captured HIP graph run concurrently on this stack?
Replays (a) one stream of 2n small kernels and (b) two forked streams of n kernels each
(joined by events), and prints both replay times.  The training step's weight-gradient
GEMMs and reverse_kld's no-grad pass are off the critical path only if (b) ~ (a) / 2."""
import json
import time

import torch


def main(n=200, reps=20):
    dev = torch.device("cuda")
    a = torch.zeros(256 * 128, device=dev)
    b = torch.zeros(256 * 128, device=dev)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def serial():
        for _ in range(2 * n):
            a.add_(1.0)

    def forked():
        side.wait_stream(torch.cuda.current_stream())
        for _ in range(n):
            a.add_(1.0)
        with torch.cuda.stream(side):
            for _ in range(n):
                b.add_(1.0)
        torch.cuda.current_stream().wait_stream(side)

    out = {}
    for name, fn in (("serial", serial), ("forked", forked)):
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            fn()
        main_s.wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        out[name + "_ms"] = (time.perf_counter() - t0) / reps * 1e3
    out["kernels"] = 2 * n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
