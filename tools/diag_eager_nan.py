"""Diagnostic for tests/test_gpu_train_graph.py::test_graphed_step_matches_eager[alpha]: the
eager loop of that test step by step, reporting per step the loss, the largest gradient, any
non-finite gradient (and the parameter it sits in) and non-finite parameters after Adam."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
from test_train_cpu import build  # noqa: E402


def main(alpha=0.7, steps=6, graphed=False):
    from flowstate.normflows import autograd_flow as AF
    from flowstate.normflows.train import GraphedTrainStep

    m, f = build("cuda")
    x = torch.from_numpy(f["x"]).cuda()
    opt = torch.optim.Adam(m.parameters(), lr=5e-3, weight_decay=1e-4)
    g = None
    if graphed:  # as the test: a second model's training step captured in a graph first
        m2, _ = build("cuda")
        g = GraphedTrainStep(m2, 64, 5e-3, 1e-4, alpha=alpha, example=x)
        print(f"after capture: splitk_pending {len(AF._splitk_pending)}, nan_flags {len(AF._nan_flags)}", flush=True)
    names = {p: n for n, p in m.named_parameters()}
    for i in range(steps):
        xb = x.roll(i, 0)
        opt.zero_grad()
        try:
            e, z = m.reverse_kld(64)
        except ValueError as err:
            print(f"step {i}: reverse_kld raised {err}; non-finite params: "
                  f"{[n for n, p in m.named_parameters() if not torch.isfinite(p).all()]}", flush=True)
            return
        s = m.forward_kld(xb)
        loss = alpha * s + (1 - alpha) * e
        E = m.p._energy(z)
        print(f"step {i}: loss {loss.item():.6g} (fwd {s.item():.6g}, rev {e.item():.6g}); target energy max "
              f"{E.max().item():.4g}", flush=True)
        if bool(~(torch.isnan(loss) | torch.isinf(loss))):
            loss.backward()
            bad = [names[p] for p in m.parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
            gmax = max(float(p.grad.abs().max()) for p in m.parameters() if p.grad is not None)
            print(f"   grad max {gmax:.4g}; non-finite grads in {bad}", flush=True)
            opt.step()
            badp = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
            print(f"   non-finite params after Adam: {badp}; splitk_pending {len(AF._splitk_pending)}", flush=True)
        if g is not None:
            l2 = g.step(xb)
            print(f"   graphed loss {l2.item():.6g}; splitk_pending {len(AF._splitk_pending)}", flush=True)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 0.7, graphed=len(sys.argv) > 2 and sys.argv[2] == "graphed")
