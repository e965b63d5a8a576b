"""Debug: which chains of the split-bf16 pass disagree with the f32 kernel."""
import sys, os, torch, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "flow-state_amd")]
from flowstate.models import build_flow, half_box

def run(N, L, H, nb, K, C=512, prec="bf16x6", variant="full"):
    torch.manual_seed(0)
    m = build_flow(N, L=L, H=H, nb=nb, K=K, device="cuda").eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for f in m.flows:
            t = f.prqct.transform_net
            w = torch.randn(t.final_layer.weight.shape, generator=g) * 0.05
            P3 = 3 * K + 1
            if variant != "full":
                keep = torch.zeros(P3, dtype=torch.bool)
                sl = {"w": slice(0, K), "h": slice(K, 2 * K), "d": slice(2 * K, 3 * K), "t": slice(3 * K, P3)}[variant]
                keep[sl] = True
                w = w * keep.repeat(N)[:, None]
            t.final_layer.weight.copy_(w)
    B = half_box(N)
    x = ((torch.rand((C, 2 * N), generator=g) * 2 - 1) * B).cuda()
    ref = m.log_prob(x).double()
    got = m.set_precision(prec).log_prob(x).double()
    rel = ((got - ref).abs() / ref.abs()).cpu().numpy()
    bad = np.nonzero(rel > 1e-5)[0]
    print(f"N={N} H={H} K={K} {variant}: {len(bad)}/{C} bad; chain%64 of bad: {np.bincount(bad % 64, minlength=64).tolist()}")
    print("   worst:", [(int(i), f"{rel[i]:.1e}") for i in np.argsort(-rel)[:6]], flush=True)

for v in ("full", "w", "h", "d", "t"):
    run(4, 1, 32, 1, 5, variant=v)
for v in ("full", "w", "d", "t"):
    run(64, 1, 256, 2, 32, variant=v)
