"""Debug: split-bf16 vs f32 with only one group of final-layer rows non-zero."""
import sys, os, torch
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "flow-state_amd")]
from flowstate.models import build_flow, half_box
torch.manual_seed(0)

def run(N, L, H, nb, K, rows, prec="bf16x6", C=128):
    m = build_flow(N, L=L, H=H, nb=nb, K=K, device="cuda").eval()
    g = torch.Generator().manual_seed(1)
    P3 = 3 * K + 1
    with torch.no_grad():
        for f in m.flows:
            w = f.prqct.transform_net.final_layer.weight
            r = torch.randn(w.shape, generator=g) * 0.05
            mask = torch.zeros(P3, dtype=torch.bool)
            mask[rows(K)] = True
            w.copy_((r.view(N, P3, H) * mask.view(1, P3, 1).to(r.device)).view(-1, H))
    B = half_box(N)
    x = ((torch.rand((C, 2 * N), generator=g) * 2 - 1) * B).cuda()
    ref = m.log_prob(x).double()
    got = m.set_precision(prec).log_prob(x).double()
    fin = torch.isfinite(ref)
    rel = ((got - ref).abs() / ref.abs())[fin]
    return rel.max().item()

groups = {"widths": lambda K: slice(0, K), "heights": lambda K: slice(K, 2 * K),
          "d0..dK-1": lambda K: slice(2 * K, 3 * K), "dK(tail)": lambda K: slice(3 * K, 3 * K + 1)}
for shape in ((4, 1, 32, 1, 5), (64, 1, 256, 2, 32)):
    for name, rows in groups.items():
        print(shape, f"{name:10s}", f"{run(*shape, rows):.3e}", flush=True)
