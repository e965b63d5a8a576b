"""Debug: split-bf16 flow vs the f32 kernel on models with parts switched off."""
import sys, os, torch, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "flow-state_amd")]
from flowstate.models import build_flow, half_box
torch.manual_seed(0)

def run(N, L, H, nb, K, variant, prec="bf16x6", C=128):
    m = build_flow(N, L=L, H=H, nb=nb, K=K, device="cuda").eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for f in m.flows:
            t = f.prqct.transform_net
            t.final_layer.weight.copy_(torch.randn(t.final_layer.weight.shape, generator=g) * (0.0 if variant == "final0" else 0.05))
            for blk in t.blocks:
                for lin in blk.linear_layers:
                    if variant == "res0":
                        lin.weight.zero_(); lin.bias.zero_()
            if variant == "init0":
                t.initial_layer.weight.zero_()
            u = f.prqct.unconditional_transform
            u.unnormalized_widths.copy_(torch.randn(u.unnormalized_widths.shape, generator=g) * 0.3)
    B = half_box(N)
    x = ((torch.rand((C, 2 * N), generator=g) * 2 - 1) * B).cuda()
    ref = m.log_prob(x).double()
    ref_ld = m.inverse_and_log_det(x)[1].double()
    got = m.set_precision(prec).log_prob(x).double()
    z_ref = m.set_precision("f32").inverse(x); z = m.set_precision(prec).inverse(x)
    fin = torch.isfinite(ref)
    rel = ((got - ref).abs() / ref.abs())[fin]
    print(f"N={N} H={H} nb={nb} K={K} L={L} {variant:7s} {prec}: max rel {rel.max().item():.3e} median {rel.median().item():.3e}  z maxdiff {(z - z_ref).abs().max().item():.3e}", flush=True)

for prec in ("bf16x6",):
    for shape in ((4, 1, 32, 1, 5), (4, 2, 32, 1, 5), (16, 1, 64, 1, 8), (64, 1, 256, 2, 32)):
        for v in ("full", "final0", "res0", "init0"):
            run(*shape, v, prec)
