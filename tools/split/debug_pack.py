"""Debug: decode the split-bf16 packed image (initial layer, first block W0, final layer) and
compare with the f32 weights it was packed from."""
import sys, os, torch, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "flow-state_amd")]
from flowstate.models import build_flow
torch.manual_seed(0)
N, L, H, nb, K = 4, 1, 32, 1, 5
m = build_flow(N, L=L, H=H, nb=nb, K=K, device="cuda").eval()
with torch.no_grad():
    w = m.flows[0].prqct.transform_net.final_layer.weight
    w.copy_(torch.randn(w.shape) * 0.05)
for prec, P in (("bf16x6", 3), ("bf16x3", 2)):
    m.set_precision(prec)
    img = m.packed().cpu().numpy().view(np.uint16)
    def frags(base_floats, ntiles, kst, kin, nrows):
        out = np.zeros((ntiles * 32, kst * 16))
        for t in range(ntiles):
            for s in range(kst):
                for p in range(P):
                    off = 2 * base_floats + ((t * kst + s) * P + p) * 512
                    blk = img[off:off + 512].reshape(64, 8).astype(np.uint32) << 16
                    vals = blk.view(np.float32).astype(np.float64)
                    for l in range(64):
                        out[32 * t + (l & 31), 16 * s + 8 * (l >> 5):16 * s + 8 * (l >> 5) + 8] += vals[l]
        return out
    kst_in, kst_h = (2 * N + 15) // 16, H // 16
    frag = 256 * P
    win = frags(0, H // 32, kst_in, 2 * N, H)
    W_in = m.flows[0].prqct.transform_net.initial_layer.weight.detach().cpu().double().numpy()
    print(prec, "W_in max abs err", np.abs(win[:H, :2 * N] - W_in).max(), "max |W|", np.abs(W_in).max(), "pad max", np.abs(win[:, 2 * N:]).max())
    blocks = (H // 32) * kst_in * frag
    w0 = frags(blocks, H // 32, kst_h, H, H)
    W0 = m.flows[0].prqct.transform_net.blocks[0].linear_layers[0].weight.detach().cpu().double().numpy()
    print(prec, "W0 max abs err", np.abs(w0[:H, :H] - W0).max(), "max |W0|", np.abs(W0).max())
    wf_off = blocks + nb * 2 * (H // 32) * kst_h * frag
    wf = frags(wf_off, 3 * N, kst_h, H, 0)
    Wf = m.flows[0].prqct.transform_net.final_layer.weight.detach().cpu().double().numpy()
    P3 = 3 * K + 1
    sc = 1.4426950408889634 / np.sqrt(H)
    err = 0
    for feat in range(N):
        for t in range(3):
            rows = Wf[feat * P3 + t * K: feat * P3 + t * K + K] * (sc if t < 2 else 1.0)
            got = wf[32 * (3 * feat + t): 32 * (3 * feat + t) + K]
            err = max(err, np.abs(got - rows).max())
    print(prec, "W_f max abs err", err)
