"""Per-launch time of the A2 training step's backward pieces (batch 256, H = 128), each
replayed 200x back to back in a HIP graph (the step's own launch pattern): the gradient
pair plus fs_bn_relu_train_bwd (r03k also timed a one-launch Linear + BatchNorm/ReLU
backward here, since removed: profiles/r03/r03k_linbn_probe.log), the BatchNorm-in-load forward product (fs_linear_f32_ex), the final
layer's input gradient (split-K vs one pass) and the graph-node floor.  FLOWSTATE_LIB
selects an A/B build (tools/build_variant.sh)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
from flowstate import _lib  # noqa: E402


def timed(fn, reps=200):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return round(best, 2)


def main(M=256, H=128, NF=2944):
    L = _lib.load()
    p = _lib.ptr
    st = _lib.stream_ptr
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rn = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x, u, gy = rn(M, H), torch.relu(rn(M, H)), rn(M, H)
    w, gamma = rn(H, H) * 0.1, rn(H).abs() + 0.5
    mean, invstd = rn(H) * 0.1, rn(H).abs() + 0.5
    add = rn(M, H)
    gx, gw, gb, gg, gbt, gu = (torch.empty_like(t) for t in (x, w, gamma, gamma, gamma, u))
    out = {"lib": os.environ.get("FLOWSTATE_LIB") or "in-tree"}
    tiny = torch.zeros(64, device=dev)
    out["node_floor_fill64"] = timed(lambda: tiny.zero_())

    g0 = _lib.GemmF32(M, H, H, p(gy), H, 1, p(w), H, 1, None, None, 0, p(gu), H, None)
    g1 = _lib.GemmF32(H, H, M, p(gy), 1, H, p(u), H, 1, None, None, 0, p(gw), H, p(gb))

    def pair():
        _lib.check(L.fs_linear_f32_pair(g0, g1, st()), "pair")

    def bnb():
        _lib.check(L.fs_bn_relu_train_bwd(M, H, p(x), p(u), p(gu), p(gamma), p(mean), p(invstd), p(gx), p(add),
                                          p(gg), p(gbt), st()), "bnbwd")

    out["pair"] = timed(pair)
    out["bn_relu_train_bwd"] = timed(bnb)
    out["pair_then_bn_bwd"] = timed(lambda: (pair(), bnb()))

    # BatchNorm-in-load forward product
    y = torch.empty(M, H, device=dev)
    stt = torch.empty((M // 32, H, 2), device=dev)
    xs = torch.empty((M // 32, H, 2), device=dev)
    L.fs_linear_f32_ex(_lib.GemmF32(M, H, H, p(x), H, 1, p(w), 1, H, p(gamma), None, 0, p(y), H, None), None,
                       p(xs), st())
    rm, rv = torch.zeros(H, device=dev), torch.ones(H, device=dev)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    mo, io = torch.empty(H, device=dev), torch.empty(H, device=dev)
    ub = torch.empty(M, H, device=dev)
    bi = _lib.BnIn(p(xs), M // 32, M, p(gamma), p(mean), 1e-5, 0.1, p(rm), p(rv), p(nbt), p(mo), p(io), p(ub), None)
    gf = _lib.GemmF32(M, H, H, p(y), H, 1, p(w), 1, H, p(gamma), None, 0, p(gu), H, None)
    out["linear_ex_bn_in_load"] = timed(lambda: L.fs_linear_f32_ex(gf, bi, p(stt), st()))
    gpl = _lib.GemmF32(M, H, H, p(y), H, 1, p(w), 1, H, p(gamma), None, 0, p(gu), H, None)
    out["linear_plain"] = timed(lambda: _lib.check(L.fs_linear_f32(gpl.M, gpl.N, gpl.K, gpl.A, gpl.sam, gpl.sak, gpl.B,
                                                                   gpl.sbk, gpl.sbn, gpl.bias, gpl.R, gpl.ldr, gpl.C,
                                                                   gpl.ldc, gpl.rowsum_a, st()), "plain"))

    # final layer's forward (736 tiles) and weight gradient (dW = dY^T h over the batch)
    hf, wff, bff = rn(M, H), rn(NF, H) * 0.05, rn(NF)
    yf = torch.empty(M, NF, device=dev)
    gff = _lib.GemmF32(M, NF, H, p(hf), H, 1, p(wff), 1, H, p(bff), None, 0, p(yf), NF, None)
    out["final_fwd"] = timed(lambda: _lib.check(L.fs_linear_f32(gff.M, gff.N, gff.K, gff.A, gff.sam, gff.sak, gff.B,
                                                                gff.sbk, gff.sbn, gff.bias, None, 0, gff.C, gff.ldc,
                                                                None, st()), "ffwd"))
    gpf = rn(M, NF)
    gwf, gbf = torch.empty(NF, H, device=dev), torch.empty(NF, device=dev)
    gdw = _lib.GemmF32(NF, H, M, p(gpf), 1, NF, p(hf), H, 1, None, None, 0, p(gwf), H, p(gbf))
    out["final_dw"] = timed(lambda: _lib.check(L.fs_linear_f32(gdw.M, gdw.N, gdw.K, gdw.A, gdw.sam, gdw.sak, gdw.B,
                                                               gdw.sbk, gdw.sbn, None, None, 0, gdw.C, gdw.ldc,
                                                               gdw.rowsum_a, st()), "fdw"))

    # final layer's input gradient: dX = dY W over K = NF
    dyf, wf = rn(M, NF), rn(NF, H) * 0.05
    gxf = torch.empty(M, H, device=dev)
    gd = _lib.GemmF32(M, H, NF, p(dyf), NF, 1, p(wf), H, 1, None, None, 0, p(gxf), H, None)
    n = L.fs_linear_f32_splitk_floats(gd)
    ws = torch.empty(max(n, 1), device=dev)
    out["final_dx_splitk"] = timed(lambda: _lib.check(L.fs_linear_f32_splitk(gd, p(ws), n, st()), "sk"))
    out["final_dx_one_pass"] = timed(lambda: _lib.check(L.fs_linear_f32(gd.M, gd.N, gd.K, gd.A, gd.sam, gd.sak, gd.B,
                                                                        gd.sbk, gd.sbn, None, None, 0, gd.C, gd.ldc,
                                                                        None, st()), "one"))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
