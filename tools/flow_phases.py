"""Per-phase time breakdown of flow_pass_kernel (A1, N=64) from the phase-timer
build (make -C flow-state_amd/csrc prof -> libflowstate_prof.so): every wave
accumulates s_memtime deltas per phase; the shares are summed over all waves."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from flowstate import _lib  # noqa: E402

PH = ["input", "periodic_features", "init_gemm", "epilogue", "resnet_gemm", "barrier_wait", "tail_gemm",
      "final_gemm", "spline_valu", "uncond_spline"]


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "f32"  # f32 | bf16x6 | bf16x3 (flow_split_kernel)
    lib = _lib.load(os.environ.get("FS_PROF_LIB") or os.path.join(REPO, "flow-state_amd", "flowstate", "lib", "libflowstate_prof.so"))
    read = lib.fs_prof_read if prec == "f32" else lib.fs_prof_read_split
    read.restype = ctypes.c_int
    read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib._lib = lib  # route the Python classes through the prof build for this run
    from bench import synthetic_model, synthetic_states
    N, C = 64, int(os.environ.get("FS_CHAINS", "65536"))
    model = synthetic_model(N, torch.device("cuda")).set_precision(prec)
    init, L = synthetic_states(N, C, 0)
    x = torch.from_numpy((init - L / 2).astype("float32").reshape(C, -1)).cuda()
    buf = (ctypes.c_ulonglong * 16)()
    out = {"precision": prec}
    def guard(f):  # timing builds with stale data may trip the NaN check after the kernels ran
        def g():
            try:
                f()
            except ValueError:
                pass
        return g

    for name, fn in (("density", guard(lambda: model.log_prob(x))), ("sample", guard(lambda: model.forward(x)))):
        fn()
        torch.cuda.synchronize()
        read(buf, 1)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        fn()
        ev1.record()
        torch.cuda.synchronize()
        read(buf, 1)
        tot = sum(buf[i] for i in range(len(PH)))
        out[name] = {"ms": ev0.elapsed_time(ev1), "share": {PH[i]: buf[i] / tot for i in range(len(PH))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
