"""Host-side checks of the conditioner precision modes (no GPU): fs_flow_dims.precision
selects the f32 image (0) or a split-bf16 image (1 = bf16x6, 3 planes; 2 = bf16x3,
2 planes) with its own size; other values are rejected with a message."""
import pytest

from flowstate import _lib
from flowstate.models import build_flow


@pytest.mark.parametrize("N,L,H,nb,K", [(4, 1, 32, 1, 5), (64, 2, 256, 3, 32), (64, 1, 128, 2, 15)])
def test_precision_modes_size_their_own_image(N, L, H, nb, K):
    m = build_flow(N, L, H, nb, K)
    lib = _lib.load()
    sizes = {}
    for name, code in (("f32", 0), ("bf16x6", 1), ("bf16x3", 2)):
        m.set_precision(name)
        assert m.precision == name and m.dims().precision == code
        sizes[name] = lib.fs_flow_packed_bytes(m.dims())
    assert sizes["f32"] > 0 and sizes["bf16x6"] > sizes["bf16x3"] > 0
    n_w = L * (2 * N * H + 2 * nb * H * H + N * (3 * K + 1) * H)  # GEMM weights
    assert sizes["bf16x6"] - sizes["bf16x3"] >= 2 * n_w  # one more bf16 plane per weight
    d = m.dims()
    d.precision = 3
    assert lib.fs_flow_packed_bytes(d) == -1 and b"precision 3" in lib.fs_last_error()


def test_unknown_precision_name_is_rejected():
    m = build_flow(4, 1, 32, 1, 5)
    with pytest.raises(ValueError):
        m.set_precision("fp8")
    assert m.dims().precision == 0
