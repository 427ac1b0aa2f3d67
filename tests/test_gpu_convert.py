"""GPU: opk_convert, the device element conversion behind the plugin functions' double
instantiations (integration/openpose_hip_shim.cpp AsFloat; the reference instantiates
resizeAndMergeGpu / nmsGpu / connectBodyPartsGpu for double: resizeAndMergeBase.cu:575-581,
nmsBase.cu:353-358, bodyPartConnectorBase.cu:252-266).  double -> float must round like numpy's
astype (nearest even, overflow to inf, NaN kept); float -> double is exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 255, 257, 1 << 20])
def test_convert_f64_f32_round_trip(ctx, n):
    import torch
    rng = np.random.default_rng(n + 7)
    x = rng.normal(0, 1e3, n) * np.exp(rng.uniform(-60, 60, n))
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e39, -1e39, 1e-46, 3.4028235677973366e38,
                        1.0000000596046448, 1.401298464324817e-45])
    if n >= len(special):
        x[:len(special)] = special
    src = torch.from_numpy(x).cuda()
    f32 = torch.empty(n, dtype=torch.float32, device="cuda")
    ctx.convert(f32, src)
    back = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.convert(back, f32)
    ctx.sync()
    with np.errstate(over="ignore"):   # 1e39 -> inf is one of the cases
        want = x.astype(np.float32)
    got = f32.cpu().numpy()
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    np.testing.assert_array_equal(back.cpu().numpy().view(np.uint64), want.astype(np.float64).view(np.uint64))


def test_convert_same_type_and_errors(ctx):
    import ctypes
    import torch
    from openpose_amd._lib import OpkError, check
    a = torch.arange(1000, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    ctx.convert(b, a)
    ctx.sync()
    assert torch.equal(a, b)
    rc = ctx.L.opk_convert(ctx.h, ctypes.c_void_p(b.data_ptr()), 2, ctypes.c_void_p(a.data_ptr()), 0, 10)
    with pytest.raises(OpkError, match="unknown element type"):
        check(rc)
