"""GPU tests of the reference's remaining v1 elementwise exports
(bagua_kernels.cu:196-266, :574-628; declared in src/kernels/mod.rs:3-137):
substract / average / divide for f32 and f16, and async_model_average.  Off the
compressed path, kept so the kernel library binds every symbol
the reference's Rust FFI declares.  Expected values restate the reference
expressions in numpy (one correctly rounded f32 op, RNE to half for f16; the
f16 divide is the correctly rounded quotient, DESIGN/elementwise.hip)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from bagua_core import _native as N
    return N.K


def _pair(dtype, n, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 3).astype(np.float32).astype(dtype)
    y = (rng.standard_normal(n) * 3).astype(np.float32).astype(dtype)
    return x, y


def _run(fn, x, y, *args):
    xd = torch.from_numpy(x.copy()).cuda()
    yd = torch.from_numpy(y.copy()).cuda() if y is not None else None
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if yd is None:
        fn(ctypes.c_void_p(xd.data_ptr()), *args, sp)
    else:
        fn(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(yd.data_ptr()), *args, sp)
    torch.cuda.synchronize()
    return xd.cpu().numpy()


@pytest.mark.parametrize("n", [1, 7, 4096 + 3, 100003])
@pytest.mark.parametrize("half", [False, True])
def test_substract_average_divide(K, n, half):
    dt = np.float16 if half else np.float32
    sfx = "f16" if half else "f32"
    x, y = _pair(dt, n, n + half)
    f32 = np.float32
    want_sub = (x.astype(f32) - y.astype(f32)).astype(dt)
    got = _run(getattr(K, f"substract_inplace_{sfx}_host"), x, y, n)
    assert np.array_equal(got.view(np.uint16 if half else np.uint32), want_sub.view(np.uint16 if half else np.uint32))
    # K:53-61 / K:198: (a + b) / 2, the sum rounded to T first for f16
    s = (x.astype(f32) + y.astype(f32)).astype(dt).astype(f32)
    want_avg = (s / f32(2)).astype(dt)
    got = _run(getattr(K, f"average_inplace_{sfx}_host"), x, y, n)
    assert np.array_equal(got.view(np.uint16 if half else np.uint32), want_avg.view(np.uint16 if half else np.uint32))
    d = 3.7
    dd = f32(np.float16(d)) if half else f32(d)  # K:251 __float2half(D_) for f16
    want_div = (x.astype(f32) / dd).astype(dt)
    got = _run(getattr(K, f"divide_inplace_{sfx}_host"), x, None, ctypes.c_float(d), n)
    assert np.array_equal(got.view(np.uint16 if half else np.uint32), want_div.view(np.uint16 if half else np.uint32))


def test_async_model_average(K):
    """K:257-266: tensor[i] += reduced[i] / nranks - copy[i] (one atomic add per element)."""
    n, nranks = 100003, 8
    rng = np.random.default_rng(9)
    t, r, c = [(rng.standard_normal(n)).astype(np.float32) for _ in range(3)]
    td, rd, cd = (torch.from_numpy(a.copy()).cuda() for a in (t, r, c))
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    K.async_model_average_host(ctypes.c_void_p(td.data_ptr()), ctypes.c_void_p(rd.data_ptr()),
                               ctypes.c_void_p(cd.data_ptr()), ctypes.c_float(nranks), n, sp)
    torch.cuda.synchronize()
    f32 = np.float32
    want = t + ((r / f32(nranks)) - c)
    assert np.array_equal(td.cpu().numpy().view(np.uint32), want.astype(f32).view(np.uint32))
