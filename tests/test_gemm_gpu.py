"""The two matmul engines against float64 on the learner's layer shapes.

x6 (csrc/gemm_x6.h: exact three-plane bf16 split, six bf16 MFMAs, f32 accumulation) must
have the error profile of the f32-MFMA engine (csrc/gemm.h): per shape, its median and
maximum error relative to the output's scale within 2x of the f32 engine's (and both
below 1e-5).  acme_dense_forward runs one dense layer on the current engine."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dense(engine, x, w, b, act=0):
    from acme_amd import _lib
    L = _lib.lib()
    prev = L.acme_matmul_engine()
    _lib.check(L.acme_set_matmul_engine(engine))
    try:
        y = torch.empty(x.shape[0], w.shape[1], dtype=torch.float32, device="cuda")
        _lib.check(L.acme_dense_forward(x.data_ptr(), x.shape[0], x.shape[1], w.data_ptr(),
                                        b.data_ptr(), w.shape[1], act, y.data_ptr(),
                                        _lib.stream_ptr()))
        torch.cuda.synchronize()
        return y.cpu().numpy().astype(np.float64)
    finally:
        L.acme_set_matmul_engine(prev)


@pytest.mark.parametrize("M,K,N,kind", [(512, 7744, 1024, "fc"), (1024, 576, 64, "conv3"),
                                        (2048, 256, 32, "conv1"), (64, 1024, 7744, "dgrad"),
                                        (96, 100, 36, "ragged")])
def test_x6_matches_f32_engine_error_profile(M, K, N, kind):
    from acme_amd import _lib
    rng = np.random.default_rng(0)
    x = np.maximum(rng.standard_normal((M, K)), 0).astype(np.float32)
    if kind == "dgrad":
        x = (1e-4 * rng.standard_normal((M, K))).astype(np.float32)  # gradient-scale values
    w = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
    b = (0.1 * rng.standard_normal(N)).astype(np.float32)
    exact = x.astype(np.float64) @ w.astype(np.float64) + b
    t = lambda a: torch.as_tensor(a).cuda()  # noqa: E731
    errs = {}
    for name, eng in (("f32", _lib.MATMUL_F32), ("x6", _lib.MATMUL_X6)):
        y = _dense(eng, t(x), t(w), t(b))
        scale = np.abs(exact).max()
        err = np.abs(y - exact) / scale
        errs[name] = (float(np.median(err)), float(err.max()))
    assert errs["f32"][1] < 1e-5 and errs["x6"][1] < 1e-5, errs
    assert errs["x6"][0] <= 2 * errs["f32"][0] + 1e-9, errs
    assert errs["x6"][1] <= 2 * errs["f32"][1] + 1e-9, errs


def test_dense_activation_epilogues():
    from acme_amd import _lib
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64, 32)).astype(np.float32)
    w = rng.standard_normal((32, 16)).astype(np.float32) / 6
    b = rng.standard_normal(16).astype(np.float32)
    z = x.astype(np.float64) @ w + b
    t = lambda a: torch.as_tensor(a).cuda()  # noqa: E731
    for act, ref in ((1, np.maximum(z, 0)), (2, np.where(z < 0, np.expm1(z), z)), (3, np.tanh(z))):
        y = _dense(_lib.lib().acme_matmul_engine(), t(x), t(w), t(b), act)
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("bk,wk", [(16, 8), (32, 4), (32, 8), (16, 16)])
@pytest.mark.parametrize("multi", [0, 1])
def test_staged_engine_configurations(bk, wk, multi):
    """The staged f32 engine at every (BK, WK) the D4PG / IMPALA layers were tried with, alone
    and through the multi-problem kernel (round 5 recorded a fault at BK 32 / 4 k-groups: the
    multi launch's block size was hard-coded for 8 k-groups; csrc/gemm.h now derives it from
    the kernel's parameters).  Shapes of the D4PG critic (rows 512, 30 -> 512; 512 -> 512;
    512 -> 256 and the ragged 256 -> 52): within the f32 engine's error of float64."""
    from acme_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(bk * 100 + wk)
    t = lambda a: torch.as_tensor(a).cuda()  # noqa: E731
    for M, K, N in ((512, 32, 512), (512, 512, 512), (512, 512, 256), (256, 256, 52)):
        x = rng.standard_normal((M, K)).astype(np.float32)
        w = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
        b = (0.1 * rng.standard_normal(N)).astype(np.float32)
        exact = np.tanh(x.astype(np.float64) @ w.astype(np.float64) + b)
        y = torch.empty(M, N, dtype=torch.float32, device="cuda")
        xd, wd, bd = t(x), t(w), t(b)
        _lib.check(L.acme_dense_forward_staged(xd.data_ptr(), M, K, wd.data_ptr(), bd.data_ptr(),
                                               N, 3, y.data_ptr(), bk, wk, multi,
                                               _lib.stream_ptr()))
        torch.cuda.synchronize()
        np.testing.assert_allclose(y.cpu().numpy(), exact, rtol=0, atol=2e-6)
