"""FP8 (E4M3) GEMM path on the GPU: the quantization kernel against PyTorch's own E4M3 cast, the projection
GEMMs against fp32 products, and a few training steps against the bf16 run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fp8_quantize_matches_torch_cast():
    from kubeoperator_amd.ops import fp8

    torch.manual_seed(0)
    for n, scale in ((8192 * 64 + 5, 1.0), (4096, 1e-3), (129, 37.0)):
        x = (torch.randn(n, device="cuda") * scale).to(torch.bfloat16)
        x[n // 3] = 11.0 * scale  # the amax
        q, s = fp8.quantize(x)
        amax = x.float().abs().max()
        torch.testing.assert_close(s, amax / 448.0, rtol=1e-6, atol=0)
        # the kernel multiplies by the fp32 reciprocal of the scale (x / s can differ by an ulp at e4m3 ties)
        ref = (x.float() * (1.0 / s)).clamp(-448, 448).to(torch.float8_e4m3fn)
        assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8)), n
    z, sz = fp8.quantize(torch.zeros(64, device="cuda", dtype=torch.bfloat16))
    assert float(sz) == 1.0 and int(z.view(torch.uint8).sum()) == 0


def test_fp8_projection_gemms_track_fp32():
    """Forward Y = X W^T and data gradient dX = dY W with E4M3 operands (per-tensor scales) against fp32:
    relative Frobenius error of a few percent (3 mantissa bits), no outliers from the scaling."""
    from kubeoperator_amd.ops import fp8

    torch.manual_seed(1)
    T, K, N = 1024, 2048, 3072
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    w8, sw = fp8.quantize(w)
    y = fp8.mm(x, w8.t(), sw)
    ref = x.float() @ w.float().t()
    assert y.dtype == torch.bfloat16 and y.shape == (T, N)
    assert ((y.float() - ref).norm() / ref.norm()).item() < 0.06
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16) * 1e-3
    wt8, swt = fp8.quantize(w.t().contiguous())
    dx = fp8.mm(dy, wt8.t(), swt)
    ref_dx = dy.float() @ w.float()
    assert ((dx.float() - ref_dx).norm() / ref_dx.norm()).item() < 0.06


def test_fp8_training_follows_bf16():
    """tiny Llama, one repeated batch: the FP8 run's loss curve stays close to the bf16 run's, and the FP8
    weight copies follow every optimizer update (bucket refresh on the optimizer stream)."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
    curves = {}
    for f8 in (False, True):
        tc = TrainConfig(model="tiny_llama", micro_batch=2, seq_len=256, lr=3e-3, warmup_steps=2, total_steps=40,
                         bucket_mb=1, fp8=f8)
        tr = Trainer(tc, info)
        batch = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=9).next()
        curves[f8] = [float(tr.train_step([batch])) for _ in range(25)]
        if f8:
            assert tr.store.has_fp8
            tr.store.await_all()
            p = tr.store.param("layers.0.w_gate_up")
            deq = p.w8.float() * p.w8_scale
            assert ((deq - p.float()).norm() / p.float().norm()).item() < 0.05
    b, f = curves[False], curves[True]
    assert f[-1] < f[0] - 1.0, f  # it learns
    assert abs(f[-1] - b[-1]) < 0.25 * (b[0] - b[-1]), (b[-1], f[-1])


def _fp8_copies(w):
    from kubeoperator_amd.ops import fp8

    w.w8, w.w8_scale = fp8.quantize(w.detach())
    w.wt = w.detach().t().contiguous()
    w.wt8, w.wt8_scale = fp8.quantize(w.wt)
    return w


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_fp8_linear_backward_tracks_bf16():
    """E4M3 forward, data gradient and weight gradient (transpose-cast operands) of one projection."""
    from kubeoperator_amd.ops import functional as kf

    torch.manual_seed(2)
    T, K, N = 1024, 2048, 4096
    x0 = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w0 = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    res = {}
    for f8 in (False, True):
        x = x0.clone().requires_grad_(True)
        w = torch.nn.Parameter(w0.clone())
        if f8:
            _fp8_copies(w)
        y = kf.linear(x, w)
        y.backward(g)
        res[f8] = (y.detach(), x.grad, w.grad)
    for a, b in zip(res[True], res[False]):
        assert _rel(a, b) < 0.06


def test_fp8_swiglu_mlp_backward_tracks_bf16():
    """All six GEMMs of the SwiGLU MLP in E4M3 (h^T and dgu^T cast with the forward / data-gradient scales)."""
    from kubeoperator_amd.ops import functional as kf

    torch.manual_seed(3)
    T, H, F = 1024, 2048, 2048
    x0 = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    wgu0 = (torch.randn(2 * F, H, device="cuda") * 0.02).to(torch.bfloat16)
    wd0 = (torch.randn(H, F, device="cuda") * 0.02).to(torch.bfloat16)
    g = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    res = {}
    for f8 in (False, True):
        x = x0.clone().requires_grad_(True)
        wgu, wd = torch.nn.Parameter(wgu0.clone()), torch.nn.Parameter(wd0.clone())
        if f8:
            _fp8_copies(wgu)
            _fp8_copies(wd)
        y = kf.swiglu_mlp(x, wgu, wd)
        y.backward(g)
        res[f8] = (y.detach(), x.grad, wgu.grad, wd.grad)
    for a, b in zip(res[True], res[False]):
        assert _rel(a, b) < 0.08
