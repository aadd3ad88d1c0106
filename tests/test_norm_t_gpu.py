"""RMSNorm kernels with transposed companion outputs (csrc/norms.hip rms_fwd_t / rms_bwd_t) against the fp32
PyTorch reference, and the Llama step that uses them (norm y^T -> QKV / gate|up weight gradients, norm dx^T ->
Wo / W_down weight gradients) against the same step with the projections transposing their own operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_fwd(x, r, w, eps):
    s = (x.float() + r.float()).bfloat16() if r is not None else x
    sf = s.float()
    rstd = torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps)
    return (sf * rstd * w.float()), s, rstd.squeeze(-1)


@pytest.mark.parametrize("T,H", [(2048, 4096), (1024, 2048), (1040, 4096)])  # 1040: row groups not dealt by XCD
@pytest.mark.parametrize("res", [False, True])
def test_rms_norm_fwd_t_matches_fp32(T, H, res):
    from kubeoperator_amd.ops.functional import _lib

    g = torch.Generator(device="cuda").manual_seed(T + H)
    x = torch.randn(T, H, device="cuda", generator=g).bfloat16()
    r = torch.randn(T, H, device="cuda", generator=g).bfloat16() if res else None
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).bfloat16()
    y, s, rstd, yt = _lib().rms_norm_fwd_t(x, r, w, 1e-5)
    ry, rs, rrstd = _ref_fwd(x, r, w, 1e-5)
    torch.testing.assert_close(y.float(), ry, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(rstd, rrstd, rtol=1e-4, atol=1e-5)
    if res:
        assert torch.equal(s, rs)
    assert yt.shape == (H, T) and torch.equal(yt, y.t())  # the companion is exactly the transpose


@pytest.mark.parametrize("T,H", [(2048, 4096), (1024, 2048), (1040, 4096)])
@pytest.mark.parametrize("dres", [False, True])
def test_rms_norm_bwd_t_matches_fp32(T, H, dres):
    from kubeoperator_amd.ops.functional import _lib

    g = torch.Generator(device="cuda").manual_seed(7 * T + H)
    s = torch.randn(T, H, device="cuda", generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).bfloat16()
    dy = torch.randn(T, H, device="cuda", generator=g).bfloat16()
    dr = torch.randn(T, H, device="cuda", generator=g).bfloat16() if dres else None
    sf = s.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    rstd = torch.rsqrt(sf.detach().pow(2).mean(-1) + 1e-5)
    ref = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    ref.backward(dy.float())
    rdx = sf.grad + (dr.float() if dres else 0)
    dw = torch.zeros(H, device="cuda", dtype=torch.bfloat16)
    dx, dxt = _lib().rms_norm_bwd_t(dy, s, w, rstd, dr, dw, False)
    torch.testing.assert_close(dx.float(), rdx, rtol=2e-2, atol=3e-2)
    assert torch.equal(dxt, dx.t())
    torch.testing.assert_close(dw.float(), wf.grad, rtol=2e-2, atol=2e-2 * wf.grad.abs().max().item())
    dx2, _ = _lib().rms_norm_bwd_t(dy, s, w, rstd, dr, dw, True)  # accumulate into the gradient
    torch.testing.assert_close(dw.float(), 2 * wf.grad, rtol=2e-2, atol=4e-2 * wf.grad.abs().max().item())


@pytest.mark.parametrize("inverse", [True, False])
@pytest.mark.parametrize("D", [128, 64])
def test_rope_transpose_matches_reference(inverse, D):
    """Inverse RoPE of the Q/K heads of dQKV fused with dQKV^T (csrc/transpose.hip rope_t) vs ops.reference."""
    from kubeoperator_amd.ops.functional import _lib
    from kubeoperator_amd.ops.reference import rope_cache, rope_ref

    B, S, Hq, Hkv = 2, 512, 8, 2
    T, C = B * S, (Hq + 2 * Hkv) * D
    cos, sin = rope_cache(S, D, 500000.0, device="cuda")
    x = torch.randn(T, C, device="cuda").bfloat16()
    ref = rope_ref(x, cos, sin, S, Hq + Hkv, D, inverse=inverse)
    out = torch.empty(C, T, device="cuda", dtype=torch.bfloat16)
    y = x.clone()
    _lib().rope_t_(y, cos, sin, S, Hq + Hkv, D, inverse, out)
    torch.testing.assert_close(y.float(), ref.float(), rtol=1e-2, atol=1e-2)
    assert torch.equal(y[:, (Hq + Hkv) * D:], x[:, (Hq + Hkv) * D:])  # V columns untouched
    assert torch.equal(out, y.t())


@pytest.mark.parametrize("D", [128, 64])
def test_flash_forward_writes_o_transpose(D):
    """The 8-wave forward's O^T tail: O^T is exactly the transpose of O, and O is unchanged by writing it."""
    from kubeoperator_amd.ops.functional import _lib

    B, S, Hq, Hkv = 2, 512, 4, 2
    T = B * S
    g = torch.Generator(device="cuda").manual_seed(D)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    o0 = torch.empty(T, Hq * D, device="cuda", dtype=torch.bfloat16)
    o1, ot = torch.empty_like(o0), torch.empty(Hq * D, T, device="cuda", dtype=torch.bfloat16)
    l0, l1 = (torch.empty(B * Hq * S, device="cuda") for _ in range(2))
    old = _lib().flash_attn_set_fwd_variant(8)  # both calls on the same kernel (pinned: the default depends on D)
    try:
        _lib().flash_attn_fwd(q, k, v, o0, l0, B, S, Hq, Hkv, D, D ** -0.5, True)
        _lib().flash_attn_fwd_t(q, k, v, o1, ot, l1, B, S, Hq, Hkv, D, D ** -0.5, True)
    finally:
        _lib().flash_attn_set_fwd_variant(old)
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
    assert torch.equal(ot, o1.t())


def test_tbox_hands_over_only_the_same_tensor():
    from kubeoperator_amd.ops.functional import TBox

    box = TBox()
    g = torch.randn(32, 16, device="cuda")
    gt = g.t().contiguous()
    box.put(g, gt)
    assert box.take(g.view(32, 16)) is gt
    assert box.take(g) is None  # taken once
    box.put(g, gt)
    g.add_(1)  # an in-place accumulation after the put: the companion is stale
    assert box.take(g) is None
    box.put(g, gt)
    assert box.take(g.clone()) is None


@pytest.mark.parametrize("recompute", [False, True])
def test_llama_gradients_with_norm_companions_match_transposes(recompute, monkeypatch):
    """2 layers of the Llama-3 1B proxy (hidden 2048) at T = 2048, one micro-batch: every parameter's gradient with
    the companions on matches the plain path to bf16 noise (the companion kernels round some activations one ulp
    differently, ~0.5 % relative per gradient; a wrong operand would be O(1)), and the companion kernels ran."""
    from kubeoperator_amd.ops import functional
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    lib = functional._lib()
    calls = {"rms_norm_fwd_t": 0, "rms_norm_bwd_t": 0, "rope_t_": 0, "transpose_": 0}

    class Spy:
        def __getattr__(self, n):
            f = getattr(lib, n)
            if n not in calls:
                return f

            def counted(*a):
                calls[n] += 1
                return f(*a)

            return counted

    spy = Spy()
    monkeypatch.setattr(functional, "_lib", lambda: spy)

    def grads(on):
        monkeypatch.setattr(functional, "_NORM_T", on)
        tr = Trainer(TrainConfig(model="llama3_1b_proxy", micro_batch=1, seq_len=2048, grad_accum=1, bucket_mb=64,
                                 grad_clip=0.0, recompute=recompute, model_overrides={"n_layers": 2}),
                     DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
        ids = torch.randint(0, tr.cfg.vocab_size, (1, 2049), generator=torch.Generator().manual_seed(5))
        for k in calls:
            calls[k] = 0
        tr.store.begin_microbatch(0)
        tr.model(ids[:, :-1].cuda(), ids[:, 1:].cuda()).backward()
        tr.store.join_side()
        torch.cuda.synchronize()
        return {n: p.main_grad.float().clone() for n, p in tr.store.named_params()}, dict(calls)

    off, c_off = grads(False)
    on, c_on = grads(True)
    assert c_off["rms_norm_fwd_t"] == 0 and c_off["rope_t_"] == 0
    fwd = 2 * 2 * (2 if recompute else 1)  # two norms per layer, forwards re-run under recompute
    assert c_on["rms_norm_fwd_t"] == fwd and c_on["rope_t_"] == 2
    assert c_on["rms_norm_bwd_t"] == 4  # norm2 of both layers, norm1 of layer 1, the final norm
    # only the LM head's two operands are still transposed (12 more per step without the companions)
    assert c_on["transpose_"] == 2 and c_off["transpose_"] == 14, (c_on, c_off)
    for n in off:
        rel = ((on[n] - off[n]).norm() / off[n].norm()).item()
        assert rel < 2e-2, (n, rel)
