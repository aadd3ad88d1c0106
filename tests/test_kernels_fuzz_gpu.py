"""Property-based fuzzing of the HIP kernels over shapes and value scales (hypothesis), each example checked
against the plain-PyTorch fp32 reference (shape/value fuzzing instead of device ASan, which
this pool cannot run). GPU only."""
import pytest
import torch

pytestmark = pytest.mark.gpu
hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

DEV = "cuda"
FAST = settings(max_examples=10, deadline=None, derandomize=True)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@FAST
@given(T=st.integers(1, 700), H=st.sampled_from([64, 256, 512, 768, 1536, 2048, 3072, 4096, 5120, 8192]),
       scale=st.sampled_from([1e-3, 1.0, 30.0]))
def test_rmsnorm_fuzz(T, H, scale):
    from kubeoperator_amd.ops.functional import rms_norm

    g = torch.Generator(device=DEV).manual_seed(T * 7 + H)
    x = (torch.randn(T, H, device=DEV, generator=g) * scale).to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16).requires_grad_(True)
    y = rms_norm(x, w, 1e-5)
    dy = torch.randn(T, H, device=DEV, generator=g).to(torch.bfloat16)
    (y.float() * dy.float()).sum().backward()
    xf, wf = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    yf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    (yf * dy.float()).sum().backward()
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 4e-2
    assert rel_err(w.grad, wf.grad) < 4e-2


@FAST
@given(T=st.integers(1, 300), V=st.integers(1000, 70000), scale=st.sampled_from([0.1, 3.0, 20.0]),
       ignore_every=st.sampled_from([0, 3, 5]))
def test_cross_entropy_fuzz(T, V, scale, ignore_every):
    from kubeoperator_amd.ops import load

    lib = load()
    g = torch.Generator(device=DEV).manual_seed(T + V)
    logits = (torch.randn(T, V, device=DEV, generator=g) * scale).to(torch.bfloat16)
    tgt = torch.randint(0, V, (T,), device=DEV, generator=g)
    if ignore_every:
        tgt[::ignore_every] = -100
    valid = tgt != -100
    n_valid = max(int(valid.sum().item()), 1)
    ref = torch.nn.functional.cross_entropy(logits.float(), tgt, ignore_index=-100, reduction="none")
    grad_ref = torch.softmax(logits.float(), -1)
    rows = torch.arange(T, device=DEV)[valid]
    grad_ref[rows, tgt[valid]] -= 1
    grad_ref[~valid] = 0
    lg = logits.clone()
    loss, lse, sc = lib.cross_entropy_fwd_(lg, tgt, -100, True, 1.0)
    assert (loss[valid] - ref[valid]).abs().max().item() < 3e-2 * max(1.0, ref.abs().max().item()) if valid.any() else True
    assert abs(sc.item() - 1.0 / n_valid) < 1e-6
    assert rel_err(lg, grad_ref / n_valid) < 3e-2
    if valid.any():
        assert (lse[valid] - torch.logsumexp(logits.float(), -1)[valid]).abs().max().item() < 2e-2 * max(1.0, scale)


@FAST
@given(S=st.sampled_from([128, 256, 384, 512, 768, 1024]), B=st.integers(1, 2),
       heads=st.sampled_from([(4, 4), (8, 2), (8, 1), (12, 12), (32, 8)]), D=st.sampled_from([64, 128]),
       causal=st.booleans(), scale=st.sampled_from([0.5, 1.0, 4.0]), rope=st.booleans())
def test_attention_fuzz(S, B, heads, D, causal, scale, rope):
    """fused (RoPE +) flash attention forward and backward, S covering both the 8-wave (S % 256 == 0) and
    the 4-wave kernels, GQA ratios 1..8, score scales that push the online-softmax rescale path."""
    from kubeoperator_amd.ops.functional import flash_attention, rope_attention
    from kubeoperator_amd.ops.reference import attention_ref, rope_cache, rope_ref

    Hq, Hkv = heads
    g = torch.Generator(device=DEV).manual_seed(S * 31 + Hq * 7 + D)
    qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, generator=g) * scale).to(torch.bfloat16)
    a, c = Hq * D, (Hq + Hkv) * D
    cos, sin = rope_cache(S, D, 500000.0, device=DEV) if rope else (None, None)
    if not rope:
        o, lse = flash_attention(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, causal)
        o_ref, lse_ref = attention_ref(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, causal)
        assert rel_err(o, o_ref) < 3e-2
        assert (lse - lse_ref).abs().max().item() < 5e-2 * max(1.0, scale * scale)
    x = qkv.clone().requires_grad_(True)
    o = rope_attention(x, cos, sin, B, S, Hq, Hkv, D, causal=causal, use_rope=rope, inplace=False)
    do = torch.randn(o.shape, device=DEV, generator=g).to(torch.bfloat16)
    (o.float() * do.float()).sum().backward()
    xf = qkv.detach().float().requires_grad_(True)
    xr = rope_ref(xf, cos, sin, S, Hq + Hkv, D) if rope else xf
    # the kernel stores rotated Q/K in bf16 before attention: round the same way (straight-through for grads)
    xr = xr + (xr.to(torch.bfloat16).float() - xr).detach()
    of, _ = attention_ref(xr[:, :a], xr[:, a:c], xr[:, c:], B, S, Hq, Hkv, D, causal)
    (of * do.float()).sum().backward()
    assert rel_err(o, of) < 3e-2
    for lo, hi in ((0, a), (a, c), (c, xf.shape[1])):
        assert rel_err(x.grad[:, lo:hi], xf.grad[:, lo:hi]) < 6e-2


@FAST
@given(T=st.integers(1, 600), F=st.sampled_from([64, 1408, 1536, 14336]), scale=st.sampled_from([0.1, 1.0, 8.0]))
def test_swiglu_fuzz(T, F, scale):
    from kubeoperator_amd.ops.functional import swiglu

    g = torch.Generator(device=DEV).manual_seed(T * 3 + F)
    gu = (torch.randn(T, 2 * F, device=DEV, generator=g) * scale).to(torch.bfloat16).requires_grad_(True)
    h = swiglu(gu)
    dh = torch.randn(h.shape, device=DEV, generator=g).to(torch.bfloat16)
    (h.float() * dh.float()).sum().backward()
    gf = gu.detach().float().requires_grad_(True)
    u, v = gf.chunk(2, -1)
    hf = torch.nn.functional.silu(u) * v
    (hf * dh.float()).sum().backward()
    assert rel_err(h, hf) < 2e-2
    assert rel_err(gu.grad, gf.grad) < 3e-2


@FAST
@given(S=st.integers(1, 300), B=st.integers(1, 3), heads=st.sampled_from([(4, 2), (8, 8), (32, 8)]),
       D=st.sampled_from([64, 128]), theta=st.sampled_from([1e4, 5e5]))
def test_rope_fuzz(S, B, heads, D, theta):
    from kubeoperator_amd.ops import load
    from kubeoperator_amd.ops.reference import rope_cache, rope_ref

    Hq, Hkv = heads
    g = torch.Generator(device=DEV).manual_seed(S + 17 * D)
    cos, sin = rope_cache(S, D, theta, device=DEV)
    x = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, generator=g).to(torch.bfloat16)
    y = x.clone()
    load().rope_(y, cos, sin, None, S, Hq + Hkv, D, False)
    assert rel_err(y, rope_ref(x, cos, sin, S, Hq + Hkv, D)) < 1e-2
    assert torch.equal(y[:, (Hq + Hkv) * D:], x[:, (Hq + Hkv) * D:])
    load().rope_(y, cos, sin, None, S, Hq + Hkv, D, True)
    assert rel_err(y, x) < 2e-2
