"""Numerics of every gfx950 HIP kernel against a plain-PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def lib():
    from kubeoperator_amd.ops import load

    return load()


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def test_extension_is_native():
    m = lib()
    assert m.__file__.endswith("_C.so")
    assert m.ARCH == "gfx950"
    props = torch.cuda.get_device_properties(0)
    assert "gfx950" in getattr(props, "gcnArchName", "gfx950")


@pytest.mark.parametrize("H", [4096, 768, 1024])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_fwd_bwd(H, with_res):
    from kubeoperator_amd.ops.functional import rms_norm

    torch.manual_seed(0)
    T = 333
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    out = rms_norm(x, w, 1e-5, residual=r)
    y, s = out if with_res else (out, None)
    dy = torch.randn_like(y)
    ds = torch.randn_like(y) if with_res else None
    loss = (y.float() * dy.float()).sum() + ((s.float() * ds.float()).sum() if with_res else 0)
    loss.backward()
    # reference
    xf = x.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if with_res else None
    wf = w.detach().float().requires_grad_(True)
    sf = xf + rf if with_res else xf
    sf_b = sf.to(torch.bfloat16).float() if with_res else sf
    yf = sf_b * torch.rsqrt(sf_b.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    lf = (yf * dy.float()).sum() + ((sf * ds.float()).sum() if with_res else 0)
    lf.backward()
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(w.grad, wf.grad) < 3e-2
    if with_res:
        assert rel_err(r.grad, rf.grad) < 3e-2


@pytest.mark.parametrize("H,T,with_res", [(768, 257, False), (4096, 257, False), (768, 9001, True),
                                          (512, 4099, True), (1024, 3, False)])
def test_layernorm_fwd_bwd(H, T, with_res):
    """H <= 1024 takes the row-per-wave narrow backward (several rows per wave once T > 4096 rows)."""
    from kubeoperator_amd.ops.functional import layer_norm

    torch.manual_seed(1)
    x = (torch.randn(T, H, device=DEV) * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    out = layer_norm(x, w, b, 1e-5, residual=r)
    y, s = out if with_res else (out, None)
    dy = torch.randn_like(y)
    ds = torch.randn_like(y) if with_res else None
    ((y.float() * dy.float()).sum() + ((s.float() * ds.float()).sum() if with_res else 0)).backward()
    xf, wf, bf = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    rf = r.detach().float().requires_grad_(True) if with_res else None
    sf = xf + rf if with_res else xf
    sf_b = sf.to(torch.bfloat16).float() if with_res else sf
    yf = torch.nn.functional.layer_norm(sf_b, (H,), wf, bf, 1e-5)
    ((yf * dy.float()).sum() + ((sf * ds.float()).sum() if with_res else 0)).backward()
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(w.grad, wf.grad) < 3e-2
    assert rel_err(b.grad, bf.grad) < 3e-2
    if with_res:
        assert rel_err(r.grad, rf.grad) < 3e-2


@pytest.mark.parametrize("D", [128, 64])
def test_rope_matches_reference_and_inverts(D):
    from kubeoperator_amd.ops.reference import rope_cache, rope_ref

    torch.manual_seed(2)
    S, B, Hq, Hkv = 64, 2, 4, 2
    cos, sin = rope_cache(S, D, 500000.0, device=DEV)
    x = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    ref = rope_ref(x, cos, sin, S, Hq + Hkv, D)
    y = x.clone()
    lib().rope_(y, cos, sin, None, S, Hq + Hkv, D, False)
    assert rel_err(y, ref) < 1e-2
    # V columns untouched
    assert torch.equal(y[:, (Hq + Hkv) * D:], x[:, (Hq + Hkv) * D:])
    lib().rope_(y, cos, sin, None, S, Hq + Hkv, D, True)
    assert rel_err(y, x) < 2e-2


def test_swiglu_fwd_bwd():
    from kubeoperator_amd.ops.functional import swiglu

    torch.manual_seed(3)
    gu = torch.randn(100, 2 * 1536, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    h = swiglu(gu)
    dh = torch.randn_like(h)
    (h.float() * dh.float()).sum().backward()
    g = gu.detach().float().requires_grad_(True)
    a, b = g.chunk(2, -1)
    hf = torch.nn.functional.silu(a) * b
    (hf * dh.float()).sum().backward()
    assert rel_err(h, hf) < 2e-2
    assert rel_err(gu.grad, g.grad) < 2e-2


@pytest.mark.parametrize("rows", [64, 2051])
def test_gelu_fwd_bwd(rows):
    """64 rows: one chunk per thread; 2051 rows: more 16-byte chunks than the 2048 x 256-thread grid holds (the
    grid-stride loop's second pass ends part-way through the grid)."""
    from kubeoperator_amd.ops.functional import gelu

    torch.manual_seed(4)
    x = (3 * torch.randn(rows, 3072, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    y = gelu(x)
    dy = torch.randn_like(y)
    (y.float() * dy.float()).sum().backward()
    xf = x.detach().float().requires_grad_(True)
    yf = torch.nn.functional.gelu(xf, approximate="tanh")
    (yf * dy.float()).sum().backward()
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 2e-2


@pytest.mark.parametrize("V", [128256, 50304, 50257, 1000])
def test_cross_entropy_lmhead(V):
    """128256: the two-pass kernel; 50304 (GPT-2's padded vocabulary) and 1000: the register-resident rows;
    50257: the scalar (unaligned) path; every seventh target ignored."""
    from kubeoperator_amd.ops.functional import cross_entropy_lmhead

    torch.manual_seed(5)
    T, H = 96, 256
    x = (0.5 * torch.randn(T, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    w = (0.05 * torch.randn(V, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (T,), device=DEV)
    tgt[::7] = -100
    loss = cross_entropy_lmhead(x, w, tgt)
    (loss * 2.0).backward()
    xf, wf = (t.detach().float().requires_grad_(True) for t in (x, w))
    logits = (xf @ wf.t()).to(torch.bfloat16).float()
    lf = torch.nn.functional.cross_entropy(logits, tgt, ignore_index=-100)
    (lf * 2.0).backward()
    assert abs(loss.item() - lf.item()) < 1e-2 * max(1.0, lf.item())
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(w.grad, wf.grad) < 3e-2


@pytest.mark.parametrize("V", [50304, 128256])
@pytest.mark.parametrize("mult", [2.0, -1.5, 0.0])
def test_cross_entropy_grad_multiplier_sign(V, mult):
    """The gradient the kernel writes in place is (softmax - onehot) * grad_multiplier / n_valid for ANY sign of the
    multiplier (its magnitude is folded into the exponent, the sign applied separately)."""
    torch.manual_seed(15)
    T = 64
    logits = (2 * torch.randn(T, V, device=DEV)).to(torch.bfloat16)
    tgt = torch.randint(0, V, (T,), device=DEV)
    tgt[::5] = -100
    ref_in = logits.float()
    x = logits.clone()
    lib().cross_entropy_fwd_(x, tgt, -100, True, mult)
    n = int((tgt != -100).sum())
    p = torch.softmax(ref_in, -1)
    oh = torch.zeros_like(p)
    valid = tgt != -100
    oh[valid.nonzero().squeeze(1), tgt[valid]] = 1.0
    ref = (p - oh) * (mult / n)
    ref[~valid] = 0.0
    if mult == 0.0:
        assert torch.count_nonzero(x[valid].float()) == 0
    else:
        assert rel_err(x[valid], ref[valid]) < 2e-2
        assert (x[valid].float() * ref[valid]).sum() > 0  # same sign pattern as the reference


def test_adamw_matches_reference():
    from kubeoperator_amd.ops.optim import FusedAdamW, Segment

    torch.manual_seed(6)
    n = 4096 * 3 + 64
    p = torch.randn(n, device=DEV).to(torch.bfloat16)
    g = (0.01 * torch.randn(n, device=DEV)).to(torch.bfloat16)
    opt = FusedAdamW([Segment(p[: n // 2], g[: n // 2], 0.1), Segment(p[n // 2:], g[n // 2:], 0.0)], lr=1e-3,
                     max_grad_norm=0.5)
    master = p.float().clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for step in range(1, 4):
        opt.step()
        gf = g.float()
        coef = min(1.0, 0.5 / (gf.norm().item() + 1e-6))
        gf = gf * coef
        m.mul_(0.9).add_(gf, alpha=0.1)
        v.mul_(0.95).addcmul_(gf, gf, value=0.05)
        wd = torch.cat([torch.full((n // 2,), 0.1, device=DEV), torch.zeros(n - n // 2, device=DEV)])
        master.mul_(1 - 1e-3 * wd)
        master.sub_(1e-3 * (m / (1 - 0.9 ** step)) / ((v / (1 - 0.95 ** step)).sqrt() + 1e-8))
    assert rel_err(opt.master, master) < 1e-5
    assert rel_err(p, master) < 1e-2
    assert abs(opt.last_grad_norm.item() - g.float().norm().item()) < 1e-3 * g.float().norm().item()


def _attn_case(B, S, Hq, Hkv, D, causal, seed=7):
    from kubeoperator_amd.ops.functional import flash_attention
    from kubeoperator_amd.ops.reference import attention_ref

    torch.manual_seed(seed)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    a, c = Hq * D, (Hq + Hkv) * D
    o, lse = flash_attention(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, causal)
    o_ref, lse_ref = attention_ref(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, causal)
    return o, lse, o_ref, lse_ref


@pytest.mark.parametrize("D", [128, 64])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_fwd(D, causal):
    o, lse, o_ref, lse_ref = _attn_case(2, 256, 8, 2, D, causal)
    assert rel_err(o, o_ref) < 2e-2
    assert (lse - lse_ref).abs().max().item() < 2e-2
    from numerics import check_against_bf16

    torch.manual_seed(7)  # the same qkv as _attn_case
    qkv = torch.randn(2 * 256, (8 + 2 * 2) * D, device=DEV, dtype=torch.bfloat16)
    ob, _ = _sdpa_bf16(qkv, torch.zeros(2 * 256, 8 * D, device=DEV), 2, 256, 8, 2, D, causal)
    check_against_bf16("o", o.reshape(-1, D), o_ref.reshape(-1, D), ob.reshape(-1, D))


@pytest.mark.parametrize("variant", [-1, 10, 8, 9, 0, 16, 12])
def test_flash_attention_fwd_spiked_rescale(variant):
    """force the online-softmax rescale branch: a large score late in the key sweep (every forward kernel:
    -1 the default, 8 / 9 / 10 the 8-wave kernel, 0 the 4-wave kernel, 16 the 16x16x32-MFMA kernel, 12 the
    hand-scheduled one-wave-per-SIMD kernel of flash_fwd4.hip)."""
    from kubeoperator_amd.ops.functional import flash_attention
    from kubeoperator_amd.ops.reference import attention_ref

    old = lib().flash_attn_set_fwd_variant(variant)
    try:
        B, S, Hq, Hkv, D = 1, 512, 4, 4, 128
        torch.manual_seed(8)
        qkv = (0.3 * torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV)).to(torch.bfloat16)
        a, c = Hq * D, (Hq + Hkv) * D
        qkv[300, a:a + D] = qkv[400, :D] * 8  # key 300 aligns strongly with query 400
        o, lse = flash_attention(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, True)
        o_ref, lse_ref = attention_ref(qkv[:, :a], qkv[:, a:c], qkv[:, c:], B, S, Hq, Hkv, D, True)
        assert rel_err(o, o_ref) < 2e-2
        assert (lse - lse_ref).abs().max().item() < 2e-2
    finally:
        lib().flash_attn_set_fwd_variant(old)


@pytest.mark.parametrize("variant,D", [(8, 128), (10, 128), (16, 128), (16, 64), (12, 128)])
@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 512, 8, 2), (1, 1024, 4, 4), (2, 256, 6, 3)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_fwd_variants_d128(variant, D, B, S, Hq, Hkv, causal):
    """the 8-wave forward (scalar / packed FMA softmax; 16: on 16x16x32 MFMAs, also at D = 64; 12: the hand-scheduled
    one-wave-per-SIMD kernel, flash_fwd4.hip) against the fp32 reference with GQA groups of 4, 1 and 2, with and without the O^T output (which must be the exact transpose of O)."""
    from kubeoperator_amd.ops.reference import attention_ref

    old = lib().flash_attn_set_fwd_variant(variant)
    try:
        torch.manual_seed(B * S + Hq)
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
        a, c = Hq * D, (Hq + Hkv) * D
        q, k, v = qkv[:, :a], qkv[:, a:c], qkv[:, c:]
        o = torch.empty(B * S, Hq * D, device=DEV, dtype=torch.bfloat16)
        lse = torch.empty(B * Hq * S, device=DEV)
        lib().flash_attn_fwd(q, k, v, o, lse, B, S, Hq, Hkv, D, D ** -0.5, causal)
        o_ref, lse_ref = attention_ref(q, k, v, B, S, Hq, Hkv, D, causal)
        assert rel_err(o, o_ref) < 2e-2
        assert (lse - lse_ref.reshape(lse.shape)).abs().max().item() < 2e-2
        o1, ot = torch.empty_like(o), torch.empty(Hq * D, B * S, device=DEV, dtype=torch.bfloat16)
        l1 = torch.empty_like(lse)
        lib().flash_attn_fwd_t(q, k, v, o1, ot, l1, B, S, Hq, Hkv, D, D ** -0.5, causal)
        assert torch.equal(o1, o) and torch.equal(l1, lse)
        assert torch.equal(ot, o1.t())
    finally:
        lib().flash_attn_set_fwd_variant(old)


@pytest.mark.parametrize("D,Hq,Hkv", [(128, 8, 2), (64, 4, 4)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_bwd(D, Hq, Hkv, causal):
    from kubeoperator_amd.ops.functional import rope_attention

    B, S = 2, 256
    torch.manual_seed(9)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=causal, use_rope=False)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    # fp32 reference through autograd
    x = qkv.detach().float().requires_grad_(True)
    a, c = Hq * D, (Hq + Hkv) * D
    qh = x[:, :a].reshape(B, S, Hq, D).transpose(1, 2)
    kh = x[:, a:c].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    vh = x[:, c:].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, device=DEV, dtype=torch.bool).triu(1), float("-inf"))
    of = (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(B * S, a)
    (of * do.float()).sum().backward()
    assert rel_err(o, of) < 2e-2
    g, gr = qkv.grad.float(), x.grad
    for name, sl in (("dq", slice(0, a)), ("dk", slice(a, c)), ("dv", slice(c, None))):
        assert rel_err(g[:, sl], gr[:, sl]) < 3e-2, name
    # no worse than plain bf16 PyTorch on the same inputs (whole tensor and smallest-norm (row, head) slices)
    from numerics import check_against_bf16

    ob, gb = _sdpa_bf16(qkv.detach(), do, B, S, Hq, Hkv, D, causal)
    check_against_bf16("o", o.reshape(-1, D), of.reshape(-1, D), ob.reshape(-1, D))
    for name, sl in (("dq", slice(0, a)), ("dk", slice(a, c)), ("dv", slice(c, None))):
        check_against_bf16(name, g[:, sl].reshape(-1, D), gr[:, sl].reshape(-1, D), gb[:, sl].reshape(-1, D))


def _sdpa_bf16(qkv, do, B, S, Hq, Hkv, D, causal):
    """Plain bf16 PyTorch attention (SDPA, GQA by repeat_interleave) forward + backward -> (o, dqkv)."""
    x = qkv.detach().clone().requires_grad_(True)
    a, c = Hq * D, (Hq + Hkv) * D
    q = x[:, :a].reshape(B, S, Hq, D).transpose(1, 2)
    k = x[:, a:c].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    v = x[:, c:].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)
    o = o.transpose(1, 2).reshape(B * S, a)
    o.backward(do.to(torch.bfloat16))
    return o.detach(), x.grad


def test_rope_attention_end_to_end_grad():
    from kubeoperator_amd.ops.functional import rope_attention
    from kubeoperator_amd.ops.reference import rope_cache

    B, S, Hq, Hkv, D = 1, 128, 4, 2, 128
    cos, sin = rope_cache(S, D, 10000.0, device=DEV)
    torch.manual_seed(10)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = rope_attention(qkv, cos, sin, B, S, Hq, Hkv, D, inplace=False)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    qc = qkv.detach().cpu().float().requires_grad_(True)
    oc = rope_attention(qc, cos.cpu(), sin.cpu(), B, S, Hq, Hkv, D)
    (oc * do.cpu().float()).sum().backward()
    assert rel_err(o.cpu(), oc) < 2e-2
    assert rel_err(qkv.grad.cpu(), qc.grad) < 3e-2


@pytest.mark.parametrize("R,C", [(64, 64), (8192, 6144), (104, 200), (8, 4104)])
def test_transpose_exact(R, C):
    from kubeoperator_amd.ops.functional import transpose

    x = torch.randn(R, C + 16, device=DEV).to(torch.bfloat16)[:, 8:C + 8]  # strided, 16-B aligned rows
    y = transpose(x)
    assert y.shape == (C, R) and y.is_contiguous()
    assert torch.equal(y, x.t())


@pytest.mark.parametrize("layout", ["tn", "nt", "auto"])
def test_weight_grad_tn_layout_matches_nt(layout, monkeypatch):
    import kubeoperator_amd.ops.functional as kf

    monkeypatch.setattr(kf, "_DW_LAYOUT", layout)
    torch.manual_seed(11)
    for T, N, K in ((2048, 768, 512), (2048, 2048, 4096)):
        x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
        dy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
        out = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
        kf._dw_into(dy, x, out, False)
        ref = dy.float().t() @ x.float()
        assert rel_err(out, ref) < 1e-2
        kf._dw_into(dy, x, out, True)
        assert rel_err(out, 2 * ref) < 1e-2


@pytest.mark.parametrize("variant,cfg", [(10, 64), (10, 66), (10, 67), (10, 640), (10, 670), (10, 42), (10, 68), (9, 64),
                                         (9, 42), (8, 42), (0, 42)],
                         ids=["ds_blk-dkdv64", "ds-dkdv66", "ds_kmaj-dkdv67", "ds_blk-dkdv64_d64", "ds_kmaj-dkdv67_d64",
                              "ds-dkdv42", "ds_kmaj-dkdv68_d64", "recompute9-dkdv64", "recompute9", "recompute8",
                              "recompute4w"])
@pytest.mark.parametrize("D,Hq,Hkv,S", [(128, 8, 2, 512), (64, 4, 4, 256), (128, 4, 1, 768), (128, 8, 1, 256),
                                        (64, 8, 4, 512), (128, 4, 4, 512), (128, 6, 2, 512), (128, 2, 1, 256)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_bwd_dq_variants(variant, cfg, D, Hq, Hkv, S, causal):
    """every dQ algorithm (recompute 8/9, materialised dS 10) and dK/dV kernel (64 / 66: one wave per SIMD
    with the wave-block / row query-major dS staged through LDS, D = 128; 640: the same at D = 64; 42: two waves per
    SIMD) against the fp32 autograd reference. The shapes cover the
    no-GQA direct path (Hq == Hkv) and every dQ head grouping (8, 4, 2, 1 heads per workgroup)."""
    from kubeoperator_amd.ops.functional import rope_attention
    from kubeoperator_amd.ops.reference import attention_ref

    old = lib().flash_attn_set_dq_variant(variant)
    old_cfg = lib().flash_attn_set_dkdv_cfg(cfg)
    try:
        B = 2
        torch.manual_seed(12)
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=causal, use_rope=False)
        do = torch.randn_like(o)
        (o.float() * do.float()).sum().backward()
        x = qkv.detach().float().requires_grad_(True)
        a, c = Hq * D, (Hq + Hkv) * D
        of, _ = attention_ref(x[:, :a], x[:, a:c], x[:, c:], B, S, Hq, Hkv, D, causal)
        (of * do.float()).sum().backward()
        for lo, hi in ((0, a), (a, c), (c, x.shape[1])):
            assert rel_err(qkv.grad[:, lo:hi], x.grad[:, lo:hi]) < 3e-2
    finally:
        lib().flash_attn_set_dq_variant(old)
        lib().flash_attn_set_dkdv_cfg(old_cfg)


@pytest.mark.parametrize("shape", [43, 44, 83])
@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 256, 4, 4), (2, 1024, 12, 12), (1, 512, 8, 2), (2, 768, 6, 3)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_bwd_d64_two_wave(shape, B, S, Hq, Hkv, causal):
    """The D = 64 dK/dV kernel with two waves per SIMD (cfg 68, csrc/flash_bwd_d64.hip; every workgroup shape) against
    the fp32 autograd reference -- direct bf16 dK / dV (Hq == Hkv) and the fp32-partial GQA path -- and against the one-wave kernel
    (cfg 67): the same products in another summation order, so the gradients agree to bf16 rounding."""
    from kubeoperator_amd.ops.functional import rope_attention
    from kubeoperator_amd.ops.reference import attention_ref

    D = 64
    torch.manual_seed(B * S + Hq)
    qkv0 = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    do = torch.randn(B * S, Hq * D, device=DEV, dtype=torch.bfloat16)
    grads = {}
    old_cfg = lib().flash_attn_set_dkdv_cfg(68)
    old_shape = lib().flash_attn_set_d64_shape(shape)
    try:
        for cfg in (670, 68):
            lib().flash_attn_set_dkdv_cfg(cfg)
            qkv = qkv0.clone().requires_grad_(True)
            o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=causal, use_rope=False)
            (o.float() * do.float()).sum().backward()
            grads[cfg] = qkv.grad.float()
    finally:
        lib().flash_attn_set_dkdv_cfg(old_cfg)
        lib().flash_attn_set_d64_shape(old_shape)
    x = qkv0.float().requires_grad_(True)
    a, c = Hq * D, (Hq + Hkv) * D
    of, _ = attention_ref(x[:, :a], x[:, a:c], x[:, c:], B, S, Hq, Hkv, D, causal)
    (of * do.float()).sum().backward()
    assert torch.isfinite(grads[68]).all()
    for lo, hi in ((0, a), (a, c), (c, x.shape[1])):
        assert rel_err(grads[68][:, lo:hi], x.grad[:, lo:hi]) < 3e-2
        assert rel_err(grads[68][:, lo:hi], grads[670][:, lo:hi]) < 1e-2


@pytest.mark.parametrize("nw", [4, 8])
@pytest.mark.parametrize("D,Hq,Hkv,S", [(64, 4, 4, 256), (64, 8, 2, 512), (128, 8, 2, 512), (64, 12, 12, 1024),
                                        (128, 4, 1, 768)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_bwd_dq_workgroup_waves(nw, D, Hq, Hkv, S, causal):
    """The dQ-from-dS kernel with 4-wave (two per CU) and 8-wave workgroups, every head grouping it takes, against
    the fp32 reference (KOP_DQ_NW / flash_attn_set_dq_nw; 8 is forced whenever a group needs more than 4 heads)."""
    from kubeoperator_amd.ops.functional import rope_attention
    from kubeoperator_amd.ops.reference import attention_ref

    old = lib().flash_attn_set_dq_nw(nw)
    try:
        B = 2
        torch.manual_seed(17)
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=causal, use_rope=False)
        do = torch.randn_like(o)
        (o.float() * do.float()).sum().backward()
        x = qkv.detach().float().requires_grad_(True)
        a, c = Hq * D, (Hq + Hkv) * D
        of, _ = attention_ref(x[:, :a], x[:, a:c], x[:, c:], B, S, Hq, Hkv, D, causal)
        (of * do.float()).sum().backward()
        for lo, hi in ((0, a), (a, c), (c, x.shape[1])):
            assert rel_err(qkv.grad[:, lo:hi], x.grad[:, lo:hi]) < 3e-2
    finally:
        lib().flash_attn_set_dq_nw(old)


@pytest.mark.parametrize("hpw", [2, 4, 8])
@pytest.mark.parametrize("D,cfg,B,S,Hq,Hkv", [(128, 64, 1, 768, 8, 2), (128, 64, 2, 512, 8, 1), (128, 64, 1, 1024, 16, 2),
                                              (64, 640, 1, 512, 8, 1), (128, 67, 1, 768, 8, 2), (128, 67, 2, 512, 8, 1),
                                              (64, 670, 1, 512, 8, 1)])
@pytest.mark.parametrize("causal", [True, False])
def test_dkdv_head_sweep_matches_one_head_per_workgroup(hpw, D, cfg, B, S, Hq, Hkv, causal):
    """The one-wave dK/dV kernel sweeping HPW query heads of a GQA group per workgroup (csrc/flash_bwd_w1.hip: the
    issue cursor steps through the heads' stages and wraps to the next head; HPW == the group size writes bf16 dK / dV
    directly, fewer heads leave grp / HPW fp32 partials for the finalize pass). The test shapes are too small for the
    automatic choice to pick HPW > 1, so it is forced: gradients against the fp32 reference and against HPW 1."""
    from kubeoperator_amd.ops.functional import rope_attention
    from kubeoperator_amd.ops.reference import attention_ref

    if (Hq // Hkv) % hpw:
        pytest.skip("HPW must divide the GQA group")
    old_cfg = lib().flash_attn_set_dkdv_cfg(cfg)
    old_hpw = lib().flash_attn_set_dkdv_hpw(1)
    try:
        torch.manual_seed(13)
        qkv0 = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
        do = torch.randn(B * S, Hq * D, device=DEV, dtype=torch.bfloat16)
        grads = {}
        for h in (1, hpw):
            lib().flash_attn_set_dkdv_hpw(h)
            qkv = qkv0.clone().requires_grad_(True)
            o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=causal, use_rope=False)
            (o.float() * do.float()).sum().backward()
            grads[h] = qkv.grad.float()
        x = qkv0.float().requires_grad_(True)
        a, c = Hq * D, (Hq + Hkv) * D
        of, _ = attention_ref(x[:, :a], x[:, a:c], x[:, c:], B, S, Hq, Hkv, D, causal)
        (of * do.float()).sum().backward()
        for lo, hi in ((0, a), (a, c), (c, x.shape[1])):
            assert rel_err(grads[hpw][:, lo:hi], x.grad[:, lo:hi]) < 3e-2
            # same products, another fp32 summation order of the heads (registers vs partials): bf16-rounding close
            assert rel_err(grads[hpw][:, lo:hi], grads[1][:, lo:hi]) < 1e-2
    finally:
        lib().flash_attn_set_dkdv_cfg(old_cfg)
        lib().flash_attn_set_dkdv_hpw(old_hpw)


@pytest.mark.parametrize("rows,H", [(8192, 768), (8192, 2304), (4096, 3072), (77, 24), (1000, 1024)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_bias_grad_matches_reference(rows, H, accumulate):
    from kubeoperator_amd.ops import load

    g = torch.Generator(device="cuda").manual_seed(rows + H)
    dy = torch.randn(rows, H, device="cuda", generator=g).to(torch.bfloat16)
    db = torch.randn(H, device="cuda", generator=g).to(torch.bfloat16)
    ref = dy.float().sum(0) + (db.float() if accumulate else 0.0)
    load().bias_grad_(dy, db, accumulate)
    torch.cuda.synchronize()
    torch.testing.assert_close(db.float(), ref, atol=0.05 + 0.01 * ref.abs().max().item() / 10, rtol=1e-2)


@pytest.mark.parametrize("T,F", [(256, 128), (1024, 448)])
def test_swiglu_bwd_transposed_matches(T, F):
    """swiglu_bwd_t = swiglu_bwd plus the exact transpose of its output."""
    from kubeoperator_amd.ops import load

    lib = load()
    torch.manual_seed(3)
    gu = torch.randn(T, 2 * F, device=DEV).to(torch.bfloat16)
    dh = torch.randn(T, F, device=DEV).to(torch.bfloat16)
    ref = lib.swiglu_bwd(gu, dh)
    dgu, dgut = lib.swiglu_bwd_t(gu, dh)
    assert torch.equal(dgu, ref)
    assert dgut.shape == (2 * F, T) and torch.equal(dgut, ref.t())


@pytest.mark.parametrize("layout", ["tn", "nt"])
def test_linear_swiglu_matches_separate_ops(layout, monkeypatch):
    """The fused gate/up projection + SwiGLU node gives the same output and gradients as linear -> swiglu."""
    import kubeoperator_amd.ops.functional as kf

    monkeypatch.setattr(kf, "_DW_LAYOUT", layout)
    torch.manual_seed(5)
    T, H, F = 1024, 256, 320
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (0.05 * torch.randn(2 * F, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    dh = torch.randn(T, F, device=DEV).to(torch.bfloat16)
    h1 = kf.linear_swiglu(x, w)
    h1.backward(dh)
    gx1, gw1 = x.grad.clone(), w.grad.clone()
    x.grad = None
    w.grad = None
    h2 = kf.swiglu(kf.linear(x, w))
    h2.backward(dh)
    assert torch.equal(h1, h2)
    assert torch.equal(gx1, x.grad)
    assert rel_err(gw1, w.grad) < 1e-2


def test_swiglu_fwd_transposed_matches():
    from kubeoperator_amd.ops import load

    lib = load()
    torch.manual_seed(4)
    gu = torch.randn(512, 2 * 192, device=DEV).to(torch.bfloat16)
    h, ht = lib.swiglu_fwd_t(gu)
    assert torch.equal(h, lib.swiglu_fwd(gu)) and torch.equal(ht, h.t())


@pytest.mark.parametrize("layout", ["tn", "nt"])
def test_swiglu_mlp_matches_separate_ops(layout, monkeypatch):
    """The fused MLP node (h^T saved, dgu^T from the SwiGLU backward) matches linear -> swiglu -> linear."""
    import kubeoperator_amd.ops.functional as kf

    monkeypatch.setattr(kf, "_DW_LAYOUT", layout)
    torch.manual_seed(6)
    T, H, F = 1024, 256, 320
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16).requires_grad_(True)
    wgu = (0.05 * torch.randn(2 * F, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    wd = (0.05 * torch.randn(H, F, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    y1 = kf.swiglu_mlp(x, wgu, wd)
    y1.backward(dy)
    g1 = [t.grad.clone() for t in (x, wgu, wd)]
    for t in (x, wgu, wd):
        t.grad = None
    y2 = kf.linear(kf.swiglu(kf.linear(x, wgu)), wd)
    y2.backward(dy)
    assert torch.equal(y1, y2)
    for a, b in zip(g1, (x.grad, wgu.grad, wd.grad)):
        assert rel_err(a, b) < 1e-2
