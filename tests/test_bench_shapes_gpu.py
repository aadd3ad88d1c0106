"""Kernel numerics at the shapes the benchmarks actually run (GPU only), each against a plain-PyTorch fp32
reference of the same op:

* flash attention forward + backward at the Llama-3-8B bench shape (B 1, S 8192, 32 / 8 heads, D 128, causal)
  and the GPT-2-small one (B 8, S 1024, 12 / 12 heads, D 64, causal) -- the grids there are 8-32x larger than
  the small-shape tests', which exercises the XCD-grouped, heaviest-first block order of ``attn_work``
  (csrc/attn_common.h) over every workgroup the bench launches;
* RMSNorm (fused residual) at T 8192, H 4096;
* the fused LM-head cross-entropy at T 8192, V 128256.

The attention reference runs one query head at a time (manual fp32 softmax backward), so its S x S matrices stay
at 256 MiB.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _attention_reference(qkv, do, B, S, Hq, Hkv, D):
    """fp32 causal attention forward + backward, one (batch, query head) at a time -> o, dqkv."""
    scale = 1.0 / math.sqrt(D)
    a, c = Hq * D, (Hq + Hkv) * D
    x = qkv.float()
    o = torch.zeros(B * S, a, device=DEV)
    dq = torch.zeros(B * S, a, device=DEV)
    dk = torch.zeros(B * S, Hkv * D, device=DEV)
    dv = torch.zeros(B * S, Hkv * D, device=DEV)
    mask = torch.ones(S, S, device=DEV, dtype=torch.bool).triu(1)
    for b in range(B):
        rows = slice(b * S, (b + 1) * S)
        for h in range(Hq):
            g = h // (Hq // Hkv)
            q = x[rows, h * D:(h + 1) * D]
            k = x[rows, a + g * D:a + (g + 1) * D]
            v = x[rows, c + g * D:c + (g + 1) * D]
            dO = do[rows, h * D:(h + 1) * D].float()
            s = (q @ k.t()) * scale
            s.masked_fill_(mask, float("-inf"))
            p = torch.softmax(s, -1)
            del s
            oh = p @ v
            o[rows, h * D:(h + 1) * D] = oh
            dv[rows, g * D:(g + 1) * D] += p.t() @ dO
            dp = dO @ v.t()
            delta = (dO * oh).sum(-1, keepdim=True)
            ds = p * (dp - delta)
            del p, dp
            dq[rows, h * D:(h + 1) * D] = (ds @ k) * scale
            dk[rows, g * D:(g + 1) * D] += (ds.t() @ q) * scale
            del ds
    return o, torch.cat([dq, dk, dv], 1)


@pytest.mark.parametrize("B,S,Hq,Hkv,D,cfg", [(1, 8192, 32, 8, 128, 64), (1, 8192, 32, 8, 128, 66),
                                               (1, 8192, 32, 8, 128, 67), (1, 8192, 32, 8, 128, 42),
                                               (8, 1024, 12, 12, 64, 42)],
                         ids=["llama3_8b", "llama3_8b-dkdv66", "llama3_8b-dkdv67_kmaj", "llama3_8b-dkdv42", "gpt2_small"])
def test_flash_attention_at_bench_shape(B, S, Hq, Hkv, D, cfg):
    from kubeoperator_amd.ops import load
    from kubeoperator_amd.ops.functional import rope_attention

    old_cfg = load().flash_attn_set_dkdv_cfg(cfg)
    try:
        _check_bench_shape(B, S, Hq, Hkv, D)
    finally:
        load().flash_attn_set_dkdv_cfg(old_cfg)


def _check_bench_shape(B, S, Hq, Hkv, D):
    from kubeoperator_amd.ops.functional import rope_attention

    torch.manual_seed(11)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = rope_attention(qkv, None, None, B, S, Hq, Hkv, D, causal=True, use_rope=False)
    do = torch.randn_like(o)
    o.backward(do)
    o_ref, dqkv_ref = _attention_reference(qkv.detach(), do, B, S, Hq, Hkv, D)
    assert rel_err(o, o_ref) < 2e-2
    a, c = Hq * D, (Hq + Hkv) * D
    g = qkv.grad.float()
    for name, sl in (("dq", slice(0, a)), ("dk", slice(a, c)), ("dv", slice(c, None))):
        err = rel_err(g[:, sl], dqkv_ref[:, sl])
        assert err < 3e-2, (name, err)
    # every query row was written: no workgroup of the remapped grid skipped (a dropped block leaves zeros)
    assert (o.float().abs().sum(1) > 0).all()
    # no worse than plain bf16 PyTorch (SDPA) on the same inputs, whole tensor and smallest-norm (row, head) slices
    from numerics import check_against_bf16

    ob, gb = _sdpa_bf16(qkv.detach(), do, B, S, Hq, Hkv, D)
    res = [check_against_bf16("o", o.reshape(-1, D), o_ref.reshape(-1, D), ob.reshape(-1, D))]
    for name, sl in (("dq", slice(0, a)), ("dk", slice(a, c)), ("dv", slice(c, None))):
        res.append(check_against_bf16(name, g[:, sl].reshape(-1, D), dqkv_ref[:, sl].reshape(-1, D),
                                      gb[:, sl].reshape(-1, D)))
    print("numerics vs plain bf16:", res)


def _sdpa_bf16(qkv, do, B, S, Hq, Hkv, D):
    x = qkv.detach().clone().requires_grad_(True)
    a, c = Hq * D, (Hq + Hkv) * D
    q = x[:, :a].reshape(B, S, Hq, D).transpose(1, 2)
    k = x[:, a:c].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    v = x[:, c:].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
    o = o.transpose(1, 2).reshape(B * S, a)
    o.backward(do)
    return o.detach().float(), x.grad.float()


def test_rmsnorm_at_bench_shape():
    from kubeoperator_amd.ops.functional import rms_norm

    torch.manual_seed(12)
    T, H = 8192, 4096
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    y, s = rms_norm(x, w, 1e-5, residual=r)
    dy, ds = torch.randn_like(y), torch.randn_like(y)
    ((y.float() * dy.float()).sum() + (s.float() * ds.float()).sum()).backward()
    xf, rf, wf = (t.detach().float().requires_grad_(True) for t in (x, r, w))
    sf = xf + rf
    sb = sf.to(torch.bfloat16).float()  # the kernel normalizes the bf16 sum it also returns
    yf = sb * torch.rsqrt(sb.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    ((yf * dy.float()).sum() + (sf * ds.float()).sum()).backward()
    assert rel_err(y, yf) < 2e-2
    assert rel_err(s, sf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(w.grad, wf.grad) < 3e-2  # column sum over 8192 rows (two-stage partials)
    # plain bf16 PyTorch on the same inputs
    from numerics import check_against_bf16

    xb, rb, wb = (t.detach().clone().requires_grad_(True) for t in (x, r, w))
    s_b = xb + rb
    yb = s_b * torch.rsqrt(s_b.pow(2).mean(-1, keepdim=True) + 1e-5) * wb
    ((yb * dy).sum() + (s_b * ds).sum()).backward()
    check_against_bf16("y", y, yf, yb)
    check_against_bf16("dx", x.grad, xf.grad, xb.grad)
    check_against_bf16("dw", w.grad.reshape(1, -1), wf.grad.reshape(1, -1), wb.grad.reshape(1, -1))


def test_cross_entropy_at_bench_shape():
    from kubeoperator_amd.ops.functional import cross_entropy_lmhead

    torch.manual_seed(13)
    T, H, V = 8192, 4096, 128256
    x = (0.5 * torch.randn(T, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    w = (0.02 * torch.randn(V, H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (T,), device=DEV)
    tgt[::97] = -100
    loss = cross_entropy_lmhead(x, w, tgt)
    loss.backward()
    xf, wf = (t.detach().float().requires_grad_(True) for t in (x, w))
    logits = (xf @ wf.t()).to(torch.bfloat16).float()
    lf = torch.nn.functional.cross_entropy(logits, tgt, ignore_index=-100)
    lf.backward()
    assert abs(loss.item() - lf.item()) < 1e-2 * max(1.0, lf.item())
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(w.grad, wf.grad) < 3e-2
    # plain bf16 PyTorch: bf16 logits, cross_entropy and its autograd on the same inputs
    from numerics import check_against_bf16

    xb, wb = (t.detach().clone().requires_grad_(True) for t in (x, w))
    torch.nn.functional.cross_entropy(xb @ wb.t(), tgt, ignore_index=-100).backward()
    check_against_bf16("dx", x.grad, xf.grad, xb.grad)
    check_against_bf16("dw", w.grad, wf.grad, wb.grad)
