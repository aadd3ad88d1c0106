"""Embedding weight gradient kernel (csrc/embedding.hip) against the fp32 PyTorch reference: overwrite and accumulate,
bf16 and fp32 gradient buffers, uniform and heavily repeated (Zipf-like) token ids, GPT-2 and Llama widths. The run sum
is in token order (stable sort), so two launches on the same inputs must agree bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(ids, dy, V):
    out = torch.zeros(V, dy.shape[1], dtype=torch.float32, device=dy.device)
    out.index_add_(0, ids, dy.float())
    return out


def _ids(kind, T, V, g):
    if kind == "uniform":
        return torch.randint(0, V, (T,), generator=g)
    # Zipf-like: a few ids hold most of the tokens (runs of hundreds) -- the long-run path of the kernel
    r = torch.rand(T, generator=g)
    return torch.clamp((V ** r).long() - 1, 0, V - 1)


@pytest.mark.parametrize("V,H,T", [(50304, 768, 4096), (1000, 4096, 2048), (64, 520, 3000)])
@pytest.mark.parametrize("kind", ["uniform", "zipf"])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_embedding_bwd_matches_reference(V, H, T, kind, out_dtype):
    from kubeoperator_amd.ops import load

    lib = load()
    g = torch.Generator().manual_seed(V + H + T)
    ids = _ids(kind, T, V, g).cuda()
    dy = (torch.randn(T, H, generator=g) * 0.5).bfloat16().cuda()
    want = _ref(ids, dy, V)
    out = torch.full((V, H), 7.0, dtype=out_dtype, device="cuda")  # overwrite must clear untouched rows
    lib.embedding_bwd_(ids, dy, out, False)
    torch.cuda.synchronize()
    tol = 2e-2 if out_dtype == torch.bfloat16 else 1e-4
    err = (out.float() - want).abs().max().item()
    scale = want.abs().max().item() + 1e-6
    assert err <= tol * scale, (err, scale)
    # accumulate onto a prior gradient
    prior = (torch.randn(V, H, generator=g) * 0.1).to(out_dtype).cuda()
    acc = prior.clone()
    lib.embedding_bwd_(ids, dy, acc, True)
    want2 = prior.float() + want
    err2 = (acc.float() - want2).abs().max().item()
    assert err2 <= tol * (want2.abs().max().item() + 1e-6), err2
    # deterministic: a second launch gives the same bits
    out2 = torch.empty_like(out)
    lib.embedding_bwd_(ids, dy, out2, False)
    assert torch.equal(out, out2)


def test_embedding_autograd_writes_the_flat_gradient():
    """Through the model path (ops.functional.embedding): the gradient of the table equals the fp32 reference."""
    from kubeoperator_amd.ops import functional as kf

    g = torch.Generator().manual_seed(3)
    V, H, T = 5000, 256, 1024
    w = (torch.randn(V, H, generator=g) * 0.02).bfloat16().cuda().requires_grad_(True)
    ids = torch.randint(0, 97, (T,), generator=g).cuda()  # many repeats
    y = kf.embedding(ids, w)
    dy = torch.randn(T, H, generator=g).bfloat16().cuda()
    y.backward(dy)
    want = _ref(ids, dy, V)
    assert (w.grad.float() - want).abs().max().item() <= 2e-2 * want.abs().max().item()
