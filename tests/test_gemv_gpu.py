"""Decode GEMV (``csrc/gemv.hip``): y = x . W^T for <= 8 token rows against an fp32 PyTorch reference, and the
generator's decode steps through it against the same steps through the library GEMMs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from kubeoperator_amd.ops import load

    return load()


@pytest.mark.parametrize("M", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1000, 1024), (28672, 4096), (13, 2048)])
def test_gemv_matches_fp32_reference(M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
    y = _lib().gemv(x, w)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_gemv_strided_rows_and_loud_refusals():
    torch.manual_seed(0)
    big = torch.randn(4, 3072, device="cuda").to(torch.bfloat16)
    x = big[:, :2048]  # row stride 3072, as a slice of a wider activation
    w = torch.randn(512, 2048, device="cuda").to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = _lib().gemv(x, w)
    assert (y.float() - ref).abs().max().item() / ref.abs().max().item() < 1e-2
    with pytest.raises(RuntimeError):  # K not a multiple of 1024
        _lib().gemv(torch.randn(2, 1000, device="cuda").to(torch.bfloat16),
                    torch.randn(8, 1000, device="cuda").to(torch.bfloat16))
    with pytest.raises(RuntimeError):  # more than 8 rows
        _lib().gemv(torch.randn(9, 1024, device="cuda").to(torch.bfloat16),
                    torch.randn(8, 1024, device="cuda").to(torch.bfloat16))


@pytest.mark.parametrize("graph", [False, True])
def test_decode_through_gemv_matches_gemm_path(graph):
    from kubeoperator_amd.models import build_model, get_config
    from kubeoperator_amd.serve import LlamaGenerator

    # head_dim 128, every projection's K a multiple of 1024: all four projections and the head take the GEMV
    cfg = get_config("tiny_llama", hidden=1024, n_heads=8, n_kv_heads=2, ffn_hidden=2048)
    m = build_model(cfg)
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_((1 + 0.1 * torch.randn(p.shape, generator=g)) if "norm" in n else 0.03 * torch.randn(p.shape, generator=g))
    m = m.to(device="cuda", dtype=torch.bfloat16)
    B, S = 3, 40
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=torch.Generator().manual_seed(1)).cuda()
    outs = []
    for use_gemv in (True, False):
        gen = LlamaGenerator(m, max_batch=B, max_seq=S + 8, graph=graph)
        gen._gemv = use_gemv
        gen.GEMV_ROWS = 8  # the default routes only batch 1; exercise the multi-row kernel through the generator
        assert gen._gemv_ok(torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16), m.layers[0].wqkv) == use_gemv
        logits = gen.prefill(ids)
        steps = []
        for t in range(4):  # fixed tokens: both paths decode the same sequences
            logits = gen.decode(ids[:, t])
            steps.append(logits)
        outs.append(torch.stack(steps))
    err = (outs[0] - outs[1]).abs().max().item() / outs[1].abs().max().item()
    assert err < 2e-2, err
