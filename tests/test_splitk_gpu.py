"""Split-K weight gradients (ops.functional._dw_into at narrow widths, csrc/splitk.hip) against the fp32 PyTorch
reference: the reduction kernel alone, the whole dW = dY^T X at the GPT-2-small shapes (bf16 and fp32 gradient
buffers, overwrite and accumulate), and a GPT-2 training run with split-K on vs off."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S", [1, 3, 4, 16])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("acc", [False, True])
def test_splitk_reduce_kernel(S, out_dtype, acc):
    from kubeoperator_amd.ops.functional import _lib

    g = torch.Generator(device="cuda").manual_seed(S)
    part = torch.randn(S, 200, 72, device="cuda", generator=g)
    out = torch.randn(200, 72, device="cuda", generator=g).to(out_dtype)
    ref = part.sum(0) + (out.float() if acc else 0)
    _lib().splitk_reduce_(part, out, acc)
    tol = 1e-2 if out_dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("N,K", [(2304, 768), (768, 768), (3072, 768), (768, 3072)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_splitk_weight_gradient_matches_fp32(N, K, out_dtype):
    from kubeoperator_amd.ops import functional as F

    T = 32768
    s = F._splitk(T, N, K)
    assert s > 1  # the GPT-2-small shapes take the split path
    g = torch.Generator(device="cuda").manual_seed(N + K)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = dy.float().t() @ x.float()
    out = torch.empty(N, K, device="cuda", dtype=out_dtype)
    F._dw_into(dy, x, out, False)
    scale = ref.abs().max().item()
    assert ((out.float() - ref).abs().max() / scale).item() < 1e-2
    F._dw_into(dy, x, out, True)  # second micro-batch accumulates
    assert ((out.float() - 2 * ref).abs().max() / (2 * scale)).item() < 1e-2


def test_splitk_leaves_wide_gradients_alone():
    from kubeoperator_amd.ops import functional as F

    assert F._splitk(8192, 4096, 4096) == 1
    assert F._splitk(32768, 50304, 768) == 1
    assert F._splitk(2048, 768, 768) == 2  # chunks keep >= 1024 rows


@pytest.mark.parametrize("stream", ["off", "on"])
def test_gpt2_training_with_splitk_matches_unsplit(stream, monkeypatch):
    from kubeoperator_amd.ops import functional
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    def run(mode):
        monkeypatch.setattr(functional, "_DW_SPLITK", mode)
        monkeypatch.delenv("KOP_WGRAD_STREAM", raising=False)
        tr = Trainer(TrainConfig(model="tiny_gpt2", micro_batch=32, seq_len=256, grad_accum=2, lr=1e-2, warmup_steps=1,
                                 total_steps=10, bucket_mb=1, grad_clip=0.0, wgrad_stream=stream),
                     DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
        init = tr.store.params.detach().float().clone()
        for step in range(2):
            gen = torch.Generator().manual_seed(7 + step)
            mbs = []
            for _ in range(2):
                ids = torch.randint(0, tr.cfg.vocab_size, (32, 257), generator=gen)
                mbs.append((ids[:, :-1].cuda(), ids[:, 1:].cuda()))
            tr.train_step(mbs)
        tr.store.await_all()
        torch.cuda.synchronize()
        return init, tr.store.params.detach().float()

    init, off = run("off")
    _, on = run("auto")
    rel = ((on - off).norm() / (off - init).norm()).item()
    assert rel < 5e-3, rel
