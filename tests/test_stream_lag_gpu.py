"""Stream-race detection by forced lag: the optimizer stream (AdamW per bucket, ZeRO-1 gathers, weight-copy refresh,
each bucket's gate for the next forward) and the weight-gradient stream are made to run deterministically behind the
compute stream (``torch.cuda._sleep`` before every launch, ``ops.optim.OPTIM_LAG_CYCLES`` /
``ops.functional.SIDE_LAG_CYCLES``). With clipping off, where two unlagged runs agree bit for bit, a correctly
ordered program ends at BIT-IDENTICAL parameters with the lag too; any missing wait (a forward reading a bucket before its
update, a backward overwriting gradients AdamW still reads, a side-stream input reused too early) shows up as a
difference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

LAG = 1_000_000  # GPU clock cycles per launch


def _train(model, accum, optim_lag, side_lag, monkeypatch, wgrad="auto"):
    from kubeoperator_amd.ops import functional, optim
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    monkeypatch.delenv("KOP_WGRAD_STREAM", raising=False)
    monkeypatch.setattr(optim, "OPTIM_LAG_CYCLES", LAG if optim_lag else 0)
    monkeypatch.setattr(functional, "SIDE_LAG_CYCLES", LAG if side_lag else 0)
    tr = Trainer(TrainConfig(model=model, micro_batch=4, seq_len=256, grad_accum=accum, lr=1e-2, warmup_steps=1,
                             total_steps=10, bucket_mb=1, grad_clip=0.0, wgrad_stream=wgrad),
                 DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
    assert tr.opt.overlap and len(tr.store.buckets) > 1
    for step in range(3):
        g = torch.Generator().manual_seed(200 + step)
        mbs = []
        for _ in range(accum):
            ids = torch.randint(0, tr.cfg.vocab_size, (4, 257), generator=g)
            mbs.append((ids[:, :-1].cuda(), ids[:, 1:].cuda()))
        tr.train_step(mbs)
    tr.store.await_all()
    torch.cuda.synchronize()
    out = tr.store.params.detach().clone()
    monkeypatch.undo()
    return out


def _same(ref, ref2, lag, init_tol=5e-3):
    """Bit-identical where the unlagged step reproduces itself bit for bit; else within bf16 noise of it."""
    if torch.equal(ref, ref2):
        assert torch.equal(ref, lag), (lag.float() - ref.float()).abs().max().item()
    else:
        rel = ((lag.float() - ref.float()).norm() / ref.float().norm()).item()
        assert rel < init_tol, rel


@pytest.mark.parametrize("model", ["tiny_llama", "tiny_gpt2"])
@pytest.mark.parametrize("accum", [1, 3])
def test_lagging_optimizer_stream(model, accum, monkeypatch):
    ref = _train(model, accum, False, False, monkeypatch)
    ref2 = _train(model, accum, False, False, monkeypatch)
    lag = _train(model, accum, True, False, monkeypatch)
    _same(ref, ref2, lag)


def test_lagging_optimizer_and_side_streams(monkeypatch):
    ref = _train("tiny_gpt2", 2, False, False, monkeypatch, wgrad="on")
    ref2 = _train("tiny_gpt2", 2, False, False, monkeypatch, wgrad="on")
    lag = _train("tiny_gpt2", 2, True, True, monkeypatch, wgrad="on")
    _same(ref, ref2, lag)
