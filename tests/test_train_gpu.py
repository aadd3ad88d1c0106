"""Training-loop properties on the GPU: the stream-overlapped optimizer (AdamW on its own stream, gated per
bucket into the next forward) must give exactly the same parameters as the serial optimizer."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(overlap: bool, steps: int = 4, bucket_mb: int = 1):
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
    tc = TrainConfig(model="tiny_llama", micro_batch=2, seq_len=256, warmup_steps=1, total_steps=10,
                     bucket_mb=bucket_mb, overlap_optimizer=overlap, grad_clip=0.0)
    tr = Trainer(tc, info)
    data = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=3)
    losses = [tr.train_step(data.batches(1)) for _ in range(steps)]
    tr.store.await_all()
    torch.cuda.synchronize()
    return tr, torch.stack(losses).float().cpu()


def test_overlapped_optimizer_matches_serial():
    """clipping off (its grad-norm uses float atomics): the serial run is then bit-reproducible, and a
    forward that read a bucket before its AdamW finished would show up as a bit difference."""
    ser, l_ser = _run(False)
    ser2, _ = _run(False)
    ovl, l_ovl = _run(True)
    assert ovl.opt.overlap and not ser.opt.overlap
    assert len(ovl.store.buckets) > 2  # small buckets: several gates per step
    assert ovl.store.use_order and ovl.store.use_order[0] != ovl.store.buckets[0].index
    noise = (ser.opt.master - ser2.opt.master).abs().max().item()
    diff = (ser.opt.master - ovl.opt.master).abs().max().item()
    assert diff <= 4 * noise, (diff, noise)
    if noise == 0:
        assert torch.equal(l_ser, l_ovl) and torch.equal(ser.store.params, ovl.store.params)



@pytest.mark.parametrize("overlap", [True, False])
def test_transposed_weight_copies_match(overlap):
    """dX through the refreshed W^T copies (forced on for the tiny model's 256-wide weights) must train like
    dX through W: same losses up to GEMM summation order, and every copy equal to its weight's transpose."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    def run(transposed):
        info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
        tc = TrainConfig(model="tiny_llama", micro_batch=2, seq_len=256, warmup_steps=1, total_steps=10,
                         bucket_mb=1, overlap_optimizer=overlap, transposed_weights=False)
        tr = Trainer(tc, info)
        if transposed:
            assert tr.store.enable_transposed(min_width=64) > 0
            tr.store.refresh_transposed()
        data = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=5)
        losses = torch.stack([tr.train_step(data.batches(2)) for _ in range(4)]).float().cpu()
        tr.store.await_all()
        torch.cuda.synchronize()
        return tr, losses

    ref, l_ref = run(False)
    tt, l_t = run(True)
    torch.testing.assert_close(l_t, l_ref, atol=2e-2, rtol=0)
    for name, p in tt.store.named_params():
        wt = getattr(p, "wt", None)
        if wt is not None:
            assert torch.equal(wt, p.detach().t()), name
    rel = ((tt.store.params.float() - ref.store.params.float()).norm() / ref.store.params.float().norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("model,transposed", [("tiny_llama", False), ("tiny_llama", True), ("tiny_gpt2", False)])
def test_model_gradients_match_cpu_reference(model, transposed):
    """Whole model, one forward + backward: the GPU path (HIP norms / RoPE / flash attention / SwiGLU or GELU
    / fused LM-head cross-entropy, hipBLASLt GEMMs, flat-buffer gradient sinks, optionally the W^T data-gradient
    path) against the CPU path (plain PyTorch ops in fp32 on the same bf16 weights)."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    tc = TrainConfig(model=model, micro_batch=2, seq_len=256, bucket_mb=1, transposed_weights=False)
    cpu = Trainer(tc, DistInfo())
    gpu = Trainer(tc, DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
    gpu.store.params.copy_(cpu.store.params.to("cuda"))
    if transposed:
        assert gpu.store.enable_transposed(min_width=64) > 0
        gpu.store.refresh_transposed()
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(0, cpu.cfg.vocab_size, (2, 257), generator=g)
    x, y = ids[:, :-1].contiguous(), ids[:, 1:].contiguous()
    for tr, dev in ((cpu, "cpu"), (gpu, "cuda")):
        tr.store.begin_microbatch(0)
        loss = tr.model(x.to(dev), y.to(dev))
        loss.backward()
        tr.loss_for_test = float(loss)
    torch.cuda.synchronize()
    assert abs(cpu.loss_for_test - gpu.loss_for_test) < 2e-2, (cpu.loss_for_test, gpu.loss_for_test)
    for name, p in cpu.store.named_params():
        gc = p.main_grad.float()
        gg = gpu.store.param(name).main_grad.float().cpu()
        rel = ((gg - gc).norm() / gc.norm().clamp_min(1e-12)).item()
        assert rel < 5e-2, (name, rel)


@pytest.mark.parametrize("model,accum", [("tiny_llama", 2), ("tiny_gpt2", 3), ("tiny_llama", 1)])
def test_hip_graph_replay_matches_eager(model, accum):
    """Micro-batches replayed as captured HIP graphs (first-micro-batch and accumulating graphs) give the same
    losses and parameters as the eager step (clipping off: bit-reproducible kernels)."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    def run(graph):
        info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
        tc = TrainConfig(model=model, micro_batch=2, seq_len=256, grad_accum=accum, warmup_steps=1, total_steps=10,
                         bucket_mb=1, grad_clip=0.0, cuda_graph=graph)
        tr = Trainer(tc, info)
        data = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=5)
        losses = [tr.train_step(data.batches(accum)) for _ in range(4)]
        tr.store.await_all()
        torch.cuda.synchronize()
        return tr, torch.stack(losses).float().cpu()

    eager, l_e = run(False)
    graphed, l_g = run(True)
    assert set(graphed._graphs) == ({0, 1} if accum > 1 else {0})
    assert torch.allclose(l_e, l_g, rtol=1e-3, atol=1e-3), (l_e, l_g)
    d = (eager.store.params.float() - graphed.store.params.float()).abs().max().item()
    assert d <= 2e-3, d


@pytest.mark.parametrize("model", ["tiny_llama", "tiny_gpt2"])
def test_fp32_gradient_buffer_matches_bf16_path(model):
    """``grad_dtype="fp32"``: every gradient sink (hipBLASLt GEMMs writing/accumulating fp32 through the
    mixed-dtype GEMM, staged norm/bias gradients, embedding) and the fp32-gradient AdamW / sum-of-squares
    kernels. Gradients after 3 accumulated micro-batches must match the bf16 buffer's to bf16 rounding, and
    an fp32 optimizer step must track the bf16 one."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    def run(gd):
        info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
        tc = TrainConfig(model=model, micro_batch=2, seq_len=256, grad_accum=3, warmup_steps=1, total_steps=10,
                         bucket_mb=1, grad_dtype=gd, transposed_weights=False)
        tr = Trainer(tc, info)
        data = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=11)
        batches = list(data.batches(3))
        for i, (x, y) in enumerate(batches):  # gradients only
            tr.store.begin_microbatch(i)
            tr.model(x, y).backward()
        torch.cuda.synchronize()
        grads = tr.store.grads.float().clone()
        loss = tr.train_step(iter(batches))
        tr.store.await_all()
        torch.cuda.synchronize()
        return tr, grads, float(loss)

    b16, g16, l16 = run("bf16")
    f32, g32, l32 = run("fp32")
    assert f32.store.grads.dtype == torch.float32
    rel = ((g32 - g16).norm() / g16.norm()).item()
    assert rel < 1e-2, rel
    assert abs(l16 - l32) < 1e-3
    assert torch.isfinite(f32.store.params.float()).all()
    prel = ((f32.store.params.float() - b16.store.params.float()).norm() / b16.store.params.float().norm()).item()
    assert prel < 1e-2, prel


def test_checkpoint_reshard_onto_gpu(tmp_path):
    """A checkpoint written by a CPU run with another bucket layout loads onto the GPU trainer through the
    resharding path (memory-mapped CPU shards copied into device state) and continues training."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer, checkpoint

    tc = dict(model="tiny_llama", micro_batch=2, seq_len=128, warmup_steps=1, total_steps=10, grad_clip=0.0)
    cpu = Trainer(TrainConfig(bucket_mb=1, **tc), DistInfo())
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, cpu.cfg.vocab_size, (2, 129), generator=g)
    batch = (ids[:, :-1].contiguous(), ids[:, 1:].contiguous())
    cpu.train_step([batch])
    checkpoint.save(cpu, str(tmp_path), DistInfo())
    info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))
    gpu = Trainer(TrainConfig(bucket_mb=0, **tc), info)
    assert gpu.layout()["pieces"] != cpu.layout()["pieces"]
    assert checkpoint.load(gpu, str(tmp_path), info) == 1
    for name, p in cpu.store.named_params():
        assert torch.equal(p, gpu.store.param(name).cpu()), name
    ma = torch.cat([cpu.opt.master[a:b] for a, b in [(x[2], x[2] + x[1] - x[0]) for x in cpu.layout()["pieces"]]])
    mg = torch.cat([gpu.opt.master[a:b].cpu() for a, b in [(x[2], x[2] + x[1] - x[0]) for x in gpu.layout()["pieces"]]])
    assert torch.equal(ma[ma != 0].sort().values, mg[mg != 0].sort().values)
    loss = gpu.train_step([(batch[0].cuda(), batch[1].cuda())])
    torch.cuda.synchronize()
    assert torch.isfinite(loss) and gpu.step == 2


@pytest.mark.parametrize("model", ["tiny_llama", "tiny_gpt2"])
def test_activation_recompute_matches_on_gpu(model):
    """Per-block recompute through the HIP kernels (flash attention forward re-run in backward, RoPE in place
    on the recomputed QKV) gives the gradients of the saved-activation run. The comparison is against the
    run-to-run noise of the same backward (the embedding gradient sums with float atomics)."""
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    info = DistInfo(0, 0, 1, "none", torch.device("cuda", 0))

    def grads(rc):
        tc = TrainConfig(model=model, micro_batch=2, seq_len=256, bucket_mb=1, recompute=rc, wgrad_stream="off",
                         seed=11)
        tr = Trainer(tc, info)
        ids, tgt = SyntheticTokens(tr.cfg.vocab_size, 2, 256, info.device, seed=5).next()
        tr.store.begin_microbatch(0)
        loss = tr.model(ids, tgt)
        loss.backward()
        tr.store.join_side()
        torch.cuda.synchronize()
        assert tr.model.recompute == rc
        return float(loss), tr.store.grads.float().clone()

    l0, g0 = grads(False)
    _, g1 = grads(False)
    l2, g2 = grads(True)
    assert l0 == l2  # the forward is the same computation
    scale = g0.norm().item()
    noise = (g0 - g1).norm().item() / scale
    diff = (g0 - g2).norm().item() / scale
    assert diff <= 4 * noise + 1e-3, (diff, noise)


@pytest.mark.gpu
def test_rccl_selftest_bench_one_rank():
    """bench.py under torchrun with KOP_RCCL_SELFTEST=1 on the GPU: the process group is RCCL ("nccl" on ROCm) and
    every data-parallel collective of the step -- ZeRO-1 reduce-scatter and all-gather, grad-norm all-reduce,
    barriers -- runs through it, matching the plain one-rank step's loss."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    args = ["--model", "tiny_llama", "--seq", "256", "--mbs", "2", "--accum", "2", "--steps", "2", "--warmup", "1",
            "--bucket-mb", "1", "--gemm-tuning", "off"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"

    def run(cmd, extra):
        p = subprocess.run(cmd, cwd=root, env={**env, **extra}, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
        assert len(lines) == 1, p.stdout[-2000:]
        return lines[0]

    r = run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
             "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "1"] + args,
            {"KOP_RCCL_SELFTEST": "1"})
    assert r["backend"] == "nccl" and r["rccl_world"] == 1
    assert r["config"]["parallelism"] == "dp1-zero1"
    assert r["grad_comm_bytes_per_step"] > 0 and r["param_gather_bytes_per_step"] > 0
    assert r["exposed_comm_ms"] is not None
    plain = run([sys.executable, "bench.py", "--gpus", "1"] + args, {})
    assert plain["backend"] == "none"
    assert abs(plain["last_loss"] - r["last_loss"]) < 2e-2, (plain["last_loss"], r["last_loss"])
