"""Tensor parallelism (``parallel.tensor``) on CPU over gloo: a TP-sharded Llama (Q/K/V split by heads, Wo /
W_down split by rows of the reduction, gate|up by FFN columns) must train exactly like one process holding the
whole model -- same losses, and every rank's shards equal to the matching slices of the single process's
weights -- alone (tp 2) and combined with ZeRO-1 data parallelism across TP groups (tp 2 x dp 2)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from kubeoperator_amd.parallel.dist import DistInfo
from kubeoperator_amd.parallel.tensor import shard_llama_weight
from kubeoperator_amd.train import TrainConfig, Trainer


def _tc(**kw):
    base = dict(model="tiny_llama", micro_batch=2, seq_len=64, lr=1e-1, eps=1.0, warmup_steps=2, total_steps=20,
                bucket_mb=1)
    base.update(kw)
    return TrainConfig(**base)


def _batch(vocab, seed, mb, seq=64):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, vocab, (mb, seq + 1), generator=g)
    return ids[:, :-1].contiguous(), ids[:, 1:].contiguous()


def _full_init():
    ref = Trainer(_tc(), DistInfo())
    return {n: p.detach().clone() for n, p in ref.store.named_params()}


def _worker(rank, world, tp, init, mode, steps, out_q, sp=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      KOP_DIST_INIT=init)
    torch.set_num_threads(1)
    from kubeoperator_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed("cpu")
    tr = Trainer(_tc(tp=tp, dp_mode=mode, sp=sp), info)
    tr.load_full_weights(_full_init())
    dp, dpr = tr.dp_info.world, tr.dp_info.rank
    losses = []
    for step in range(steps):
        ids, tgt = _batch(tr.cfg.vocab_size, step, 2 * dp)
        losses.append(float(tr.train_step([(ids[2 * dpr:2 * dpr + 2], tgt[2 * dpr:2 * dpr + 2])])))
    out_q.put((rank, losses, {n: p.detach().float().numpy() for n, p in tr.store.named_params()},
               float(tr.opt.last_grad_norm)))
    shutdown(info)


def _run(world, tp, mode, tmp_path, steps=3, sp=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = f"file://{tmp_path}/rdzv-{world}-{tp}-{int(sp)}"
    procs = [ctx.Process(target=_worker, args=(r, world, tp, init, mode, steps, q, sp)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, losses, params, gn = q.get(timeout=600)
        res[r] = (losses, params, gn)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,tp,mode,sp", [(2, 2, "allreduce", False), (4, 2, "zero1", False),
                                              (2, 2, "zero1", True), (4, 2, "zero1", True), (4, 2, "allreduce", True)])
def test_tensor_parallel_matches_single_process(world, tp, mode, sp, tmp_path):
    """sp: sequence parallelism on top (norms / residual stream / LM head on 1/tp of the token rows)."""
    res = _run(world, tp, mode, tmp_path, sp=sp)
    dp = world // tp
    single = Trainer(_tc(micro_batch=2 * dp), DistInfo())
    single.load_full_weights(_full_init())
    init = {n: p.detach().float().clone() for n, p in single.store.named_params()}
    want_losses = [float(single.train_step([_batch(single.cfg.vocab_size, s, 2 * dp)])) for s in range(3)]
    want = {n: p.detach().float() for n, p in single.store.named_params()}
    cfg = single.cfg
    for rank, (losses, params, gn) in res.items():
        if dp == 1:  # one data stream: the TP job's loss is the single process's
            assert max(abs(a - b) for a, b in zip(losses, want_losses)) < 2e-2, (losses, want_losses)
        assert abs(gn - float(single.opt.last_grad_norm)) < 0.02 * float(single.opt.last_grad_norm)
        t = rank % tp
        num = den = 0.0
        for n, got in params.items():
            w = shard_llama_weight(n, want[n], cfg, tp, t)
            w0 = shard_llama_weight(n, init[n], cfg, tp, t)
            assert got.shape == tuple(w.shape), n
            num += float((torch.from_numpy(got) - w).pow(2).sum())
            den += float((w - w0).pow(2).sum())
        # eps >> |grad|: Adam's update is ~linear in the gradient, so a lost / doubled / misrouted shard
        # gradient is an O(1) error while bf16 reduction-order noise stays ~1 %
        assert (num / den) ** 0.5 < 0.05, (rank, (num / den) ** 0.5)


def test_tensor_parallel_shards_are_a_partition():
    """The shard map covers every element of every sharded weight exactly once."""
    from kubeoperator_amd.models import get_config

    cfg = get_config("tiny_llama")
    tp = 2
    D, F = cfg.head_dim, cfg.ffn_hidden
    for name, shape in (("layers.0.wqkv", ((cfg.n_heads + 2 * cfg.n_kv_heads) * D, cfg.hidden)),
                        ("layers.0.wo", (cfg.hidden, cfg.n_heads * D)), ("layers.0.w_gate_up", (2 * F, cfg.hidden)),
                        ("layers.0.w_down", (cfg.hidden, F))):
        full = torch.arange(shape[0] * shape[1], dtype=torch.float64).reshape(shape)
        parts = [shard_llama_weight(name, full, cfg, tp, r) for r in range(tp)]
        got = torch.cat([p.reshape(-1) for p in parts]).sort().values
        assert torch.equal(got, full.reshape(-1)), name
    with pytest.raises(ValueError, match="divisible"):
        Trainer(_tc(tp=3), DistInfo(world=3))


def test_llama3_70b_tp8_shards_fit_one_mi355x():
    """Llama-3-70B (70.55 B parameters) at tp 8: every rank holds 1/8 of the block projections plus the
    replicated embeddings / LM head / norms (10.66 B parameters), so weights + gradients + fp32 AdamW state
    (2 + 2 + 12 bytes per parameter) take ~171 GB of a rank's 288 GB of HBM before activations."""
    from kubeoperator_amd.models import build_model, get_config
    from kubeoperator_amd.parallel.tensor import TPContext

    cfg = get_config("llama3_70b")
    assert abs(cfg.num_params() - 70.55e9) < 0.01e9
    with torch.device("meta"):
        full = build_model(cfg)
        shard = build_model(cfg, TPContext(8, 0, None))
    blk = lambda m: sum(p.numel() for n, p in m.named_parameters() if n.startswith("layers.") and "norm" not in n)
    rest = lambda m: sum(p.numel() for n, p in m.named_parameters()) - blk(m)
    assert blk(shard) * 8 == blk(full) and rest(shard) == rest(full)
    per_rank = sum(p.numel() for p in shard.parameters())
    assert 16 * per_rank < 180e9, per_rank


def _ckpt_worker(rank, world, tp, sp, init, ckpt, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      KOP_DIST_INIT=init)
    torch.set_num_threads(1)
    from kubeoperator_amd.parallel.dist import init_distributed, shutdown
    from kubeoperator_amd.train import checkpoint

    info = init_distributed("cpu")
    a = Trainer(_tc(tp=tp, sp=sp, dp_mode="zero1"), info)
    dpr, dp = a.dp_info.rank, a.dp_info.world
    batches = [_batch(a.cfg.vocab_size, s, 2 * dp) for s in range(4)]
    mine = [(ids[2 * dpr:2 * dpr + 2], tgt[2 * dpr:2 * dpr + 2]) for ids, tgt in batches]
    for b in mine[:2]:
        a.train_step([b])
    checkpoint.save(a, ckpt, info)
    for b in mine[2:]:
        a.train_step([b])
    # a second trainer resumes from the step-2 checkpoint and replays steps 3-4
    b_ = Trainer(_tc(tp=tp, sp=sp, dp_mode="zero1", seed=99), info)
    assert checkpoint.load(b_, ckpt, info) == 2
    for b in mine[2:]:
        b_.train_step([b])
    same = bool(torch.equal(a.store.params, b_.store.params) and torch.equal(a.opt.exp_avg, b_.opt.exp_avg))
    out_q.put((rank, same, sorted(os.listdir(ckpt))))
    shutdown(info)


@pytest.mark.parametrize("world,tp,sp", [(2, 2, False), (4, 2, True)])
def test_tensor_parallel_checkpoint_resume_is_exact(world, tp, sp, tmp_path):
    """Per-TP-rank checkpoint trees: a resumed TP (+SP, x DP with ZeRO-1) job continues bit-identically."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ckpt = str(tmp_path / "ckpt")
    init = f"file://{tmp_path}/rdzv-ckpt"
    procs = [ctx.Process(target=_ckpt_worker, args=(r, world, tp, sp, init, ckpt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    for rank, same, listing in res:
        assert same, rank
        assert listing == [f"tp{t}_of{tp}" for t in range(tp)], listing
