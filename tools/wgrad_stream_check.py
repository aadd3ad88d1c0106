"""Single-GPU check of the weight-gradient side stream: the same 3 training steps (tiny Llama, GPT-2) with the
side stream off, on, on again -- parameters must agree to bf16 reduction noise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model, stream, accum):
    os.environ["KOP_WGRAD_STREAM"] = "1" if stream else "0"
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    tr = Trainer(TrainConfig(model=model, micro_batch=8, seq_len=256, grad_accum=accum, lr=1e-1, eps=1.0,
                             warmup_steps=1, total_steps=10, bucket_mb=1), DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
    assert tr.store.wgrad_stream == stream
    init = torch.cat([p.detach().reshape(-1).float().cpu() for _, p in tr.store.named_params()])
    for step in range(3):
        g = torch.Generator().manual_seed(100 + step)
        mbs = []
        for i in range(accum):
            ids = torch.randint(0, tr.cfg.vocab_size, (8, 257), generator=g)
            mbs.append((ids[:, :-1].cuda(), ids[:, 1:].cuda()))
        tr.train_step(mbs)
    tr.store.await_all()
    torch.cuda.synchronize()
    return init, torch.cat([p.detach().reshape(-1).float().cpu() for _, p in tr.store.named_params()])


for model in ("tiny_llama", "tiny_gpt2"):
    for accum in (1, 4):
        init, off = run(model, False, accum)
        _, on1 = run(model, True, accum)
        _, on2 = run(model, True, accum)
        upd = (off - init).norm().item()
        print(f"{model} accum{accum}: on-vs-off {((on1 - off).norm() / upd).item():.4f} "
              f"on-vs-on {((on2 - on1).norm() / upd).item():.4f}", flush=True)
