"""Probe: torch._scaled_mm (hipBLASLt FP8) vs bf16 torch.mm at Llama-3-8B GEMM shapes on one MI355X."""
import json
import time

import torch


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it


dev = "cuda"
for fp8 in (torch.float8_e4m3fn, torch.float8_e4m3fnuz):
    try:
        a = torch.randn(64, 64, device=dev).to(fp8)
        b = torch.randn(64, 64, device=dev).to(fp8).t()
        one = torch.ones((), device=dev)
        torch._scaled_mm(a, b, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        print(json.dumps({"dtype": str(fp8), "ok": True}))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"dtype": str(fp8), "ok": False, "err": str(e)[:300]}))
for (m, n, k) in ((8192, 6144, 4096), (8192, 4096, 4096), (8192, 28672, 4096), (8192, 4096, 14336),
                  (8192, 128256, 4096), (4096, 4096, 8192), (14336, 4096, 8192)):
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    t_bf = bench(lambda: torch.mm(x, w.t()))
    rec = {"m": m, "n": n, "k": k, "bf16_tflops": round(2 * m * n * k / t_bf / 1e12, 1)}
    try:
        xf = x.to(torch.float8_e4m3fn)
        wf = w.to(torch.float8_e4m3fn)
        one = torch.ones((), device=dev)
        t8 = bench(lambda: torch._scaled_mm(xf, wf.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
        rec["fp8_tflops"] = round(2 * m * n * k / t8 / 1e12, 1)
        ref = (x.float() @ w.float().t())
        got = torch._scaled_mm(xf, wf.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16).float()
        rec["rel_err"] = round(((got - ref).norm() / ref.norm()).item(), 4)
    except Exception as e:  # noqa: BLE001
        rec["fp8_err"] = str(e)[:200]
    print(json.dumps(rec), flush=True)
