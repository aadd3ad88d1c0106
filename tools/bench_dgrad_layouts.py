"""dX = dY @ W at Llama-3-8B shapes: W as stored ([N_out, K_in], the reduction dim strided: hipBLASLt "NN")
against a transposed copy W^T ([K_in, N_out], reduction dim contiguous: the forward's "TN" form).
Prints ms and TFLOP/s per shape; TunableOp off (heuristic) and on (tuning both layouts briefly)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    T = 8192
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    tot = {"nn": 0.0, "tn": 0.0}
    for name, (N, K) in shapes.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        a = timeit(lambda: torch.mm(dy, w))
        b = timeit(lambda: torch.mm(dy, wt.t()))
        f = 2 * T * N * K
        tot["nn"] += a
        tot["tn"] += b
        print(json.dumps({"gemm": f"dgrad_{name}", "nn_ms": round(a, 4), "tn_ms": round(b, 4),
                          "nn_tflops": round(f / a / 1e9, 1), "tn_tflops": round(f / b / 1e9, 1)}), flush=True)
        del dy, w, wt
    print(json.dumps({"per_layer_set_ms": {k: round(v, 4) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
