"""SwiGLU backward at Llama-3-8B shape (8192 x 14336): swiglu_bwd + transpose of dgu vs swiglu_bwd_t."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeoperator_amd.ops import load  # noqa: E402
from kubeoperator_amd.ops.functional import transpose  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


lib = load()
T, F = 8192, 14336
gu = torch.randn(T, 2 * F, device="cuda").to(torch.bfloat16)
dh = torch.randn(T, F, device="cuda").to(torch.bfloat16)
a = timeit(lambda: lib.swiglu_bwd(gu, dh))
b = timeit(lambda: transpose(lib.swiglu_bwd(gu, dh)))
c = timeit(lambda: lib.swiglu_bwd_t(gu, dh))
print(json.dumps({"swiglu_bwd_us": round(a, 1), "swiglu_bwd+transpose_us": round(b, 1), "swiglu_bwd_t_us": round(c, 1)}))
