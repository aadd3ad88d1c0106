"""FP8 GEMMs (OCP E4M3, gfx950) for the forward and data-gradient products of the Llama projections.

``--fp8`` (opt-in; the headline benchmark stays bf16): the four projections of every block (QKV, O, gate|up,
down) multiply E4M3 operands on the matrix cores at twice the bf16 rate -- hipBLASLt reaches 2.6-3.3 PF/s at
these shapes against 1.2-1.55 PF/s in bf16 (``tools/fp8_gemm_probe.py``). Per-tensor *current* scaling:
every operand is quantized right before its GEMM with scale = amax / 448 (``csrc/fp8.hip``: amax pass +
cast pass), so no amax history and no overflow. The weights are quantized once per optimizer step, per
bucket, right after the update lands (``FlatParamStore.refresh_fp8``), in both orientations (W for the
forward, the W^T copy for dX = dY . W). Weight gradients, attention, norms, the LM head and the optimizer
stay bf16 / fp32. Activations saved for backward stay bf16.
"""
from __future__ import annotations

import torch

FP8 = torch.float8_e4m3fn


def _lib():
    from . import load

    return load()


def quantize(x: torch.Tensor):
    """bf16 -> (E4M3 tensor of the same shape, fp32 dequantization scale), both on x's device."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=FP8, device=x.device)
    scale = torch.empty((), dtype=torch.float32, device=x.device)
    ws = torch.empty(1, dtype=torch.int32, device=x.device)
    _lib().fp8_quant_(x, out.view(torch.uint8), scale, ws)
    return out, scale


def quantize_into(x: torch.Tensor, out: torch.Tensor, scale: torch.Tensor) -> None:
    ws = torch.empty(1, dtype=torch.int32, device=x.device)
    _lib().fp8_quant_(x, out.view(torch.uint8), scale, ws)


def mm(a: torch.Tensor, b8_t: torch.Tensor, scale_b: torch.Tensor, out_dtype=torch.bfloat16) -> torch.Tensor:
    """a (bf16, quantized here) @ b8_t, where ``b8_t`` is the column-major view ``B8.t()`` of a row-major
    E4M3 matrix B8 with dequantization scale ``scale_b``."""
    a8, sa = quantize(a)
    return torch._scaled_mm(a8, b8_t, scale_a=sa, scale_b=scale_b, out_dtype=out_dtype)
