"""FP8 GEMMs (OCP E4M3, gfx950) for the forward and data-gradient products of the Llama projections.

``--fp8`` (opt-in; the headline benchmark stays bf16): the four projections of every block (QKV, O, gate|up,
down) multiply E4M3 operands on the matrix cores at twice the bf16 rate -- hipBLASLt reaches 2.6-3.3 PF/s at
these shapes against 1.2-1.55 PF/s in bf16 (``tools/fp8_gemm_probe.py``). Per-tensor *current* scaling:
every operand is quantized right before its GEMM with scale = amax / 448 (``csrc/fp8.hip``: amax pass +
cast pass), so no amax history and no overflow. The weights are quantized once per optimizer step, per
bucket, right after the update lands (``FlatParamStore.refresh_fp8``), in both orientations (W for the
forward, the W^T copy for dX = dY . W). The weight gradient dW = dY^T X runs in E4M3 too: its K-contiguous
operands come from a transpose that writes E4M3 directly with the scale the operand already got for the
forward / data-gradient GEMM (``csrc/fp8.hip`` fp8_transpose_cast), or, where a kernel already produced the
transposed bf16 operand (SwiGLU's h^T and dgu^T), from a one-pass cast. Attention, norms, the LM head and
the optimizer stay bf16 / fp32; activations saved for backward stay bf16.
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
    quantize_into(x, out, scale)
    return out, scale


def quantize_into(x: torch.Tensor, out: torch.Tensor, scale: torch.Tensor) -> None:
    lib = _lib()
    ws = torch.empty(lib.FP8_AMAX_BLOCKS, dtype=torch.float32, device=x.device)  # per-workgroup partial maxima
    lib.fp8_quant_(x, out.view(torch.uint8), scale, ws)


def mm(a: torch.Tensor, b8_t: torch.Tensor, scale_b: torch.Tensor, out_dtype=torch.bfloat16) -> torch.Tensor:
    """a (bf16, quantized here) @ b8_t, where ``b8_t`` is the column-major view ``B8.t()`` of a row-major
    E4M3 matrix B8 with dequantization scale ``scale_b``."""
    a8, sa = quantize(a)
    return torch._scaled_mm(a8, b8_t, scale_a=sa, scale_b=scale_b, out_dtype=out_dtype)


def cast_scaled(x: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """E4M3 copy of bf16 ``x`` with a known dequantization scale (one pass)."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=FP8, device=x.device)
    _lib().fp8_cast_scaled_(x, scale, out.view(torch.uint8))
    return out


def transpose_cast(x: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """E4M3 [C, R] transpose of a bf16 [R, C] row view, with a known scale (one pass)."""
    out = torch.empty(x.shape[1], x.shape[0], dtype=FP8, device=x.device)
    _lib().fp8_transpose_cast_(x, scale, out.view(torch.uint8))
    return out


def mm8(a8, sa, b8_t, sb, out_dtype=torch.bfloat16) -> torch.Tensor:
    return torch._scaled_mm(a8, b8_t, scale_a=sa, scale_b=sb, out_dtype=out_dtype)


def wgrad_into(dyt8: torch.Tensor, sdy: torch.Tensor, xt8: torch.Tensor, sx: torch.Tensor, out: torch.Tensor,
               accumulate: bool) -> None:
    """out (+)= dY^T X from the E4M3 transposed operands dY^T [N, T] and X^T [K, T]."""
    if not accumulate and out.is_contiguous():
        torch.ops.aten._scaled_mm.out(dyt8, xt8.t(), sdy, sx, None, None, out.dtype, False, out=out)
        return
    res = torch._scaled_mm(dyt8, xt8.t(), scale_a=sdy, scale_b=sx, out_dtype=out.dtype)
    if accumulate:
        out.add_(res)
    else:
        out.copy_(res)

