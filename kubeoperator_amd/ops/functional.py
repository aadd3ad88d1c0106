"""Autograd wrappers around the gfx950 kernels.

GPU tensors always take the HIP path (``ops.load()`` raises if the extension is missing); CPU tensors take
the fp32 reference path so the whole trainer can be exercised in CPU-only CI.

Weight gradients follow the flat-buffer protocol of :class:`kubeoperator_amd.parallel.flat.FlatParamStore`:
a parameter that carries ``main_grad`` (a view into the store's flat bf16 -- or, with ``grad_dtype=fp32``,
fp32 -- gradient buffer) gets its gradient
written (or accumulated, for gradient-accumulation micro-batches) straight into that view by the backward
kernel / GEMM (``torch.mm(..., out=main_grad)``), and the store is notified so the data-parallel layer can
launch the bucket's collective immediately -- no AccumulateGrad pass, no extra copy.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import reference as ref


def _lib():
    from . import load

    return load()


# ---------------------------------------------------------------------------------------------------
# weight-gradient sink
# ---------------------------------------------------------------------------------------------------
# Weight gradients on a second HIP stream: the backward's critical path is the data-gradient chain (dX feeds
# the next layer); the weight-gradient GEMMs (and their operand transposes) only feed the flat gradient buffer.
# Issued on the store's side stream, they run beside the next layer's kernels instead of between them.
# ``inputs`` are the tensors ``produce`` reads. Two hazards follow from reading them on another stream:
#
# * memory reuse: the store keeps a reference to every input until the side stream has passed the launch that reads
#   it (``FlatParamStore.hold_side``), so the caching allocator cannot hand the memory out earlier (no
#   ``record_stream``: it would hold each block until the side stream's whole queue at free time has run);
# * in-place accumulation by autograd: when a gradient tensor reaches a node that already holds another
#   contribution for the same input, autograd adds the two IN PLACE into whichever buffer it holds the last
#   reference to (``InputBuffer::accumulate``, ``can_accumulate_inplace``). The residual stream makes that
#   happen: block 0's first norm reads the embedding output ``x`` and passes it on as the residual ``x1``, so
#   ``x`` gets two gradients -- the second norm's (which is also the ``dY`` of the Wo / proj projection) and the
#   first norm's. With the side stream lagging, ``dY += dX1`` ran on the compute stream before the side stream's
#   dW_o read ``dY``, so Wo of layer 0 received the gradient of dY + dX1 (the round-2 divergence: rel. error 0.29,
#   identical across runs). The same references make autograd allocate a fresh sum instead of writing into it.
#
# Measured on one MI355X (profiles/r2_wgrad_stream_ab.log): GPT-2-small +8 % (its 768-wide GEMMs leave the chip
# partly idle), Llama-3-8B -30..-50 % (two full-chip stream-K GEMMs contend), so the trainer enables it per
# parameter store for narrow models only (``FlatParamStore.wgrad_stream``; ``KOP_WGRAD_STREAM=0/1`` forces it).

# test hook: GPU cycles of ``torch.cuda._sleep`` enqueued on the side stream before every weight gradient, so the
# side stream deterministically lags the compute stream (tests/test_wgrad_stream_gpu.py)
SIDE_LAG_CYCLES = int(os.environ.get("KOP_SIDE_LAG_CYCLES", "0"))


# norm weight / bias gradient folds on the side stream (KOP_NORM_SIDE=1). Round 5 kept them there (+0.7 % on GPT-2-small);
# with the grouped side launches, no record_stream and the 64 x 2 shape they are cheaper inside the norm backward:
# off +0.2..1.3 % over five same-box alternations (profiles/r6_gpt2_norm_side_ab_1.jsonl, _2.jsonl)
_NORM_SIDE = os.environ.get("KOP_NORM_SIDE", "0") == "1"


def _side_active(w) -> bool:
    """The weight-gradient side stream takes launches for ``w`` (the flat store runs one, not under capture)."""
    hooks = getattr(w, "_kop_hooks", None)
    return (hooks is not None and hooks.store.wgrad_stream and w.is_cuda
            and not torch.cuda.is_current_stream_capturing())


def _lagged(launch):
    """``launch`` behind the forced side-stream lag (race tests; no-op by default)."""
    def run():
        if SIDE_LAG_CYCLES > 0:
            torch.cuda._sleep(SIDE_LAG_CYCLES)
        launch()
    return run


def _side_launch(w, launch, *inputs, ready=()) -> None:
    """Run ``launch()`` on ``w``'s weight-gradient stream once it has caught up with the compute stream; ``inputs``
    stay alive (and their memory unreused) until that stream has passed them; the parameters in ``ready`` are marked
    ready once it is issued (``FlatParamStore.side_submit``: possibly grouped with the next launches)."""
    w._kop_hooks.store.side_submit(_lagged(launch), inputs, ready)


def _sink(w: torch.Tensor, produce, *inputs, defer: bool = False):
    """``produce(out, accumulate)`` writes the gradient of ``w``; returns what autograd should receive.

    ``defer``: with the side stream on and a later micro-batch to come (``FlatParamStore.defer_ok``), only the
    bookkeeping happens now (accumulate flag, readiness, an event marking the inputs ready on the compute stream) and
    the launches are issued by ``FlatParamStore.run_deferred`` after the NEXT micro-batch's forward has been queued:
    a gradient whose host-side launch sequence is long (the embedding's sort + run sum) then no longer holds the host
    while the compute stream runs dry at the micro-batch boundary."""
    mg = getattr(w, "main_grad", None)
    if mg is None:
        g = torch.empty_like(w)
        produce(g, False)
        return g
    hooks = w._kop_hooks
    acc = hooks.accumulate_for(w)
    store = hooks.store
    if defer and store.wgrad_stream and store.defer_ok and mg.is_cuda and not torch.cuda.is_current_stream_capturing():
        ready = torch.cuda.Event()
        ready.record()

        def launch():
            side = store.side_stream()
            side.wait_event(ready)
            with torch.cuda.stream(side):
                if SIDE_LAG_CYCLES > 0:
                    torch.cuda._sleep(SIDE_LAG_CYCLES)
                produce(mg, acc)
            store.hold_side(inputs)

        store.defer(launch)
        hooks.ready(w)
        return None
    if hooks.store.wgrad_stream and mg.is_cuda and not torch.cuda.is_current_stream_capturing():
        store.side_submit(_lagged(lambda: produce(mg, acc)), inputs, (w,))
        return None
    produce(mg, acc)
    hooks.ready(w)
    return None


def _gate(*ws):
    """Order the compute stream after the optimizer stream's update of these weights (parallel.flat gates)."""
    for w in ws:
        h = getattr(w, "_kop_hooks", None)
        if h is not None:
            h.store.await_param(w)


_MM_DTYPE_OUT = [True]  # aten's mixed-dtype GEMM (bf16 operands, fp32 output) available on this build


def _mm_into(a, b, out, accumulate):
    if out.dtype != a.dtype:
        # fp32 gradient buffer (``--grad-dtype fp32``) fed by bf16 operands: the GEMM accumulates in fp32 and
        # writes / adds fp32 directly; without the mixed-dtype kernel the bf16 product is added in fp32
        if _MM_DTYPE_OUT[0]:
            try:
                if accumulate:
                    torch.ops.aten.addmm.dtype_out(out, a, b, out.dtype, beta=1, alpha=1, out=out)
                else:
                    torch.ops.aten.mm.dtype_out(a, b, out.dtype, out=out)
                return
            except (RuntimeError, NotImplementedError):
                _MM_DTYPE_OUT[0] = False
        prod = torch.mm(a, b)
        if accumulate:
            out.add_(prod)
        else:
            out.copy_(prod)
        return
    if accumulate:
        out.addmm_(a, b)
    else:
        torch.mm(a, b, out=out)


# weight gradients dW = dY^T X through the forward ("TN") GEMM layout: hipBLASLt runs the strided "NT"
# form at ~1.15 PF/s and the K-contiguous form at ~1.55 PF/s on MI355X at Llama-3-8B widths; two HIP
# transposes at HBM speed cost far less than the difference there (tools/bench_gemm_layouts.py,
# csrc/transpose.hip). At GPT-2-small widths (768-3072) the GEMMs are short and the transposes are not
# repaid: the step is 4.6 % faster without them (profiles/r1_experiments.md). "auto" picks per GEMM by
# the narrower of its two output dimensions.
_DW_LAYOUT = os.environ.get("KOP_DW_LAYOUT", "auto")
_DW_TN_MIN_ROWS = 1024
_DW_TN_MIN_WIDTH = 2048


def _rows_ok(t: torch.Tensor) -> bool:
    return (t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.shape[1] % 8 == 0 and t.data_ptr() % 16 == 0)


def transpose(x: torch.Tensor) -> torch.Tensor:
    """Contiguous [C, R] copy of a bf16 [R, C] row view (HIP kernel)."""
    out = torch.empty(x.shape[1], x.shape[0], dtype=x.dtype, device=x.device)
    _lib().transpose_(x, out)
    return out


def transpose_into(x: torch.Tensor, out: torch.Tensor) -> None:
    """out[c, r] = x[r, c] (bf16, HIP kernel on GPU)."""
    if x.is_cuda:
        _lib().transpose_(x, out)
    else:
        out.copy_(x.t())


def _dx(dy2, w):
    """dX = dY . W through the transposed copy when the flat store keeps one (K-contiguous GEMM layout);
    in E4M3 when the store keeps an FP8 copy of it (``--fp8``, ops/fp8.py)."""
    wt8 = getattr(w, "wt8", None)
    if wt8 is not None:
        from . import fp8

        return fp8.mm(dy2, wt8.t(), w.wt8_scale, out_dtype=dy2.dtype)
    wt = getattr(w, "wt", None)
    return torch.mm(dy2, wt.t()) if wt is not None else torch.mm(dy2, w)


def _fwd(x2, w):
    """Y = X . W^T (E4M3 operands when the store keeps an FP8 copy of W)."""
    return _fwd8(x2, w)[0]


def _fwd8(x2, w):
    """(Y = X . W^T, X's E4M3 dequantization scale or None): the scale is kept for the E4M3 weight gradient."""
    w8 = getattr(w, "w8", None)
    if w8 is not None:
        from . import fp8

        M = x2.shape[0]
        if M % 16:  # hipBLASLt's E4M3 GEMMs want 16-row multiples: pad (decode steps of a few sequences)
            x2 = torch.cat([x2, x2.new_zeros(16 - M % 16, x2.shape[1])])
        x8, sx = fp8.quantize(x2)
        return fp8.mm8(x8, sx, w8.t(), w.w8_scale, out_dtype=x2.dtype)[:M], sx
    return torch.mm(x2, w.t()), None


def _fp8_bwd(w, sx) -> bool:
    """E4M3 data- and weight-gradient GEMMs: W has its E4M3 transposed copy and X was quantized in forward."""
    return sx is not None and getattr(w, "wt8", None) is not None


def _dx8(dy2, w):
    """dX = dY . W in E4M3 -> (dX, dY contiguous, dY's scale)."""
    from . import fp8

    dy2 = dy2.contiguous()
    dy8, sdy = fp8.quantize(dy2)
    return fp8.mm8(dy8, sdy, w.wt8.t(), w.wt8_scale, out_dtype=dy2.dtype), dy2, sdy


# Narrow weight gradients (GPT-2-small: 768 x 768 ... 3072 x 768 over T = 32768 rows) are a few dozen 256 x 256
# output tiles for 256 CUs: split the token rows into s chunks as ONE batched GEMM with fp32 outputs, then fold
# the partial planes into the gradient with one HIP pass (csrc/splitk.hip). s doubles while s x tiles stays
# within half the CUs' worth of tiles, up to 16; at Llama widths (>= 256 tiles) s = 1. One MI355X
# (profiles/r3_wgrad_splitk_probe.jsonl): proj 0.124 -> 0.059 ms, qkv 0.230 -> 0.155, out 0.232 -> 0.176.
_DW_SPLITK = os.environ.get("KOP_DW_SPLITK", "auto")  # auto | off | fixed split count
_DW_SPLITK_MIN_ROWS = 1024  # rows per chunk


def _splitk(T: int, N: int, K: int) -> int:
    if _DW_SPLITK == "off":
        return 1
    if _DW_SPLITK.isdigit():
        s = int(_DW_SPLITK)
    else:
        tiles = -(-N // 256) * -(-K // 256)
        s = 1
        while s < 16 and tiles * s * 2 <= 256:
            s *= 2
    while s > 1 and (T % s or T // s < _DW_SPLITK_MIN_ROWS or (T // s) % 8):
        s //= 2
    return s


def _dw_splitk_into(dy2, x2, out, accumulate, s):
    T, N = dy2.shape
    c = T // s
    part = torch.bmm(dy2.view(s, c, N).transpose(1, 2), x2.view(s, c, x2.shape[1]), out_dtype=torch.float32)
    _lib().splitk_reduce_(part, out, accumulate)


def _dw_into(dy2, x2, out, accumulate):
    """out (+)= dy2^T @ x2, the reduction running over the token rows."""
    wide = min(dy2.shape[1], x2.shape[1]) >= _DW_TN_MIN_WIDTH
    if ((_DW_LAYOUT == "tn" or (_DW_LAYOUT == "auto" and wide)) and dy2.shape[0] >= _DW_TN_MIN_ROWS
            and dy2.shape[0] % 8 == 0 and _rows_ok(dy2) and _rows_ok(x2)):
        _mm_into(transpose(dy2), transpose(x2).t(), out, accumulate)
        return
    s = _splitk(dy2.shape[0], dy2.shape[1], x2.shape[1])
    if (s > 1 and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and dy2.is_contiguous()
            and x2.is_contiguous() and out.is_contiguous() and out.numel() % 8 == 0):
        _dw_splitk_into(dy2, x2, out, accumulate, s)
    else:
        _mm_into(dy2.t(), x2, out, accumulate)


_BIAS_HIP = os.environ.get("KOP_BIAS_GRAD", "hip") == "hip"


def _bias_grad_into(dy2, out, accumulate):
    """out (+)= dy2.sum(0): HIP row-chunk partials + column reduce (csrc/norms.hip) for bf16 row matrices."""
    if (_BIAS_HIP and dy2.dtype == torch.bfloat16 and dy2.is_contiguous() and dy2.shape[1] % 8 == 0 and dy2.data_ptr() % 16 == 0
            and out.dtype == torch.bfloat16 and out.is_contiguous()):
        _lib().bias_grad_(dy2, out, accumulate)
        return
    s = dy2.sum(0, dtype=torch.float32)
    if accumulate:
        out.add_(s.to(out.dtype))
    else:
        out.copy_(s)


# ---------------------------------------------------------------------------------------------------
# linear
# ---------------------------------------------------------------------------------------------------
def _tp_reduce_async(dx, group):
    """Tensor parallelism, column-split projection: start summing the input gradient over the TP group on
    RCCL's stream (returns the work, or None) so it overlaps the weight-gradient GEMM that follows."""
    if group is None or dx is None:
        return None
    import torch.distributed as dist

    return dist.all_reduce(dx, group=group, async_op=True)


def _dw_t_into(dy2, x2, xt, dyt, out, acc):
    """dW (+)= dY^T X with either K-contiguous operand possibly supplied by its producer (``xt`` = X^T from the
    norm forward, ``dyt`` = dY^T from the norm backward); the missing one is transposed here."""
    if dyt is None:
        dyt = transpose(dy2) if _rows_ok(dy2) else None
    if dyt is None:
        _mm_into(dy2.t(), xt.t() if xt is not None else x2, out, acc)
        return
    _mm_into(dyt, xt.t() if xt is not None else (transpose(x2).t() if _rows_ok(x2) else x2), out, acc)


class _Linear(Function):
    @staticmethod
    def forward(ctx, x, w, b, tp_group=None, xt=None, box=None):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.tp_group = tp_group
        ctx.sx = None
        if b is not None:
            y = torch.addmm(b, x2, w.t())
        else:
            y, ctx.sx = _fwd8(x2, w)
        ctx.has_xt = xt is not None and ctx.sx is None
        # with X^T from the producer only X^T is kept for backward (the same bytes as X)
        ctx.save_for_backward(xt if ctx.has_xt else x2, w)
        ctx.has_b = b is not None
        if b is not None:
            ctx.b = b
        ctx.in_shape = x.shape
        ctx.box = box
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        dyt = ctx.box.take(dy2) if ctx.box is not None else None
        if _fp8_bwd(w, ctx.sx):
            from . import fp8

            dx, dy2, sdy = _dx8(dy2, w)
            work = _tp_reduce_async(dx, ctx.tp_group)
            dx = dx.view(ctx.in_shape)
            sx = ctx.sx
            dw = _sink(w, lambda out, acc: fp8.wgrad_into(fp8.transpose_cast(dy2, sdy), sdy,
                                                          fp8.transpose_cast(x2, sx), sx, out, acc),
                       dy2, x2, sdy, sx) if ctx.needs_input_grad[1] else None
            if work is not None:
                work.wait()
            return dx, dw, None, None, None, None
        dx = _dx(dy2, w) if ctx.needs_input_grad[0] else None
        work = _tp_reduce_async(dx, ctx.tp_group)
        dx = dx.view(ctx.in_shape) if dx is not None else None
        dw = None
        if ctx.needs_input_grad[1]:
            if ctx.has_xt or dyt is not None:
                xt = x2 if ctx.has_xt else None
                xr = None if ctx.has_xt else x2
                dw = _sink(w, lambda out, acc: _dw_t_into(dy2, xr, xt, dyt, out, acc),
                           *[t for t in (dy2, x2, dyt) if t is not None])
            else:
                dw = _sink(w, lambda out, acc: _dw_into(dy2, x2, out, acc), dy2, x2)
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = _sink(ctx.b, lambda out, acc: _bias_grad_into(dy2, out, acc), dy2)
        if work is not None:
            work.wait()
        return dx, dw, db, None, None, None


def linear(x, w, b=None, tp_group=None, xt=None, box=None):
    """``tp_group``: ``w`` is a column shard of a tensor-parallel projection (``parallel.tensor``) whose input is
    replicated over the group; the input gradient is summed over it, overlapped with the weight gradient.
    ``xt``: X^T from the producer of ``x`` (``rms_norm(want_t=True)``); ``box``: a ``TBox`` that the consumer of
    the output fills with dY^T in backward (``rms_norm(box=)``). Both feed the weight-gradient GEMM."""
    if not x.is_cuda:
        if tp_group is not None:
            from ..parallel.tensor import _CopyToTP

            x = _CopyToTP.apply(x, tp_group)
        return F.linear(x, w, b)
    _gate(w, b)
    return _Linear.apply(x, w, b, tp_group, xt, box)


# ---------------------------------------------------------------------------------------------------
# RMSNorm / LayerNorm with fused residual add
# ---------------------------------------------------------------------------------------------------
class TBox:
    """Hands the transposed copy of a gradient from the autograd node that produced it to the node that consumes it
    as dY (the model creates one per producer / consumer pair in forward). The norm backward fills it
    (``rms_norm_bwd_t``), the projection's backward takes it for its weight-gradient GEMM. ``take`` returns it
    only for the very tensor that was put -- same storage, shape and version: if autograd summed another
    contribution into the gradient in place, or handed the consumer a new tensor, the consumer transposes as
    before."""

    __slots__ = ("t", "key")

    def __init__(self):
        self.t = None
        self.key = None

    def put(self, g, gt):
        self.t, self.key = gt, (g.data_ptr(), tuple(g.shape), g._version)

    def take(self, g):
        t, key = self.t, self.key
        self.t = self.key = None
        if t is not None and key == (g.data_ptr(), tuple(g.shape), g._version):
            return t
        return None


_NORM_T = os.environ.get("KOP_NORM_T", "1") != "0"


def norm_t_enabled() -> bool:
    """Transposed-companion norms on (``KOP_NORM_T=0`` turns them off: the projections transpose as before)."""
    return _NORM_T and _DW_LAYOUT != "nt"


def _t_ok(x2) -> bool:
    """Shapes the transposed-companion RMSNorm kernels take (csrc/norms.hip rms_fwd_t / rms_bwd_t)."""
    return x2.dim() == 2 and x2.shape[1] in (2048, 4096) and x2.shape[0] % 16 == 0 and x2.shape[0] >= _DW_TN_MIN_ROWS


class _Norm(Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, eps, layernorm, want_t=False, box=None):
        lib = _lib()
        x = x.contiguous()
        has_res = residual is not None
        yt = None
        if want_t:
            y, s, rstd, yt = lib.rms_norm_fwd_t(x, residual.contiguous() if has_res else None, w, eps)
            mean = None
            ctx.mark_non_differentiable(yt)
            ctx.set_materialize_grads(False)  # no zero-filled [H, T] "gradient" of y^T
        else:
            y, s, rstd, mean = lib.norm_fwd(x, residual.contiguous() if has_res else None, w, b, eps, layernorm)
        if not has_res:
            s = x
        ctx.save_for_backward(s, w, rstd, mean if layernorm else None)
        ctx.layernorm = layernorm
        ctx.has_res = has_res
        ctx.b = b
        ctx.box = box
        ctx.want_t = want_t
        out = (y, s) if has_res else (y,)
        if want_t:
            out = out + (yt,)
        return out if len(out) > 1 else y

    @staticmethod
    def backward(ctx, dy, *rest):
        lib = _lib()
        s, w, rstd, mean = ctx.saved_tensors
        ds_extra = rest[0] if ctx.has_res else None
        dy = dy.contiguous()
        dres = ds_extra.contiguous() if ds_extra is not None else None

        b = ctx.b
        need_w = ctx.needs_input_grad[2]
        mg_w = getattr(w, "main_grad", None) if need_w else None
        mg_b = getattr(b, "main_grad", None) if (b is not None and ctx.needs_input_grad[3]) else None
        # fp32 gradient buffers: the kernel writes bf16 partials, added into the fp32 buffer below
        staged = mg_w is not None and mg_w.dtype != w.dtype
        dw_buf = mg_w if (mg_w is not None and not staged) else torch.empty_like(w)
        db_buf = None
        if ctx.layernorm:
            db_buf = mg_b if (mg_b is not None and not staged) else torch.empty_like(b)
        acc = w._kop_hooks.accumulate_for(w) if mg_w is not None else False
        side_fold = False  # the side-stream fold marks w (and b) ready itself
        if ctx.box is not None and not ctx.layernorm and _t_ok(s):
            # also write dx^T: the dY operand of the weight gradient of the projection that produced x
            dx, dxt = lib.rms_norm_bwd_t(dy, s, w, rstd, dres, dw_buf, acc and not staged)
            ctx.box.put(dx, dxt)
        elif (_NORM_SIDE and mg_w is not None and not staged and _side_active(w)
              and (not ctx.layernorm or db_buf is mg_b)):
            # the weight / bias gradient fold (two column reductions) goes to the weight-gradient stream: it is not on
            # the data-gradient chain, and there it no longer waits for CUs behind that stream's GEMMs. Only when both
            # outputs are the parameters' main_grad views: a temporary bias buffer (frozen bias, no main_grad) would be
            # freed to the compute stream's allocator while the side-stream kernel still writes it
            dx, part = lib.norm_bwd_parts(dy, s, w, rstd, mean, dres, ctx.layernorm)
            side_fold = True
            _side_launch(w, lambda: lib.norm_bwd_reduce_(part, dw_buf, db_buf, ctx.layernorm, acc), part,
                         ready=(w, b) if ctx.layernorm else (w,))
        else:
            dx = lib.norm_bwd(dy, s, w, rstd, mean, dres, dw_buf, db_buf, ctx.layernorm, acc and not staged)
        if staged:
            for mg, buf in ((mg_w, dw_buf), (mg_b, db_buf)):
                if mg is not None and buf is not None:
                    mg.add_(buf) if acc else mg.copy_(buf)
        dw = None
        if need_w:
            if mg_w is not None:
                if not side_fold:
                    w._kop_hooks.ready(w)
            else:
                dw = dw_buf
        db = None
        if ctx.layernorm and ctx.needs_input_grad[3]:
            if mg_b is not None:
                if not side_fold:
                    b._kop_hooks.ready(b)
            else:
                db = db_buf
        dres_out = dx if ctx.has_res else None
        return dx, dres_out, dw, db, None, None, None, None


def rms_norm(x, w, eps=1e-5, residual=None, want_t=False, box=None):
    """y = rmsnorm(x (+ residual)) * w; returns y, or (y, x + residual) when residual is given.

    ``want_t``: also return y^T ([H, T], last in the tuple; None where the kernel does not take the shape), the
    X operand of the next projection's weight-gradient GEMM (``linear(..., xt=)``). ``box`` (a ``TBox``): the
    backward also writes dx^T into it, for the projection whose output is ``x`` / ``residual``."""
    if not x.is_cuda:
        y, s = ref.rms_norm_ref(x, w, eps, residual)
        out = (y, s) if residual is not None else (y,)
        out = out + (None,) if want_t else out
        return out if len(out) > 1 else y
    _gate(w)
    t = bool(want_t) and _t_ok(x.reshape(-1, x.shape[-1]))
    out = _Norm.apply(x, residual, w, None, eps, False, t, box)
    if want_t and not t:
        out = (out if isinstance(out, tuple) else (out,)) + (None,)
    return out


def layer_norm(x, w, b, eps=1e-5, residual=None):
    if not x.is_cuda:
        y, s = ref.layer_norm_ref(x, w, b, eps, residual)
        return (y, s) if residual is not None else y
    _gate(w, b)
    return _Norm.apply(x, residual, w, b, eps, True, False, None)


# ---------------------------------------------------------------------------------------------------
# SwiGLU / GELU
# ---------------------------------------------------------------------------------------------------
class _SwiGLU(Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return _lib().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        return _lib().swiglu_bwd(gu, dh.contiguous())


def swiglu(gu):
    if not gu.is_cuda:
        g, u = gu.chunk(2, dim=-1)
        return F.silu(g) * u
    return _SwiGLU.apply(gu)


_SWIGLU_T = os.environ.get("KOP_SWIGLU_T", "1") != "0"


class _LinearSwiGLU(Function):
    """h = swiglu(x . W_gu^T) as one autograd node, so the backward can take dgu^T (the K-contiguous operand
    of the weight-gradient GEMM) from the SwiGLU backward kernel itself instead of transposing dgu afterwards
    (``swiglu_bwd_t``: one read + one write of the [T, 2F] gradient saved per layer and micro-batch)."""

    @staticmethod
    def forward(ctx, x, w):
        x2 = x.reshape(-1, x.shape[-1])
        gu = _fwd(x2, w)
        ctx.save_for_backward(x2, w, gu)
        ctx.in_shape = x.shape
        h = _lib().swiglu_fwd(gu)
        return h.view(*x.shape[:-1], h.shape[-1])

    @staticmethod
    def backward(ctx, dh):
        x2, w, gu = ctx.saved_tensors
        dh2 = dh.reshape(-1, gu.shape[1] // 2).contiguous()
        T, F2 = gu.shape
        fused_t = _SWIGLU_T and ((_DW_LAYOUT == "tn" or (_DW_LAYOUT == "auto" and min(F2, x2.shape[1]) >= _DW_TN_MIN_WIDTH))
                   and T >= _DW_TN_MIN_ROWS and T % 64 == 0 and (F2 // 2) % 64 == 0 and _rows_ok(x2))
        if fused_t:
            dgu, dgut = _lib().swiglu_bwd_t(gu, dh2)
        else:
            dgu, dgut = _lib().swiglu_bwd(gu, dh2), None
        dx = _dx(dgu, w).view(ctx.in_shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if dgut is not None:
                dw = _sink(w, lambda out, acc: _mm_into(dgut, transpose(x2).t(), out, acc), dgut, x2)
            else:
                dw = _sink(w, lambda out, acc: _dw_into(dgu, x2, out, acc), dgu, x2)
        return dx, dw


def linear_swiglu(x, w):
    """swiglu(linear(x, w)) with w = [gate | up] stacked on the output dimension."""
    if not x.is_cuda:
        return swiglu(F.linear(x, w))
    _gate(w)
    return _LinearSwiGLU.apply(x, w)



def _tn_ok(T: int, F2: int, H: int) -> bool:
    """Weight gradient of a [T] x [F2, H] projection through transposed operands (see _dw_into)."""
    return ((_DW_LAYOUT == "tn" or (_DW_LAYOUT == "auto" and min(F2, H) >= _DW_TN_MIN_WIDTH))
            and T >= _DW_TN_MIN_ROWS and T % 64 == 0)


class _SwiGLUMLP(Function):
    """y = swiglu(x . W_gu^T) . W_d^T as one autograd node. With the transposed weight-gradient layout the
    SwiGLU kernels also emit the K-contiguous operands of both weight-gradient GEMMs: the forward writes h^T
    (saved INSTEAD of h: the down projection's backward only needs h for dW_d) and the backward writes dgu^T,
    so neither h nor dgu is transposed separately."""

    @staticmethod
    def forward(ctx, x, w_gu, w_d, tp_group=None, xt=None, box=None):
        lib = _lib()
        x2 = x.reshape(-1, x.shape[-1])
        ctx.tp_group = tp_group
        gu, ctx.sx = _fwd8(x2, w_gu)
        T, F2 = gu.shape
        F = F2 // 2
        ht = None
        if _SWIGLU_T and F % 64 == 0 and _tn_ok(T, w_d.shape[0], F):
            h, ht = lib.swiglu_fwd_t(gu)
        else:
            h = lib.swiglu_fwd(gu)
        y, ctx.sh = _fwd8(h, w_d)
        # X^T from the norm forward replaces X (only the gate|up weight gradient reads it; the FP8 path keeps X)
        ctx.has_xt = xt is not None and ctx.sx is None
        ctx.save_for_backward(xt if ctx.has_xt else x2, w_gu, w_d, gu, ht if ht is not None else h)
        ctx.has_ht = ht is not None
        ctx.in_shape = x.shape
        ctx.box = box
        return y.view(*x.shape[:-1], w_d.shape[0])

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        x2, w_gu, w_d, gu, h_or_ht = ctx.saved_tensors
        T, F2 = gu.shape
        dy2 = dy.reshape(-1, w_d.shape[0])
        dyt = ctx.box.take(dy2) if ctx.box is not None else None
        if ctx.has_ht and _fp8_bwd(w_d, ctx.sh) and _fp8_bwd(w_gu, ctx.sx):
            return _SwiGLUMLP._backward_fp8(ctx, lib, x2, w_gu, w_d, gu, h_or_ht, dy2)
        dh = _dx(dy2, w_d)
        dw_d = None
        if ctx.needs_input_grad[2]:
            if ctx.has_ht:
                a = dyt if dyt is not None else (transpose(dy2) if _rows_ok(dy2) else dy2.t())
                dw_d = _sink(w_d, lambda out, acc: _mm_into(a, h_or_ht.t(), out, acc), a, h_or_ht)
            else:
                dw_d = _sink(w_d, lambda out, acc: _dw_into(dy2, h_or_ht, out, acc), dy2, h_or_ht)
        dh = dh.contiguous()
        H = x2.shape[0] if ctx.has_xt else x2.shape[1]
        if _SWIGLU_T and (F2 // 2) % 64 == 0 and _tn_ok(T, F2, H) and (ctx.has_xt or _rows_ok(x2)):
            dgu, dgut = lib.swiglu_bwd_t(gu, dh)
        else:
            dgu, dgut = lib.swiglu_bwd(gu, dh), None
        dx = _dx(dgu, w_gu) if ctx.needs_input_grad[0] else None
        work = _tp_reduce_async(dx, ctx.tp_group)
        dx = dx.view(ctx.in_shape) if dx is not None else None
        dw_gu = None
        if ctx.needs_input_grad[1]:
            if ctx.has_xt:
                if dgut is not None:
                    dw_gu = _sink(w_gu, lambda out, acc: _mm_into(dgut, x2.t(), out, acc), dgut, x2)
                else:
                    dw_gu = _sink(w_gu, lambda out, acc: _mm_into(dgu.t(), x2.t(), out, acc), dgu, x2)
            elif dgut is not None:
                dw_gu = _sink(w_gu, lambda out, acc: _mm_into(dgut, transpose(x2).t(), out, acc), dgut, x2)
            else:
                dw_gu = _sink(w_gu, lambda out, acc: _dw_into(dgu, x2, out, acc), dgu, x2)
        if work is not None:
            work.wait()
        return dx, dw_gu, dw_d, None, None, None


    @staticmethod
    def _backward_fp8(ctx, lib, x2, w_gu, w_d, gu, ht, dy2):
        """All four backward GEMMs in E4M3: the data gradients quantize dY / dgu (current scaling), the weight
        gradients reuse those scales for dY^T (transpose-cast) and dgu^T (one-pass cast of the SwiGLU kernel's
        transposed output), and the forward's scales for h^T and X^T."""
        from . import fp8

        dh, dy2, sdy = _dx8(dy2, w_d)
        dw_d = None
        if ctx.needs_input_grad[2]:
            sh = ctx.sh
            dw_d = _sink(w_d, lambda out, acc: fp8.wgrad_into(fp8.transpose_cast(dy2, sdy), sdy,
                                                              fp8.cast_scaled(ht, sh), sh, out, acc),
                         dy2, ht, sdy, sh)
        dgu, dgut = lib.swiglu_bwd_t(gu, dh.contiguous())
        dx, dgu, sdgu = _dx8(dgu, w_gu)
        work = _tp_reduce_async(dx, ctx.tp_group)
        dw_gu = None
        if ctx.needs_input_grad[1]:
            sx = ctx.sx
            dw_gu = _sink(w_gu, lambda out, acc: fp8.wgrad_into(fp8.cast_scaled(dgut, sdgu), sdgu,
                                                                fp8.transpose_cast(x2, sx), sx, out, acc),
                          dgut, x2, sdgu, sx)
        if work is not None:
            work.wait()
        return dx.view(ctx.in_shape) if ctx.needs_input_grad[0] else None, dw_gu, dw_d, None, None, None


def swiglu_mlp(x, w_gu, w_d, tp_group=None, xt=None, box=None):
    """linear(swiglu(linear(x, w_gu)), w_d): the Llama MLP (w_gu = [gate | up] on the output dimension).
    ``tp_group``: w_gu / w_d are the FFN-column / FFN-row shards of a tensor-parallel MLP; the input gradient
    is summed over the group, overlapped with the gate|up weight gradient (the output sum is the caller's).
    ``xt`` / ``box``: transposed operands from the neighbouring norms, as in ``linear``."""
    if not x.is_cuda:
        if tp_group is not None:
            from ..parallel.tensor import _CopyToTP

            x = _CopyToTP.apply(x, tp_group)
        return F.linear(swiglu(F.linear(x, w_gu)), w_d)
    _gate(w_gu, w_d)
    return _SwiGLUMLP.apply(x, w_gu, w_d, tp_group, xt, box)


class _GELU(Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        ctx.save_for_backward(x)
        return _lib().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _lib().gelu_bwd(x, dy.contiguous())


def gelu(x):
    if not x.is_cuda:
        return F.gelu(x, approximate="tanh")
    return _GELU.apply(x)


# ---------------------------------------------------------------------------------------------------
# attention (RoPE + flash attention on the fused QKV activation)
# ---------------------------------------------------------------------------------------------------
class _RopeAttention(Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, Hq, Hkv, D, causal, scale, use_rope, inplace, box=None, want_ot=False):
        lib = _lib()
        qkv = qkv.contiguous()
        if use_rope and not inplace:
            qkv = qkv.clone()
        if use_rope:
            lib.rope_(qkv, cos, sin, None, S, Hq + Hkv, D, False)
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:]
        T = qkv.shape[0]
        o = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * Hq * S, dtype=torch.float32, device=qkv.device)
        if want_ot:
            ot = torch.empty(Hq * D, T, dtype=qkv.dtype, device=qkv.device)
            lib.flash_attn_fwd_t(q, k, v, o, ot, lse, B, S, Hq, Hkv, D, scale, causal)
            ctx.mark_non_differentiable(ot)
            ctx.set_materialize_grads(False)  # no zero-filled [Hq*D, T] "gradient" of o^T
        else:
            lib.flash_attn_fwd(q, k, v, o, lse, B, S, Hq, Hkv, D, scale, causal)
        ctx.save_for_backward(qkv, o, lse, cos, sin)
        ctx.cfg = (B, S, Hq, Hkv, D, causal, scale, use_rope)
        ctx.box = box
        return (o, ot) if want_ot else o

    @staticmethod
    def backward(ctx, do, dot=None):
        lib = _lib()
        qkv, o, lse, cos, sin = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, scale, use_rope = ctx.cfg
        do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        ws = torch.empty(lib.flash_attn_bwd_workspace(B, S, Hq, D), dtype=torch.uint8, device=qkv.device)
        a, c = Hq * D, (Hq + Hkv) * D
        lib.flash_attn_bwd(qkv[:, :a], qkv[:, a:c], qkv[:, c:], o, do, lse, dqkv[:, :a], dqkv[:, a:c], dqkv[:, c:], ws,
                           B, S, Hq, Hkv, D, scale, causal)
        T, C = dqkv.shape
        if ctx.box is not None and D in (64, 128) and T % 64 == 0 and C % 128 == 0 and ((Hq + Hkv) * D) % 128 == 0:
            # inverse RoPE fused with dQKV^T for the QKV projection's weight gradient (csrc/transpose.hip rope_t)
            dqkvt = torch.empty(C, T, dtype=dqkv.dtype, device=dqkv.device)
            lib.rope_t_(dqkv, cos, sin, S, Hq + Hkv if use_rope else 0, D, True, dqkvt)
            ctx.box.put(dqkv, dqkvt)
        elif use_rope:
            lib.rope_(dqkv, cos, sin, None, S, Hq + Hkv, D, True)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None, None


def rope_attention(qkv, cos, sin, B, S, Hq, Hkv, D, causal=True, scale=None, use_rope=True, inplace=True, box=None,
                   want_ot=False):
    """Fused-QKV activation [B*S, (Hq+2Hkv)*D] -> attention output [B*S, Hq*D] (RoPE on Q,K if use_rope).

    With ``inplace`` (the model's setting) RoPE overwrites the Q/K columns of ``qkv`` -- safe there because
    the QKV projection's output has no other consumer -- saving one [T, (Hq+Hkv)D] copy per layer.
    ``box`` (a ``TBox``): the backward also writes dQKV^T into it, for the QKV projection (``linear(box=)``).
    ``want_ot``: return (o, o^T) -- o^T [Hq*D, B*S] from the forward kernel, the Wo projection's ``xt`` -- with
    None in place of o^T where the kernel does not take the shape (S not a multiple of 256).
    """
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not qkv.is_cuda:
        x = ref.rope_ref(qkv, cos, sin, S, Hq + Hkv, D) if use_rope else qkv
        a, c = Hq * D, (Hq + Hkv) * D
        o, _ = _attn_ref_autograd(x[:, :a], x[:, a:c], x[:, c:], B, S, Hq, Hkv, D, causal, scale)
        return (o, None) if want_ot else o
    ot = bool(want_ot) and S % 256 == 0 and D in (64, 128) and os.environ.get("KOP_FWD_VARIANT", "10") in ("8", "9", "10", "12", "16")
    out = _RopeAttention.apply(qkv, cos, sin, B, S, Hq, Hkv, D, causal, scale, use_rope, inplace, box, ot)
    if want_ot and not ot:
        return out, None
    return out


def _attn_ref_autograd(q, k, v, B, S, Hq, Hkv, D, causal, scale):
    qh = q.reshape(B, S, Hq, D).transpose(1, 2)
    kh = k.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    vh = v.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    o = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal, scale=scale)
    return o.transpose(1, 2).reshape(B * S, Hq * D), None


def flash_attention(q, k, v, B, S, Hq, Hkv, D, causal=True, scale=None):
    """Attention on already-positioned q/k/v row views; returns (o, lse). Forward only helper for tests."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not q.is_cuda:
        return ref.attention_ref(q, k, v, B, S, Hq, Hkv, D, causal, scale)
    lib = _lib()
    o = torch.empty(B * S, Hq * D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B * Hq * S, dtype=torch.float32, device=q.device)
    lib.flash_attn_fwd(q, k, v, o, lse, B, S, Hq, Hkv, D, scale, causal)
    return o, lse.view(B, Hq, S)


def decode_attention(q, k_cache, v_cache, lens, max_len: int, scale=None):
    """Serving: attention of one new query row per sequence (q [B, Hq*D], a row view of the fused QKV output)
    over its KV cache ([B, Hkv, Smax, D], ``lens`` [B] int32 valid keys, ``max_len`` >= every lens on the host).
    HIP split-K kernel on the GPU (csrc/decode_attn.hip); forward only."""
    D = k_cache.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not q.is_cuda:
        return ref.decode_attention_ref(q, k_cache, v_cache, lens, scale)
    return _lib().decode_attn(q, k_cache, v_cache, lens, int(max_len), scale)


def rope_positions_(x, cos, sin, pos, nheads, D):
    """RoPE in place on the first ``nheads`` heads of each row of x at explicit positions ``pos`` [T] int32."""
    if not x.is_cuda:
        x.copy_(ref.rope_ref(x, cos, sin, 1, nheads, D, pos=pos))
        return x
    _lib().rope_(x, cos, sin, pos, 1, nheads, D, False)
    return x


# ---------------------------------------------------------------------------------------------------
# embedding
# ---------------------------------------------------------------------------------------------------
_EMB_HIP = os.environ.get("KOP_EMB_BWD", "hip") == "hip"


class _Embedding(Function):
    @staticmethod
    def forward(ctx, ids, w):
        ctx.save_for_backward(ids)
        ctx.V = w.shape[0]
        ctx.w = w
        return F.embedding(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        H = w.shape[1]
        dy2 = dy.reshape(-1, H)
        if _EMB_HIP and dy2.is_cuda and dy2.dtype == torch.bfloat16 and H % 8 == 0:
            # csrc/embedding.hip: one stable sort of the ids + a run-sum kernel straight into the gradient buffer (no
            # dense fp32 [V, H] scratch, no fill / copy of the whole table)
            dy2 = dy2.contiguous()

            def prod(out, acc):
                _lib().embedding_bwd_(ids.reshape(-1), dy2, out.view(-1, H), acc)

            return None, _sink(w, prod, dy2, ids, defer=True)

        def prod(out, acc):
            g = torch.ops.aten.embedding_dense_backward(dy2, ids.reshape(-1), ctx.V, -1, False)
            if acc:
                out.add_(g)
            else:
                out.copy_(g)

        return None, _sink(w, prod, dy, ids)


def embedding(ids, w):
    if not w.is_cuda:
        return F.embedding(ids, w)
    _gate(w)
    return _Embedding.apply(ids, w)


# ---------------------------------------------------------------------------------------------------
# LM head + cross entropy (fused: logits buffer is overwritten by its own gradient)
# ---------------------------------------------------------------------------------------------------
class _LMHeadCE(Function):
    @staticmethod
    def forward(ctx, x, w, targets, ignore_index):
        lib = _lib()
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        logits = torch.mm(x2, w.t())
        loss_rows, lse, scale = lib.cross_entropy_fwd_(logits, targets.reshape(-1).contiguous(), ignore_index, True, 1.0)
        loss = loss_rows.sum() * scale[0]
        ctx.save_for_backward(x2, w, logits)
        ctx.in_shape = x.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        x2, w, dlogits = ctx.saved_tensors
        g = g.to(torch.float32)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (_dx(dlogits, w) * g).view(ctx.in_shape)
        dw = None
        if ctx.needs_input_grad[1]:
            xg = x2 * g
            dw = _sink(w, lambda out, acc: _dw_into(dlogits, xg, out, acc), dlogits, xg)
        return dx, dw, None, None


def cross_entropy_lmhead(x, w, targets, ignore_index=-100):
    """mean cross-entropy of softmax(x @ w^T) against targets, computed without fp32 logits."""
    if not x.is_cuda:
        logits = F.linear(x.reshape(-1, x.shape[-1]), w)
        return F.cross_entropy(logits.float(), targets.reshape(-1), ignore_index=ignore_index)
    _gate(w)
    return _LMHeadCE.apply(x, w, targets, ignore_index)
