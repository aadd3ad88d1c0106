// PyTorch bindings for the kubeoperator_amd gfx950 kernels.
//
// Thin adapters only: validate dtype / device / alignment / strides, pick the current HIP stream,
// call the raw-pointer launcher from kernels.h. Activations are passed as 2-D [tokens, features]
// views whose rows may be strided (e.g. the Q, K and V column slices of the fused QKV output), so
// the attention / RoPE paths never copy or transpose.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include "kernels.h"

namespace {

using at::Tensor;
using kop::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be on the GPU (HIP device)");
}
void check_bf16(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_f32(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}
void check_aligned(const Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
// 2-D view with unit inner stride, 16-B aligned rows
void check_rows(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D [rows, features]");
  TORCH_CHECK(t.stride(1) == 1, name, " must have a contiguous last dimension");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  check_aligned(t, name);
}
bf16_t* bp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
const bf16_t* cbp(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<const bf16_t*>(t->data_ptr()) : nullptr;
}
void rc(int code, const char* what) { TORCH_CHECK(code == 0, what, " failed with code ", code, " (unsupported shape)"); }

// ------------------------------------------------------------------ decode projections
Tensor gemv(const Tensor& x, const Tensor& w) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  check_rows(x, "x");
  check_rows(w, "weight");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemv: x and weight disagree on K");
  auto y = at::empty({M, N}, x.options());
  rc(kop::gemv_bf16(bp(x), bp(w), bp(y), M, N, K, x.stride(0), w.stride(0), y.stride(0), cur_stream()),
     "gemv (M <= 8, K a multiple of 1024)");
  return y;
}

// ------------------------------------------------------------------ norms
std::vector<Tensor> norm_fwd(const Tensor& x, const c10::optional<Tensor>& residual, const Tensor& w,
                             const c10::optional<Tensor>& b, double eps, bool layernorm) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "norm inputs must be contiguous");
  const int H = (int)x.size(-1);
  const int rows = (int)(x.numel() / H);
  auto y = at::empty_like(x);
  Tensor s;
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes(), "residual shape");
    s = at::empty_like(x);
  }
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  Tensor mean;
  if (layernorm) {
    TORCH_CHECK(b.has_value(), "layernorm needs a bias");
    check_bf16(*b, "bias");
    mean = at::empty({rows}, x.options().dtype(at::kFloat));
  }
  rc(kop::norm_fwd(bp(x), cbp(residual), bp(w), cbp(b), bp(y), s.defined() ? bp(s) : nullptr, rstd.data_ptr<float>(),
                   layernorm ? mean.data_ptr<float>() : nullptr, rows, H, (float)eps, layernorm, cur_stream()),
     "norm_fwd");
  return {y, s, rstd, mean};
}

Tensor norm_bwd(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& rstd,
                const c10::optional<Tensor>& mean, const c10::optional<Tensor>& dres, const Tensor& dw,
                const c10::optional<Tensor>& db, bool layernorm, bool accumulate) {
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  check_bf16(dw, "dw");
  TORCH_CHECK(dy.is_contiguous() && s.is_contiguous() && dw.is_contiguous(), "norm_bwd inputs must be contiguous");
  const int H = (int)s.size(-1);
  const int rows = (int)(s.numel() / H);
  auto dx = at::empty_like(s);
  const int parts = kop::norm_bwd_partial_rows(rows, H);
  auto part = at::empty({(layernorm ? 2 : 1) * (int64_t)parts * H}, s.options().dtype(at::kFloat));
  rc(kop::norm_bwd(bp(dy), bp(s), bp(w), rstd.data_ptr<float>(),
                   mean.has_value() && mean->defined() ? mean->data_ptr<float>() : nullptr, cbp(dres), bp(dx),
                   part.data_ptr<float>(), bp(dw), db.has_value() ? bp(*db) : nullptr, rows, H, layernorm,
                   accumulate ? 1 : 0, cur_stream()),
     "norm_bwd");
  return dx;
}

// the norm backward without its weight-gradient fold: [dx, fp32 partials]; norm_bwd_reduce_ folds the partials into
// dw (and db for LayerNorm) -- on the weight-gradient stream, off the data-gradient chain (ops/functional.py)
std::vector<Tensor> norm_bwd_parts(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& rstd,
                                   const c10::optional<Tensor>& mean, const c10::optional<Tensor>& dres,
                                   bool layernorm) {
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  TORCH_CHECK(dy.is_contiguous() && s.is_contiguous(), "norm_bwd_parts inputs must be contiguous");
  const int H = (int)s.size(-1);
  const int rows = (int)(s.numel() / H);
  auto dx = at::empty_like(s);
  const int parts = kop::norm_bwd_partial_rows(rows, H);
  auto part = at::empty({(layernorm ? 2 : 1) * (int64_t)parts, (int64_t)H}, s.options().dtype(at::kFloat));
  rc(kop::norm_bwd(bp(dy), bp(s), bp(w), rstd.data_ptr<float>(),
                   mean.has_value() && mean->defined() ? mean->data_ptr<float>() : nullptr, cbp(dres), bp(dx),
                   part.data_ptr<float>(), nullptr, nullptr, rows, H, layernorm, 0, cur_stream()),
     "norm_bwd_parts");
  return {dx, part};
}

void norm_bwd_reduce_(const Tensor& part, const Tensor& dw, const c10::optional<Tensor>& db, bool layernorm,
                      bool accumulate) {
  check_f32(part, "part");
  check_bf16(dw, "dw");
  TORCH_CHECK(part.dim() == 2 && part.is_contiguous() && dw.is_contiguous() && part.size(1) == dw.numel(),
              "norm_bwd_reduce_: part must be [k * parts, H] with H = dw.numel()");
  TORCH_CHECK(!layernorm || (db.has_value() && db->defined() && db->numel() == dw.numel()), "LayerNorm needs db");
  const int H = (int)part.size(1);
  const int parts = (int)(part.size(0) / (layernorm ? 2 : 1));
  rc(kop::norm_bwd_reduce(part.data_ptr<float>(), parts, H, bp(dw), layernorm ? bp(*db) : nullptr, layernorm,
                          accumulate ? 1 : 0, cur_stream()),
     "norm_bwd_reduce_");
}

// RMSNorm with the transposed companion: [y, s, rstd, y^T] (s undefined without a residual)
std::vector<Tensor> rms_norm_fwd_t(const Tensor& x, const c10::optional<Tensor>& residual, const Tensor& w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && x.dim() == 2, "rms_norm_fwd_t: contiguous [rows, H] input");
  const int H = (int)x.size(1), rows = (int)x.size(0);
  TORCH_CHECK(kop::rms_norm_t_parts(rows, H) > 0, "rms_norm_fwd_t: H must be 2048 or 4096 and rows a multiple of 16");
  auto y = at::empty_like(x);
  auto yt = at::empty({H, rows}, x.options());
  Tensor s;
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes(), "residual shape");
    s = at::empty_like(x);
  }
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  rc(kop::rms_norm_fwd_t(bp(x), cbp(residual), bp(w), bp(y), s.defined() ? bp(s) : nullptr, bp(yt),
                         rstd.data_ptr<float>(), rows, H, (float)eps, cur_stream()),
     "rms_norm_fwd_t");
  return {y, s, rstd, yt};
}

// backward: [dx, dx^T]; the weight gradient is written to / accumulated into dw
std::vector<Tensor> rms_norm_bwd_t(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& rstd,
                                   const c10::optional<Tensor>& dres, const Tensor& dw, bool accumulate) {
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  check_bf16(dw, "dw");
  TORCH_CHECK(dy.is_contiguous() && s.is_contiguous() && dw.is_contiguous() && s.dim() == 2 && dy.sizes() == s.sizes(),
              "rms_norm_bwd_t: contiguous [rows, H] inputs");
  const int H = (int)s.size(1), rows = (int)s.size(0);
  const int parts = kop::rms_norm_t_parts(rows, H);
  TORCH_CHECK(parts > 0, "rms_norm_bwd_t: H must be 2048 or 4096 and rows a multiple of 16");
  if (dres.has_value()) {
    check_bf16(*dres, "dres");
    TORCH_CHECK(dres->is_contiguous() && dres->sizes() == s.sizes(), "dres shape");
  }
  auto dx = at::empty_like(s);
  auto dxt = at::empty({H, rows}, s.options());
  auto part = at::empty({(int64_t)parts * H}, s.options().dtype(at::kFloat));
  rc(kop::rms_norm_bwd_t(bp(dy), bp(s), bp(w), rstd.data_ptr<float>(), cbp(dres), bp(dx), bp(dxt),
                         part.data_ptr<float>(), bp(dw), rows, H, accumulate ? 1 : 0, cur_stream()),
     "rms_norm_bwd_t");
  return {dx, dxt};
}

void bias_grad_(const Tensor& dy, const Tensor& db, bool accumulate) {
  check_bf16(dy, "dy");
  check_bf16(db, "db");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous() && db.is_contiguous() && db.numel() == dy.size(1),
              "bias_grad: dy must be a contiguous [rows, H] matrix and db a contiguous [H] vector");
  check_aligned(dy, "dy");
  const int rows = (int)dy.size(0), H = (int)dy.size(1);
  auto part = at::empty({(int64_t)kop::bias_grad_parts(rows, H) * H}, dy.options().dtype(at::kFloat));
  rc(kop::bias_grad(bp(dy), rows, H, part.data_ptr<float>(), bp(db), accumulate ? 1 : 0, cur_stream()),
     "bias_grad (H must be a multiple of 8)");
}

// ------------------------------------------------------------------ elementwise
void rope_(const Tensor& x, const Tensor& cos_t, const Tensor& sin_t, const c10::optional<Tensor>& pos, int64_t S,
           int64_t nheads, int64_t D, bool inverse) {
  check_bf16(x, "x");
  check_rows(x, "x");
  check_f32(cos_t, "cos");
  check_f32(sin_t, "sin");
  TORCH_CHECK(cos_t.is_contiguous() && sin_t.is_contiguous(), "cos/sin tables must be contiguous");
  TORCH_CHECK(x.size(1) >= nheads * D, "rope: row narrower than nheads*D");
  const int* pp = nullptr;
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kInt && pos->is_contiguous(), "positions must be contiguous int32");
    pp = pos->data_ptr<int>();
  }
  rc(kop::rope_inplace(bp(x), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp, x.size(0), (int)S, (int)nheads,
                       (int)D, x.stride(0), inverse, cur_stream()),
     "rope");
}

Tensor swiglu_fwd(const Tensor& gu) {
  check_bf16(gu, "gate_up");
  TORCH_CHECK(gu.is_contiguous(), "gate_up must be contiguous");
  const int64_t F = gu.size(-1) / 2;
  const int64_t T = gu.numel() / (2 * F);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto h = at::empty(sizes, gu.options());
  rc(kop::swiglu_fwd(bp(gu), bp(h), T, (int)F, cur_stream()), "swiglu_fwd");
  return h;
}
Tensor swiglu_bwd(const Tensor& gu, const Tensor& dh) {
  check_bf16(gu, "gate_up");
  check_bf16(dh, "dh");
  TORCH_CHECK(gu.is_contiguous() && dh.is_contiguous(), "swiglu_bwd inputs must be contiguous");
  const int64_t F = gu.size(-1) / 2;
  const int64_t T = gu.numel() / (2 * F);
  auto dgu = at::empty_like(gu);
  rc(kop::swiglu_bwd(bp(gu), bp(dh), bp(dgu), T, (int)F, cur_stream()), "swiglu_bwd");
  return dgu;
}
std::vector<Tensor> swiglu_fwd_t(const Tensor& gu) {
  check_bf16(gu, "gate_up");
  TORCH_CHECK(gu.is_contiguous(), "gate_up must be contiguous");
  const int64_t F = gu.size(-1) / 2;
  const int64_t T = gu.numel() / (2 * F);
  auto h = at::empty({T, F}, gu.options());
  auto ht = at::empty({F, T}, gu.options());
  rc(kop::swiglu_fwd_t(bp(gu), bp(h), bp(ht), T, (int)F, cur_stream()),
     "swiglu_fwd_t (tokens and F must be multiples of 64)");
  return {h, ht};
}
std::vector<Tensor> swiglu_bwd_t(const Tensor& gu, const Tensor& dh) {
  check_bf16(gu, "gate_up");
  check_bf16(dh, "dh");
  TORCH_CHECK(gu.is_contiguous() && dh.is_contiguous(), "swiglu_bwd_t inputs must be contiguous");
  const int64_t F = gu.size(-1) / 2;
  const int64_t T = gu.numel() / (2 * F);
  auto dgu = at::empty_like(gu);
  auto dgut = at::empty({2 * F, T}, gu.options());
  rc(kop::swiglu_bwd_t(bp(gu), bp(dh), bp(dgu), bp(dgut), T, (int)F, cur_stream()),
     "swiglu_bwd_t (tokens and F must be multiples of 64)");
  return {dgu, dgut};
}
Tensor gelu_fwd(const Tensor& x) {
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
  auto y = at::empty_like(x);
  rc(kop::gelu_fwd(bp(x), bp(y), x.numel(), cur_stream()), "gelu_fwd");
  return y;
}
Tensor gelu_bwd(const Tensor& x, const Tensor& dy) {
  check_bf16(x, "x");
  check_bf16(dy, "dy");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous(), "gelu_bwd inputs must be contiguous");
  auto dx = at::empty_like(x);
  rc(kop::gelu_bwd(bp(x), bp(dy), bp(dx), x.numel(), cur_stream()), "gelu_bwd");
  return dx;
}

// ------------------------------------------------------------------ cross entropy
std::vector<Tensor> cross_entropy_fwd_(const Tensor& logits, const Tensor& targets, int64_t ignore_index,
                                       bool write_grad, double grad_multiplier) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be 2-D with a contiguous last dim");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous(), "targets must be contiguous int64");
  const int64_t T = logits.size(0);
  TORCH_CHECK(targets.numel() == T, "targets / logits row mismatch");
  auto f32 = logits.options().dtype(at::kFloat);
  auto loss = at::empty({T}, f32), lse = at::empty({T}, f32), scale = at::empty({1}, f32);
  rc(kop::cross_entropy_fwd(bp(logits), logits.stride(0), T, (int)logits.size(1), targets.data_ptr<int64_t>(),
                            ignore_index, scale.data_ptr<float>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                            write_grad, (float)grad_multiplier, cur_stream()),
     "cross_entropy");
  return {loss, lse, scale};
}

// ------------------------------------------------------------------ embedding gradient
// out (+)= the embedding weight gradient of (ids, dy), written straight into ``out`` (the flat gradient buffer's view of
// the table): one stable radix sort of the int32 ids + the run-sum kernel; no dense fp32 scratch
void embedding_bwd_(const Tensor& ids, const Tensor& dy, const Tensor& out, bool accumulate) {
  check_gpu(ids, "ids");
  check_bf16(dy, "dy");
  check_rows(dy, "dy");
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out must be bf16 or fp32");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.stride(0) % 8 == 0, "out must be [V, H] with contiguous rows");
  check_aligned(out, "out");
  TORCH_CHECK(ids.numel() == dy.size(0) && out.size(1) == dy.size(1), "embedding_bwd: shape mismatch");
  const int64_t T = ids.numel();
  TORCH_CHECK(T < ((int64_t)1 << 31), "embedding_bwd: too many tokens");
  if (!accumulate) out.zero_();
  if (T == 0) return;
  auto sr = at::sort(ids.reshape({-1}).to(at::kInt), /*stable=*/true, /*dim=*/0, /*descending=*/false);
  const Tensor& sid = std::get<0>(sr);
  const Tensor& perm = std::get<1>(sr);
  rc(kop::embedding_bwd(sid.data_ptr<int>(), perm.data_ptr<int64_t>(), bp(dy), dy.stride(0), out.data_ptr(),
                        out.scalar_type() == at::kFloat, out.stride(0), (int)T, (int)dy.size(1), accumulate, cur_stream()),
     "embedding_bwd (H a multiple of 8)");
}

// ------------------------------------------------------------------ transpose
void transpose_(const Tensor& in, const Tensor& out) {
  check_bf16(in, "in");
  check_bf16(out, "out");
  check_rows(in, "in");
  check_rows(out, "out");
  TORCH_CHECK(out.size(0) == in.size(1) && out.size(1) == in.size(0), "out must be [in.cols, in.rows]");
  rc(kop::transpose2d(bp(in), bp(out), in.size(0), in.size(1), in.stride(0), out.stride(0), cur_stream()),
     "transpose (rows and columns must be multiples of 8)");
}

// RoPE in place on the Q/K heads of x [T, C] fused with out = x^T [C, T] (the attention backward's dQKV)
void rope_t_(const Tensor& x, const Tensor& cos_t, const Tensor& sin_t, int64_t S, int64_t nheads, int64_t D,
             bool inverse, const Tensor& out) {
  check_bf16(x, "x");
  check_bf16(out, "out");
  check_rows(x, "x");
  check_rows(out, "out");
  check_f32(cos_t, "cos");
  check_f32(sin_t, "sin");
  TORCH_CHECK(cos_t.is_contiguous() && sin_t.is_contiguous(), "cos/sin tables must be contiguous");
  TORCH_CHECK(cos_t.size(-1) == D / 2 && cos_t.size(0) >= S, "cos/sin tables must be [>= S, D/2]");
  TORCH_CHECK(out.size(0) == x.size(1) && out.size(1) == x.size(0), "out must be [x.cols, x.rows]");
  rc(kop::rope_transpose(bp(x), bp(out), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), x.size(0), x.size(1),
                         x.stride(0), out.stride(0), (int)S, (int)nheads, (int)D, inverse, cur_stream()),
     "rope_t (head_dim 128 or 64, rows a multiple of 64, columns and rotated columns of 128)");
}

// ------------------------------------------------------------------ split-K weight-gradient reduction
// part [S, N, K] fp32 partial planes of one weight gradient -> out [N, K] (bf16 or fp32), overwritten or accumulated
void splitk_reduce_(const Tensor& part, const Tensor& out, bool accumulate) {
  check_f32(part, "part");
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out must be bf16 or fp32");
  TORCH_CHECK(part.is_contiguous() && out.is_contiguous(), "splitk_reduce: part and out must be contiguous");
  TORCH_CHECK(part.dim() >= 2 && part.numel() == part.size(0) * out.numel(), "part must be [S, *out.shape]");
  check_aligned(part, "part");
  check_aligned(out, "out");
  rc(kop::splitk_reduce(part.data_ptr<float>(), (int)part.size(0), out.numel(), out.data_ptr(),
                        out.scalar_type() == at::kFloat, accumulate, cur_stream()),
     "splitk_reduce (element count must be a multiple of 8)");
}

// ------------------------------------------------------------------ fp8
void fp8_quant_(const Tensor& x, const Tensor& out, const Tensor& scale, const Tensor& amax_ws) {
  check_bf16(x, "x");
  check_gpu(out, "out");
  check_f32(scale, "scale");
  check_gpu(amax_ws, "amax_ws");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "fp8_quant: contiguous tensors only");
  TORCH_CHECK(out.element_size() == 1 && out.numel() == x.numel(), "fp8_quant: out must be 1-byte, x.numel()");
  TORCH_CHECK(scale.numel() == 1 && amax_ws.nbytes() >= kop::kFp8AmaxBlocks * sizeof(float),
              "fp8_quant: scale / workspace size");
  rc(kop::fp8_quantize(bp(x), x.numel(), reinterpret_cast<uint8_t*>(out.data_ptr()), scale.data_ptr<float>(),
                       reinterpret_cast<float*>(amax_ws.data_ptr()), cur_stream()),
     "fp8_quant (x 16-byte and out 8-byte aligned)");
}

void fp8_cast_scaled_(const Tensor& x, const Tensor& scale, const Tensor& out) {
  check_bf16(x, "x");
  check_f32(scale, "scale");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && out.is_cuda(), "fp8_cast: contiguous GPU tensors");
  TORCH_CHECK(out.element_size() == 1 && out.numel() == x.numel(), "fp8_cast: out must be 1-byte, x.numel()");
  rc(kop::fp8_cast_scaled(bp(x), x.numel(), scale.data_ptr<float>(), reinterpret_cast<uint8_t*>(out.data_ptr()),
                          cur_stream()),
     "fp8_cast (numel a multiple of 8, aligned)");
}
void fp8_transpose_cast_(const Tensor& in, const Tensor& scale, const Tensor& out) {
  check_bf16(in, "in");
  check_rows(in, "in");
  check_f32(scale, "scale");
  TORCH_CHECK(out.is_cuda() && out.element_size() == 1 && out.dim() == 2 && out.stride(1) == 1,
              "fp8_transpose_cast: out must be a 2-D 1-byte GPU tensor with contiguous rows");
  TORCH_CHECK(out.size(0) == in.size(1) && out.size(1) == in.size(0), "out must be [in.cols, in.rows]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0, "out must be 8-byte aligned");
  rc(kop::fp8_transpose_cast(bp(in), reinterpret_cast<uint8_t*>(out.data_ptr()), in.size(0), in.size(1),
                             in.stride(0), out.stride(0), scale.data_ptr<float>(), cur_stream()),
     "fp8_transpose_cast (rows and columns multiples of 8)");
}

// ------------------------------------------------------------------ optimizer
void adamw_(const Tensor& p, const Tensor& g, const Tensor& master, const Tensor& m, const Tensor& v, double lr,
            double b1, double b2, double eps, double wd, int64_t step, double gscale,
            const c10::optional<Tensor>& gscale_dev) {
  check_bf16(p, "param");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat, "grad must be bf16 or fp32");
  TORCH_CHECK(g.device() == p.device(), "grad on another device");
  check_f32(master, "master");
  check_f32(m, "exp_avg");
  check_f32(v, "exp_avg_sq");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && master.numel() == n && m.numel() == n && v.numel() == n, "adamw size mismatch");
  for (auto* t : {&p, &g, &master, &m, &v}) {
    TORCH_CHECK(t->is_contiguous(), "adamw buffers must be contiguous");
    check_aligned(*t, "adamw buffer");
  }
  const float* gd = nullptr;
  if (gscale_dev.has_value() && gscale_dev->defined()) {
    check_f32(*gscale_dev, "gscale_dev");
    gd = gscale_dev->data_ptr<float>();
  }
  if (g.scalar_type() == at::kFloat)
    rc(kop::adamw_step(bp(p), g.data_ptr<float>(), master.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                       n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step, (float)gscale, gd,
                       cur_stream()),
       "adamw");
  else
    rc(kop::adamw_step(bp(p), bp(g), master.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), n,
                       (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step, (float)gscale, gd,
                       cur_stream()),
       "adamw");
}
void grad_sumsq_(const Tensor& g, const Tensor& out) {
  TORCH_CHECK(g.is_cuda() && (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat),
              "grad must be a bf16 or fp32 GPU tensor");
  check_f32(out, "out");
  TORCH_CHECK(g.is_contiguous(), "grad must be contiguous");
  check_aligned(g, "grad");
  if (g.scalar_type() == at::kFloat)
    rc(kop::grad_sumsq(g.data_ptr<float>(), g.numel(), out.data_ptr<float>(), cur_stream()), "grad_sumsq");
  else
    rc(kop::grad_sumsq(bp(g), g.numel(), out.data_ptr<float>(), cur_stream()), "grad_sumsq");
}
void clip_coef_(const Tensor& sumsq, double max_norm, const Tensor& coef, const Tensor& norm) {
  rc(kop::clip_coef(sumsq.data_ptr<float>(), (float)max_norm, coef.data_ptr<float>(), norm.data_ptr<float>(),
                    cur_stream()),
     "clip_coef");
}

// ------------------------------------------------------------------ attention
void flash_attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& lse, int64_t B,
                    int64_t S, int64_t Hq, int64_t Hkv, int64_t D, double scale, bool causal) {
  for (auto* t : {&q, &k, &v, &o}) {
    check_bf16(*t, "q/k/v/o");
    check_rows(*t, "q/k/v/o");
    TORCH_CHECK(t->size(0) == B * S, "attention tensors must have B*S rows");
  }
  check_f32(lse, "lse");
  TORCH_CHECK(lse.numel() == B * Hq * S, "lse size");
  TORCH_CHECK(q.size(1) >= Hq * D && k.size(1) >= Hkv * D && v.size(1) >= Hkv * D && o.size(1) >= Hq * D,
              "attention head width");
  rc(kop::flash_attn_fwd(bp(q), bp(k), bp(v), bp(o), lse.data_ptr<float>(), (int)B, (int)S, (int)Hq, (int)Hkv,
                         (int)D, q.stride(0), k.stride(0), v.stride(0), o.stride(0), (float)scale, causal,
                         cur_stream()),
     "flash_attn_fwd");
}

// forward that also writes O^T [Hq*D, B*S] (8-wave kernel shapes: S a multiple of 256)
void flash_attn_fwd_t(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& ot,
                      const Tensor& lse, int64_t B, int64_t S, int64_t Hq, int64_t Hkv, int64_t D, double scale,
                      bool causal) {
  for (auto* t : {&q, &k, &v, &o}) {
    check_bf16(*t, "q/k/v/o");
    check_rows(*t, "q/k/v/o");
    TORCH_CHECK(t->size(0) == B * S, "attention tensors must have B*S rows");
  }
  check_bf16(ot, "ot");
  TORCH_CHECK(ot.is_contiguous() && ot.size(0) == Hq * D && ot.size(1) == B * S, "ot must be a contiguous [Hq*D, B*S]");
  check_f32(lse, "lse");
  TORCH_CHECK(lse.numel() == B * Hq * S, "lse size");
  TORCH_CHECK(q.size(1) >= Hq * D && k.size(1) >= Hkv * D && v.size(1) >= Hkv * D && o.size(1) >= Hq * D,
              "attention head width");
  rc(kop::flash_attn_fwd(bp(q), bp(k), bp(v), bp(o), lse.data_ptr<float>(), (int)B, (int)S, (int)Hq, (int)Hkv,
                         (int)D, q.stride(0), k.stride(0), v.stride(0), o.stride(0), (float)scale, causal,
                         cur_stream(), bp(ot)),
     "flash_attn_fwd_t (S must be a multiple of 256)");
}

int64_t flash_attn_bwd_workspace(int64_t B, int64_t S, int64_t Hq, int64_t D) {
  return (int64_t)kop::flash_attn_bwd_workspace((int)B, (int)S, (int)Hq, (int)D);
}

void flash_attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& dout,
                    const Tensor& lse, const Tensor& dq, const Tensor& dk, const Tensor& dv, const Tensor& workspace,
                    int64_t B, int64_t S, int64_t Hq, int64_t Hkv, int64_t D, double scale, bool causal) {
  for (auto* t : {&q, &k, &v, &o, &dout, &dq, &dk, &dv}) {
    check_bf16(*t, "attention tensor");
    check_rows(*t, "attention tensor");
    TORCH_CHECK(t->size(0) == B * S, "attention tensors must have B*S rows");
  }
  check_f32(lse, "lse");
  TORCH_CHECK(workspace.nbytes() >= (size_t)flash_attn_bwd_workspace(B, S, Hq, D), "attention workspace too small");
  check_aligned(workspace, "workspace");
  rc(kop::flash_attn_bwd(bp(q), bp(k), bp(v), bp(o), bp(dout), lse.data_ptr<float>(), bp(dq), bp(dk), bp(dv),
                         workspace.data_ptr(), (int)B, (int)S, (int)Hq, (int)Hkv, (int)D, q.stride(0), k.stride(0),
                         v.stride(0), o.stride(0), dout.stride(0), dq.stride(0), dk.stride(0), dv.stride(0),
                         (float)scale, causal, cur_stream()),
     "flash_attn_bwd");
}

}  // namespace

// ------------------------------------------------------------------ decode attention (serving)
// q: [B, Hq*D] rows (strided view allowed); k_cache / v_cache: [B, Hkv, Smax, D] contiguous; lens: [B] int32
// (valid keys per sequence, 1 <= lens <= Smax); max_len bounds lens (host value: sizes the split grid)
Tensor decode_attn(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& lens, int64_t max_len,
                   double scale) {
  check_bf16(q, "q");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_rows(q, "q");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous() &&
                  k_cache.sizes() == v_cache.sizes(), "caches must be contiguous [B, Hkv, Smax, D] and equal");
  check_aligned(k_cache, "k_cache");
  check_aligned(v_cache, "v_cache");
  TORCH_CHECK(lens.is_cuda() && lens.scalar_type() == at::kInt && lens.is_contiguous(), "lens must be int32 on the GPU");
  const int B = (int)k_cache.size(0), Hkv = (int)k_cache.size(1), Smax = (int)k_cache.size(2), D = (int)k_cache.size(3);
  TORCH_CHECK(q.size(0) == B && lens.numel() == B, "batch mismatch");
  TORCH_CHECK(q.size(1) % D == 0, "q width must be a multiple of head_dim");
  const int Hq = (int)(q.size(1) / D);
  TORCH_CHECK(max_len >= 1 && max_len <= Smax, "max_len must be in [1, Smax]");
  const int nsplit = kop::decode_attn_splits((int)max_len);
  auto o = at::empty({B, (int64_t)Hq * D}, q.options());
  auto part_o = at::empty({(int64_t)B * Hq * nsplit * D}, q.options().dtype(at::kFloat));
  auto part_ml = at::empty({(int64_t)B * Hq * nsplit * 2}, q.options().dtype(at::kFloat));
  rc(kop::decode_attn(bp(q), q.stride(0), bp(k_cache), bp(v_cache), lens.data_ptr<int>(), bp(o), o.stride(0),
                      part_o.data_ptr<float>(), part_ml.data_ptr<float>(), B, Smax, Hq, Hkv, D, nsplit, (float)scale,
                      cur_stream()),
     "decode_attn");
  return o;
}

// qkv: [B, (Hq + 2 Hkv) D] fused rows; caches [B, Hkv, Smax, D]; pos: [B] int32 (cache row to append at)
void decode_rope_append_(const Tensor& qkv, const Tensor& cos_t, const Tensor& sin_t, const Tensor& pos,
                         const Tensor& k_cache, const Tensor& v_cache, int64_t Hq) {
  check_bf16(qkv, "qkv");
  check_rows(qkv, "qkv");
  check_f32(cos_t, "cos");
  check_f32(sin_t, "sin");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous() &&
                  k_cache.sizes() == v_cache.sizes(), "caches must be contiguous [B, Hkv, Smax, D] and equal");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kInt && pos.is_contiguous(), "pos must be int32 on the GPU");
  const int B = (int)qkv.size(0), Hkv = (int)k_cache.size(1), Smax = (int)k_cache.size(2), D = (int)k_cache.size(3);
  TORCH_CHECK(k_cache.size(0) >= B && pos.numel() == B, "batch mismatch");
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width must be (Hq + 2 Hkv) * D");
  TORCH_CHECK(cos_t.size(0) >= Smax && cos_t.size(1) == D / 2, "rope tables must cover the cache");
  rc(kop::decode_rope_append(bp(qkv), qkv.stride(0), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(),
                             pos.data_ptr<int>(), bp(k_cache), bp(v_cache), B, Smax, (int)Hq, Hkv, D, cur_stream()),
     "decode_rope_append");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "kubeoperator_amd gfx950 (MI355X) HIP kernels";
  m.attr("ARCH") = "gfx950";
  m.def("norm_fwd", &norm_fwd);
  m.def("norm_bwd", &norm_bwd);
  m.def("norm_bwd_parts", &norm_bwd_parts);
  m.def("norm_bwd_reduce_", &norm_bwd_reduce_);
  m.def("rms_norm_fwd_t", &rms_norm_fwd_t);
  m.def("rms_norm_bwd_t", &rms_norm_bwd_t);
  m.def("bias_grad_", &bias_grad_);
  m.def("rope_", &rope_);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("swiglu_bwd_t", &swiglu_bwd_t);
  m.def("swiglu_fwd_t", &swiglu_fwd_t);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("cross_entropy_fwd_", &cross_entropy_fwd_);
  m.def("transpose_", &transpose_);
  m.def("embedding_bwd_", &embedding_bwd_);
  m.def("rope_t_", &rope_t_);
  m.def("splitk_reduce_", &splitk_reduce_);
  m.def("fp8_quant_", &fp8_quant_);
  m.attr("FP8_AMAX_BLOCKS") = kop::kFp8AmaxBlocks;
  m.def("fp8_cast_scaled_", &fp8_cast_scaled_);
  m.def("fp8_transpose_cast_", &fp8_transpose_cast_);
  m.def("adamw_", &adamw_);
  m.def("grad_sumsq_", &grad_sumsq_);
  m.def("clip_coef_", &clip_coef_);
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_attn_fwd_t", &flash_attn_fwd_t);
  m.def("decode_attn", &decode_attn);
  m.def("decode_rope_append_", &decode_rope_append_);
  m.def("gemv", &gemv);
  m.def("flash_attn_bwd_workspace", &flash_attn_bwd_workspace);
  m.def("flash_attn_bwd", &flash_attn_bwd);
  m.def("flash_attn_set_dq_variant", [](int64_t v) { return (int64_t)kop::flash_attn_set_dq_variant((int)v); });
  m.def("flash_attn_set_fwd_variant", [](int64_t v) { return (int64_t)kop::flash_attn_set_fwd_variant((int)v); });
  m.def("decode_attn_set_mfma", [](int64_t on) { return (int64_t)kop::decode_attn_set_mfma((int)on); });
  m.def("flash_attn_set_dkdv_cfg", [](int64_t c) { return (int64_t)kop::flash_attn_set_dkdv_cfg((int)c); });
  m.def("flash_attn_set_dq_nw", [](int64_t c) { return (int64_t)kop::flash_attn_set_dq_nw((int)c); });
  m.def("flash_attn_set_d64_shape", [](int64_t c) { return (int64_t)kop::flash_attn_set_d64_shape((int)c); });
  m.def("flash_attn_set_dkdv_hpw", [](int64_t h) { return (int64_t)kop::flash_attn_set_dkdv_hpw((int)h); });
}
