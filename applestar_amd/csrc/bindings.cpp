// PyTorch bindings for the applestar_amd HIP kernels.  Tensor checks happen here; the launchers in
// kernels/*.hip only see raw pointers and the current HIP stream (graph-capturable).
#include <cstring>
#include <cstdlib>
#include <map>
#include <string>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "kernels.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dt(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return as::DT_F32;
  if (t.scalar_type() == at::kBFloat16) return as::DT_BF16;
  TORCH_CHECK(false, "applestar_amd: unsupported dtype ", t.scalar_type());
}

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "applestar_amd: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "applestar_amd: ", name, " must be contiguous");
}

// ---------------------------------------------------------------- layer norm
std::vector<at::Tensor> layer_norm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                       const at::Tensor& w, const at::Tensor& b, int64_t out_dtype, double eps,
                                       int64_t act, bool save_sum) {
  check_cuda(x, "x");
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 64 == 0 && C <= 1536, "layer_norm: cols must be a multiple of 64 and <= 1536");
  TORCH_CHECK(w.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat, "layer_norm: fp32 affine");
  const int64_t rows = x.numel() / C;
  c10::hip::HIPGuard g(x.device().index());
  auto y = at::empty(x.sizes(), x.options().dtype(out_dtype == 1 ? at::kBFloat16 : at::kFloat));
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor xsum;
  const void* rp = nullptr;
  int rdt = as::DT_F32;
  if (res.has_value()) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes(), "layer_norm: residual shape");
    rp = res->data_ptr();
    rdt = dt(*res);
    if (save_sum) xsum = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  }
  as::layer_norm_fwd(x.data_ptr(), dt(x), rp, rdt, w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr(), dt(y),
                     xsum.defined() ? xsum.data_ptr<float>() : nullptr, mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), rows, static_cast<int>(C), static_cast<float>(eps),
                     static_cast<int>(act), stream());
  return {y, mean, rstd, xsum.defined() ? xsum : at::Tensor()};
}

std::vector<at::Tensor> layer_norm_bwd(const at::Tensor& dy, const at::Tensor& xin, const at::Tensor& y,
                                       const at::Tensor& w, const at::Tensor& mean, const at::Tensor& rstd,
                                       int64_t dx_dtype, int64_t act, const c10::optional<at::Tensor>& mask_src) {
  check_cuda(dy, "dy");
  check_cuda(xin, "xin");
  const int64_t C = xin.size(-1);
  const int64_t rows = xin.numel() / C;
  c10::hip::HIPGuard g(xin.device().index());
  auto dx = at::empty(xin.sizes(), xin.options().dtype(dx_dtype == 1 ? at::kBFloat16 : at::kFloat));
  const int nblk = as::layer_norm_bwd_blocks(rows);
  auto part = at::empty({nblk, 2 * C}, xin.options().dtype(at::kFloat));
  auto dwb = at::empty({2 * C}, xin.options().dtype(at::kFloat));
  const at::Tensor& yy = act != 0 ? y : dy;
  at::Tensor dxm;
  if (mask_src.has_value()) {
    TORCH_CHECK(mask_src->scalar_type() == at::kFloat && mask_src->is_contiguous() && mask_src->numel() == rows * C,
                "layer_norm_bwd: mask_src fp32 contiguous, x's size");
    dxm = at::empty(xin.sizes(), xin.options().dtype(at::kFloat));
  }
  as::layer_norm_bwd(dy.data_ptr(), dt(dy), xin.data_ptr(), dt(xin), yy.data_ptr(), dt(yy), w.data_ptr<float>(),
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(), dt(dx),
                     part.data_ptr<float>(), part.data_ptr<float>() + C, rows, static_cast<int>(C),
                     static_cast<int>(act), nblk, stream(), dxm.defined() ? mask_src->data_ptr<float>() : nullptr,
                     dxm.defined() ? dxm.data_ptr<float>() : nullptr);
  as::column_reduce(part.data_ptr<float>(), dwb.data_ptr<float>(), nblk, static_cast<int>(2 * C), stream());
  if (dxm.defined()) return {dx, dwb.narrow(0, 0, C), dwb.narrow(0, C, C), dxm};
  return {dx, dwb.narrow(0, 0, C), dwb.narrow(0, C, C)};
}

// ---------------------------------------------------------------- reverse scan
at::Tensor reverse_scan(const at::Tensor& a, const at::Tensor& b, const at::Tensor& init) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  check_cuda(init, "init");
  TORCH_CHECK(a.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat && init.scalar_type() == at::kFloat,
              "reverse_scan: fp32");
  TORCH_CHECK(a.sizes() == b.sizes() && a.dim() >= 2, "reverse_scan: a/b shape");
  const int64_t B = a.size(-1), T = a.size(-2);
  const int64_t K = a.numel() / (B * T);
  TORCH_CHECK(init.numel() == K * B, "reverse_scan: init shape");
  c10::hip::HIPGuard g(a.device().index());
  auto y = at::empty_like(b);
  as::reverse_scan(a.data_ptr<float>(), b.data_ptr<float>(), init.data_ptr<float>(), y.data_ptr<float>(),
                   static_cast<int>(K), static_cast<int>(T), static_cast<int>(B), stream());
  return y;
}

// ---------------------------------------------------------------- gated residual
// post (optional): added to the block output in the same pass
at::Tensor gated_residual_fwd(const at::Tensor& y, const at::Tensor& gt, const at::Tensor& sp, const at::Tensor& x,
                              const c10::optional<at::Tensor>& post) {
  check_cuda(y, "y");
  check_cuda(gt, "g");
  check_cuda(x, "x");
  TORCH_CHECK(y.scalar_type() == gt.scalar_type() && y.scalar_type() == x.scalar_type(), "gated_residual: dtypes");
  TORCH_CHECK(y.sizes() == gt.sizes() && y.sizes() == x.sizes(), "gated_residual: shapes");
  TORCH_CHECK(y.is_contiguous() && gt.is_contiguous() && x.is_contiguous(), "gated_residual: contiguous operands");
  TORCH_CHECK(sp.scalar_type() == at::kFloat, "gated_residual: sp fp32");
  const void* pp = nullptr;
  if (post && post->defined()) {
    check_cuda(*post, "post");
    TORCH_CHECK(post->scalar_type() == y.scalar_type() && post->sizes() == y.sizes() && post->is_contiguous(),
                "gated_residual: post must match y (dtype, shape, contiguous)");
    pp = post->data_ptr();
  }
  c10::hip::HIPGuard g(y.device().index());
  auto out = at::empty_like(y);
  as::gated_residual_fwd(y.data_ptr(), gt.data_ptr(), sp.data_ptr<float>(), x.data_ptr(), pp, out.data_ptr(), dt(y),
                         y.numel(), stream());
  return out;
}

// out: the saved block output (its ReLU mask); with xin (the block input) the mask comes from the recomputed
// pre-activation instead (the forward carried a post-add, so the saved tensor is not the ReLU output)
std::vector<at::Tensor> gated_residual_bwd(const at::Tensor& dout, const at::Tensor& y, const at::Tensor& gt,
                                           const at::Tensor& sp, const c10::optional<at::Tensor>& out,
                                           const c10::optional<at::Tensor>& xin) {
  check_cuda(dout, "dout");
  TORCH_CHECK(dout.scalar_type() == y.scalar_type(), "gated_residual_bwd: dtype");
  const bool use_x = xin && xin->defined();
  TORCH_CHECK(use_x || (out && out->defined()), "gated_residual_bwd: needs the saved output or the block input");
  const at::Tensor& mref = use_x ? *xin : *out;
  TORCH_CHECK(mref.scalar_type() == y.scalar_type() && mref.sizes() == y.sizes() && mref.is_contiguous() &&
                  dout.sizes() == y.sizes() && dout.is_contiguous() && y.is_contiguous() && gt.is_contiguous(),
              "gated_residual_bwd: operands must match y (dtype, shape, contiguous)");
  c10::hip::HIPGuard g(y.device().index());
  auto dy = at::empty_like(y), dg = at::empty_like(y), dx = at::empty_like(y);
  const int nblk = as::elementwise_blocks(y.numel());
  auto part = at::empty({nblk}, y.options().dtype(at::kFloat));
  as::gated_residual_bwd(dout.data_ptr(), y.data_ptr(), gt.data_ptr(), sp.data_ptr<float>(),
                         use_x ? nullptr : out->data_ptr(), use_x ? xin->data_ptr() : nullptr, dt(y), dy.data_ptr(),
                         dg.data_ptr(), dx.data_ptr(), part.data_ptr<float>(), y.numel(), nblk, stream());
  return {dy, dg, dx, part.sum().reshape({1})};
}

// ---------------------------------------------------------------- LN-LSTM recurrence
// ---------------------------------------------------------------- layer-norm LSTM recurrence
// Split (multi-workgroup) recurrence for H = 384 and small batches; APPLESTAR_LSTM_SPLIT=0 disables it.
bool lstm_split_enabled(int64_t H, int64_t B) {
  static const bool env_on = [] {
    const char* v = std::getenv("APPLESTAR_LSTM_SPLIT");
    return v == nullptr || std::string(v) != "0";
  }();
  return env_on && H == 384 && B >= 1 && B <= 16;
}

// sticky device-side timeout flag of the split recurrence's cross-workgroup poll (never reset)
at::Tensor& lstm_split_err(const at::Device& dev) {
  static std::map<int, at::Tensor> flags;
  auto it = flags.find(dev.index());
  if (it == flags.end())
    it = flags.emplace(dev.index(), at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(dev))).first;
  return it->second;
}

at::Tensor lstm_split_error(int64_t device) {
  return lstm_split_err(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device))).clone();
}

// the flag itself (not a copy): the trainers gate the optimizer update on it and log it with the step's
// other scalars, so a timed-out exchange never reaches the weights unnoticed
at::Tensor lstm_split_flag(int64_t device) {
  return lstm_split_err(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
}

struct SplitBufs {
  at::Tensor slab;
  as::LstmSplit s;
};

// granule slab, zeroed per launch (epoch tags start at 1)
SplitBufs make_split(const at::Tensor& like, int64_t B, int64_t width) {
  SplitBufs r;
  const int64_t Bp = (B + 7) / 8 * 8;
  // granules [2, Bp, 8, width] u64 (backward) or data [2, Bp, 8, width] u32 + flags [Bp, 8] (forward):
  // one zeroed buffer sized for either
  const int64_t KS = std::getenv("APPLESTAR_LSTM_KS") != nullptr && std::atoi(std::getenv("APPLESTAR_LSTM_KS")) == 16
                       ? 16 : 8;     // workgroups per row (lstm.hip lstm_ks)
  r.slab = at::zeros({2 * Bp * KS * width + Bp * KS}, like.options().dtype(at::kLong));
  r.s = {reinterpret_cast<unsigned long long*>(r.slab.data_ptr<int64_t>()), lstm_split_err(like.device()).data_ptr<int>()};
  return r;
}

// want_bf16: also return a bf16 copy of out written by the split recurrence itself (inference: the next layer's input
// projection and the heads take bf16 operands - no cast launch per layer); undefined when the split path is not taken
std::vector<at::Tensor> lnlstm_fwd(const at::Tensor& xp, const at::Tensor& h0, const at::Tensor& c0,
                                   const at::Tensor& wT, const at::Tensor& lnh_w, const at::Tensor& lnh_b,
                                   const at::Tensor& lnc_w, const at::Tensor& lnc_b, double eps, bool want_bf16) {
  for (auto* t : {&xp, &h0, &c0, &wT, &lnh_w, &lnh_b, &lnc_w, &lnc_b}) check_cuda(*t, "lnlstm input");
  TORCH_CHECK(xp.scalar_type() == at::kFloat && h0.scalar_type() == at::kFloat && c0.scalar_type() == at::kFloat,
              "lnlstm: fp32 activations");
  const int64_t T = xp.size(0), B = xp.size(1), G = xp.size(2), H = G / 4;
  TORCH_CHECK(as::lnlstm_supported(static_cast<int>(H)), "lnlstm: unsupported hidden size ", H);
  TORCH_CHECK(wT.size(0) == H && wT.size(1) == G, "lnlstm: wT must be [H, 4H]");
  TORCH_CHECK(h0.size(0) == B && h0.size(1) == H && c0.sizes() == h0.sizes(), "lnlstm: state shape");
  c10::hip::HIPGuard g(xp.device().index());
  auto f = xp.options().dtype(at::kFloat);
  auto out = at::empty({T, B, H}, f);
  auto c_all = at::empty({T + 1, B, H}, f);
  auto xhat_h = at::empty({T, B, G}, f);
  auto gates = at::empty({T, B, G}, f);
  auto xhat_c = at::empty({T, B, H}, f);
  auto rstd_h = at::empty({T, B}, f);
  auto rstd_c = at::empty({T, B}, f);
  auto hT = at::empty({B, H}, f);
  auto cT = at::empty({B, H}, f);
  SplitBufs sb;
  const bool split = lstm_split_enabled(H, B);
  if (split) sb = make_split(xp, B, G);
  at::Tensor out_bf;
  if (split && want_bf16) out_bf = at::empty({T, B, H}, xp.options().dtype(at::kBFloat16));
  as::lnlstm_fwd(xp.data_ptr<float>(), h0.data_ptr<float>(), c0.data_ptr<float>(), wT.data_ptr(), dt(wT),
                 lnh_w.data_ptr<float>(), lnh_b.data_ptr<float>(), lnc_w.data_ptr<float>(), lnc_b.data_ptr<float>(),
                 static_cast<int>(T), static_cast<int>(B), static_cast<int>(H), static_cast<float>(eps),
                 out.data_ptr<float>(), c_all.data_ptr<float>(), xhat_h.data_ptr<float>(), rstd_h.data_ptr<float>(),
                 gates.data_ptr<float>(), xhat_c.data_ptr<float>(), rstd_c.data_ptr<float>(), hT.data_ptr<float>(),
                 cT.data_ptr<float>(), stream(), split ? &sb.s : nullptr,
                 out_bf.defined() ? reinterpret_cast<unsigned short*>(out_bf.data_ptr()) : nullptr);
  return {out, hT, cT, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, out_bf};
}

std::vector<at::Tensor> lnlstm_bwd(const at::Tensor& dout, const at::Tensor& dhT, const at::Tensor& dcT,
                                   const at::Tensor& gates, const at::Tensor& c_all, const at::Tensor& xhat_c,
                                   const at::Tensor& rstd_c, const at::Tensor& xhat_h, const at::Tensor& rstd_h,
                                   const at::Tensor& w, const at::Tensor& lnh_w, const at::Tensor& lnc_w) {
  for (auto* t : {&dout, &dhT, &dcT, &gates, &c_all, &xhat_c, &rstd_c, &xhat_h, &rstd_h, &w, &lnh_w, &lnc_w})
    check_cuda(*t, "lnlstm_bwd input");
  const int64_t T = gates.size(0), B = gates.size(1), G = gates.size(2), H = G / 4;
  TORCH_CHECK(w.size(0) == G && w.size(1) == H, "lnlstm_bwd: w must be [4H, H]");
  TORCH_CHECK(dout.scalar_type() == at::kFloat && dout.size(0) == T && dout.size(1) == B && dout.size(2) == H,
              "lnlstm_bwd: dout");
  c10::hip::HIPGuard g(gates.device().index());
  auto f = gates.options().dtype(at::kFloat);
  auto dgates = at::empty({T, B, G}, f);
  auto dhg = at::empty({T, B, G}, f);
  auto dc_ln = at::empty({T, B, H}, f);
  auto dh0 = at::empty({B, H}, f);
  auto dc0 = at::empty({B, H}, f);
  SplitBufs sb;
  const bool split = lstm_split_enabled(H, B);
  if (split) sb = make_split(gates, B, H);
  as::lnlstm_bwd(dout.data_ptr<float>(), dhT.data_ptr<float>(), dcT.data_ptr<float>(), gates.data_ptr<float>(),
                 c_all.data_ptr<float>(), xhat_c.data_ptr<float>(), rstd_c.data_ptr<float>(), xhat_h.data_ptr<float>(),
                 rstd_h.data_ptr<float>(), w.data_ptr(), dt(w), lnh_w.data_ptr<float>(), lnc_w.data_ptr<float>(),
                 static_cast<int>(T), static_cast<int>(B), static_cast<int>(H), dgates.data_ptr<float>(),
                 dhg.data_ptr<float>(), dc_ln.data_ptr<float>(), dh0.data_ptr<float>(), dc0.data_ptr<float>(),
                 stream(), split ? &sb.s : nullptr);
  return {dgates, dhg, dc_ln, dh0, dc0};
}

// ---------------------------------------------------------------- LayerNorm affine gradients (column sums)
// [2, C] fp32: row 0 = sum_r dy * xh, row 1 = sum_r dy (the LN weight / bias gradients) for fp32 dy, xh of equal
// shape (rows = every leading dim); one launch (+ one column reduction past 512 rows)
at::Tensor ln_affine_grads(const at::Tensor& dy, const at::Tensor& xh) {
  check_cuda(dy, "dy");
  check_cuda(xh, "xh");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && xh.scalar_type() == at::kFloat && dy.sizes() == xh.sizes() &&
                  dy.is_contiguous() && xh.is_contiguous() && dy.dim() >= 1, "ln_affine_grads: contiguous fp32, same shape");
  c10::hip::HIPGuard g(dy.device().index());
  const int64_t C = dy.size(-1), R = C ? dy.numel() / C : 0;
  auto out = at::empty({2, C}, dy.options());
  if (R == 0) return out.zero_();
  const int S = as::ln_affine_slices(R);
  at::Tensor part = S == 1 ? out : at::empty({S, 2 * C}, dy.options());
  as::ln_affine_grads(dy.data_ptr<float>(), xh.data_ptr<float>(), part.data_ptr<float>(), R, static_cast<int>(C), stream());
  if (S > 1) as::column_reduce(part.data_ptr<float>(), out.data_ptr<float>(), S, static_cast<int>(2 * C), stream());
  return out;
}

// ---------------------------------------------------------------- entity embedding
int src_dt(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kByte: case at::kBool: return as::SRC_U8;
    case at::kChar: return as::SRC_I8;
    case at::kShort: return as::SRC_I16;
    case at::kInt: return as::SRC_I32;
    case at::kLong: return as::SRC_I64;
    case at::kHalf: return as::SRC_F16;
    case at::kFloat: return as::SRC_F32;
    default: TORCH_CHECK(false, "entity field dtype ", t.scalar_type());
  }
}

as::EntityFields make_fields(const std::vector<at::Tensor>& fields, const std::vector<int64_t>& kind,
                             const std::vector<int64_t>& offset, const std::vector<int64_t>& width, int64_t numel) {
  TORCH_CHECK(fields.size() <= as::kMaxFields && fields.size() == kind.size() && kind.size() == offset.size() &&
                  offset.size() == width.size(), "entity fields table");
  as::EntityFields f{};
  f.n = static_cast<int>(fields.size());
  for (size_t i = 0; i < fields.size(); ++i) {
    check_cuda(fields[i], "entity field");
    TORCH_CHECK(fields[i].numel() == numel, "entity field numel mismatch");
    f.ptr[i] = fields[i].data_ptr();
    f.dtype[i] = src_dt(fields[i]);
    f.kind[i] = static_cast<int>(kind[i]);
    f.offset[i] = static_cast<int>(offset[i]);
    f.width[i] = static_cast<int>(width[i]);
  }
  return f;
}

at::Tensor entity_embed_fwd(const std::vector<at::Tensor>& fields, const std::vector<int64_t>& kind,
                            const std::vector<int64_t>& offset, const std::vector<int64_t>& width,
                            const at::Tensor& index, const at::Tensor& wT, const at::Tensor& bias, int64_t out_dtype) {
  check_cuda(index, "index");
  check_cuda(wT, "wT");
  TORCH_CHECK(index.scalar_type() == at::kLong, "index int64");
  TORCH_CHECK(wT.size(1) == 256 && bias.numel() == 256 && bias.scalar_type() == at::kFloat, "entity embed: 256 channels");
  auto f = make_fields(fields, kind, offset, width, fields.empty() ? 0 : fields[0].numel());
  for (int i = 0; i < f.n; ++i) TORCH_CHECK(f.offset[i] + (f.kind[i] == as::FIELD_SCALAR ? 1 : f.width[i]) <= wT.size(0), "field offset");
  c10::hip::HIPGuard g(wT.device().index());
  const int64_t T = index.numel();
  auto out = at::empty({T, 256}, wT.options().dtype(out_dtype == 1 ? at::kBFloat16 : at::kFloat));
  if (T > 0)
    as::entity_embed_fwd(f, index.data_ptr<int64_t>(), wT.data_ptr(), dt(wT), bias.data_ptr<float>(), out.data_ptr(),
                         dt(out), T, stream());
  return out;
}

at::Tensor entity_onehot(const std::vector<at::Tensor>& fields, const std::vector<int64_t>& kind,
                         const std::vector<int64_t>& offset, const std::vector<int64_t>& width, const at::Tensor& index,
                         int64_t k_in, int64_t out_dtype) {
  check_cuda(index, "index");
  auto f = make_fields(fields, kind, offset, width, fields.empty() ? 0 : fields[0].numel());
  c10::hip::HIPGuard g(index.device().index());
  const int64_t T = index.numel();
  auto X = at::zeros({T, k_in}, index.options().dtype(out_dtype == 1 ? at::kBFloat16 : at::kFloat));
  as::entity_onehot(f, index.data_ptr<int64_t>(), X.data_ptr(), dt(X), T, static_cast<int>(k_in), stream());
  return X;
}

// a [R, 32] @ W [32, N] (bf16) given wT = W^T [N, 32]
at::Tensor mm_k32(const at::Tensor& a, const at::Tensor& wT) {
  check_cuda(a, "a");
  check_cuda(wT, "wT");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && wT.scalar_type() == at::kBFloat16 && a.is_contiguous() &&
                  wT.is_contiguous() && a.dim() == 2 && a.size(1) == 32 && wT.dim() == 2 && wT.size(1) == 32 &&
                  wT.size(0) % 16 == 0, "mm_k32: a [R, 32], wT [N, 32] bf16 contiguous, N % 16 == 0");
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({a.size(0), wT.size(0)}, a.options());
  as::mm_k32(a.data_ptr(), wT.data_ptr(), out.data_ptr(), a.size(0), static_cast<int>(wT.size(0)), stream());
  return out;
}

// (dW [256, k_in] fp32, db [256] fp32) of relu(X W^T + b) from dout and the ReLU output (same dtype)
std::vector<at::Tensor> entity_embed_wgrad(const std::vector<at::Tensor>& fields, const std::vector<int64_t>& kind,
                                           const std::vector<int64_t>& offset, const std::vector<int64_t>& width,
                                           const at::Tensor& index, const at::Tensor& dout, const at::Tensor& out,
                                           int64_t k_in) {
  check_cuda(index, "index");
  check_cuda(dout, "dout");
  check_cuda(out, "out");
  const int64_t T = index.numel();
  TORCH_CHECK(dout.scalar_type() == out.scalar_type() && dout.is_contiguous() && out.is_contiguous() &&
                  dout.numel() == T * 256 && out.numel() == T * 256, "entity_embed_wgrad: dout / out [T, 256] contiguous");
  TORCH_CHECK(k_in >= 1 && k_in < 1024, "entity_embed_wgrad: K_in < 1024 (column K_in carries db)");
  auto f = make_fields(fields, kind, offset, width, fields.empty() ? 0 : fields[0].numel());
  for (int i = 0; i < f.n; ++i)
    TORCH_CHECK(f.offset[i] + (f.kind[i] == as::FIELD_SCALAR ? 1 : f.width[i]) <= k_in, "field offset");
  c10::hip::HIPGuard g(index.device().index());
  auto f32 = dout.options().dtype(at::kFloat);
  const int nchunk = as::entity_wgrad_chunks(T);
  const int64_t width_row = 256 * k_in + 256;
  auto part = at::empty({nchunk, width_row}, f32);
  as::entity_embed_wgrad(f, index.data_ptr<int64_t>(), dout.data_ptr(), out.data_ptr(), dt(dout), part.data_ptr<float>(),
                         T, static_cast<int>(k_in), nchunk, stream());
  auto red = at::empty({width_row}, f32);
  as::column_reduce(part.data_ptr<float>(), red.data_ptr<float>(), nchunk, width_row, stream());
  return {red.narrow(0, 0, 256 * k_in).view({256, k_in}), red.narrow(0, 256 * k_in, 256)};
}

// ---------------------------------------------------------------- spatial path (NHWC)
at::Tensor upsample2x_fwd(const at::Tensor& x) {  // x [B,H,W,C]
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 4 == 0, "upsample2x: NHWC with C % 4 == 0");
  c10::hip::HIPGuard g(x.device().index());
  auto y = at::empty({x.size(0), 2 * x.size(1), 2 * x.size(2), x.size(3)}, x.options());
  as::upsample2x_fwd(x.data_ptr(), y.data_ptr(), dt(x), x.size(0), x.size(1), x.size(2), x.size(3), stream());
  return y;
}

// mask (optional): the forward input x (NHWC, a ReLU output): dx *= [x > 0]
at::Tensor upsample2x_bwd(const at::Tensor& dy, const c10::optional<at::Tensor>& mask) {  // dy [B,2H,2W,C]
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.dim() == 4 && dy.size(3) % 4 == 0 && dy.size(1) % 2 == 0 && dy.size(2) % 2 == 0, "upsample2x_bwd");
  c10::hip::HIPGuard g(dy.device().index());
  auto dx = at::empty({dy.size(0), dy.size(1) / 2, dy.size(2) / 2, dy.size(3)}, dy.options());
  const void* mp = nullptr;
  if (mask && mask->defined()) {
    TORCH_CHECK(mask->sizes() == dx.sizes() && mask->scalar_type() == dy.scalar_type() && mask->is_contiguous(),
                "upsample2x_bwd: mask");
    mp = mask->data_ptr();
  }
  as::upsample2x_bwd(dy.data_ptr(), dx.data_ptr(), dt(dy), dx.size(0), dx.size(1), dx.size(2), dx.size(3), stream(),
                     mp);
  return dx;
}

as::SpatialPlanes make_planes(const std::vector<at::Tensor>& planes, const std::vector<at::Tensor>& effects) {
  TORCH_CHECK(planes.size() == 7 && effects.size() == 6, "spatial: 7 planes (height + 6 one-hot) and 6 effects");
  as::SpatialPlanes sp{};
  for (const auto& t : planes) {
    check_cuda(t, "plane");
    TORCH_CHECK(t.scalar_type() == at::kByte, "spatial planes must be uint8");
  }
  for (const auto& t : effects) {
    check_cuda(t, "effect");
    TORCH_CHECK(t.scalar_type() == at::kShort, "effects must be int16");
  }
  sp.height = planes[0].data_ptr<uint8_t>();
  for (int k = 0; k < 6; ++k) {
    TORCH_CHECK(planes[k + 1].numel() == planes[0].numel(), "plane size");
    sp.plane[k] = planes[k + 1].data_ptr<uint8_t>();
    sp.effect[k] = effects[k].data_ptr<int16_t>();
  }
  return sp;
}

// returns (effect bits [B,HW] u8, out [B,H,W,32] relu'd)
std::vector<at::Tensor> spatial_embed_fwd(const std::vector<at::Tensor>& planes, const std::vector<at::Tensor>& effects,
                                          const at::Tensor& w_dense, const at::Tensor& bias, const at::Tensor& rows,
                                          const at::Tensor& ex, const at::Tensor& ey, const at::Tensor& entity_num,
                                          int64_t out_dtype) {
  auto sp = make_planes(planes, effects);
  const int64_t B = planes[0].size(0), H = planes[0].size(1), W = planes[0].size(2), HW = H * W;
  const int64_t L = effects[0].size(1);
  TORCH_CHECK(w_dense.size(0) == 32 && w_dense.size(1) == 24 && w_dense.scalar_type() == at::kFloat, "w_dense [32,24]");
  check_cuda(rows, "rows");
  TORCH_CHECK(rows.dim() == 3 && rows.size(0) == B && rows.size(2) == 32, "rows [B,N,32]");
  TORCH_CHECK(ex.scalar_type() == at::kByte && ey.scalar_type() == at::kByte && entity_num.scalar_type() == at::kLong,
              "entity x/y uint8, entity_num int64");
  c10::hip::HIPGuard g(rows.device().index());
  TORCH_CHECK(rows.is_contiguous() && ex.is_contiguous() && ey.is_contiguous() && entity_num.is_contiguous(),
              "spatial: contiguous rows / entity coordinates");
  auto out = at::empty({B, H, W, 32}, rows.options().dtype(out_dtype == 1 ? at::kBFloat16 : at::kFloat));
  as::spatial_embed_fused(sp, w_dense.data_ptr<float>(), bias.data_ptr<float>(), rows.data_ptr(), dt(rows),
                          ex.data_ptr<uint8_t>(), ey.data_ptr<uint8_t>(), entity_num.data_ptr<int64_t>(),
                          out.data_ptr(), dt(out), static_cast<int>(B), static_cast<int>(rows.size(1)),
                          static_cast<int>(H), static_cast<int>(W), static_cast<int>(L), stream());
  return {at::Tensor(), out};
}

// relu(embed) -> max_pool2x2 fused: {pooled [B,H/2,W/2,32] bf16, pos [B,H/2,W/2,32] uint8}
std::vector<at::Tensor> spatial_embed_pool_fwd(const std::vector<at::Tensor>& planes, const std::vector<at::Tensor>& effects,
                                               const at::Tensor& w_dense, const at::Tensor& bias, const at::Tensor& rows,
                                               const at::Tensor& ex, const at::Tensor& ey, const at::Tensor& entity_num) {
  auto sp = make_planes(planes, effects);
  const int64_t B = planes[0].size(0), H = planes[0].size(1), W = planes[0].size(2);
  const int64_t L = effects[0].size(1);
  TORCH_CHECK(as::spatial_pool_supported(static_cast<int>(H), static_cast<int>(W)), "spatial_embed_pool: H, W");
  TORCH_CHECK(w_dense.size(0) == 32 && w_dense.size(1) == 24 && w_dense.scalar_type() == at::kFloat &&
              bias.scalar_type() == at::kFloat && bias.numel() == 32, "spatial_embed_pool: w_dense [32,24], bias fp32");
  check_cuda(rows, "rows");
  TORCH_CHECK(rows.dim() == 3 && rows.size(0) == B && rows.size(2) == 32 && rows.is_contiguous() &&
              (rows.scalar_type() == at::kBFloat16 || rows.scalar_type() == at::kFloat),
              "spatial_embed_pool: rows [B,N,32] bf16 / fp32 (the pooled map takes rows' dtype)");
  TORCH_CHECK(ex.scalar_type() == at::kByte && ey.scalar_type() == at::kByte && entity_num.scalar_type() == at::kLong &&
              ex.is_contiguous() && ey.is_contiguous() && entity_num.is_contiguous(),
              "spatial_embed_pool: entity x/y uint8, entity_num int64, contiguous");
  c10::hip::HIPGuard g(rows.device().index());
  auto pooled = at::empty({B, H / 2, W / 2, 32}, rows.options());
  auto pos = at::empty({B, H / 2, W / 2, 32}, rows.options().dtype(at::kByte));
  as::spatial_embed_pool(sp, w_dense.data_ptr<float>(), bias.data_ptr<float>(), rows.data_ptr(), ex.data_ptr<uint8_t>(),
                         ey.data_ptr<uint8_t>(), entity_num.data_ptr<int64_t>(), pooled.data_ptr(),
                         pos.data_ptr<uint8_t>(), static_cast<int>(B), static_cast<int>(rows.size(1)),
                         static_cast<int>(H), static_cast<int>(W), static_cast<int>(L), stream(),
                         rows.scalar_type() == at::kFloat);
  return {pooled, pos};
}

// (dWd fp32 [32, 24], db fp32 [32]) of the spatial 1x1 projection's dense columns from dpre [B,H,W,32]
// gate (optional): the embedding's ReLU output; dpre is then dout and the ReLU mask is applied on the fly
std::vector<at::Tensor> spatial_dense_wgrad(const std::vector<at::Tensor>& planes, const std::vector<at::Tensor>& effects,
                                            const at::Tensor& dpre, const c10::optional<at::Tensor>& gate) {
  auto sp = make_planes(planes, effects);
  const int64_t B = planes[0].size(0), H = planes[0].size(1), W = planes[0].size(2);
  const int64_t L = effects[0].size(1);
  check_cuda(dpre, "dpre");
  TORCH_CHECK(dpre.is_contiguous() && dpre.numel() == B * H * W * 32, "spatial_dense_wgrad: dpre [B,H,W,32] contiguous");
  const void* gp = nullptr;
  if (gate.has_value()) {
    TORCH_CHECK(gate->is_contiguous() && gate->sizes() == dpre.sizes() && gate->scalar_type() == dpre.scalar_type(),
                "spatial_dense_wgrad: gate like dpre");
    gp = gate->data_ptr();
  }
  c10::hip::HIPGuard g(dpre.device().index());
  const int nb = as::spatial_wgrad_blocks(static_cast<int>(B));
  auto f32 = dpre.options().dtype(at::kFloat);
  auto part = at::empty({nb, 32 * 24 + 32}, f32);
  as::spatial_dense_wgrad(sp, dpre.data_ptr(), gp, dt(dpre), part.data_ptr<float>(), static_cast<int>(B),
                          static_cast<int>(H), static_cast<int>(W), static_cast<int>(L), stream());
  auto red = at::empty({32 * 24 + 32}, f32);
  as::column_reduce(part.data_ptr<float>(), red.data_ptr<float>(), nb, 32 * 24 + 32, stream());
  return {red.narrow(0, 0, 32 * 24).view({32, 24}), red.narrow(0, 32 * 24, 32)};
}

at::Tensor spatial_gather_rows(const at::Tensor& dpre, const at::Tensor& ex, const at::Tensor& ey,
                               const at::Tensor& entity_num, int64_t N, const c10::optional<at::Tensor>& gate) {
  check_cuda(dpre, "dpre");
  TORCH_CHECK(dpre.is_contiguous() && dpre.dim() == 4 && dpre.size(3) == 32, "spatial_gather_rows: dpre [B,H,W,32]");
  const void* gp = nullptr;
  if (gate.has_value()) {
    TORCH_CHECK(gate->is_contiguous() && gate->sizes() == dpre.sizes() && gate->scalar_type() == dpre.scalar_type(),
                "spatial_gather_rows: gate like dpre");
    gp = gate->data_ptr();
  }
  const int64_t B = dpre.size(0), H = dpre.size(1), W = dpre.size(2);
  c10::hip::HIPGuard g(dpre.device().index());
  auto drows = at::empty({B, N, 32}, dpre.options());
  as::gather_rows(dpre.data_ptr(), gp, dt(dpre), ex.data_ptr<uint8_t>(), ey.data_ptr<uint8_t>(),
                  entity_num.data_ptr<int64_t>(), drows.data_ptr(), B, N, H, W, stream());
  return drows;
}

// the fused embed + pool stage's backward without the full-resolution dpre (fp32): dy, y [B, H/2, W/2, 32] fp32 (pooled
// gradient, pooled ReLU output), pos [B, H/2, W/2, 32] uint8 (per-channel argmax in the 2x2 window)
std::vector<at::Tensor> spatial_dense_wgrad_pooled(const std::vector<at::Tensor>& planes,
                                                   const std::vector<at::Tensor>& effects, const at::Tensor& dy,
                                                   const at::Tensor& y, const at::Tensor& pos) {
  auto sp = make_planes(planes, effects);
  const int64_t B = planes[0].size(0), H = planes[0].size(1), W = planes[0].size(2);
  const int64_t L = effects[0].size(1);
  for (auto* t : {&dy, &y, &pos}) check_cuda(*t, "pooled operand");
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0, "spatial_dense_wgrad_pooled: even H, W");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat && pos.scalar_type() == at::kByte,
              "spatial_dense_wgrad_pooled: fp32 dy / y, uint8 pos");
  for (auto* t : {&dy, &y, &pos})
    TORCH_CHECK(t->is_contiguous() && t->numel() == B * (H / 2) * (W / 2) * 32, "spatial_dense_wgrad_pooled: [B,H/2,W/2,32]");
  c10::hip::HIPGuard g(dy.device().index());
  const int nb = as::spatial_wgrad_blocks(static_cast<int>(B));
  auto f32 = dy.options().dtype(at::kFloat);
  auto part = at::empty({nb, 32 * 24 + 32}, f32);
  as::spatial_dense_wgrad_pooled(sp, dy.data_ptr<float>(), y.data_ptr<float>(), pos.data_ptr<uint8_t>(),
                                 part.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                                 static_cast<int>(L), stream());
  auto red = at::empty({32 * 24 + 32}, f32);
  as::column_reduce(part.data_ptr<float>(), red.data_ptr<float>(), nb, 32 * 24 + 32, stream());
  return {red.narrow(0, 0, 32 * 24).view({32, 24}), red.narrow(0, 32 * 24, 32)};
}

at::Tensor spatial_gather_rows_pooled(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& pos,
                                      const at::Tensor& ex, const at::Tensor& ey, const at::Tensor& entity_num, int64_t N,
                                      int64_t H, int64_t W) {
  for (auto* t : {&dy, &y, &pos}) check_cuda(*t, "pooled operand");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat && pos.scalar_type() == at::kByte &&
                  dy.is_contiguous() && y.is_contiguous() && pos.is_contiguous() && dy.dim() == 4 && dy.size(3) == 32 &&
                  y.sizes() == dy.sizes() && pos.sizes() == dy.sizes() && dy.size(1) == H / 2 && dy.size(2) == W / 2,
              "spatial_gather_rows_pooled: fp32 dy / y, uint8 pos [B,H/2,W/2,32]");
  TORCH_CHECK(ex.scalar_type() == at::kByte && ey.scalar_type() == at::kByte && entity_num.scalar_type() == at::kLong,
              "spatial_gather_rows_pooled: uint8 ex / ey, int64 entity_num");
  const int64_t B = dy.size(0);
  TORCH_CHECK(ex.numel() == B * N && ey.numel() == B * N && entity_num.numel() == B, "spatial_gather_rows_pooled: rows");
  c10::hip::HIPGuard g(dy.device().index());
  auto drows = at::empty({B, N, 32}, dy.options());
  as::gather_rows_pooled(dy.data_ptr<float>(), y.data_ptr<float>(), pos.data_ptr<uint8_t>(), ex.data_ptr<uint8_t>(),
                         ey.data_ptr<uint8_t>(), entity_num.data_ptr<int64_t>(), drows.data_ptr<float>(),
                         static_cast<int>(B), static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), stream());
  return drows;
}

at::Tensor spatial_dense_input(const std::vector<at::Tensor>& planes, const std::vector<at::Tensor>& effects,
                               const at::Tensor& bits, int64_t x_dtype) {
  auto sp = make_planes(planes, effects);
  const int64_t npix = planes[0].numel();
  c10::hip::HIPGuard g(bits.device().index());
  auto X = at::empty({npix, 24}, bits.options().dtype(x_dtype == 1 ? at::kBFloat16 : at::kFloat));
  as::spatial_dense_input(sp, bits.data_ptr<uint8_t>(), X.data_ptr(), dt(X), npix, stream());
  return X;
}

// ---------------------------------------------------------------- varlen attention
std::vector<at::Tensor> varlen_attn_fwd(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_len, int64_t H) {
  check_cuda(qkv, "qkv");
  check_cuda(cu, "cu_seqlens");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 2 && qkv.size(1) == 3 * H * 128,
              "varlen_attn: qkv bf16 [T, 3*H*128]");
  TORCH_CHECK(cu.scalar_type() == at::kInt, "cu_seqlens int32");
  const int64_t T = qkv.size(0), S = cu.numel() - 1;
  c10::hip::HIPGuard g(qkv.device().index());
  auto out = at::empty({T, H * 128}, qkv.options());
  auto lse = at::empty({H, T}, qkv.options().dtype(at::kFloat));
  if (T > 0 && S > 0)
    as::varlen_attn_fwd(qkv.data_ptr(), cu.data_ptr<int>(), out.data_ptr(), lse.data_ptr<float>(), S, max_len, H, T,
                        1.0f / std::sqrt(128.0f), stream());
  return {out, lse};
}

at::Tensor varlen_attn_bwd(const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& dout, const at::Tensor& lse,
                           const at::Tensor& cu, int64_t max_len, int64_t H) {
  check_cuda(dout, "dout");
  TORCH_CHECK(dout.scalar_type() == at::kBFloat16 && dout.sizes() == out.sizes(), "varlen_attn_bwd: dout");
  const int64_t T = qkv.size(0), S = cu.numel() - 1;
  c10::hip::HIPGuard g(qkv.device().index());
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({H, T}, qkv.options().dtype(at::kFloat));
  if (T > 0 && S > 0)
    as::varlen_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), cu.data_ptr<int>(),
                        dqkv.data_ptr(), delta.data_ptr<float>(), S, max_len, H, T, 1.0f / std::sqrt(128.0f), stream());
  return dqkv;
}


std::vector<at::Tensor> varlen_attn_fwd_f32(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_len, int64_t H) {
  check_cuda(qkv, "qkv");
  check_cuda(cu, "cu_seqlens");
  TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.dim() == 2 && qkv.size(1) == 3 * H * 128 && qkv.is_contiguous(),
              "varlen_attn_f32: qkv fp32 contiguous [T, 3*H*128]");
  TORCH_CHECK(cu.scalar_type() == at::kInt && cu.is_contiguous(), "cu_seqlens int32");
  const int64_t T = qkv.size(0), S = cu.numel() - 1;
  c10::hip::HIPGuard g(qkv.device().index());
  auto out = at::empty({T, H * 128}, qkv.options());
  auto lse = at::empty({H, T}, qkv.options());
  if (T > 0 && S > 0)
    as::varlen_attn_fwd_f32(qkv.data_ptr<float>(), cu.data_ptr<int>(), out.data_ptr<float>(), lse.data_ptr<float>(), S,
                            max_len, H, T, 1.0f / std::sqrt(128.0f), stream());
  return {out, lse};
}

at::Tensor varlen_attn_bwd_f32(const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& dout,
                               const at::Tensor& lse, const at::Tensor& cu, int64_t max_len, int64_t H) {
  check_cuda(dout, "dout");
  TORCH_CHECK(qkv.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && dout.scalar_type() == at::kFloat &&
              dout.sizes() == out.sizes() && dout.is_contiguous() && out.is_contiguous(), "varlen_attn_bwd_f32: fp32");
  const int64_t T = qkv.size(0), S = cu.numel() - 1;
  c10::hip::HIPGuard g(qkv.device().index());
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({H, T}, qkv.options());
  if (T > 0 && S > 0)
    as::varlen_attn_bwd_f32(qkv.data_ptr<float>(), out.data_ptr<float>(), dout.data_ptr<float>(), lse.data_ptr<float>(),
                            cu.data_ptr<int>(), dqkv.data_ptr<float>(), delta.data_ptr<float>(), S, max_len, H, T,
                            1.0f / std::sqrt(128.0f), stream());
  return dqkv;
}


// ---------------------------------------------------------------- selected-units sampler
std::vector<at::Tensor> su_sample(const at::Tensor& key, const at::Tensor& c0, const at::Tensor& u,
                                  const at::Tensor& entity_num, const at::Tensor& su_mask, const at::Tensor& wf,
                                  const at::Tensor& bf, const at::Tensor& wq2, const at::Tensor& bq2,
                                  const at::Tensor& wih, const at::Tensor& whh, const at::Tensor& lni_w,
                                  const at::Tensor& lni_b, const at::Tensor& lnh_w, const at::Tensor& lnh_b,
                                  const at::Tensor& lnc_w, const at::Tensor& lnc_b, const at::Tensor& we1,
                                  const at::Tensor& be1, double temperature, double eps, int64_t max_steps,
                                  bool extra_units) {
  for (auto* t : {&key, &c0, &u, &entity_num, &su_mask, &wf, &bf, &wq2, &bq2, &wih, &whh, &lni_w, &lni_b, &lnh_w,
                  &lnh_b, &lnc_w, &lnc_b, &we1, &be1})
    check_cuda(*t, "su_sample input");
  const int64_t B = key.size(0), N1 = key.size(1);
  TORCH_CHECK(key.dim() == 3 && key.size(2) == 32, "su_sample: key must be [B, N+1, 32]");
  TORCH_CHECK(N1 >= 1 && N1 <= 513, "su_sample: N+1 must be in [1, 513]");
  TORCH_CHECK(c0.scalar_type() == at::kFloat && c0.size(0) == B && c0.size(1) == 256, "su_sample: c0 [B,256] fp32");
  TORCH_CHECK(u.scalar_type() == at::kFloat && u.size(0) == B && u.size(1) == max_steps, "su_sample: u [B,steps]");
  TORCH_CHECK(max_steps >= 1 && max_steps <= 64, "su_sample: 1..64 steps (the kernel stages the uniforms in LDS)");
  TORCH_CHECK(entity_num.scalar_type() == at::kLong && entity_num.numel() == B, "su_sample: entity_num int64 [B]");
  TORCH_CHECK(su_mask.scalar_type() == at::kByte && su_mask.numel() == B, "su_sample: su_mask uint8 [B]");
  TORCH_CHECK(wf.scalar_type() == at::kBFloat16 && wf.size(0) == 256 && wf.size(1) == 256, "su_sample: wf bf16");
  TORCH_CHECK(wq2.size(0) == 32 && wq2.size(1) == 256 && wih.size(0) == 128 && wih.size(1) == 32 &&
              whh.size(0) == 128 && whh.size(1) == 32 && we1.size(0) == 256 && we1.size(1) == 32,
              "su_sample: weight shapes");
  for (auto* t : {&bf, &wq2, &bq2, &wih, &whh, &lni_w, &lni_b, &lnh_w, &lnh_b, &lnc_w, &lnc_b, &we1, &be1})
    TORCH_CHECK(t->scalar_type() == at::kFloat, "su_sample: fp32 weights");
  c10::hip::HIPGuard g(key.device().index());
  auto f = key.options().dtype(at::kFloat);
  // every element is written by the kernel (its prologue fills the steps a row does not run)
  auto logits = at::empty({B, max_steps, N1}, f);
  auto results = at::empty({B, max_steps}, key.options().dtype(at::kLong));
  auto logp = at::empty({B, max_steps}, f);
  auto su_num = at::empty({B}, key.options().dtype(at::kLong));
  auto emb = at::empty({B, 32}, f);
  auto extra = extra_units ? at::empty({B, 513}, f) : at::zeros({B, 1}, f);   // [B, 513]: the padded entity width
  as::su_sample(key.data_ptr(), dt(key), N1 * 32, c0.data_ptr<float>(), u.data_ptr<float>(),
                entity_num.data_ptr<int64_t>(), su_mask.data_ptr<uint8_t>(),
                reinterpret_cast<const uint16_t*>(wf.data_ptr()), bf.data_ptr<float>(), wq2.data_ptr<float>(),
                bq2.data_ptr<float>(), wih.data_ptr<float>(), whh.data_ptr<float>(), lni_w.data_ptr<float>(),
                lni_b.data_ptr<float>(), lnh_w.data_ptr<float>(), lnh_b.data_ptr<float>(), lnc_w.data_ptr<float>(),
                lnc_b.data_ptr<float>(), we1.data_ptr<float>(), be1.data_ptr<float>(),
                static_cast<float>(1.0 / temperature), static_cast<float>(eps), static_cast<int>(B),
                static_cast<int>(N1), static_cast<int>(max_steps), extra_units ? 1 : 0, logits.data_ptr<float>(),
                results.data_ptr<int64_t>(), logp.data_ptr<float>(), su_num.data_ptr<int64_t>(), emb.data_ptr<float>(),
                extra.data_ptr<float>(), stream());
  return {logits, results, logp, su_num, emb, extra};
}


// ---------------------------------------------------------------- trajectory ring gather
void segment_copy(const at::Tensor& arena, const at::Tensor& out, const at::Tensor& seg) {
  check_cuda(arena, "arena");
  check_cuda(out, "out");
  check_cuda(seg, "seg");
  TORCH_CHECK(arena.scalar_type() == at::kByte && out.scalar_type() == at::kByte, "segment_copy: uint8 buffers");
  TORCH_CHECK(seg.scalar_type() == at::kLong && seg.dim() == 2 && seg.size(1) == 3, "segment_copy: seg [n,3] int64");
  c10::hip::HIPGuard g(arena.device().index());
  as::segment_copy(arena.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), seg.data_ptr<int64_t>(), seg.size(0), stream());
}


// ---------------------------------------------------------------- flipped / transposed conv3x3 weight
at::Tensor conv_wt(const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda(), "conv_wt: w must be a GPU tensor");   // any strides: read through them
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3,
              "conv_wt: bf16 [Cout,Cin,3,3] weight");
  c10::hip::HIPGuard g(w.device().index());
  const int cout = (int)w.size(0), cin = (int)w.size(1);
  auto out = at::empty({cin, 3, 3, cout}, w.options().memory_format(at::MemoryFormat::Contiguous));
  as::conv_wt(reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()), cout, cin,
              w.stride(0), w.stride(1), w.stride(2), w.stride(3), stream());
  return out;
}

// ---------------------------------------------------------------- fused upsample x2 + conv3x3 -> 1 channel
void check_upconv_x(const at::Tensor& x) {
  TORCH_CHECK(x.dim() == 4 && x.size(3) == as::upconv1_channels() && x.is_contiguous(),
              "upconv1: x must be contiguous NHWC [B,H,W,32]");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "upconv1: x fp32 or bf16");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "upconv1: x must be 16-byte aligned");
}

at::Tensor upconv1_fwd(const at::Tensor& x_nhwc, const at::Tensor& w, const at::Tensor& bias) {
  check_cuda(x_nhwc, "x");
  check_cuda(w, "w");
  check_upconv_x(x_nhwc);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == as::upconv1_channels() * 9,
              "upconv1: w fp32 contiguous [32*9]");
  check_cuda(bias, "bias");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == 1, "upconv1: bias fp32 [1]");
  const int64_t B = x_nhwc.size(0), H = x_nhwc.size(1), W = x_nhwc.size(2);
  c10::hip::HIPGuard g(x_nhwc.device().index());
  auto y = at::empty({B, 2 * H, 2 * W}, x_nhwc.options().dtype(at::kFloat));
  as::upconv1_fwd(x_nhwc.data_ptr(), dt(x_nhwc), w.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr<float>(),
                  static_cast<int>(B), static_cast<int>(H), static_cast<int>(W), stream());
  return y;
}

std::vector<at::Tensor> upconv1_bwd(const at::Tensor& x_nhwc, const at::Tensor& w, const at::Tensor& dy,
                                    bool relu_mask) {
  check_cuda(x_nhwc, "x");
  check_cuda(w, "w");
  check_cuda(dy, "dy");
  const int64_t B = x_nhwc.size(0), H = x_nhwc.size(1), W = x_nhwc.size(2);
  check_upconv_x(x_nhwc);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == as::upconv1_channels() * 9,
              "upconv1_bwd: w fp32 contiguous [32*9]");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && dy.is_contiguous() && dy.numel() == B * 4 * H * W,
              "upconv1_bwd: dy contiguous [B,2H,2W] fp32");
  c10::hip::HIPGuard g(x_nhwc.device().index());
  auto dx = at::empty_like(x_nhwc);
  const int64_t tiles = as::upconv1_tiles(static_cast<int>(B), static_cast<int>(H), static_cast<int>(W));
  auto part = at::empty({tiles, as::upconv1_channels() * 9 + 1}, dy.options());
  auto dwb = at::empty({as::upconv1_channels() * 9 + 1}, dy.options());
  as::upconv1_bwd(x_nhwc.data_ptr(), dt(x_nhwc), w.data_ptr<float>(), dy.data_ptr<float>(), dx.data_ptr(),
                  part.data_ptr<float>(), dwb.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H),
                  static_cast<int>(W), stream(), relu_mask);
  return {dx, dwb};
}

// ---------------------------------------------------------------- max-pool 2x2 (NHWC)
std::vector<at::Tensor> maxpool2_fwd(const at::Tensor& x) {  // x [B,H,W,C]
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "maxpool2: NHWC with C % 8 == 0");
  c10::hip::HIPGuard g(x.device().index());
  auto y = at::empty({x.size(0), x.size(1) / 2, x.size(2) / 2, x.size(3)}, x.options());
  auto pos = at::empty(y.sizes(), x.options().dtype(at::kByte));
  as::maxpool2_fwd(x.data_ptr(), y.data_ptr(), pos.data_ptr<uint8_t>(), dt(x), x.size(0), x.size(1), x.size(2),
                   x.size(3), stream());
  return {y, pos};
}

// mask (optional): the forward input x (NHWC, a ReLU output): dx *= [x > 0]
at::Tensor maxpool2_bwd(const at::Tensor& dy, const at::Tensor& pos, int64_t H, int64_t W,
                        const c10::optional<at::Tensor>& mask) {
  check_cuda(dy, "dy");
  check_cuda(pos, "pos");
  TORCH_CHECK(dy.dim() == 4 && dy.sizes() == pos.sizes() && dy.size(1) == H / 2 && dy.size(2) == W / 2,
              "maxpool2_bwd: shapes");
  c10::hip::HIPGuard g(dy.device().index());
  auto dx = at::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  const void* mp = nullptr;
  if (mask && mask->defined()) {
    TORCH_CHECK(mask->sizes() == dx.sizes() && mask->scalar_type() == dy.scalar_type() && mask->is_contiguous(),
                "maxpool2_bwd: mask");
    mp = mask->data_ptr();
  }
  as::maxpool2_bwd(dy.data_ptr(), pos.data_ptr<uint8_t>(), dx.data_ptr(), dt(dy), dy.size(0), H, W, dy.size(3),
                   stream(), mp);
  return dx;
}

at::Tensor maxpool2_bwd_relu(const at::Tensor& dy, const at::Tensor& pos, const at::Tensor& y, int64_t H, int64_t W) {
  check_cuda(dy, "dy");
  check_cuda(pos, "pos");
  check_cuda(y, "y");
  TORCH_CHECK(((dy.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16) ||
               (dy.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat)) && dy.dim() == 4 &&
              dy.is_contiguous() && y.is_contiguous() && pos.is_contiguous() &&
              dy.sizes() == pos.sizes() && dy.sizes() == y.sizes() && H % 2 == 0 && W % 2 == 0 &&
              dy.size(1) == H / 2 && dy.size(2) == W / 2 && dy.size(3) % 8 == 0, "maxpool2_bwd_relu: shapes");
  TORCH_CHECK(dy.numel() < (1L << 31) - (1L << 24), "maxpool2_bwd_relu: size");
  c10::hip::HIPGuard g(dy.device().index());
  auto dx = at::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  as::maxpool2_bwd_relu(dy.data_ptr(), pos.data_ptr<uint8_t>(), y.data_ptr(), dx.data_ptr(), dy.size(0), H, W,
                        dy.size(3), stream(), dy.scalar_type() == at::kFloat);
  return dx;
}

// ---------------------------------------------------------------- segment sum / table gradient
at::Tensor segment_sum(const at::Tensor& x, const at::Tensor& cu) {  // x [T,C], cu [S+1] int32 -> [S,C] fp32
  check_cuda(x, "x");
  check_cuda(cu, "cu");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 4 == 0 && x.size(1) <= 1024, "segment_sum: x [T, C<=1024]");
  TORCH_CHECK(cu.scalar_type() == at::kInt, "segment_sum: cu int32");
  c10::hip::HIPGuard g(x.device().index());
  const int64_t S = cu.numel() - 1;
  auto out = at::empty({S, x.size(1)}, x.options().dtype(at::kFloat));
  as::segment_sum(x.data_ptr(), dt(x), cu.data_ptr<int>(), out.data_ptr<float>(), S, x.size(1), stream());
  return out;
}

// x [B,N,C] bf16 / fp32, valid [B,N] bool, num [B] int64 / int32 -> [B,C] in x's dtype (inference, no autograd)
at::Tensor entity_mean_pool(const at::Tensor& x, const at::Tensor& valid, const at::Tensor& num) {
  check_cuda(x, "x");
  check_cuda(valid, "valid");
  check_cuda(num, "num");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "entity_mean_pool: contiguous x [B, N, C] bf16 / fp32");
  TORCH_CHECK(valid.scalar_type() == at::kBool && valid.is_contiguous() && valid.size(0) == x.size(0) &&
                  valid.size(1) == x.size(1) && valid.dim() == 2, "entity_mean_pool: valid [B, N] bool");
  TORCH_CHECK((num.scalar_type() == at::kLong || num.scalar_type() == at::kInt) && num.numel() == x.size(0) &&
                  num.is_contiguous(), "entity_mean_pool: num [B] int64 / int32");
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({x.size(0), x.size(2)}, x.options());
  as::entity_mean_pool(x.data_ptr(), dt(x), valid.data_ptr<bool>(), num.data_ptr(), num.scalar_type() == at::kLong,
                       out.data_ptr(), static_cast<int>(x.size(0)), static_cast<int>(x.size(1)),
                       static_cast<int>(x.size(2)), stream());
  return out;
}

at::Tensor table_grad(const at::Tensor& src, const at::Tensor& idx, int64_t V) {  // src [U,D], idx [U] int64
  check_cuda(src, "src");
  check_cuda(idx, "idx");
  TORCH_CHECK(src.dim() == 2 && idx.scalar_type() == at::kLong && idx.numel() == src.size(0), "table_grad: shapes");
  TORCH_CHECK(V * src.size(1) <= 16384, "table_grad: table too large for LDS accumulation");
  c10::hip::HIPGuard g(src.device().index());
  auto out = at::zeros({V, src.size(1)}, src.options().dtype(at::kFloat));
  as::table_grad(src.data_ptr(), dt(src), idx.data_ptr<int64_t>(), out.data_ptr<float>(), src.size(0), V, src.size(1),
                 stream());
  return out;
}

namespace {
int idx_dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kLong: return 0;
    case at::kInt: return 1;
    case at::kShort: return 2;
    case at::kByte: return 3;
    case at::kChar: return 4;
    default: TORCH_CHECK(false, "embed_relu: integer index tensor expected");
  }
  return 0;
}
}  // namespace

// relu(table[clamp(idx)]) -> [U, D] (table fp32 or bf16 [V, D]; idx any integer dtype, contiguous)
at::Tensor embed_relu_fwd(const at::Tensor& table, const at::Tensor& idx) {
  check_cuda(table, "table");
  check_cuda(idx, "idx");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous() && idx.is_contiguous(), "embed_relu: contiguous [V, D] table");
  TORCH_CHECK(table.scalar_type() == at::kFloat || table.scalar_type() == at::kBFloat16, "embed_relu: fp32 / bf16");
  c10::hip::HIPGuard g(table.device().index());
  auto out = at::empty({idx.numel(), table.size(1)}, table.options());
  as::embed_relu_fwd(table.data_ptr(), dt(table), idx.data_ptr(), idx_dtype_code(idx), out.data_ptr(), idx.numel(),
                     static_cast<int>(table.size(0)), static_cast<int>(table.size(1)), stream());
  return out;
}

// d table (fp32 [V, D]) of embed_relu_fwd: rows of dout masked by out > 0, summed per (clamped) index
at::Tensor embed_relu_bwd(const at::Tensor& dout, const at::Tensor& out, const at::Tensor& idx, int64_t V) {
  check_cuda(dout, "dout");
  TORCH_CHECK(dout.sizes() == out.sizes() && dout.scalar_type() == out.scalar_type() && dout.is_contiguous() &&
                  out.is_contiguous() && out.dim() == 2 && idx.numel() == out.size(0) && idx.is_contiguous(),
              "embed_relu_bwd: dout / out [U, D] contiguous, idx [U]");
  TORCH_CHECK(V * out.size(1) <= 16384, "embed_relu_bwd: table too large for LDS accumulation");
  c10::hip::HIPGuard g(out.device().index());
  const long U = out.size(0), D = out.size(1);
  const bool direct = U * D <= 2048;
  auto dtab = direct ? at::empty({V, D}, out.options().dtype(at::kFloat))
                     : at::zeros({V, D}, out.options().dtype(at::kFloat));
  as::embed_relu_bwd(dout.data_ptr(), out.data_ptr(), dt(out), idx.data_ptr(), idx_dtype_code(idx),
                     dtab.data_ptr<float>(), U, static_cast<int>(V), static_cast<int>(D), direct, stream());
  return dtab;
}

// (valid bool [B, N], flat int64 [total], seg int64 [total], cu int32 [B + 1]) of the entity packing
std::vector<at::Tensor> entity_pack(const at::Tensor& num, int64_t N, int64_t total) {
  check_cuda(num, "entity_num");
  TORCH_CHECK(num.dim() == 1 && num.is_contiguous() && (num.scalar_type() == at::kLong || num.scalar_type() == at::kInt),
              "entity_pack: entity_num int64 / int32 [B]");
  TORCH_CHECK(N > 0 && total >= 0 && num.size(0) * N < (1L << 31), "entity_pack: sizes");
  c10::hip::HIPGuard g(num.device().index());
  const int64_t B = num.size(0);
  auto o = num.options();
  auto valid = at::empty({B, N}, o.dtype(at::kBool));
  auto flat = at::empty({total}, o.dtype(at::kLong));
  auto seg = at::empty({total}, o.dtype(at::kLong));
  auto cu = at::empty({B + 1}, o.dtype(at::kInt));
  if (B == 0) {
    cu.zero_();
    return {valid, flat, seg, cu};
  }
  as::entity_pack(num.data_ptr(), num.scalar_type() == at::kLong, static_cast<int>(B), static_cast<int>(N), total,
                  valid.data_ptr<bool>(), flat.data_ptr<int64_t>(), seg.data_ptr<int64_t>(), cu.data_ptr<int>(),
                  stream());
  return {valid, flat, seg, cu};
}

// B [N, K] fp32 (or, trans, B^T given as [K, N]) -> its bf16 fragment planes (uint8 [presplit_b_bytes]) for
// gemm_f32_psb; out: an existing planes buffer of that size to rebuild in place
at::Tensor presplit_b(const at::Tensor& b, bool trans, const c10::optional<at::Tensor>& out) {
  check_cuda(b, "b");
  TORCH_CHECK(b.dim() == 2 && b.scalar_type() == at::kFloat && b.is_contiguous(), "presplit_b: contiguous fp32 matrix");
  c10::hip::HIPGuard g(b.device().index());
  const int N = static_cast<int>(trans ? b.size(1) : b.size(0)), K = static_cast<int>(trans ? b.size(0) : b.size(1));
  const long bytes = as::presplit_b_bytes(N, K);
  at::Tensor o;
  if (out && out->defined()) {
    TORCH_CHECK(out->scalar_type() == at::kByte && out->numel() == bytes && out->is_contiguous() &&
                    out->device() == b.device(), "presplit_b: out must be a uint8 planes buffer of the right size");
    o = *out;
  } else {
    o = at::empty({bytes}, b.options().dtype(at::kByte));
  }
  as::presplit_b(b.data_ptr<float>(), N, K, trans, o.data_ptr(), stream());
  return o;
}

// presplit_b(srcs[i], trans[i], outs[i]) for every i, in launches of up to 48 weights
void multi_presplit(const std::vector<at::Tensor>& srcs, const std::vector<bool>& trans,
                    const std::vector<at::Tensor>& outs) {
  TORCH_CHECK(srcs.size() == trans.size() && srcs.size() == outs.size(), "multi_presplit: list sizes");
  if (srcs.empty()) return;
  c10::hip::HIPGuard g(srcs[0].device().index());
  as::PresplitArgs a;
  a.n = 0;
  a.block_start[0] = 0;
  auto flush = [&]() {
    if (a.n > 0) as::multi_presplit(a, stream());
    a.n = 0;
    a.block_start[0] = 0;
  };
  for (size_t i = 0; i < srcs.size(); ++i) {
    const at::Tensor& b = srcs[i];
    check_cuda(b, "src");
    TORCH_CHECK(b.dim() == 2 && b.scalar_type() == at::kFloat && b.is_contiguous(), "multi_presplit: fp32 matrices");
    const int N = static_cast<int>(trans[i] ? b.size(1) : b.size(0)), K = static_cast<int>(trans[i] ? b.size(0) : b.size(1));
    TORCH_CHECK(outs[i].scalar_type() == at::kByte && outs[i].is_contiguous() &&
                    outs[i].numel() == as::presplit_b_bytes(N, K) && outs[i].device() == b.device(),
                "multi_presplit: out buffer size");
    const long total = static_cast<long>((N + 31) / 32) * ((K + 15) / 16) * 64;
    if (total == 0) continue;
    if (a.n == as::kPresplitMax) flush();
    a.src[a.n] = b.data_ptr<float>();
    a.dst[a.n] = outs[i].data_ptr();
    a.N[a.n] = N;
    a.K[a.n] = K;
    a.trans[a.n] = trans[i] ? 1 : 0;
    a.block_start[a.n + 1] = a.block_start[a.n] + static_cast<int>((total + 255) / 256);
    ++a.n;
  }
  flush();
}

bool gemm_f32_psb_supported(int64_t M, int64_t N, int64_t K) {
  return as::gemm_f32_psb_supported(M, static_cast<int>(N), static_cast<int>(K));
}

// act(a [M, K] b^T + bias (+ res)) with b given as its presplit_b planes of an [N, K] matrix
at::Tensor gemm_f32_psb(const at::Tensor& a, const at::Tensor& bsplit, int64_t N, int64_t K,
                        const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res, int64_t act,
                        int64_t variant) {
  check_cuda(a, "a");
  check_cuda(bsplit, "bsplit");
  TORCH_CHECK(a.scalar_type() == at::kFloat && a.dim() == 2 && a.size(1) == K && a.is_contiguous(),
              "gemm_f32_psb: contiguous fp32 a [M, K]");
  TORCH_CHECK(bsplit.scalar_type() == at::kByte && bsplit.numel() == as::presplit_b_bytes(N, K) &&
                  bsplit.is_contiguous(), "gemm_f32_psb: bsplit must be presplit_b of an [N, K] matrix");
  TORCH_CHECK(as::gemm_f32_psb_supported(a.size(0), static_cast<int>(N), static_cast<int>(K)),
              "gemm_f32_psb: N % 128 == 0, K % 4 == 0");
  const float* bp = nullptr;
  const float* rp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(), "gemm_f32_psb: bias");
    bp = bias->data_ptr<float>();
  }
  if (res && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kFloat && res->numel() == a.size(0) * N && res->is_contiguous(),
                "gemm_f32_psb: res [M, N]");
    rp = res->data_ptr<float>();
  }
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({a.size(0), N}, a.options());
  as::gemm_f32_psb(a.data_ptr<float>(), bsplit.data_ptr(), bp, rp, out.data_ptr<float>(), a.size(0),
                   static_cast<int>(N), static_cast<int>(K), static_cast<int>(act), static_cast<int>(variant), stream());
  return out;
}

// log-probability of the taken action per head in one launch: logits[h] [..., C_h] (fp32 / bf16, contiguous),
// actions[h] int64 of the logits' leading shape -> fp32 tensors of that shape
std::vector<at::Tensor> multi_logp(const std::vector<at::Tensor>& logits, const std::vector<at::Tensor>& actions) {
  TORCH_CHECK(logits.size() == actions.size() && !logits.empty() && logits.size() <= as::kLogpMaxH,
              "multi_logp: 1..8 heads");
  c10::hip::HIPGuard g(logits[0].device().index());
  as::LogpArgs a;
  a.nheads = static_cast<int>(logits.size());
  a.row_start[0] = 0;
  std::vector<at::Tensor> outs;
  for (size_t h = 0; h < logits.size(); ++h) {
    const at::Tensor& l = logits[h];
    const at::Tensor& ac = actions[h];
    check_cuda(l, "logits");
    TORCH_CHECK((l.scalar_type() == at::kFloat || l.scalar_type() == at::kBFloat16) && l.is_contiguous() &&
                    l.dim() >= 1 && l.size(-1) > 0, "multi_logp: contiguous fp32 / bf16 logits");
    TORCH_CHECK(ac.scalar_type() == at::kLong && ac.is_contiguous() && ac.device() == l.device() &&
                    ac.numel() * l.size(-1) == l.numel(), "multi_logp: int64 actions of the logits' leading shape");
    auto o = at::empty(ac.sizes(), l.options().dtype(at::kFloat));
    a.logits[h] = l.data_ptr();
    a.action[h] = ac.data_ptr<int64_t>();
    a.out[h] = o.data_ptr<float>();
    a.cols[h] = static_cast<int>(l.size(-1));
    a.bf16[h] = l.scalar_type() == at::kBFloat16 ? 1 : 0;
    a.row_start[h + 1] = a.row_start[h] + ac.numel();
    outs.push_back(o);
  }
  as::multi_logp(a, stream());
  return outs;
}

// fp32 3 x 3 conv of NHWC x on the pre-split planes of a [Cout, 3, 3, Cin] weight (presplit_b of its [Cout, 9 Cin]
// view): bias / res / act as conv3x3_f32, res2 (first rows) / mask as conv3x3_f32_epi2
at::Tensor conv3x3_f32_psb(const at::Tensor& x, const at::Tensor& wsplit, int64_t Cout,
                           const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
                           const c10::optional<at::Tensor>& res2, const c10::optional<at::Tensor>& mask, int64_t act) {
  check_cuda(x, "x");
  check_cuda(wsplit, "wsplit");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 4 && x.is_contiguous(), "conv3x3_f32_psb: NHWC fp32 x");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), M = B * H * W;
  TORCH_CHECK(as::conv3x3_f32_psb_supported(M, static_cast<int>(Cin), static_cast<int>(Cout)),
              "conv3x3_f32_psb: Cout % 128, Cin % 16");
  TORCH_CHECK(wsplit.scalar_type() == at::kByte && wsplit.is_contiguous() &&
                  wsplit.numel() == as::presplit_b_bytes(static_cast<int>(Cout), static_cast<int>(9 * Cin)),
              "conv3x3_f32_psb: wsplit must be presplit_b of the [Cout, 9 Cin] weight");
  auto fp = [&](const c10::optional<at::Tensor>& t, int64_t rows, const char* what) -> const float* {
    if (!t || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->device() == x.device() &&
                    (rows < 0 ? t->numel() == Cout : (t->numel() % Cout == 0 && t->numel() / Cout <= rows)), what);
    return t->data_ptr<float>();
  };
  const float* bp = fp(bias, -1, "conv3x3_f32_psb: bias [Cout]");
  const float* rp = fp(res, M, "conv3x3_f32_psb: res [B, H, W, Cout]");
  if (rp) TORCH_CHECK(res->numel() == M * Cout, "conv3x3_f32_psb: res [B, H, W, Cout]");
  const float* r2 = fp(res2, M, "conv3x3_f32_psb: res2 [b <= B, H, W, Cout]");
  const float* mk = fp(mask, M, "conv3x3_f32_psb: mask [B, H, W, Cout]");
  if (mk) TORCH_CHECK(mask->numel() == M * Cout, "conv3x3_f32_psb: mask [B, H, W, Cout]");
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({B, H, W, Cout}, x.options());
  as::conv3x3_f32_psb(x.data_ptr<float>(), wsplit.data_ptr(), bp, rp, r2, r2 ? res2->numel() / Cout : 0, mk,
                      out.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                      static_cast<int>(Cin), static_cast<int>(Cout), static_cast<int>(act), stream());
  return out;
}

at::Tensor conv3x3_f32_v2(const at::Tensor& x, const at::Tensor& wsplit, int64_t Cout,
                           const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
                           const c10::optional<at::Tensor>& res2, const c10::optional<at::Tensor>& mask, int64_t act,
                          int64_t variant) {
  check_cuda(x, "x");
  check_cuda(wsplit, "wsplit");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 4 && x.is_contiguous(), "conv3x3_f32_psb: NHWC fp32 x");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), M = B * H * W;
  TORCH_CHECK(as::conv3x3_f32_psb_supported(M, static_cast<int>(Cin), static_cast<int>(Cout)),
              "conv3x3_f32_psb: Cout % 128, Cin % 16");
  TORCH_CHECK(wsplit.scalar_type() == at::kByte && wsplit.is_contiguous() &&
                  wsplit.numel() == as::presplit_b_bytes(static_cast<int>(Cout), static_cast<int>(9 * Cin)),
              "conv3x3_f32_psb: wsplit must be presplit_b of the [Cout, 9 Cin] weight");
  auto fp = [&](const c10::optional<at::Tensor>& t, int64_t rows, const char* what) -> const float* {
    if (!t || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->device() == x.device() &&
                    (rows < 0 ? t->numel() == Cout : (t->numel() % Cout == 0 && t->numel() / Cout <= rows)), what);
    return t->data_ptr<float>();
  };
  const float* bp = fp(bias, -1, "conv3x3_f32_psb: bias [Cout]");
  const float* rp = fp(res, M, "conv3x3_f32_psb: res [B, H, W, Cout]");
  if (rp) TORCH_CHECK(res->numel() == M * Cout, "conv3x3_f32_psb: res [B, H, W, Cout]");
  const float* r2 = fp(res2, M, "conv3x3_f32_psb: res2 [b <= B, H, W, Cout]");
  const float* mk = fp(mask, M, "conv3x3_f32_psb: mask [B, H, W, Cout]");
  if (mk) TORCH_CHECK(mask->numel() == M * Cout, "conv3x3_f32_psb: mask [B, H, W, Cout]");
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({B, H, W, Cout}, x.options());
  as::conv3x3_f32_v2(x.data_ptr<float>(), wsplit.data_ptr(), bp, rp, r2, r2 ? res2->numel() / Cout : 0, mk,
                      out.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                      static_cast<int>(Cin), static_cast<int>(Cout), static_cast<int>(act),
                     static_cast<int>(variant), stream());
  return out;
}

bool conv3x3_f32_psb_supported(int64_t M, int64_t Cin, int64_t Cout) {
  return as::conv3x3_f32_psb_supported(M, static_cast<int>(Cin), static_cast<int>(Cout));
}

// ---------------------------------------------------------------- conv3x3 implicit GEMM (NHWC bf16)
at::Tensor conv3x3_fwd(const at::Tensor& x, const at::Tensor& wk, const c10::optional<at::Tensor>& bias,
                       const c10::optional<at::Tensor>& res, int64_t act) {
  check_cuda(x, "x");
  check_cuda(wk, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && wk.scalar_type() == at::kBFloat16, "conv3x3: bf16 x / w");
  TORCH_CHECK(x.dim() == 4 && wk.dim() == 4 && wk.size(1) == 3 && wk.size(2) == 3 && wk.size(3) == x.size(3),
              "conv3x3: x NHWC [B,H,W,Cin], w [Cout,3,3,Cin]");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = wk.size(0);
  TORCH_CHECK(as::conv3x3_supported(Cin, Cout), "conv3x3: unsupported channels ", Cin, "->", Cout);
  TORCH_CHECK(x.is_contiguous() && wk.is_contiguous(), "conv3x3: contiguous NHWC x / w");
  // 32-bit buffer offsets: every byte offset (and the out-of-range sentinel) must stay below 2^31 - 16
  TORCH_CHECK(B * H * W * Cin * 2 < 0x7ffffff0LL && Cout * 9 * Cin * 2 < 0x7ffffff0LL, "conv3x3: tensor too large");
  const float* bp = nullptr;
  if (bias.has_value()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == Cout, "conv3x3: bias fp32 [Cout]");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  if (res.has_value()) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->dim() == 4 && res->size(0) == B && res->size(1) == H &&
                    res->size(2) == W && res->size(3) == Cout && res->is_contiguous(),
                "conv3x3: residual NHWC bf16 [B,H,W,Cout] contiguous");
    rp = res->data_ptr();
  }
  TORCH_CHECK(act >= 0 && act <= 4 && (act != 4 || rp != nullptr), "conv3x3: act 0..4; act 4 (ReLU gradient gate) needs res");
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({B, H, W, Cout}, x.options());
  as::conv3x3_fwd(x.data_ptr(), wk.data_ptr(), bp, rp, out.data_ptr(), B, H, W, Cin, Cout, static_cast<int>(act),
                  stream());
  return out;
}

}  // namespace

// ---------------------------------------------------------------- split-R MFMA weight gradient
// dy [R, N] bf16; x [R, K] bf16 (cin == 0) or NHWC [B, H, W, cin] bf16 (3x3 conv, K = 9 cin).
// Returns (dW fp32 [N, K], db fp32 [N] or undefined); bf16_out: both in bf16, the cast fused into the
// split reduction (the gradients of bf16 compute parameters under master weights).
// ---------------------------------------------------------------- head sampling tails
std::vector<at::Tensor> head_sample(const at::Tensor& logits, double temperature, const c10::optional<at::Tensor>& mask,
                                    const c10::optional<at::Tensor>& lens, const at::Tensor& u,
                                    const c10::optional<at::Tensor>& table, const c10::optional<at::Tensor>& tbias) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "head_sample: logits [B, C] with unit inner stride");
  const int64_t B = logits.size(0), C = logits.size(1);
  TORCH_CHECK(u.scalar_type() == at::kFloat && u.is_contiguous() && u.numel() == B, "head_sample: u fp32 [B]");
  const uint8_t* mp = nullptr;
  int64_t mld = 0;
  if (mask && mask->defined()) {
    TORCH_CHECK((mask->scalar_type() == at::kBool || mask->scalar_type() == at::kByte) && mask->is_contiguous() &&
                (mask->numel() == C || mask->numel() == B * C), "head_sample: mask bool [C] or [B, C]");
    mp = reinterpret_cast<const uint8_t*>(mask->data_ptr());
    mld = mask->numel() == C ? 0 : C;
  }
  const int64_t* lp = nullptr;
  if (lens && lens->defined()) {
    TORCH_CHECK(lens->scalar_type() == at::kLong && lens->numel() == B && lens->is_contiguous(), "head_sample: lens");
    lp = lens->data_ptr<int64_t>();
  }
  const void* tp = nullptr;
  int tdt = 0, D = 0;
  const float* bp = nullptr;
  if (table && table->defined()) {
    TORCH_CHECK(table->dim() == 2 && table->size(0) == C && table->is_contiguous(), "head_sample: table [C, D]");
    TORCH_CHECK(tbias && tbias->defined() && tbias->scalar_type() == at::kFloat && tbias->numel() == table->size(1),
                "head_sample: table bias fp32 [D]");
    tp = table->data_ptr();
    tdt = dt(*table);
    D = static_cast<int>(table->size(1));
    bp = tbias->data_ptr<float>();
  }
  c10::hip::HIPGuard g(logits.device().index());
  auto f = logits.options().dtype(at::kFloat);
  auto out = at::empty({B, C}, f);
  auto act = at::empty({B}, logits.options().dtype(at::kLong));
  auto emb = at::empty({B, std::max<int64_t>(D, 1)}, f);
  as::head_sample(logits.data_ptr(), dt(logits), logits.stride(0), static_cast<int>(B), static_cast<int>(C),
                  static_cast<float>(1.0 / temperature), mp, mld, lp, u.data_ptr<float>(), tp, tdt, bp, D,
                  out.data_ptr<float>(), act.data_ptr<int64_t>(), emb.data_ptr<float>(), stream());
  return {out, act, emb};
}

std::vector<at::Tensor> target_unit_sample(const at::Tensor& e, const at::Tensor& w1, const at::Tensor& b1,
                                           const at::Tensor& w2, const at::Tensor& b2, const at::Tensor& key,
                                           const at::Tensor& lens, double temperature, const at::Tensor& u) {
  check_cuda(e, "embedding");
  TORCH_CHECK(e.dim() == 2 && e.size(1) == 1024 && e.is_contiguous(), "target_unit: embedding [B, 1024]");
  const int64_t B = e.size(0);
  TORCH_CHECK(key.dim() == 3 && key.size(0) == B && key.size(2) == 32 && key.is_contiguous(), "target_unit: key [B,N,32]");
  for (auto* t : {&w1, &b1, &w2, &b2})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "target_unit: fp32 weights");
  TORCH_CHECK(w1.numel() == 32 * 1024 && b1.numel() == 32 && w2.numel() == 32 * 32 && b2.numel() == 32, "target_unit: shapes");
  TORCH_CHECK(lens.scalar_type() == at::kLong && lens.numel() == B && u.scalar_type() == at::kFloat && u.numel() == B,
              "target_unit: lens int64 [B], u fp32 [B]");
  const int64_t N = key.size(1);
  c10::hip::HIPGuard g(e.device().index());
  auto out = at::empty({B, N}, e.options().dtype(at::kFloat));
  auto act = at::empty({B}, e.options().dtype(at::kLong));
  as::target_unit_sample(e.data_ptr(), dt(e), w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(),
                         b2.data_ptr<float>(), key.data_ptr(), dt(key), static_cast<int>(B), static_cast<int>(N),
                         lens.data_ptr<int64_t>(), static_cast<float>(1.0 / temperature), u.data_ptr<float>(),
                         out.data_ptr<float>(), act.data_ptr<int64_t>(), stream());
  return {out, act};
}

// ---------------------------------------------------------------- fused clip + Adam
void fused_clip_adam(const at::Tensor& table, const at::Tensor& chunks, const at::Tensor& part,
                     const c10::optional<at::Tensor>& gate, const at::Tensor& norm_out, double max_norm,
                     const c10::optional<at::Tensor>& mom, const c10::optional<at::Tensor>& scale,
                     const c10::optional<at::Tensor>& mom_init, const c10::optional<at::Tensor>& hp, double lr_bc1, double b1, double b2, double inv_sqrt_bc2,
                     double eps, double wd, bool decoupled) {
  check_cuda(table, "table");
  TORCH_CHECK(table.scalar_type() == at::kLong && chunks.scalar_type() == at::kLong && table.is_contiguous() &&
              chunks.is_contiguous() && table.numel() % 6 == 0 && chunks.numel() % 2 == 0, "fused_clip_adam: tables");
  const int64_t nch = chunks.numel() / 2, nt = table.numel() / 6;
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= nch, "fused_clip_adam: part");
  TORCH_CHECK(norm_out.scalar_type() == at::kFloat && norm_out.numel() >= 1, "fused_clip_adam: norm_out");
  const float* gp = nullptr;
  if (gate && gate->defined()) {
    TORCH_CHECK(gate->scalar_type() == at::kFloat && gate->numel() == 1, "fused_clip_adam: gate fp32 scalar");
    gp = gate->data_ptr<float>();
  }
  float* mp = nullptr;
  float* sp = nullptr;
  float* ip = nullptr;
  if (mom && mom->defined()) {
    TORCH_CHECK(scale && scale->defined() && mom_init && mom_init->defined(),
                "fused_clip_adam: momentum_norm needs mom, scale and the init flag");
    TORCH_CHECK(mom_init->scalar_type() == at::kFloat && mom_init->numel() == 1 && mom_init->is_cuda() &&
                mom->is_cuda() && mom->device() == table.device(), "fused_clip_adam: mom / init flag on the device");
    ip = mom_init->data_ptr<float>();
    TORCH_CHECK(mom->scalar_type() == at::kFloat && mom->numel() == nt && mom->is_contiguous() &&
                scale->scalar_type() == at::kFloat && scale->numel() == nt && scale->is_contiguous(),
                "fused_clip_adam: mom / scale fp32 [ntensors]");
    mp = mom->data_ptr<float>();
    sp = scale->data_ptr<float>();
  }
  const float* hpp = nullptr;
  if (hp && hp->defined()) {
    TORCH_CHECK(hp->scalar_type() == at::kFloat && hp->numel() == 3 && hp->is_cuda(), "fused_clip_adam: hp fp32 [3]");
    hpp = hp->data_ptr<float>();
  }
  c10::hip::HIPGuard g(table.device().index());
  as::fused_clip_adam(table.data_ptr(), reinterpret_cast<const long*>(chunks.data_ptr<int64_t>()),
                      static_cast<int>(nch), static_cast<int>(nt), part.data_ptr<float>(), gp,
                      norm_out.data_ptr<float>(), static_cast<float>(max_norm), mp, sp, ip, hpp,
                      static_cast<float>(lr_bc1), static_cast<float>(b1), static_cast<float>(b2),
                      static_cast<float>(inv_sqrt_bc2), static_cast<float>(eps), static_cast<float>(wd),
                      decoupled ? 1 : 0, stream());
}

// ---------------------------------------------------------------- fp32 conv3x3 / weight gradients
at::Tensor conv3x3_f32(const at::Tensor& x, const at::Tensor& wk, const c10::optional<at::Tensor>& bias,
                       const c10::optional<at::Tensor>& res, int64_t act) {
  check_cuda(x, "x");
  check_cuda(wk, "w");
  TORCH_CHECK(x.scalar_type() == at::kFloat && wk.scalar_type() == at::kFloat, "conv3x3_f32: fp32 x / w");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "conv3x3_f32: x contiguous NHWC [B, H, W, Cin]");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  TORCH_CHECK(wk.dim() == 4 && wk.size(1) == 3 && wk.size(2) == 3 && wk.size(3) == Cin && wk.is_contiguous(),
              "conv3x3_f32: w contiguous [Cout, 3, 3, Cin]");
  const int64_t Cout = wk.size(0);
  TORCH_CHECK(as::conv3x3_f32_supported(static_cast<int>(Cin), static_cast<int>(Cout)), "conv3x3_f32: Cin % 16");
  TORCH_CHECK(B * H * W * std::max(Cin, Cout) * 4 < 0x7ffffff0LL && Cout * 9 * Cin * 4 < 0x7ffffff0LL,
              "conv3x3_f32: tensor too large for 32-bit buffer offsets");
  const float* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == Cout && bias->is_contiguous(), "conv3x3_f32: bias");
    bp = bias->data_ptr<float>();
  }
  const float* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kFloat && res->dim() == 4 && res->size(0) == B && res->size(1) == H &&
                res->size(2) == W && res->size(3) == Cout && res->is_contiguous(), "conv3x3_f32: residual NHWC");
    rp = res->data_ptr<float>();
  }
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({B, H, W, Cout}, x.options());
  as::conv3x3_f32_fwd(x.data_ptr<float>(), wk.data_ptr<float>(), bp, rp, out.data_ptr<float>(), static_cast<int>(B),
                      static_cast<int>(H), static_cast<int>(W), static_cast<int>(Cin), static_cast<int>(Cout),
                      static_cast<int>(act), stream());
  return out;
}

// input gradient with the extended epilogue: conv(x) + res + (first res2_rows rows) res2, masked by (mask > 0)
at::Tensor conv3x3_f32_epi2(const at::Tensor& x, const at::Tensor& wk, const at::Tensor& res,
                            const c10::optional<at::Tensor>& res2, const c10::optional<at::Tensor>& mask) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && wk.scalar_type() == at::kFloat && x.dim() == 4 && x.is_contiguous(),
              "conv3x3_f32_epi2: fp32 NHWC x");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  TORCH_CHECK(wk.dim() == 4 && wk.size(1) == 3 && wk.size(2) == 3 && wk.size(3) == Cin && wk.is_contiguous(),
              "conv3x3_f32_epi2: w contiguous [Cout, 3, 3, Cin]");
  const int64_t Cout = wk.size(0);
  TORCH_CHECK(as::conv3x3_f32_epi2_supported(static_cast<int>(Cin), static_cast<int>(Cout)),
              "conv3x3_f32_epi2: shape / mode not covered (Cout % 128, split mode)");
  TORCH_CHECK(B * H * W * std::max(Cin, Cout) * 4 < 0x7ffffff0LL, "conv3x3_f32_epi2: 32-bit offsets");
  auto full = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 4 && t.size(0) == B && t.size(1) == H && t.size(2) == W &&
                t.size(3) == Cout && t.is_contiguous() && t.device() == x.device(), what);
  };
  full(res, "conv3x3_f32_epi2: residual NHWC [B, H, W, Cout]");
  const float* r2 = nullptr;
  long r2_rows = 0;
  if (res2 && res2->defined()) {
    TORCH_CHECK(res2->scalar_type() == at::kFloat && res2->dim() == 4 && res2->size(0) <= B && res2->size(1) == H &&
                res2->size(2) == W && res2->size(3) == Cout && res2->is_contiguous() && res2->device() == x.device(),
                "conv3x3_f32_epi2: res2 NHWC [B2 <= B, H, W, Cout]");
    r2 = res2->data_ptr<float>();
    r2_rows = static_cast<long>(res2->size(0) * H * W);
  }
  const float* mp = nullptr;
  if (mask && mask->defined()) {
    full(*mask, "conv3x3_f32_epi2: mask NHWC [B, H, W, Cout]");
    mp = mask->data_ptr<float>();
  }
  c10::hip::HIPGuard g(x.device().index());
  auto out = at::empty({B, H, W, Cout}, x.options());
  as::conv3x3_f32_fwd_epi2(x.data_ptr<float>(), wk.data_ptr<float>(), res.data_ptr<float>(), r2, r2_rows, mp,
                           out.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                           static_cast<int>(Cin), static_cast<int>(Cout), stream());
  return out;
}

bool conv3x3_f32_epi2_supported(int64_t cin, int64_t cout) {
  return as::conv3x3_f32_epi2_supported(static_cast<int>(cin), static_cast<int>(cout));
}

at::Tensor gemm_f32(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                    const c10::optional<at::Tensor>& res, int64_t act) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat && a.dim() == 2 && b.dim() == 2 &&
              a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1), "gemm_f32: fp32 contiguous A [M,K], B [N,K]");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(K % 4 == 0, "gemm_f32: K % 4");
  TORCH_CHECK(M * K * 4 < 0x7ffffff0LL && N * K * 4 < 0x7ffffff0LL && M * N < (1LL << 40), "gemm_f32: too large");
  const float* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(), "gemm_f32: bias");
    bp = bias->data_ptr<float>();
  }
  const float* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kFloat && res->numel() == M * N && res->is_contiguous(), "gemm_f32: res");
    rp = res->data_ptr<float>();
  }
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({M, N}, a.options());
  as::gemm_f32(a.data_ptr<float>(), b.data_ptr<float>(), bp, rp, out.data_ptr<float>(), M, static_cast<int>(N),
               static_cast<int>(K), static_cast<int>(act), stream());
  return out;
}

at::Tensor gemm_bf16_impl(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                          const c10::optional<at::Tensor>& res, int64_t act, bool small_only) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && a.dim() == 2 && b.dim() == 2 &&
              a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "gemm_bf16_small: bf16 contiguous A [M,K], B [N,K]");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(K % 8 == 0, "gemm_bf16_small: K % 8");
  TORCH_CHECK(M * K * 2 < 0x7ffffff0LL && N * K * 2 < 0x7ffffff0LL && M * N < (1LL << 31), "gemm_bf16_small: too large");
  const float* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(), "gemm_bf16_small: fp32 bias");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->numel() == M * N && res->is_contiguous(),
                "gemm_bf16_small: bf16 res");
    rp = res->data_ptr();
  }
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({M, N}, a.options());
  if (small_only)
    as::gemm_bf16_small(a.data_ptr(), b.data_ptr(), bp, rp, out.data_ptr(), M, static_cast<int>(N),
                        static_cast<int>(K), static_cast<int>(act), stream());
  else
    as::gemm_bf16(a.data_ptr(), b.data_ptr(), bp, rp, out.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                  static_cast<int>(act), stream());
  return out;
}

// few-row kernel only / size-dispatched (LDS-DMA ring for >= 128 tiles)
at::Tensor gemm_bf16_small(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                           const c10::optional<at::Tensor>& res, int64_t act) {
  return gemm_bf16_impl(a, b, bias, res, act, true);
}
at::Tensor gemm_bf16(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                     const c10::optional<at::Tensor>& res, int64_t act) {
  return gemm_bf16_impl(a, b, bias, res, act, false);
}

// ---------------------------------------------------------------- few-row products of any shape (gemm_small.hip)
// out [M, N] = epi(mask(a) . b^T): a [M, K], b [N, K] (fp32 or bf16, same dtype), fp32 bias [N], res [M, N] and
// amask [M, K] in a's dtype; mask_mode / act: as::Act codes (mask: 0 none, 1 ReLU, 2 sigmoid of the saved output)
at::Tensor small_gemm(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                      const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& amask, int64_t mask_mode,
                      int64_t act) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  const bool bf = a.scalar_type() == at::kBFloat16;
  TORCH_CHECK((bf || a.scalar_type() == at::kFloat) && b.scalar_type() == a.scalar_type() && a.dim() == 2 &&
                  b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "small_gemm: contiguous A [M,K], B [N,K] of one dtype (fp32 / bf16)");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(M * K < (1LL << 31) && N * K < (1LL << 31) && M * N < (1LL << 31), "small_gemm: too large");
  TORCH_CHECK(mask_mode >= 0 && mask_mode <= 2 && (act == 0 || act == 1 || act == 2 || act == 4), "small_gemm: codes");
  const float* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous() && bias->is_cuda(),
                "small_gemm: fp32 bias [N]");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->scalar_type() == a.scalar_type() && res->numel() == M * N && res->is_contiguous() && res->is_cuda(),
                "small_gemm: res [M, N] in A's dtype");
    rp = res->data_ptr();
  }
  TORCH_CHECK(act != 4 || rp != nullptr, "small_gemm: the DRELU epilogue masks by res");
  const void* mp = nullptr;
  if (amask && amask->defined() && mask_mode > 0) {
    TORCH_CHECK(amask->scalar_type() == a.scalar_type() && amask->numel() == M * K && amask->is_contiguous() &&
                    amask->is_cuda(), "small_gemm: amask [M, K] in A's dtype");
    mp = amask->data_ptr();
  }
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({M, N}, a.options());
  as::small_nt(a.data_ptr(), b.data_ptr(), bp, rp, mp, static_cast<int>(mask_mode), out.data_ptr(), M,
               static_cast<int>(N), static_cast<int>(K), static_cast<int>(act), bf, stream());
  return out;
}

// few rows, long K (the spatial encoder's 48,640-wide fc): split-K over S workgroup slices + an ordered sum with
// the bias / act epilogue (deterministic); S == 1 -> the one-pass kernel
at::Tensor small_gemm_splitk(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                             int64_t act) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  const bool bf = a.scalar_type() == at::kBFloat16;
  TORCH_CHECK((bf || a.scalar_type() == at::kFloat) && b.scalar_type() == a.scalar_type() && a.dim() == 2 &&
                  b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "small_gemm_splitk: contiguous A [M,K], B [N,K] of one dtype (fp32 / bf16)");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(M * K < (1LL << 31) && N * K < (1LL << 31) && M * N < (1LL << 28), "small_gemm_splitk: too large");
  TORCH_CHECK(act == 0 || act == 1 || act == 2, "small_gemm_splitk: act code");
  const float* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous() && bias->is_cuda(),
                "small_gemm_splitk: fp32 bias [N]");
    bp = bias->data_ptr<float>();
  }
  c10::hip::HIPGuard g(a.device().index());
  auto out = at::empty({M, N}, a.options());
  const int S = as::small_nt_splits(M, static_cast<int>(N), static_cast<int>(K));
  if (S <= 1) {
    as::small_nt(a.data_ptr(), b.data_ptr(), bp, nullptr, nullptr, 0, out.data_ptr(), M, static_cast<int>(N),
                 static_cast<int>(K), static_cast<int>(act), bf, stream());
    return out;
  }
  auto part = at::empty({S, M, N}, a.options().dtype(at::kFloat));
  as::small_nt_splitk(a.data_ptr(), b.data_ptr(), bp, part.data_ptr<float>(), S, out.data_ptr(), M,
                      static_cast<int>(N), static_cast<int>(K), static_cast<int>(act), bf, stream());
  return out;
}

// dW [N, K] = mask(dy)^T . x and db [N] = column sums of mask(dy) over R rows (dy [R, N], x [R, K], ymask [R, N]:
// the layer output whose activation gradient masks dy); dW / db in bf16 when out_bf16 (bf16 inputs only)
std::vector<at::Tensor> small_wgrad(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& ymask,
                                    int64_t mask_mode, bool want_bias, bool out_bf16) {
  check_cuda(dy, "dy");
  check_cuda(x, "x");
  const bool bf = dy.scalar_type() == at::kBFloat16;
  TORCH_CHECK((bf || dy.scalar_type() == at::kFloat) && x.scalar_type() == dy.scalar_type() && dy.dim() == 2 &&
                  x.dim() == 2 && dy.is_contiguous() && x.is_contiguous() && dy.size(0) == x.size(0),
              "small_wgrad: contiguous dy [R, N], x [R, K] of one dtype");
  TORCH_CHECK(!out_bf16 || bf, "small_wgrad: bf16 output needs bf16 inputs");
  TORCH_CHECK(mask_mode >= 0 && mask_mode <= 2, "small_wgrad: mask code");
  const int64_t R = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(R * N < (1LL << 31) && R * K < (1LL << 31) && N * K < (1LL << 31), "small_wgrad: too large");
  const void* mp = nullptr;
  if (ymask && ymask->defined() && mask_mode > 0) {
    TORCH_CHECK(ymask->scalar_type() == dy.scalar_type() && ymask->numel() == R * N && ymask->is_contiguous() &&
                    ymask->is_cuda(), "small_wgrad: ymask [R, N] in dy's dtype");
    mp = ymask->data_ptr();
  }
  c10::hip::HIPGuard g(dy.device().index());
  auto opts = out_bf16 ? dy.options() : dy.options().dtype(at::kFloat);
  auto dw = at::empty({N, K}, opts);
  at::Tensor db = want_bias ? at::empty({N}, opts) : at::Tensor();
  if (R == 0) {
    dw.zero_();
    if (want_bias) db.zero_();
    return {dw, db};
  }
  as::small_tn(dy.data_ptr(), x.data_ptr(), mp, static_cast<int>(mask_mode), dw.data_ptr(),
               want_bias ? db.data_ptr() : nullptr, R, static_cast<int>(N), static_cast<int>(K), bf, out_bf16, stream());
  return {dw, db};
}

std::vector<at::Tensor> wgrad_f32(const at::Tensor& dy, const at::Tensor& x, int64_t cin, bool want_bias,
                                  const c10::optional<at::Tensor>& out) {
  check_cuda(dy, "dy");
  check_cuda(x, "x");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && x.scalar_type() == at::kFloat, "wgrad_f32: fp32 dy / x");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous() && x.is_contiguous(), "wgrad_f32: contiguous dy [R, N], x");
  const int64_t R = dy.size(0), N = dy.size(1);
  int64_t K, H = 1, W = 1;
  if (cin > 0) {
    TORCH_CHECK(x.dim() == 4 && x.size(3) == cin && x.size(0) * x.size(1) * x.size(2) == R, "wgrad_f32: x NHWC");
    H = x.size(1);
    W = x.size(2);
    K = 9 * cin;
    TORCH_CHECK(cin % 4 == 0, "wgrad_f32: Cin % 4");
  } else {
    TORCH_CHECK(x.dim() == 2 && x.size(0) == R, "wgrad_f32: x [R, K]");
    K = x.size(1);
  }
  TORCH_CHECK(N % 4 == 0 && K % 4 == 0, "wgrad_f32: N and K must be multiples of 4");
  TORCH_CHECK(R * N * 4 < 0x7ffffff0LL && x.numel() * 4 < 0x7ffffff0LL, "wgrad_f32: tensor too large");
  c10::hip::HIPGuard g(dy.device().index());
  auto opts = dy.options();
  const int64_t NK = N * K, stride = NK + (want_bias ? N : 0);
  // out: a caller-provided flat [N K (+ N)] fp32 result buffer (the deferred weight gradients, ops/native.py)
  at::Tensor flat;
  if (out && out->defined()) {
    TORCH_CHECK(out->scalar_type() == at::kFloat && out->is_contiguous() && out->numel() == stride &&
                out->device() == dy.device(), "wgrad_f32: out must be a contiguous fp32 [N K (+ N)] buffer");
    flat = *out;
  }
  if (R == 0) {
    if (flat.defined()) {
      flat.zero_();
      return {flat.narrow(0, 0, NK).view({N, K}), want_bias ? flat.narrow(0, NK, N) : at::Tensor()};
    }
    return {at::zeros({N, K}, opts), want_bias ? at::zeros({N}, opts) : at::Tensor()};
  }
  const int S = as::wgrad_f32_splits(R, static_cast<int>(N), static_cast<int>(K));
  auto part = (S == 1 && flat.defined()) ? flat.view({1, stride}) : at::empty({S, stride}, opts);
  as::wgrad_f32(dy.data_ptr<float>(), x.data_ptr<float>(), part.data_ptr<float>(),
                want_bias ? part.data_ptr<float>() + NK : nullptr, stride, R, static_cast<int>(N), static_cast<int>(K),
                static_cast<int>(H), static_cast<int>(W), static_cast<int>(cin), S, stream());
  if (S == 1) {
    if (!flat.defined()) flat = part.view({stride});
  } else {
    if (!flat.defined()) flat = at::empty({stride}, opts);
    as::column_reduce(part.data_ptr<float>(), flat.data_ptr<float>(), S, static_cast<int>(stride), stream());
  }
  return {flat.narrow(0, 0, NK).view({N, K}), want_bias ? flat.narrow(0, NK, N) : at::Tensor()};
}

std::vector<at::Tensor> wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t cin, bool want_bias, bool bf16_out) {
  check_cuda(dy, "dy");
  check_cuda(x, "x");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "wgrad: bf16 dy / x");
  TORCH_CHECK(dy.dim() == 2, "wgrad: dy [R, N]");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "wgrad: dy and x must be contiguous");
  const int64_t R = dy.size(0), N = dy.size(1);
  int64_t K, H = 1, W = 1;
  if (cin > 0) {
    TORCH_CHECK(x.dim() == 4 && x.size(3) == cin && x.size(0) * x.size(1) * x.size(2) == R, "wgrad: x NHWC");
    H = x.size(1);
    W = x.size(2);
    K = 9 * cin;
    TORCH_CHECK(cin % 8 == 0, "wgrad: Cin % 8");
  } else {
    TORCH_CHECK(x.dim() == 2 && x.size(0) == R, "wgrad: x [R, K]");
    K = x.size(1);
  }
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "wgrad: N and K must be multiples of 8");
  TORCH_CHECK(R * N * 2 < 0x7ffffff0LL && x.numel() * 2 < 0x7ffffff0LL, "wgrad: tensor too large");
  c10::hip::HIPGuard g(dy.device().index());
  const int S = R > 0 ? as::wgrad_splits(R, static_cast<int>(N), static_cast<int>(K)) : 1;
  auto opts = dy.options().dtype(at::kFloat);
  if (R == 0) {
    auto zo = bf16_out ? dy.options() : opts;
    return {at::zeros({N, K}, zo), want_bias ? at::zeros({N}, zo) : at::Tensor()};
  }
  // one [S, N*K (+ N)] partial buffer: dW and db of a slice side by side, reduced by ONE column pass
  const int64_t NK = N * K, stride = NK + (want_bias ? N : 0);
  if (bf16_out && S == 1) {   // one slice: the kernel writes the final bf16 gradient (no reduce / cast pass)
    auto flat = at::empty({stride}, dy.options());
    as::wgrad(dy.data_ptr(), x.data_ptr(), reinterpret_cast<float*>(flat.data_ptr()),
              want_bias ? reinterpret_cast<float*>(static_cast<at::BFloat16*>(flat.data_ptr()) + NK) : nullptr, 0, R,
              static_cast<int>(N), static_cast<int>(K), static_cast<int>(H), static_cast<int>(W), static_cast<int>(cin),
              1, stream(), true);
    return {flat.narrow(0, 0, NK).view({N, K}), want_bias ? flat.narrow(0, NK, N) : at::Tensor()};
  }
  auto part = at::empty({S, stride}, opts);
  // debug: poison the partials so any slot the kernel leaves unwritten shows up as NaN on every run
  static const bool nan_fill = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_NANFILL");
    return e != nullptr && e[0] == '1';
  }();
  if (nan_fill) part.fill_(std::numeric_limits<float>::quiet_NaN());
  as::wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), want_bias ? part.data_ptr<float>() + NK : nullptr,
            stride, R, static_cast<int>(N), static_cast<int>(K), static_cast<int>(H), static_cast<int>(W),
            static_cast<int>(cin), S, stream());
  at::Tensor flat;
  if (bf16_out && S <= 1024) {
    flat = at::empty({stride}, dy.options());
    as::column_reduce_bf16(part.data_ptr<float>(), flat.data_ptr(), S, static_cast<int>(stride), stream());
  } else if (S == 1) {
    flat = part.view({stride});
  } else {
    flat = at::empty({stride}, opts);
    as::column_reduce(part.data_ptr<float>(), flat.data_ptr<float>(), S, static_cast<int>(stride), stream());
  }
  if (bf16_out && flat.scalar_type() != at::kBFloat16) flat = flat.to(at::kBFloat16);
  return {flat.narrow(0, 0, NK).view({N, K}), want_bias ? flat.narrow(0, NK, N) : at::Tensor()};
}

// ---------------------------------------------------------------- fused build-order transformer
// params: w0, b0, then per layer ln1w, ln1b, wqkv, bqkv, wp, bp, ln2w, ln2b, w1, b1, w2, b2 (38 tensors):
// linear weights / biases all bf16 or all fp32, LayerNorm affines fp32
namespace {
int idx_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kShort) return 0;
  if (t.scalar_type() == at::kInt) return 1;
  TORCH_CHECK(t.scalar_type() == at::kLong, "bo_encoder: index dtype int16 / int32 / int64");
  return 2;
}

as::BoWeights bo_weights(const std::vector<at::Tensor>& p, int* wdt) {
  TORCH_CHECK(p.size() == 2 + 12 * as::kBoLayers, "bo_encoder: 38 parameter tensors");
  const auto lin_t = p[0].scalar_type();
  TORCH_CHECK(lin_t == at::kFloat || lin_t == at::kBFloat16, "bo_encoder: linear dtype");
  auto lin = [&](const at::Tensor& t, int64_t numel) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == lin_t && t.numel() == numel,
                "bo_encoder: linear parameter (dtype / shape / contiguity)");
    return static_cast<const void*>(t.data_ptr());
  };
  auto ln = [&](const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.numel() == 64,
                "bo_encoder: LayerNorm parameter fp32 [64]");
    return t.data_ptr<float>();
  };
  as::BoWeights w;
  w.w0 = lin(p[0], 64 * 214);
  w.b0 = lin(p[1], 64);
  for (int l = 0; l < as::kBoLayers; ++l) {
    const int o = 2 + 12 * l;
    w.ln1w[l] = ln(p[o]);
    w.ln1b[l] = ln(p[o + 1]);
    w.wqkv[l] = lin(p[o + 2], 48 * 64);
    w.bqkv[l] = lin(p[o + 3], 48);
    w.wp[l] = lin(p[o + 4], 64 * 16);
    w.bp[l] = lin(p[o + 5], 64);
    w.ln2w[l] = ln(p[o + 6]);
    w.ln2b[l] = ln(p[o + 7]);
    w.w1[l] = lin(p[o + 8], 128 * 64);
    w.b1[l] = lin(p[o + 9], 128);
    w.w2[l] = lin(p[o + 10], 64 * 128);
    w.b2[l] = lin(p[o + 11], 64);
  }
  *wdt = lin_t == at::kBFloat16 ? as::DT_BF16 : as::DT_F32;
  return w;
}
}  // namespace

// bo, loc [B, 20] -> (mean [B, 64] fp32, save [B, 3, kBoRecord] fp32 or undefined)
std::vector<at::Tensor> bo_encoder_fwd(const at::Tensor& bo, const at::Tensor& loc, const std::vector<at::Tensor>& params,
                                       bool save) {
  check_cuda(bo, "bo");
  check_cuda(loc, "loc");
  TORCH_CHECK(bo.dim() == 2 && bo.size(1) == as::kBoTokens && bo.is_contiguous() && loc.sizes() == bo.sizes() &&
                  loc.is_contiguous() && loc.scalar_type() == bo.scalar_type(),
              "bo_encoder: bo / loc [B, 20] contiguous, same dtype");
  int wdt = 0;
  const as::BoWeights w = bo_weights(params, &wdt);
  const int64_t B = bo.size(0);
  c10::hip::HIPGuard g(bo.device().index());
  auto opts = bo.options().dtype(at::kFloat);
  auto out = at::empty({B, 64}, opts);
  at::Tensor rec;
  if (save) rec = at::empty({B, as::kBoLayers, as::kBoRecord}, opts);
  as::bo_encoder_fwd(bo.data_ptr(), loc.data_ptr(), idx_code(bo), w, wdt, out.data_ptr<float>(),
                     save ? rec.data_ptr<float>() : nullptr, B, stream());
  return {out, rec};
}

// -> flat fp32 parameter gradient [kBoGradSize] in the params order
at::Tensor bo_encoder_bwd(const at::Tensor& bo, const at::Tensor& loc, const std::vector<at::Tensor>& params,
                          const at::Tensor& save, const at::Tensor& dmean) {
  check_cuda(dmean, "dmean");
  const int64_t B = bo.size(0);
  TORCH_CHECK(dmean.scalar_type() == at::kFloat && dmean.is_contiguous() && dmean.numel() == B * 64,
              "bo_encoder_bwd: dmean fp32 [B, 64]");
  TORCH_CHECK(save.scalar_type() == at::kFloat && save.numel() == B * as::kBoLayers * as::kBoRecord,
              "bo_encoder_bwd: saved record");
  int wdt = 0;
  const as::BoWeights w = bo_weights(params, &wdt);
  c10::hip::HIPGuard g(bo.device().index());
  const int reps = static_cast<int>(std::min<int64_t>(B, 32));
  auto rep = at::zeros({reps, as::kBoGradSize}, dmean.options());
  as::bo_encoder_bwd(bo.data_ptr(), loc.data_ptr(), idx_code(bo), w, wdt, save.data_ptr<float>(),
                     dmean.data_ptr<float>(), rep.data_ptr<float>(), B, reps, stream());
  auto grad = at::empty({as::kBoGradSize}, dmean.options());
  as::column_reduce(rep.data_ptr<float>(), grad.data_ptr<float>(), reps, as::kBoGradSize, stream());
  return grad;
}

// ---------------------------------------------------------------- residual MLP stack (value baseline)
// params: per block w1, b1, w2, b2 (bf16 [256,256] / [256]), ln weight, ln bias (fp32 [256])
namespace {
as::ResMlpW resmlp_weights(const std::vector<at::Tensor>& p, int* nblk) {
  TORCH_CHECK(p.size() % 6 == 0 && p.size() / 6 >= 1 && p.size() / 6 <= as::kResMax, "resmlp: 6 tensors per block");
  const int n = static_cast<int>(p.size() / 6);
  as::ResMlpW w{};
  for (int k = 0; k < n; ++k) {
    for (int j = 0; j < 4; ++j) {
      const at::Tensor& t = p[6 * k + j];
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kBFloat16 &&
                      t.numel() == ((j % 2) == 0 ? 256 * 256 : 256),
                  "resmlp: bf16 contiguous fc weights [256,256] / biases [256]");
    }
    for (int j = 4; j < 6; ++j) {
      const at::Tensor& t = p[6 * k + j];
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.numel() == 256,
                  "resmlp: fp32 LayerNorm affine [256]");
    }
    w.w1[k] = p[6 * k].data_ptr();
    w.b1[k] = p[6 * k + 1].data_ptr();
    w.w2[k] = p[6 * k + 2].data_ptr();
    w.b2[k] = p[6 * k + 3].data_ptr();
    w.g[k] = p[6 * k + 4].data_ptr<float>();
    w.be[k] = p[6 * k + 5].data_ptr<float>();
  }
  *nblk = n;
  return w;
}
}  // namespace

// x0 [R, 256] fp32 / bf16 -> (out fp32 [R, 256], sv_x, sv_h, sv_xhat, sv_rstd) (saved tensors undefined if !save)
std::vector<at::Tensor> resmlp_fwd(const at::Tensor& x0, const std::vector<at::Tensor>& params, bool save) {
  check_cuda(x0, "x0");
  TORCH_CHECK(x0.dim() == 2 && x0.size(1) == 256 && x0.is_contiguous() &&
                  (x0.scalar_type() == at::kFloat || x0.scalar_type() == at::kBFloat16),
              "resmlp: x0 [R, 256] fp32 / bf16 contiguous");
  int n = 0;
  as::ResMlpW w = resmlp_weights(params, &n);
  const int64_t R = x0.size(0);
  c10::hip::HIPGuard g(x0.device().index());
  auto f32 = x0.options().dtype(at::kFloat), b16 = x0.options().dtype(at::kBFloat16);
  auto out = at::empty({R, 256}, f32);
  auto pk = at::empty({2 * n, 256, 256}, b16);
  as::resmlp_pack(w, n, false, reinterpret_cast<uint16_t*>(pk.data_ptr()), stream());
  w.pk = pk.data_ptr();
  at::Tensor sx, sh, sxh, srs;
  if (save) {
    sx = at::empty({n, R, 256}, b16);
    sh = at::empty({n, R, 256}, b16);
    sxh = at::empty({n, R, 256}, f32);
    srs = at::empty({n, R}, f32);
  }
  as::resmlp_fwd(x0.data_ptr(), dt(x0), w, n, out.data_ptr<float>(),
                 save ? reinterpret_cast<uint16_t*>(sx.data_ptr()) : nullptr,
                 save ? reinterpret_cast<uint16_t*>(sh.data_ptr()) : nullptr, save ? sxh.data_ptr<float>() : nullptr,
                 save ? srs.data_ptr<float>() : nullptr, R, stream());
  return {out, sx, sh, sxh, srs};
}

// -> (dx0 fp32 [R, 256], weight grads fp32 [2n, 256*256 + 256] (W1_k | b1_k, W2_k | b2_k), LN grads fp32 [n, 512])
std::vector<at::Tensor> resmlp_bwd(const at::Tensor& dout, const std::vector<at::Tensor>& params, const at::Tensor& sx,
                                   const at::Tensor& sh, const at::Tensor& sxh, const at::Tensor& srs) {
  check_cuda(dout, "dout");
  int n = 0;
  as::ResMlpW w = resmlp_weights(params, &n);
  const int64_t R = dout.size(0);
  TORCH_CHECK(dout.scalar_type() == at::kFloat && dout.is_contiguous() && dout.numel() == R * 256,
              "resmlp_bwd: dout fp32 [R, 256]");
  TORCH_CHECK(sx.numel() == n * R * 256 && sh.numel() == n * R * 256 && sxh.numel() == n * R * 256 && srs.numel() == n * R,
              "resmlp_bwd: saved tensors");
  c10::hip::HIPGuard g(dout.device().index());
  auto f32 = dout.options(), b16 = dout.options().dtype(at::kBFloat16);
  auto pk = at::empty({2 * n, 256, 256}, b16);
  as::resmlp_pack(w, n, true, reinterpret_cast<uint16_t*>(pk.data_ptr()), stream());
  w.pk = pk.data_ptr();
  auto dy = at::empty({n, R, 256}, b16), dh = at::empty({n, R, 256}, b16);
  const int nrb = as::resmlp_row_blocks(R);
  auto part = at::empty({nrb, n * 512}, f32);
  auto dx0 = at::empty({R, 256}, f32);
  as::resmlp_bwd(dout.data_ptr<float>(), w, n, reinterpret_cast<const uint16_t*>(sh.data_ptr()), sxh.data_ptr<float>(),
                 srs.data_ptr<float>(), reinterpret_cast<uint16_t*>(dy.data_ptr()),
                 reinterpret_cast<uint16_t*>(dh.data_ptr()), part.data_ptr<float>(), dx0.data_ptr<float>(), R, stream());
  const int64_t stride = 65536 + 256;
  auto gw = at::empty({2 * n, stride}, f32);
  as::WgBatch P;
  for (int k = 0; k < n; ++k) {
    const long o = static_cast<long>(k) * R * 256;
    P.dy[2 * k] = static_cast<const uint16_t*>(dh.data_ptr()) + o;       // W1_k: dH^T x_in
    P.x[2 * k] = static_cast<const uint16_t*>(sx.data_ptr()) + o;
    P.dy[2 * k + 1] = static_cast<const uint16_t*>(dy.data_ptr()) + o;   // W2_k: dY^T h
    P.x[2 * k + 1] = static_cast<const uint16_t*>(sh.data_ptr()) + o;
    for (int j = 0; j < 2; ++j) {
      P.dw[2 * k + j] = gw.data_ptr<float>() + (2 * k + j) * stride;
      P.db[2 * k + j] = gw.data_ptr<float>() + (2 * k + j) * stride + 65536;
    }
  }
  as::wgrad_batched(P, 2 * n, 0, R, 256, 256, 1, 1, 0, 1, stream());
  auto gln = at::empty({n, 512}, f32);
  as::column_reduce(part.data_ptr<float>(), gln.data_ptr<float>(), nrb, n * 512, stream());
  return {dx0, gw, gln};
}

// ---------------------------------------------------------------- fused categorical head statistics
// logits [R, C] fp32/bf16, teacher [R, C] fp32/bf16 (optional), action [R] int64
// -> out [3, R] fp32 (logp_a, entropy, KL(teacher || logits)), stats [R, 6] fp32
std::vector<at::Tensor> head_stats_fwd(const at::Tensor& logits, const c10::optional<at::Tensor>& teacher,
                                       const at::Tensor& action) {
  check_cuda(logits, "logits");
  check_cuda(action, "action");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "head_stats: logits [R, C] contiguous");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "head_stats: logits dtype");
  TORCH_CHECK(action.scalar_type() == at::kLong && action.is_contiguous() && action.numel() == logits.size(0),
              "head_stats: action int64 [R]");
  const int64_t R = logits.size(0), C = logits.size(1);
  TORCH_CHECK(C > 0 && C < (1 << 30), "head_stats: C");
  const void* tp = nullptr;
  int tdt = 0;
  if (teacher.has_value()) {
    const at::Tensor& t = *teacher;
    check_cuda(t, "teacher");
    TORCH_CHECK(t.sizes() == logits.sizes() && t.is_contiguous(), "head_stats: teacher [R, C] contiguous");
    TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "head_stats: teacher dtype");
    tp = t.data_ptr();
    tdt = dt(t);
  }
  c10::hip::HIPGuard g(logits.device().index());
  auto out = at::empty({3, R}, logits.options().dtype(at::kFloat));
  auto stats = at::empty({R, 6}, logits.options().dtype(at::kFloat));
  as::head_stats_fwd(logits.data_ptr(), dt(logits), tp, tdt, action.data_ptr<int64_t>(), out.data_ptr<float>(),
                     stats.data_ptr<float>(), R, static_cast<int>(C), stream());
  return {out, stats};
}

at::Tensor head_stats_bwd(const at::Tensor& logits, const c10::optional<at::Tensor>& teacher, const at::Tensor& action,
                          const at::Tensor& stats, const at::Tensor& grad) {
  check_cuda(grad, "grad");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.is_contiguous() && grad.numel() == 3 * logits.size(0),
              "head_stats_bwd: grad fp32 [3, R]");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == 6 * logits.size(0),
              "head_stats_bwd: stats");
  const int64_t R = logits.size(0), C = logits.size(1);
  const void* tp = teacher.has_value() ? teacher->data_ptr() : nullptr;
  const int tdt = teacher.has_value() ? dt(*teacher) : 0;
  c10::hip::HIPGuard g(logits.device().index());
  auto dl = at::empty_like(logits);
  as::head_stats_bwd(logits.data_ptr(), dt(logits), tp, tdt, action.data_ptr<int64_t>(), stats.data_ptr<float>(),
                     grad.data_ptr<float>(), dl.data_ptr(), R, static_cast<int>(C), stream());
  return dl;
}

// ---------------------------------------------------------------- conv epilogue backward -> NHWC bf16
// dout: [B, H, W, C] view (NHWC- or NCHW-contiguous underneath); out: NHWC bf16 (used when relu).
at::Tensor act_grad_nhwc(const at::Tensor& dout, const c10::optional<at::Tensor>& out, bool relu) {
  TORCH_CHECK(dout.is_cuda() && dout.dim() == 4, "act_grad: dout [B,H,W,C] GPU");
  const int64_t B = dout.size(0), H = dout.size(1), W = dout.size(2), C = dout.size(3);
  at::Tensor d = dout;
  bool nchw = false;
  if (!d.is_contiguous()) {
    if (d.permute({0, 3, 1, 2}).is_contiguous() && C % 32 == 0) nchw = true;
    else d = d.contiguous();
  }
  TORCH_CHECK(C % 8 == 0, "act_grad: C % 8");
  const void* op = nullptr;
  if (relu) {
    TORCH_CHECK(out.has_value(), "act_grad: relu needs out");
    check_cuda(*out, "out");
    TORCH_CHECK(out->scalar_type() == at::kBFloat16 && out->sizes() == dout.sizes(), "act_grad: out NHWC bf16");
    op = out->data_ptr();
  }
  c10::hip::HIPGuard g(dout.device().index());
  auto dpre = at::empty({B, H, W, C}, dout.options().dtype(at::kBFloat16));
  as::act_grad_nhwc(d.data_ptr(), dt(d), nchw, op, dpre.data_ptr(), static_cast<int>(B), static_cast<int>(C),
                    static_cast<int>(H * W), relu ? 1 : 0, stream());
  return dpre;
}

// ---------------------------------------------------------------- value-encoder spatial input (value_spatial.hip)
// sc [P, 8] bf16 (NHWC scatter map), own / enemy [P] bool or uint8, w [16, 10] fp32, b [16] fp32 -> [P, 16] bf16
at::Tensor vsp_fwd(const at::Tensor& sc, const at::Tensor& own, const at::Tensor& enemy, const at::Tensor& w,
                   const at::Tensor& b) {
  check_cuda(sc, "sc");
  check_cuda(own, "own");
  check_cuda(enemy, "enemy");
  check_cuda(w, "w");
  check_cuda(b, "b");
  const int64_t P = sc.size(0);
  TORCH_CHECK((sc.scalar_type() == at::kBFloat16 || sc.scalar_type() == at::kFloat) && sc.dim() == 2 &&
              sc.size(1) == as::vsp_in_channels() - 2 && sc.is_contiguous(), "vsp: sc [P, 8] bf16 / fp32");
  TORCH_CHECK(own.element_size() == 1 && enemy.element_size() == 1 && own.numel() == P && enemy.numel() == P,
              "vsp: own / enemy [P] bool");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.size(0) == as::vsp_out_channels() && w.size(1) == as::vsp_in_channels()
              && b.scalar_type() == at::kFloat && b.numel() == as::vsp_out_channels(), "vsp: w [16, 10], b [16] fp32");
  c10::hip::HIPGuard g(sc.device().index());
  auto out = at::empty({P, as::vsp_out_channels()}, sc.options());
  as::vsp_fwd(sc.data_ptr(), own.data_ptr(), enemy.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(),
              out.data_ptr(), P, stream(), dt(sc));
  return out;
}

// -> {dSc [P, 8] bf16, [dW | db] [16, 11] fp32}
std::vector<at::Tensor> vsp_bwd(const at::Tensor& dout, const at::Tensor& out, const at::Tensor& sc,
                                const at::Tensor& own, const at::Tensor& enemy, const at::Tensor& w) {
  check_cuda(dout, "dout");
  check_cuda(out, "out");
  check_cuda(sc, "sc");
  check_cuda(own, "own");
  check_cuda(enemy, "enemy");
  check_cuda(w, "w");
  const int64_t P = sc.size(0);
  TORCH_CHECK(dout.scalar_type() == sc.scalar_type() && out.scalar_type() == sc.scalar_type() &&
              dout.sizes() == out.sizes() && out.size(0) == P && out.size(1) == as::vsp_out_channels() &&
              dout.is_contiguous() && out.is_contiguous(), "vsp_bwd: dout / out [P, 16] of sc's dtype");
  TORCH_CHECK((sc.scalar_type() == at::kBFloat16 || sc.scalar_type() == at::kFloat) &&
              sc.size(1) == as::vsp_in_channels() - 2 && sc.is_contiguous(), "vsp_bwd: sc [P, 8] bf16 / fp32");
  TORCH_CHECK(own.element_size() == 1 && enemy.element_size() == 1 && own.numel() == P && enemy.numel() == P,
              "vsp_bwd: own / enemy [P] bool");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.size(0) == as::vsp_out_channels() && w.size(1) == as::vsp_in_channels(),
              "vsp_bwd: w [16, 10] fp32");
  c10::hip::HIPGuard g(sc.device().index());
  const int nblk = as::vsp_bwd_blocks(P);
  auto dsc = at::empty_like(sc);
  auto part = at::empty({nblk, as::vsp_out_channels() * (as::vsp_in_channels() + 1)}, sc.options().dtype(at::kFloat));
  as::vsp_bwd(dout.data_ptr(), out.data_ptr(), sc.data_ptr(), own.data_ptr(), enemy.data_ptr(), w.data_ptr<float>(),
              dsc.data_ptr(), part.data_ptr<float>(), P, nblk, stream(), dt(sc));
  return {dsc, part.sum(0).view({as::vsp_out_channels(), as::vsp_in_channels() + 1})};
}

// pooled forms (even H, W): sc [B*H*W, 8], own / enemy [B*H*W] -> {pooled [B*(H/2)*(W/2), 16] bf16, pos uint8}
std::vector<at::Tensor> vsp_pool_fwd(const at::Tensor& sc, const at::Tensor& own, const at::Tensor& enemy,
                                     const at::Tensor& w, const at::Tensor& b, int64_t B, int64_t H, int64_t W) {
  check_cuda(sc, "sc");
  check_cuda(own, "own");
  check_cuda(enemy, "enemy");
  check_cuda(w, "w");
  check_cuda(b, "b");
  const int64_t P = B * H * W;
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && sc.dim() == 2 && sc.size(0) == P && sc.size(1) == as::vsp_in_channels() - 2 &&
              (sc.scalar_type() == at::kBFloat16 || sc.scalar_type() == at::kFloat) && sc.is_contiguous(),
              "vsp_pool: sc [B*H*W, 8] bf16 / fp32, even H / W");
  TORCH_CHECK(own.element_size() == 1 && enemy.element_size() == 1 && own.numel() == P && enemy.numel() == P,
              "vsp_pool: own / enemy [B*H*W] bool");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.size(0) == as::vsp_out_channels() && w.size(1) == as::vsp_in_channels()
              && b.scalar_type() == at::kFloat && b.numel() == as::vsp_out_channels(), "vsp_pool: w [16, 10], b [16] fp32");
  c10::hip::HIPGuard g(sc.device().index());
  const int64_t Po = B * (H / 2) * (W / 2);
  auto pooled = at::empty({Po, as::vsp_out_channels()}, sc.options());
  auto pos = at::empty({Po, as::vsp_out_channels()}, sc.options().dtype(at::kByte));
  as::vsp_pool_fwd(sc.data_ptr(), own.data_ptr(), enemy.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(),
                   pooled.data_ptr(), pos.data_ptr<uint8_t>(), static_cast<int>(B), static_cast<int>(H),
                   static_cast<int>(W), stream(), dt(sc));
  return {pooled, pos};
}

// -> {dSc [B*H*W, 8] bf16, [dW | db] [16, 11] fp32}
std::vector<at::Tensor> vsp_pool_bwd(const at::Tensor& dpooled, const at::Tensor& pos, const at::Tensor& pooled,
                                     const at::Tensor& sc, const at::Tensor& own, const at::Tensor& enemy,
                                     const at::Tensor& w, int64_t B, int64_t H, int64_t W) {
  check_cuda(dpooled, "dpooled");
  check_cuda(pos, "pos");
  check_cuda(pooled, "pooled");
  check_cuda(sc, "sc");
  check_cuda(w, "w");
  const int64_t P = B * H * W, Po = B * (H / 2) * (W / 2);
  TORCH_CHECK(dpooled.scalar_type() == sc.scalar_type() && pooled.scalar_type() == sc.scalar_type() &&
              dpooled.is_contiguous() && sc.is_contiguous() && dpooled.sizes() == pooled.sizes() && pos.sizes() == pooled.sizes() && pooled.size(0) == Po &&
              pooled.size(1) == as::vsp_out_channels(), "vsp_pool_bwd: dpooled / pooled / pos [Po, 16]");
  TORCH_CHECK(sc.size(0) == P && sc.size(1) == as::vsp_in_channels() - 2 && own.numel() == P && enemy.numel() == P &&
              own.element_size() == 1 && enemy.element_size() == 1 && own.is_contiguous() && enemy.is_contiguous(),
              "vsp_pool_bwd: sc / own / enemy");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.size(0) == as::vsp_out_channels() && w.size(1) == as::vsp_in_channels(),
              "vsp_pool_bwd: w [16, 10] fp32");
  c10::hip::HIPGuard g(sc.device().index());
  const int nblk = as::vsp_bwd_blocks(Po);
  auto dsc = at::empty_like(sc);
  auto part = at::empty({nblk, as::vsp_out_channels() * (as::vsp_in_channels() + 1)}, sc.options().dtype(at::kFloat));
  as::vsp_pool_bwd(dpooled.data_ptr(), pos.data_ptr<uint8_t>(), pooled.data_ptr(), sc.data_ptr(), own.data_ptr(),
                   enemy.data_ptr(), w.data_ptr<float>(), dsc.data_ptr(), part.data_ptr<float>(), static_cast<int>(B),
                   static_cast<int>(H), static_cast<int>(W), nblk, stream(), dt(sc));
  return {dsc, part.sum(0).view({as::vsp_out_channels(), as::vsp_in_channels() + 1})};
}

// ---------------------------------------------------------------- gate chain (gate_chain.hip)
// x [P,128] bf16; m: 4 x [128,128] bf16 (row n = output channel); bias: 4 x fp32 [128] or None; mask / res:
// 4 x bf16 [P,128] or None; relu_mask bit L: ReLU after layer L -> 4 outputs [P,128] bf16
std::vector<at::Tensor> gate_chain(const at::Tensor& x, const std::vector<at::Tensor>& m,
                                   const std::vector<c10::optional<at::Tensor>>& bias,
                                   const std::vector<c10::optional<at::Tensor>>& mask,
                                   const std::vector<c10::optional<at::Tensor>>& res, int64_t relu_mask) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.size(1) == 128 && x.is_contiguous(),
              "gate_chain: x [P,128] bf16 contiguous");
  TORCH_CHECK(m.size() == 4 && bias.size() == 4 && mask.size() == 4 && res.size() == 4, "gate_chain: 4 layers");
  const int64_t P = x.size(0);
  as::GateChainArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.relu_mask = static_cast<int>(relu_mask);
  std::vector<at::Tensor> outs;
  for (int L = 0; L < 4; ++L) {
    check_cuda(m[L], "m");
    TORCH_CHECK(m[L].scalar_type() == at::kBFloat16 && m[L].size(0) == 128 && m[L].numel() == 128 * 128 &&
                m[L].is_contiguous(), "gate_chain: m [128,128] bf16 contiguous");
    a.m[L] = reinterpret_cast<const uint16_t*>(m[L].data_ptr());
    a.bias[L] = nullptr;
    if (bias[L].has_value()) {
      check_cuda(*bias[L], "bias");
      TORCH_CHECK(bias[L]->scalar_type() == at::kFloat && bias[L]->numel() == 128, "gate_chain: bias fp32 [128]");
      a.bias[L] = bias[L]->data_ptr<float>();
    }
    a.mask[L] = nullptr;
    if (mask[L].has_value()) {
      check_cuda(*mask[L], "mask");
      TORCH_CHECK(mask[L]->scalar_type() == at::kBFloat16 && mask[L]->sizes() == x.sizes() &&
                  mask[L]->is_contiguous(), "gate_chain: mask like x");
      a.mask[L] = reinterpret_cast<const uint16_t*>(mask[L]->data_ptr());
    }
    a.res[L] = nullptr;
    if (res[L].has_value()) {
      check_cuda(*res[L], "res");
      TORCH_CHECK(res[L]->scalar_type() == at::kBFloat16 && res[L]->sizes() == x.sizes() &&
                  res[L]->is_contiguous(), "gate_chain: res like x");
      a.res[L] = reinterpret_cast<const uint16_t*>(res[L]->data_ptr());
    }
    outs.push_back(at::empty_like(x));
    a.out[L] = reinterpret_cast<uint16_t*>(outs.back().data_ptr());
  }
  c10::hip::HIPGuard g(x.device().index());
  as::gate_chain(a, P, stream());
  return outs;
}

// fp32 chain: x [P,128] fp32; m: 4 x [128,128] fp32 (row n = output channel); bias: 4 x fp32 [128] or None;
// mask / res: 4 x fp32 [P,128] or None -> 4 outputs [P,128] fp32
std::vector<at::Tensor> gate_chain_f32(const at::Tensor& x, const std::vector<at::Tensor>& m,
                                       const std::vector<c10::optional<at::Tensor>>& bias,
                                       const std::vector<c10::optional<at::Tensor>>& mask,
                                       const std::vector<c10::optional<at::Tensor>>& res, int64_t relu_mask) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 2 && x.size(1) == 128 && x.is_contiguous(),
              "gate_chain_f32: x [P,128] fp32 contiguous");
  TORCH_CHECK(m.size() == 4 && bias.size() == 4 && mask.size() == 4 && res.size() == 4, "gate_chain_f32: 4 layers");
  const int64_t P = x.size(0);
  TORCH_CHECK(P * 128 < (1LL << 31), "gate_chain_f32: 32-bit element offsets");
  as::GateChainF32Args a{};
  a.x = x.data_ptr<float>();
  a.relu_mask = static_cast<int>(relu_mask);
  auto opt = [&](const c10::optional<at::Tensor>& t, bool rows, const char* what) -> const float* {
    if (!t.has_value()) return nullptr;
    check_cuda(*t, what);
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() &&
                (rows ? t->sizes() == x.sizes() : t->numel() == 128), "gate_chain_f32: ", what, rows ? " like x" : " [128]");
    return t->data_ptr<float>();
  };
  std::vector<at::Tensor> outs;
  for (int L = 0; L < 4; ++L) {
    check_cuda(m[L], "m");
    TORCH_CHECK(m[L].scalar_type() == at::kFloat && m[L].size(0) == 128 && m[L].numel() == 128 * 128 &&
                m[L].is_contiguous(), "gate_chain_f32: m [128,128] fp32 contiguous");
    a.m[L] = m[L].data_ptr<float>();
    a.bias[L] = opt(bias[L], false, "bias");
    a.mask[L] = opt(mask[L], true, "mask");
    a.res[L] = opt(res[L], true, "res");
    outs.push_back(at::empty_like(x));
    a.out[L] = outs.back().data_ptr<float>();
  }
  c10::hip::HIPGuard g(x.device().index());
  as::gate_chain_f32(a, P, stream());
  return outs;
}

// ---------------------------------------------------------------- RL loss tail (rl_loss.hip)
// -> {info [rl_loss_info_size(F)], dalp, dent, dkl [6,T,B], dv [F,T+1,B]}
std::vector<at::Tensor> rl_loss(const at::Tensor& alp, const at::Tensor& blp, const at::Tensor& hm, const at::Tensor& ent,
                                const at::Tensor& kl, const at::Tensor& v, const at::Tensor& r, const at::Tensor& wm,
                                const at::Tensor& atflag, const at::Tensor& sc, int64_t upgo_f, bool only_value) {
  for (const at::Tensor* t : {&alp, &blp, &hm, &ent, &kl, &v, &r, &wm, &atflag, &sc}) {
    check_cuda(*t, "rl_loss operand");
    TORCH_CHECK(t->scalar_type() == at::kFloat, "rl_loss: fp32 operands");
  }
  TORCH_CHECK(alp.dim() == 3 && alp.size(0) == 6, "rl_loss: alp [6,T,B]");
  const int64_t T = alp.size(1), B = alp.size(2), F = v.size(0);
  TORCH_CHECK(blp.sizes() == alp.sizes() && hm.sizes() == alp.sizes() && ent.sizes() == alp.sizes() &&
              kl.sizes() == alp.sizes(), "rl_loss: per-head operands [6,T,B]");
  TORCH_CHECK(F >= 1 && F <= 6 && v.dim() == 3 && v.size(1) == T + 1 && v.size(2) == B && r.dim() == 3 &&
              r.size(0) == F && r.size(1) == T && r.size(2) == B && wm.sizes() == r.sizes(), "rl_loss: fields");
  TORCH_CHECK(atflag.numel() == T * B && T * B <= as::rl_loss_max_tb() && T >= 1, "rl_loss: [T,B] size");
  TORCH_CHECK(sc.numel() == 4 * F + 4 * 6 + 4 && upgo_f >= -1 && upgo_f < F, "rl_loss: scalars");
  c10::hip::HIPGuard g(alp.device().index());
  auto info = at::empty({as::rl_loss_info_size(static_cast<int>(F))}, alp.options());
  auto dalp = at::empty_like(alp), dent = at::empty_like(alp), dkl = at::empty_like(alp), dv = at::empty_like(v);
  as::rl_loss(alp.data_ptr<float>(), blp.data_ptr<float>(), hm.data_ptr<float>(), ent.data_ptr<float>(),
              kl.data_ptr<float>(), v.data_ptr<float>(), r.data_ptr<float>(), wm.data_ptr<float>(),
              atflag.data_ptr<float>(), sc.data_ptr<float>(), static_cast<int>(F), static_cast<int>(T),
              static_cast<int>(B), static_cast<int>(upgo_f), only_value ? 1 : 0, dalp.data_ptr<float>(),
              dent.data_ptr<float>(), dkl.data_ptr<float>(), dv.data_ptr<float>(), info.data_ptr<float>(), stream());
  return {info, dalp, dent, dkl, dv};
}

// ---------------------------------------------------------------- location-head input (locin.hip)
// y0 [P, 128] bf16 (skip W_s^T + b), p [B, 4*HW] bf16 (fc output), wp [128, 4] fp32 -> relu(y0 + W_p relu(p))
at::Tensor loc_in_fwd(const at::Tensor& y0, const at::Tensor& p, const at::Tensor& wp, int64_t HW) {
  check_cuda(y0, "y0");
  check_cuda(p, "p");
  check_cuda(wp, "wp");
  TORCH_CHECK(y0.scalar_type() == at::kBFloat16 && p.scalar_type() == at::kBFloat16 && wp.scalar_type() == at::kFloat,
              "loc_in: bf16 y0 / p, fp32 wp");
  TORCH_CHECK(y0.dim() == 2 && wp.dim() == 2 && as::loc_in_supported(static_cast<int>(y0.size(1)),
              static_cast<int>(wp.size(1))) && wp.size(0) == y0.size(1), "loc_in: [P,128] x [128,4]");
  TORCH_CHECK(HW > 0 && y0.size(0) % HW == 0 && p.numel() == (y0.size(0) / HW) * wp.size(1) * HW, "loc_in: p shape");
  c10::hip::HIPGuard g(y0.device().index());
  auto out = at::empty_like(y0);
  as::loc_in_fwd(y0.data_ptr(), p.data_ptr(), wp.data_ptr<float>(), out.data_ptr(), y0.size(0), static_cast<int>(HW),
                 stream());
  return out;
}

// -> {dY * (y > 0) [P,128] bf16, dp [B, 4*HW] bf16, dW_p [128, 4] fp32}
std::vector<at::Tensor> loc_in_bwd(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& p, const at::Tensor& wp,
                                   int64_t HW) {
  check_cuda(dy, "dy");
  check_cuda(y, "y");
  check_cuda(p, "p");
  check_cuda(wp, "wp");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 && dy.sizes() == y.sizes(),
              "loc_in_bwd: bf16 dy / y of one shape");
  TORCH_CHECK(p.scalar_type() == at::kBFloat16 && wp.scalar_type() == at::kFloat, "loc_in_bwd: dtypes");
  TORCH_CHECK(y.dim() == 2 && as::loc_in_supported(static_cast<int>(y.size(1)), static_cast<int>(wp.size(1))) &&
              wp.size(0) == y.size(1), "loc_in_bwd: [P,128] x [128,4]");
  TORCH_CHECK(HW > 0 && y.size(0) % HW == 0 && p.numel() == (y.size(0) / HW) * wp.size(1) * HW, "loc_in_bwd: p shape");
  c10::hip::HIPGuard g(y.device().index());
  const long P = y.size(0);
  const int nblk = as::loc_in_bwd_blocks(P);
  auto dym = at::empty_like(y);
  auto dp = at::empty_like(p);
  auto part = at::empty({nblk, wp.size(0) * wp.size(1)}, y.options().dtype(at::kFloat));
  as::loc_in_bwd(dy.data_ptr(), y.data_ptr(), p.data_ptr(), wp.data_ptr<float>(), dym.data_ptr(), dp.data_ptr(),
                 part.data_ptr<float>(), P, static_cast<int>(HW), nblk, stream());
  return {dym, dp, part.sum(0).view({wp.size(0), wp.size(1)})};
}

// ---------------------------------------------------------------- multi-tensor copy (+ dtype conversion)
// dst[i].copy_(src[i]) for same-shape, same-stride, non-overlapping-and-dense pairs (storage order copy);
// pairs that do not qualify are copied with copy_.  One H2D upload of the chunk table + one launch.
void multi_copy(const std::vector<at::Tensor>& dsts, const std::vector<at::Tensor>& srcs) {
  TORCH_CHECK(dsts.size() == srcs.size(), "multi_copy: list sizes");
  if (dsts.empty()) return;
  c10::hip::HIPGuard g(dsts[0].device().index());
  as::CopyArgs a;
  a.ntensors = 0;
  a.chunk_start[0] = 0;
  auto flush = [&]() {
    if (a.ntensors > 0) as::multi_copy(a, stream());
    a.ntensors = 0;
    a.chunk_start[0] = 0;
  };
  for (size_t i = 0; i < dsts.size(); ++i) {
    const at::Tensor& d = dsts[i];
    const at::Tensor& s = srcs[i];
    TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.sizes() == s.sizes(), "multi_copy: GPU tensors of equal shape");
    const bool same = d.scalar_type() == s.scalar_type();
    const auto st = s.scalar_type();
    const bool ok = d.strides() == s.strides() && d.is_non_overlapping_and_dense() &&
                    (same || ((d.scalar_type() == at::kFloat || d.scalar_type() == at::kBFloat16) &&
                              (st == at::kFloat || st == at::kBFloat16 || st == at::kByte || st == at::kShort)));
    if (!ok) {
      at::Tensor dd = d;
      dd.copy_(s);
      continue;
    }
    const long n = d.numel();
    if (n == 0) continue;
    // storage-order copy: the lowest address of a non-overlapping dense tensor is its data_ptr; equal dtypes
    // (any dtype) travel as raw bytes
    const int t = a.ntensors++;
    a.src[t] = s.data_ptr();
    a.dst[t] = d.data_ptr();
    if (same) {
      a.n[t] = n * static_cast<long>(d.element_size());
      a.dts[t] = 4;
      a.chunk_start[t + 1] = a.chunk_start[t] + static_cast<int>((a.n[t] + as::kCopyRawChunk - 1) / as::kCopyRawChunk);
    } else {
      a.n[t] = n;
      a.dts[t] = static_cast<unsigned char>((st == at::kFloat ? 1 : 0) | (d.scalar_type() == at::kFloat ? 2 : 0) |
                                            (st == at::kByte ? 8 : 0) | (st == at::kShort ? 16 : 0));
      a.chunk_start[t + 1] = a.chunk_start[t] + static_cast<int>((n + as::kCopyChunk - 1) / as::kCopyChunk);
    }
    if (a.ntensors == as::kCopyMaxT) flush();
  }
  flush();
}

// ---------------------------------------------------------------- strided multi-tensor copy (derived weight forms)
// dsts[t] (contiguous, fp32/bf16) <- srcs[t] read through spec[9 t .. 9 t + 8] = {size0..3, stride0..3, base}
// (element units, relative to srcs[t].data_ptr(); strides may be negative).  Every reachable source offset is
// checked against the source tensor's own extent before anything is launched.
// Column-block assembly (as::col_sum): pieces[k] = (dst, dst_col, width, [(src, src_col), ...] (1..3)); every
// tensor fp32 2-D [rows, *] with unit column stride (row pitch = stride(0)), all on one device.
void col_sum(const std::vector<at::Tensor>& dsts, const std::vector<int64_t>& dcols, const std::vector<int64_t>& widths,
             const std::vector<std::vector<at::Tensor>>& srcs, const std::vector<std::vector<int64_t>>& scols) {
  const size_t P = dsts.size();
  TORCH_CHECK(P > 0 && P <= as::kColMaxP && dcols.size() == P && widths.size() == P && srcs.size() == P &&
                  scols.size() == P, "col_sum: 1..32 pieces, matching lists");
  c10::hip::HIPGuard g(dsts[0].device().index());
  as::ColSumArgs a;
  a.npieces = static_cast<int>(P);
  a.rows = dsts[0].size(0);
  a.block_start[0] = 0;
  auto check = [&](const at::Tensor& t, int64_t col, int64_t w) {
    TORCH_CHECK(t.is_cuda() && t.device() == dsts[0].device() && t.scalar_type() == at::kFloat && t.dim() == 2 &&
                    t.size(0) == a.rows && t.stride(1) == 1 && col >= 0 && w >= 1 && col + w <= t.size(1) &&
                    t.stride(0) >= t.size(1) && t.stride(0) < (1L << 31),
                "col_sum: fp32 [rows, *] tensors with unit column stride, column block in range");
  };
  for (size_t p = 0; p < P; ++p) {
    check(dsts[p], dcols[p], widths[p]);
    TORCH_CHECK(srcs[p].size() >= 1 && srcs[p].size() <= 3 && scols[p].size() == srcs[p].size(),
                "col_sum: 1..3 sources per piece");
    a.dst[p] = dsts[p].data_ptr<float>();
    a.dld[p] = static_cast<int>(dsts[p].stride(0));
    a.doff[p] = static_cast<int>(dcols[p]);
    a.width[p] = static_cast<int>(widths[p]);
    a.nsrc[p] = static_cast<int>(srcs[p].size());
    for (size_t k = 0; k < srcs[p].size(); ++k) {
      check(srcs[p][k], scols[p][k], widths[p]);
      a.src[p][k] = srcs[p][k].data_ptr<float>();
      a.sld[p][k] = static_cast<int>(srcs[p][k].stride(0));
      a.soff[p][k] = static_cast<int>(scols[p][k]);
    }
    const long n = a.rows * widths[p];
    a.block_start[p + 1] = a.block_start[p] + static_cast<int>(std::min<long>((n + 1023) / 1024, 256));
  }
  as::col_sum(a, stream());
}

void multi_strided_copy(const std::vector<at::Tensor>& dsts, const std::vector<at::Tensor>& srcs,
                        const std::vector<int64_t>& spec) {
  TORCH_CHECK(dsts.size() == srcs.size() && spec.size() == 9 * dsts.size(), "multi_strided_copy: list sizes");
  if (dsts.empty()) return;
  c10::hip::HIPGuard g(dsts[0].device().index());
  as::StridedCopyArgs a;
  a.ntensors = 0;
  a.chunk_start[0] = 0;
  auto flush = [&]() {
    if (a.ntensors > 0) as::multi_strided_copy(a, stream());
    a.ntensors = 0;
    a.chunk_start[0] = 0;
  };
  for (size_t i = 0; i < dsts.size(); ++i) {
    const at::Tensor& d = dsts[i];
    const at::Tensor& s = srcs[i];
    TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.device() == s.device(), "multi_strided_copy: GPU tensors");
    TORCH_CHECK(d.is_contiguous(), "multi_strided_copy: contiguous destination");
    TORCH_CHECK((d.scalar_type() == at::kFloat || d.scalar_type() == at::kBFloat16) &&
                (s.scalar_type() == at::kFloat || s.scalar_type() == at::kBFloat16), "multi_strided_copy: fp32/bf16");
    const int64_t* sp = spec.data() + 9 * i;
    int64_t n = 1, lo = sp[8], hi = sp[8];
    for (int k = 0; k < 4; ++k) {
      TORCH_CHECK(sp[k] >= 1, "multi_strided_copy: sizes >= 1");
      n *= sp[k];
      const int64_t reach = (sp[k] - 1) * sp[4 + k];
      if (reach < 0) lo += reach; else hi += reach;
    }
    TORCH_CHECK(n == d.numel() && n < (int64_t{1} << 31), "multi_strided_copy: spec / destination size");
    int64_t extent = 1;                 // elements spanned by the source view itself
    for (int64_t k = 0; k < s.dim(); ++k) extent += (s.size(k) - 1) * s.stride(k);
    TORCH_CHECK(lo >= 0 && hi < extent, "multi_strided_copy: spec reaches outside the source");
    const int t = a.ntensors++;
    a.src[t] = s.data_ptr();
    a.dst[t] = d.data_ptr();
    a.n[t] = static_cast<int>(n);
    for (int k = 0; k < 4; ++k) {
      a.size[t][k] = static_cast<int>(sp[k]);
      a.stride[t][k] = sp[4 + k];
    }
    a.base[t] = sp[8];
    // a transpose of the last two dims (dst rows contiguous in the source) of a large tensor: LDS-tiled path,
    // one 64 x 128 tile per block
    const bool tiled = sp[0] == 1 && sp[1] == 1 && sp[6] == 1 && sp[7] > 1 && n >= (1 << 16);
    a.dts[t] = static_cast<unsigned char>((s.scalar_type() == at::kFloat ? 1 : 0) | (d.scalar_type() == at::kFloat ? 2 : 0) |
                                          (tiled ? 4 : 0));
    const int64_t chunks = tiled ? ((sp[2] + 63) / 64) * ((sp[3] + 127) / 128) : (n + as::kCopyChunk - 1) / as::kCopyChunk;
    a.chunk_start[t + 1] = a.chunk_start[t] + static_cast<int>(chunks);
    if (a.ntensors == as::kSCopyMaxT) flush();
  }
  flush();
}

// ---------------------------------------------------------------- narrow 1x1 conv on NHWC pixels
at::Tensor pointwise_conv(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act) {
  check_cuda(x, "x");
  check_cuda(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "pointwise: x [P, cin] bf16");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.dim() == 2 && w.size(1) == x.size(1), "pointwise: w fp32 [cout, cin]");
  const int64_t P = x.size(0), cin = x.size(1), cout = w.size(0);
  TORCH_CHECK(as::pointwise_supported(static_cast<int>(cin), static_cast<int>(cout)), "pointwise: channels");
  const float* bp = nullptr;
  if (bias.has_value()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == cout, "pointwise: bias fp32 [cout]");
    bp = bias->data_ptr<float>();
  }
  c10::hip::HIPGuard g(x.device().index());
  auto y = at::empty({P, cout}, x.options());
  as::pointwise_conv(x.data_ptr(), w.data_ptr<float>(), bp, y.data_ptr(), P, static_cast<int>(cin),
                     static_cast<int>(cout), static_cast<int>(act), stream());
  return y;
}

void register_codec(pybind11::module& m);   // codec.cpp: native tensor-tree frames (utils/serialize.py)

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "applestar_amd HIP kernels for gfx950 (MI355X)";
  register_codec(m);
  m.def("layer_norm_fwd", &layer_norm_fwd);
  m.def("layer_norm_bwd", &layer_norm_bwd, py::arg("dy"), py::arg("xin"), py::arg("y"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("dx_dtype"), py::arg("act"), py::arg("mask_src") = py::none());
  m.def("reverse_scan", &reverse_scan);
  m.def("col_sum", &col_sum);
  m.def("multi_logp", &multi_logp);
  m.def("presplit_b", &presplit_b, py::arg("b"), py::arg("trans") = false, py::arg("out") = py::none());
  m.def("gemm_f32_psb_supported", &gemm_f32_psb_supported);
  m.def("multi_presplit", &multi_presplit);
  m.def("conv3x3_f32_psb_supported", &conv3x3_f32_psb_supported);
  m.def("conv3x3_f32_psb", &conv3x3_f32_psb, py::arg("x"), py::arg("wsplit"), py::arg("Cout"),
        py::arg("bias") = py::none(), py::arg("res") = py::none(), py::arg("res2") = py::none(),
        py::arg("mask") = py::none(), py::arg("act") = 0);
  m.def("conv3x3_f32_v2", &conv3x3_f32_v2, py::arg("x"), py::arg("wsplit"), py::arg("Cout"),
        py::arg("bias") = py::none(), py::arg("res") = py::none(), py::arg("res2") = py::none(),
        py::arg("mask") = py::none(), py::arg("act") = 0, py::arg("variant") = 0);
  m.def("gemm_f32_psb", &gemm_f32_psb, py::arg("a"), py::arg("bsplit"), py::arg("N"), py::arg("K"),
        py::arg("bias") = py::none(), py::arg("res") = py::none(), py::arg("act") = 0, py::arg("variant") = 0);
  m.def("entity_pack", &entity_pack);
  m.def("embed_relu_fwd", &embed_relu_fwd);
  m.def("embed_relu_bwd", &embed_relu_bwd);
  m.def("gated_residual_fwd", &gated_residual_fwd, py::arg("y"), py::arg("g"), py::arg("sp"), py::arg("x"),
        py::arg("post") = py::none());
  m.def("gated_residual_bwd", &gated_residual_bwd, py::arg("dout"), py::arg("y"), py::arg("g"), py::arg("sp"),
        py::arg("out"), py::arg("xin") = py::none());
  m.def("lnlstm_fwd", &lnlstm_fwd, py::arg("xp"), py::arg("h0"), py::arg("c0"), py::arg("wT"),
        py::arg("lnh_w"), py::arg("lnh_b"), py::arg("lnc_w"), py::arg("lnc_b"),
        py::arg("eps"), py::arg("want_bf16") = false);
  m.def("lnlstm_bwd", &lnlstm_bwd);
  m.def("entity_embed_fwd", &entity_embed_fwd);
  m.def("entity_onehot", &entity_onehot);
  m.def("upsample2x_fwd", &upsample2x_fwd);
  m.def("upsample2x_bwd", &upsample2x_bwd, py::arg("dy"), py::arg("mask") = py::none());
  m.def("entity_embed_wgrad", &entity_embed_wgrad);
  m.def("mm_k32", &mm_k32);
  m.def("spatial_embed_fwd", &spatial_embed_fwd);
  m.def("spatial_gather_rows", &spatial_gather_rows, py::arg("dpre"), py::arg("ex"), py::arg("ey"),
        py::arg("entity_num"), py::arg("N"), py::arg("gate") = py::none());
  m.def("spatial_dense_input", &spatial_dense_input);
  m.def("spatial_dense_wgrad", &spatial_dense_wgrad, py::arg("planes"), py::arg("effects"), py::arg("dpre"),
        py::arg("gate") = py::none());
  m.def("varlen_attn_fwd", &varlen_attn_fwd);
  m.def("varlen_attn_bwd", &varlen_attn_bwd);
  m.def("varlen_attn_fwd_f32", &varlen_attn_fwd_f32);
  m.def("conv3x3_f32_epi2", &conv3x3_f32_epi2);
  m.def("conv3x3_f32_epi2_supported", &conv3x3_f32_epi2_supported);
  m.def("conv3x3_f32", &conv3x3_f32);
  m.def("fused_clip_adam", &fused_clip_adam);
  m.def("head_sample", &head_sample);
  m.def("target_unit_sample", &target_unit_sample);
  m.def("fused_adam_chunk", &as::fused_adam_chunk);
  m.def("wgrad_f32", &wgrad_f32, py::arg("dy"), py::arg("x"), py::arg("cin"), py::arg("want_bias"),
        py::arg("out") = py::none());
  m.def("gemm_f32", &gemm_f32);
  m.def("gemm_bf16_small", &gemm_bf16_small);
  m.def("gemm_bf16", &gemm_bf16);
  m.def("small_gemm", &small_gemm);
  m.def("small_wgrad", &small_wgrad);
  m.def("small_gemm_splitk", &small_gemm_splitk);
  m.def("f32_mfma_mode", &as::f32_mfma_mode);
  m.def("set_f32_pipe_variant", &as::set_f32_pipe_variant);
  m.def("set_f32_conv_variant", &as::set_f32_conv_variant);
  m.def("set_f32_mfma_mode", &as::set_f32_mfma_mode);
  m.def("conv3x3_f32_supported", &as::conv3x3_f32_supported);
  m.def("varlen_attn_bwd_f32", &varlen_attn_bwd_f32);
  m.def("attn_f32_variant", [](int64_t v) { return static_cast<int64_t>(as::attn_f32_variant(static_cast<int>(v))); });
  m.def("su_sample", &su_sample);
  m.def("segment_copy", &segment_copy);
  m.def("conv_wt", &conv_wt);
  m.def("upconv1_fwd", &upconv1_fwd);
  m.def("upconv1_bwd", &upconv1_bwd, py::arg("x_nhwc"), py::arg("w"), py::arg("dy"), py::arg("relu_mask") = false);
  m.def("maxpool2_fwd", &maxpool2_fwd);
  m.def("maxpool2_bwd", &maxpool2_bwd, py::arg("dy"), py::arg("pos"), py::arg("H"), py::arg("W"),
        py::arg("mask") = py::none());
  m.def("maxpool2_bwd_relu", &maxpool2_bwd_relu);
  m.def("spatial_embed_pool_fwd", &spatial_embed_pool_fwd);
  m.def("spatial_pool_supported", [](int64_t h, int64_t w) { return as::spatial_pool_supported(static_cast<int>(h), static_cast<int>(w)); });
  m.def("segment_sum", &segment_sum);
  m.def("spatial_dense_wgrad_pooled", &spatial_dense_wgrad_pooled);
  m.def("spatial_gather_rows_pooled", &spatial_gather_rows_pooled);
  m.def("entity_mean_pool", &entity_mean_pool);
  m.def("table_grad", &table_grad);
  m.def("conv3x3_fwd", &conv3x3_fwd);
  m.def("wgrad", &wgrad, py::arg("dy"), py::arg("x"), py::arg("cin"), py::arg("want_bias"),
        py::arg("bf16_out") = false);
  m.def("pointwise_conv", &pointwise_conv);
  m.def("pointwise_supported", [](int64_t ci, int64_t co) { return as::pointwise_supported(static_cast<int>(ci), static_cast<int>(co)); });
  m.def("lstm_split_error", &lstm_split_error);
  m.def("lstm_split_flag", &lstm_split_flag);
  m.def("multi_copy", &multi_copy);
  m.def("ln_affine_grads", &ln_affine_grads);
  m.def("multi_strided_copy", &multi_strided_copy);
  m.def("loc_in_fwd", &loc_in_fwd);
  m.def("vsp_fwd", &vsp_fwd);
  m.def("rl_loss", &rl_loss);
  m.def("gate_chain", &gate_chain);
  m.def("gate_chain_f32", &gate_chain_f32);
  m.def("vsp_pool_fwd", &vsp_pool_fwd);
  m.def("vsp_pool_bwd", &vsp_pool_bwd);
  m.def("vsp_in_channels", []() { return as::vsp_in_channels(); });
  m.def("vsp_out_channels", []() { return as::vsp_out_channels(); });
  m.def("vsp_bwd", &vsp_bwd);
  m.def("loc_in_supported", [](int64_t c, int64_t p) { return as::loc_in_supported(static_cast<int>(c), static_cast<int>(p)); });
  m.def("loc_in_bwd", &loc_in_bwd);
  m.def("head_stats_fwd", &head_stats_fwd);
  m.def("resmlp_fwd", &resmlp_fwd);
  m.def("resmlp_bwd", &resmlp_bwd);
  m.def("bo_encoder_fwd", &bo_encoder_fwd);
  m.def("bo_encoder_bwd", &bo_encoder_bwd);
  m.def("head_stats_bwd", &head_stats_bwd);
  m.def("act_grad_nhwc", &act_grad_nhwc);
  m.def("conv3x3_supported", [](int64_t cin, int64_t cout) { return as::conv3x3_supported(static_cast<int>(cin), static_cast<int>(cout)); });
}
