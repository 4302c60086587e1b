#include <cmath>
#include <cstdlib>
// Python bindings for the gfx950 kernels. Every op checks device, dtype,
// contiguity and alignment on the host before launching (a mis-shaped launch
// of a hand-written kernel must fail loudly here, never fault on the GPU), and
// launches on the caller's current HIP stream so ops compose with torch
// streams, events and hipGraph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "geom_guard.h"
#include "launchers.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous() || t.is_contiguous(at::MemoryFormat::ChannelsLast), name,
              " must be dense (contiguous or channels_last)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " must be 16-byte aligned");
}

void check_flat(const Tensor& t, at::ScalarType dt, int64_t n, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.numel() == n, name, " has ", t.numel(), " elements, expected ", n);
}

template <typename T>
T* ptr_or_null(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// BatchNorm slot sums [2][kBnSlots][C]: a persistent per-layer buffer (zeroed
// once, re-zeroed by every finalize) or a fresh zeroed one
Tensor bn_slots(const optional<Tensor>& slots, int64_t C, const at::TensorOptions& opt) {
  if (slots.has_value() && slots->defined()) {
    TORCH_CHECK(slots->is_cuda() && slots->scalar_type() == at::kFloat && slots->is_contiguous() &&
                    slots->numel() == 2 * dmp::kBnSlots * C + dmp::kBnTail,
                "BN slot buffer must be a contiguous fp32 GPU tensor of 2*", dmp::kBnSlots,
                "*C+", dmp::kBnTail, " elements");
    return *slots;
  }
  return at::zeros({2 * dmp::kBnSlots * C + dmp::kBnTail}, opt.dtype(at::kFloat));
}

// ----------------------------------------------------------------- optimizer
void asgd_fused_step(Tensor g, Tensor p, optional<Tensor> acc, optional<Tensor> mom,
                     optional<Tensor> w16, double lr, double wd, double momentum,
                     double dampening, bool nesterov) {
  const int64_t n = p.numel();
  TORCH_CHECK(n % 4 == 0, "flat arena length must be a multiple of 4");
  check_flat(p, at::kFloat, n, "p");
  check_flat(g, at::kFloat, n, "g");
  if (acc) check_flat(*acc, at::kFloat, n, "acc");
  if (mom) check_flat(*mom, at::kFloat, n, "mom");
  if (w16) check_flat(*w16, at::kBFloat16, n, "w16");
  dmp::launch_asgd_fused_step(g.data_ptr<float>(), p.data_ptr<float>(), ptr_or_null<float>(acc),
                              ptr_or_null<float>(mom), ptr_or_null<uint16_t>(w16), n, (float)lr,
                              (float)wd, (float)momentum, (float)dampening, nesterov,
                              cur_stream());
}

void ps_apply(Tensor shard, Tensor delta, optional<Tensor> mirror, double scale, bool atomic) {
  const int64_t n = shard.numel();
  TORCH_CHECK(n % 4 == 0, "shard length must be a multiple of 4");
  check_flat(shard, at::kFloat, n, "shard");
  if (mirror) check_flat(*mirror, at::kBFloat16, n, "mirror");
  if (atomic) {
    // concurrent applies on several streams: no mirror (it would race)
    TORCH_CHECK(!mirror, "ps_apply: atomic applies take no bf16 mirror");
    const bool bf = delta.scalar_type() == at::kBFloat16;
    check_flat(delta, bf ? at::kBFloat16 : at::kFloat, n, "delta");
    dmp::launch_ps_apply_atomic(shard.data_ptr<float>(), delta.data_ptr(), bf, n, (float)scale,
                                cur_stream());
    return;
  }
  if (delta.scalar_type() == at::kFloat) {
    check_flat(delta, at::kFloat, n, "delta");
    dmp::launch_ps_apply_f32(shard.data_ptr<float>(), delta.data_ptr<float>(),
                             ptr_or_null<uint16_t>(mirror), n, (float)scale, cur_stream());
  } else {
    check_flat(delta, at::kBFloat16, n, "delta");
    dmp::launch_ps_apply_bf16(shard.data_ptr<float>(),
                              reinterpret_cast<uint16_t*>(delta.data_ptr()),
                              ptr_or_null<uint16_t>(mirror), n, (float)scale, cur_stream());
  }
}

// PS applied-count (server.py / async_sharded.py version stamps): ps_count adds
// `add` to (or, set=True, sets) the int32 counter on the current stream;
// ps_stamp writes float(counter) into the 1-element fp32 `dst`
void ps_count(Tensor cnt, int64_t add, bool set) {
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && cnt.numel() == 1,
              "ps_count: counter must be a 1-element int32 GPU tensor");
  dmp::launch_ps_count(cnt.data_ptr<int>(), (int)add, set, cur_stream());
}

void ps_stamp(Tensor cnt, Tensor dst) {
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && cnt.numel() == 1,
              "ps_stamp: counter must be a 1-element int32 GPU tensor");
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.numel() == 1 &&
                  dst.device() == cnt.device(),
              "ps_stamp: dst must be a 1-element fp32 tensor on the counter's device");
  dmp::launch_ps_stamp(cnt.data_ptr<int>(), dst.data_ptr<float>(), cur_stream());
}

void pull_land(Tensor p, Tensor src, optional<Tensor> acc, optional<Tensor> w16) {
  const int64_t n = p.numel();
  TORCH_CHECK(n % 4 == 0, "arena length must be a multiple of 4");
  check_flat(p, at::kFloat, n, "p");
  if (acc) check_flat(*acc, at::kFloat, n, "acc");
  if (w16) check_flat(*w16, at::kBFloat16, n, "w16");
  if (src.scalar_type() == at::kFloat) {
    check_flat(src, at::kFloat, n, "src");
    dmp::launch_pull_land_f32(p.data_ptr<float>(), src.data_ptr<float>(), ptr_or_null<float>(acc),
                              ptr_or_null<uint16_t>(w16), n, cur_stream());
  } else {
    check_flat(src, at::kBFloat16, n, "src");
    dmp::launch_pull_land_bf16(p.data_ptr<float>(), reinterpret_cast<uint16_t*>(src.data_ptr()),
                               ptr_or_null<float>(acc), ptr_or_null<uint16_t>(w16), n,
                               cur_stream());
  }
}

void push_handoff(Tensor acc, optional<Tensor> out32, optional<Tensor> out16) {
  const int64_t n = acc.numel();
  TORCH_CHECK(n % 4 == 0, "arena length must be a multiple of 4");
  check_flat(acc, at::kFloat, n, "acc");
  if (out32) check_flat(*out32, at::kFloat, n, "out32");
  if (out16) check_flat(*out16, at::kBFloat16, n, "out16");
  dmp::launch_push_handoff(acc.data_ptr<float>(), ptr_or_null<float>(out32),
                           ptr_or_null<uint16_t>(out16), n, cur_stream());
}

void cast_f32_bf16(Tensor src, Tensor dst) {
  const int64_t n = src.numel();
  TORCH_CHECK(n % 4 == 0, "length must be a multiple of 4");
  check_flat(src, at::kFloat, n, "src");
  check_flat(dst, at::kBFloat16, n, "dst");
  dmp::launch_cast_f32_bf16(src.data_ptr<float>(), reinterpret_cast<uint16_t*>(dst.data_ptr()), n,
                            cur_stream());
}

Tensor sumsq(Tensor x) {
  const int64_t n = x.numel();
  TORCH_CHECK(n % 4 == 0, "length must be a multiple of 4");
  check_flat(x, at::kFloat, n, "x");
  auto part = at::empty({1024}, x.options());
  const int g = dmp::launch_sumsq_partial(x.data_ptr<float>(), part.data_ptr<float>(), n,
                                          cur_stream());
  return part.narrow(0, 0, g).sum();
}

// ------------------------------------------------------------ cross-entropy
std::vector<Tensor> softmax_xent(Tensor logits, Tensor labels, bool want_grad, double smoothing,
                                 int64_t ignore_index) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits must be contiguous [B, C]");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous(),
              "labels must be a contiguous int64 GPU tensor");
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  TORCH_CHECK(labels.numel() == B, "labels length mismatch");
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({}, fopt);
  auto hits = at::empty({}, logits.options().dtype(at::kInt));
  auto row_loss = at::empty({B}, fopt);
  auto row_hit = at::empty({B}, logits.options().dtype(at::kInt));
  Tensor dlogits;
  if (want_grad) dlogits = at::empty_like(logits);
  // <= 0: the kernels count the non-ignored rows on device and scale the
  // gradient by 1/#valid (the mean the reported loss uses)
  const float grad_scale = -1.f;
  if (logits.scalar_type() == at::kBFloat16) {
    dmp::launch_softmax_xent_bf16(
        reinterpret_cast<const uint16_t*>(logits.data_ptr()), labels.data_ptr<int64_t>(),
        want_grad ? reinterpret_cast<uint16_t*>(dlogits.data_ptr()) : nullptr,
        row_loss.data_ptr<float>(), row_hit.data_ptr<int>(), loss.data_ptr<float>(),
        hits.data_ptr<int>(), B, C, grad_scale, (float)smoothing, (int)ignore_index, cur_stream());
  } else {
    TORCH_CHECK(logits.scalar_type() == at::kFloat, "logits must be bf16 or f32");
    dmp::launch_softmax_xent_f32(
        logits.data_ptr<float>(), labels.data_ptr<int64_t>(),
        want_grad ? dlogits.data_ptr<float>() : nullptr, row_loss.data_ptr<float>(),
        row_hit.data_ptr<int>(), loss.data_ptr<float>(), hits.data_ptr<int>(), B, C, grad_scale,
        (float)smoothing, (int)ignore_index, cur_stream());
  }
  return {loss, hits, want_grad ? dlogits : Tensor()};
}

// ---------------------------------------------------------------- batchnorm
// x is a channels-last activation (N,C,H,W logical) or a [M, C] matrix.
int64_t channels_of(const Tensor& x) { return x.dim() == 2 ? x.size(1) : x.size(1); }

void check_nhwc_bf16(const Tensor& x, const char* name) {
  check_gpu(x, name);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, name, " must be bf16");
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last");
  } else {
    TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), name, " must be [M, C] contiguous");
  }
}

std::vector<Tensor> bn_fwd(Tensor x, optional<Tensor> res, optional<Tensor> gamma,
                           optional<Tensor> beta, optional<Tensor> running_mean,
                           optional<Tensor> running_var, double momentum, double eps,
                           bool training, bool relu, optional<Tensor> slots, bool want_mask) {
  check_nhwc_bf16(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: C must be a multiple of 8 and <= 2048, got ", C);
  if (res) {
    check_nhwc_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
  }
  for (auto* t : {&gamma, &beta, &running_mean, &running_var}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn affine/running tensors must be contiguous fp32 [C] on the GPU");
    }
  }
  TORCH_CHECK(training || (running_mean && running_var), "eval-mode bn needs running stats");
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto stats = at::empty({4, C}, fopt);
  auto part = bn_slots(slots, C, fopt);
  // 1-bit ReLU mask [M][C/8] for the backward (instead of re-reading y)
  Tensor mask;
  if (want_mask && relu) mask = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  dmp::launch_bn_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                     res ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr,
                     reinterpret_cast<uint16_t*>(y.data_ptr()), ptr_or_null<float>(gamma),
                     ptr_or_null<float>(beta), ptr_or_null<float>(running_mean),
                     ptr_or_null<float>(running_var), stats.data_ptr<float>(),
                     part.data_ptr<float>(), M, (int)C, (float)momentum, (float)eps, training,
                     relu, cur_stream(), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, stats, mask};
}

std::vector<Tensor> bn_bwd(Tensor x, Tensor dy, optional<Tensor> y, optional<Tensor> gamma,
                           Tensor stats, optional<Tensor> dgamma, optional<Tensor> dbeta,
                           bool relu, bool want_dres, optional<Tensor> slots,
                           optional<Tensor> mask) {
  check_nhwc_bf16(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: bad C");
  if (!dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.dim() == 4)
    dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  // relu without y: the mask is recomputed from x and stats (forward had no residual)
  const bool have_y = relu && y.has_value() && y->defined();
  if (have_y) {
    check_nhwc_bf16(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes(), "y shape mismatch");
  }
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * C, "bad stats");
  for (auto* t : {&gamma, &dgamma, &dbeta}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn gamma/dgamma/dbeta must be contiguous fp32 [C]");
    }
  }
  auto dx = at::empty_like(x);
  Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto part = bn_slots(slots, C, fopt);
  auto coef = at::empty({3, C}, fopt);
  const uint8_t* mptr = nullptr;
  if (relu && mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == M * C / 8,
                "bn: ReLU bit mask must be a contiguous uint8 [M, C/8] GPU tensor");
    mptr = mask->data_ptr<uint8_t>();
  }
  dmp::launch_bn_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                     reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                     have_y ? reinterpret_cast<const uint16_t*>(y->data_ptr()) : nullptr,
                     ptr_or_null<float>(gamma), stats.data_ptr<float>(),
                     ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta), coef.data_ptr<float>(),
                     part.data_ptr<float>(), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                     want_dres ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr, M,
                     (int)C, relu, cur_stream(), mptr);
  return {dx, want_dres ? dres : Tensor()};
}

// dz: the already ReLU-masked output gradient; part: the slot sums the consuming
// conv's dgrad epilogue accumulated (re-zeroed here)
Tensor bn_bwd_from_partials(Tensor x, Tensor dz, optional<Tensor> gamma, Tensor stats,
                            optional<Tensor> dgamma, optional<Tensor> dbeta, Tensor part) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dz, "dz");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: bad C");
  TORCH_CHECK(dz.sizes() == x.sizes(), "dz shape mismatch");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * C, "bad stats");
  for (auto* t : {&gamma, &dgamma, &dbeta}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn gamma/dgamma/dbeta must be contiguous fp32 [C]");
    }
  }
  auto fopt = x.options().dtype(at::kFloat);
  part = bn_slots(part, C, fopt);
  auto dx = at::empty_like(x);
  auto coef = at::empty({3, C}, fopt);
  dmp::launch_bn_bwd_from_partials(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(dz.data_ptr()),
                                   ptr_or_null<float>(gamma), stats.data_ptr<float>(),
                                   ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta),
                                   coef.data_ptr<float>(), part.data_ptr<float>(),
                                   reinterpret_cast<uint16_t*>(dx.data_ptr()), M, (int)C,
                                   cur_stream());
  return dx;
}

// ------------------------------------------------------------------ pooling
// fused GAP + Linear head: [y [B, N] bf16, f [B, C] bf16 (pooled features, kept
// for the weight gradient)]
std::vector<Tensor> gap_linear_fwd(Tensor x, Tensor w, optional<Tensor> bias) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "gap_linear expects NCHW (channels_last) input");
  const int B = (int)x.size(0), C = (int)x.size(1), HW = (int)(x.size(2) * x.size(3));
  check_gpu(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.size(1) == C &&
                  w.is_contiguous(), "gap_linear: w must be contiguous bf16 [N, C]");
  const int N = (int)w.size(0);
  TORCH_CHECK(dmp::gap_linear_supported(C, N), "gap_linear: unsupported C / N");
  if (bias) {
    check_gpu(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous(),
                "gap_linear: bias must be contiguous bf16 [N]");
  }
  auto y = at::empty({B, N}, x.options().memory_format(at::MemoryFormat::Contiguous));
  auto f = at::empty({B, C}, x.options().memory_format(at::MemoryFormat::Contiguous));
  dmp::launch_gap_linear_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                             reinterpret_cast<const uint16_t*>(w.data_ptr()),
                             bias ? reinterpret_cast<const uint16_t*>(bias->data_ptr()) : nullptr,
                             reinterpret_cast<uint16_t*>(y.data_ptr()),
                             reinterpret_cast<uint16_t*>(f.data_ptr()), B, HW, C, N, cur_stream());
  return {y, f};
}

// dx [B, C, H, W] channels-last; gw [N, C] fp32 (+=), gb [N] fp32 (+=)
Tensor gap_linear_bwd(Tensor dy, Tensor f, Tensor w, Tensor gw, optional<Tensor> gb, int64_t H,
                      int64_t W) {
  dy = dy.contiguous();
  check_gpu(dy, "dy");
  check_gpu(f, "f");
  check_gpu(w, "w");
  check_gpu(gw, "gw");
  const int B = (int)f.size(0), C = (int)f.size(1), N = (int)w.size(0);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 && dy.size(0) == B &&
                  dy.size(1) == N, "gap_linear_bwd: dy must be bf16 [B, N]");
  TORCH_CHECK(f.scalar_type() == at::kBFloat16 && f.is_contiguous(), "gap_linear_bwd: f bf16 [B, C]");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.size(1) == C,
              "gap_linear_bwd: w bf16 [N, C]");
  TORCH_CHECK(gw.scalar_type() == at::kFloat && gw.is_contiguous() && gw.numel() == (int64_t)N * C,
              "gap_linear_bwd: gw fp32 [N, C]");
  TORCH_CHECK(dmp::gap_linear_supported(C, N), "gap_linear: unsupported C / N");
  if (gb) {
    check_gpu(*gb, "gb");
    TORCH_CHECK(gb->scalar_type() == at::kFloat && gb->numel() == N && gb->is_contiguous(),
                "gap_linear_bwd: gb fp32 [N]");
  }
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  dmp::launch_gap_linear_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                             reinterpret_cast<const uint16_t*>(f.data_ptr()),
                             reinterpret_cast<const uint16_t*>(w.data_ptr()),
                             reinterpret_cast<uint16_t*>(dx.data_ptr()), gw.data_ptr<float>(),
                             gb ? gb->data_ptr<float>() : nullptr, B, (int)(H * W), C, N,
                             cur_stream());
  return dx;
}

Tensor gap_fwd(Tensor x) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "gap expects NCHW (channels_last) input");
  const int N = (int)x.size(0), C = (int)x.size(1), HW = (int)(x.size(2) * x.size(3));
  TORCH_CHECK(C % 8 == 0, "gap: C must be a multiple of 8");
  auto y = at::empty({N, C}, x.options().memory_format(at::MemoryFormat::Contiguous));
  dmp::launch_gap_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                      reinterpret_cast<uint16_t*>(y.data_ptr()), N, HW, C, cur_stream());
  return y;
}

Tensor gap_bwd(Tensor dy, int64_t H, int64_t W) {
  dy = dy.contiguous();
  check_gpu(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.dim() == 2, "gap_bwd expects bf16 [N, C]");
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  TORCH_CHECK(C % 8 == 0, "gap: C must be a multiple of 8");
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  dmp::launch_gap_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                      reinterpret_cast<uint16_t*>(dx.data_ptr()), N, (int)(H * W), C,
                      cur_stream());
  return dx;
}

std::vector<Tensor> maxpool_fwd(Tensor x, int64_t K, int64_t S, int64_t P, bool nchw_out,
                                bool relu_in) {
  if (S < 0) S = K;
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "maxpool expects 4-D input");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(K >= 1 && K <= 15 && S >= 1 && P >= 0 && 2 * P <= K,
              "maxpool: 1 <= K <= 15, S >= 1, 0 <= P <= K/2");
  const int Ho = dmp::maxpool_out(H, (int)K, (int)S, (int)P);
  const int Wo = dmp::maxpool_out(W, (int)K, (int)S, (int)P);
  TORCH_CHECK(Ho > 0 && Wo > 0, "maxpool: window larger than input");
  auto mf = at::MemoryFormat::ChannelsLast;
  const bool nchw = nchw_out && C % 8 == 0;
  auto y = at::empty({N, C, Ho, Wo},
                     x.options().memory_format(nchw ? at::MemoryFormat::Contiguous : mf));
  auto idx = at::empty({N, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(mf));
  dmp::launch_maxpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                          reinterpret_cast<uint16_t*>(y.data_ptr()), idx.data_ptr<uint8_t>(), N, H,
                          W, C, (int)K, (int)S, (int)P, cur_stream(), nchw, relu_in);
  if (nchw_out && !nchw) y = y.contiguous();
  return {y, idx};
}

Tensor maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t K, int64_t S, int64_t P) {
  if (S < 0) S = K;
  auto mf = at::MemoryFormat::ChannelsLast;
  // an NCHW-contiguous dy (gradient of an nchw_out forward) is read in place
  const bool nchw = dy.dim() == 4 && dy.size(1) % 8 == 0 && dy.is_contiguous() &&
                    !dy.is_contiguous(mf);
  if (!nchw) {
    dy = dy.contiguous(mf);
    check_nhwc_bf16(dy, "dy");
  } else {
    check_gpu(dy, "dy");
  }
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.is_contiguous(mf), "maxpool idx mismatch");
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  TORCH_CHECK(dy.size(2) == dmp::maxpool_out((int)H, (int)K, (int)S, (int)P) &&
                  dy.size(3) == dmp::maxpool_out((int)W, (int)K, (int)S, (int)P),
              "maxpool_bwd: shape mismatch");
  // gather-form kernel writes every input element (un-pooled borders get 0)
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(mf));
  dmp::launch_maxpool_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                          reinterpret_cast<uint16_t*>(dx.data_ptr()), N, (int)H, (int)W, C, (int)K,
                          (int)S, (int)P, cur_stream(), nchw);
  return dx;
}

// ----------------------------------------------------------- im2col / relu
// x: bf16 channels_last [B, CI, H, W] -> [B*OH*OW, Kp] patch rows, k = (r, s, ci)
Tensor im2col(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Kp) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "im2col: 4-D input");
  const int B = (int)x.size(0), CI = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(R >= 1 && S >= 1 && stride >= 1 && pad >= 0, "im2col: bad geometry");
  const int OH = (int)((H + 2 * pad - R) / stride + 1), OW = (int)((W + 2 * pad - S) / stride + 1);
  TORCH_CHECK(OH > 0 && OW > 0, "im2col: window larger than the padded input");
  const int64_t K = R * S * CI;
  TORCH_CHECK(Kp >= K && Kp % 8 == 0, "im2col: Kp must be >= R*S*CI and a multiple of 8");
  TORCH_CHECK(2LL * B * OH * OW * Kp < (1LL << 40), "im2col: patch matrix too large");
  Tensor cols = at::empty({(int64_t)B * OH * OW, Kp}, x.options());
  dmp::launch_im2col(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                     reinterpret_cast<uint16_t*>(cols.data_ptr()), B, H, W, CI, OH, OW, (int)R,
                     (int)S, (int)stride, (int)pad, (int)K, (int)Kp, cur_stream());
  return cols;
}

// dcols [B*OH*OW, Kp] -> dX bf16 channels_last [B, CI, H, W]
Tensor col2im(Tensor dcols, int64_t B, int64_t CI, int64_t H, int64_t W, int64_t R, int64_t S,
              int64_t stride, int64_t pad) {
  check_gpu(dcols, "dcols");
  TORCH_CHECK(dcols.scalar_type() == at::kBFloat16 && dcols.dim() == 2 && dcols.is_contiguous(),
              "col2im: dcols must be a contiguous bf16 [M, Kp] tensor");
  const int OH = (int)((H + 2 * pad - R) / stride + 1), OW = (int)((W + 2 * pad - S) / stride + 1);
  TORCH_CHECK(dcols.size(0) == B * OH * OW && dcols.size(1) >= R * S * CI,
              "col2im: dcols shape does not match the conv geometry");
  Tensor dx = at::empty({B, CI, H, W}, dcols.options().memory_format(at::MemoryFormat::ChannelsLast));
  dmp::launch_col2im(reinterpret_cast<const uint16_t*>(dcols.data_ptr()),
                     reinterpret_cast<uint16_t*>(dx.data_ptr()), (int)B, (int)H, (int)W, (int)CI,
                     OH, OW, (int)R, (int)S, (int)stride, (int)pad, (int)dcols.size(1),
                     cur_stream());
  return dx;
}

// dx = y > 0 ? dy : 0 over dense bf16 tensors of one layout (out may alias dy)
Tensor relu_bwd(Tensor dy, Tensor y, optional<Tensor> out) {
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16, "relu_bwd: bf16 GPU tensors");
  const auto mf = y.dim() == 4 && y.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                          !y.is_contiguous()
                      ? at::MemoryFormat::ChannelsLast
                      : at::MemoryFormat::Contiguous;
  // the kernel reads / writes 16-B vectors over one dense layout: a strided y is
  // made dense in the layout dy is brought to, and an operand that is dense but
  // not 16-B aligned (an offset slice such as x[..., 1:]) goes through an aligned
  // copy (fresh allocations are 256-B aligned)
  auto aligned = [](const Tensor& t) {
    return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15u) == 0;
  };
  y = y.contiguous(mf);
  dy = dy.contiguous(mf);
  if (!aligned(y)) y = y.clone(mf);
  if (!aligned(dy)) dy = dy.clone(mf);
  TORCH_CHECK(dy.sizes() == y.sizes() && dy.scalar_type() == at::kBFloat16, "relu_bwd: dy shape");
  Tensor dst = out.has_value() && out->defined() ? *out : at::empty_like(dy);
  TORCH_CHECK(dst.sizes() == y.sizes() && dst.is_contiguous(mf) &&
                  dst.scalar_type() == at::kBFloat16,
              "relu_bwd: out layout");
  Tensor dx = aligned(dst) ? dst : at::empty_like(dy);
  dmp::launch_relu_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                       reinterpret_cast<const uint16_t*>(y.data_ptr()),
                       reinterpret_cast<uint16_t*>(dx.data_ptr()), y.numel(), cur_stream());
  if (!dx.is_same(dst)) dst.copy_(dx);
  return dst;
}

// ---------------------------------------------------------------- convolution
// x: bf16 channels_last [B, CI, H, W]; w: bf16 channels_last [CO, CI, R, S].
struct ConvGeom {
  int B, CI, H, W, CO, R, S, OH, OW;
};

ConvGeom conv_geom(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad) {
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv: 4-D tensors expected");
  TORCH_CHECK(w.size(1) == x.size(1), "conv: weight/input channel mismatch");
  TORCH_CHECK(stride >= 1 && pad >= 0, "conv: bad stride/pad");
  const int64_t OH = dmp::guard::conv_out(x.size(2), pad, w.size(2), stride);
  const int64_t OW = dmp::guard::conv_out(x.size(3), pad, w.size(3), stride);
  TORCH_CHECK(OH > 0 && OW > 0, "conv: empty output");
  // the kernels address operands with 32-bit byte offsets into buffer descriptors
  // (checked on the 64-bit sizes, before anything is narrowed to int)
  TORCH_CHECK(dmp::guard::conv_offsets_ok(x.size(0), x.size(2), x.size(3), x.size(1), OH, OW,
                                          w.size(0), w.size(2), w.size(3)),
              "native conv: tensor too large for 32-bit byte offsets");
  ConvGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)w.size(0),
             (int)w.size(2), (int)w.size(3), (int)OH, (int)OW};
  TORCH_CHECK(g.CI % 64 == 0 && g.CO % 64 == 0,
              "native conv needs CI % 64 == 0 and CO % 64 == 0 (got ", g.CI, ", ", g.CO, ")");
  return g;
}

std::vector<Tensor> conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, bool want_stats,
                             int64_t cfg, optional<Tensor> slots, optional<Tensor> bias,
                             bool relu, optional<Tensor> addend) {
  check_nhwc_bf16(x, "x");
  check_gpu(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv weight must be bf16 channels_last");
  auto g = conv_geom(x, w, stride, pad);
  auto y = at::empty({g.B, g.CO, g.OH, g.OW},
                     x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() == g.CO,
                "conv bias must be a contiguous fp32 [CO] GPU tensor");
  } else {
    bias.reset();
  }
  Tensor part;
  int64_t G = 0;
  if (want_stats) {
    G = dmp::kBnSlots;
    part = bn_slots(slots, g.CO, x.options());
  }
  const uint16_t* add_ptr = nullptr;
  Tensor add_t;
  if (addend.has_value() && addend->defined()) {
    // residual added before the ReLU (inference-time BatchNorm fold, ops/eval_fold.py)
    add_t = addend->contiguous(at::MemoryFormat::ChannelsLast);
    check_nhwc_bf16(add_t, "addend");
    TORCH_CHECK(add_t.sizes() == y.sizes(), "conv_fwd: addend must have the output's shape");
    add_ptr = reinterpret_cast<const uint16_t*>(add_t.data_ptr());
  }
  dmp::launch_conv_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       reinterpret_cast<const uint16_t*>(w.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()),
                       want_stats ? part.data_ptr<float>() : nullptr, g.B, g.H, g.W, g.CI, g.OH,
                       g.OW, g.CO, g.R, g.S, (int)stride, (int)pad, (int)cfg, cur_stream(),
                       bias ? bias->data_ptr<float>() : nullptr, relu, add_ptr);
  return {y, part, at::scalar_tensor(G, at::kLong)};
}

// Inference-time BatchNorm fold into the producing conv / GEMM (csrc/bn.hip):
// returns (w16 = bf16(w * s) with w's shape and memory format, t fp32 [CO],
// t bf16 [CO]), s = gamma / sqrt(running_var + eps), t = beta + (cbias - mean) * s.
std::vector<Tensor> bn_fold_weights(Tensor w, optional<Tensor> gamma, optional<Tensor> beta,
                                    Tensor rmean, Tensor rvar, optional<Tensor> cbias,
                                    double eps) {
  check_gpu(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kFloat, "bn_fold_weights: fp32 master weight");
  const bool cl = w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(cl || w.is_contiguous(), "bn_fold_weights: contiguous or channels_last weight");
  const int64_t CO = w.size(0);
  const int64_t n = w.numel();
  TORCH_CHECK(n % CO == 0, "bn_fold_weights: weight [CO, ...] expected");
  for (auto* t : {&gamma, &beta, &cbias}) {
    if (t->has_value() && (*t)->defined()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat &&
                      (*t)->is_contiguous() && (*t)->numel() == CO,
                  "bn_fold_weights: affine / bias tensors must be contiguous fp32 [CO]");
    } else {
      t->reset();
    }
  }
  for (auto* t : {&rmean, &rvar})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == CO,
                "bn_fold_weights: running stats must be contiguous fp32 [CO]");
  auto w16 = at::empty_like(w, w.options().dtype(at::kBFloat16));
  auto b32 = at::empty({CO}, w.options());
  auto b16 = at::empty({CO}, w.options().dtype(at::kBFloat16));
  dmp::launch_bn_fold_weights(w.data_ptr<float>(), ptr_or_null<float>(gamma),
                              ptr_or_null<float>(beta), rmean.data_ptr<float>(),
                              rvar.data_ptr<float>(), ptr_or_null<float>(cbias),
                              reinterpret_cast<uint16_t*>(w16.data_ptr()), b32.data_ptr<float>(),
                              reinterpret_cast<uint16_t*>(b16.data_ptr()), n, (int)CO, (float)eps,
                              cur_stream());
  return {w16, b32, b16};
}

void conv_weight_transpose_batched(Tensor src, Tensor dst, Tensor table, int64_t max_elems) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kBFloat16 &&
                  src.numel() == dst.numel(),
              "batched transpose: src/dst must be equal-size bf16 buffers");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.dim() == 2 &&
                  table.size(1) == 4 && table.is_contiguous(),
              "batched transpose: table must be a [n, 4] int64 GPU tensor");
  dmp::launch_conv_weight_transpose_batched(reinterpret_cast<const uint16_t*>(src.data_ptr()),
                                            reinterpret_cast<uint16_t*>(dst.data_ptr()),
                                            reinterpret_cast<const long long*>(table.data_ptr()),
                                            (int)table.size(0), (long long)max_elems,
                                            cur_stream());
}

void pad_rows_batched(Tensor src, Tensor dst, Tensor table, int64_t max_elems) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kBFloat16,
              "pad_rows_batched: bf16 buffers");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.dim() == 2 &&
                  table.size(1) == 5 && table.is_contiguous(),
              "pad_rows_batched: table must be a [n, 5] int64 GPU tensor");
  dmp::launch_pad_rows_batched(reinterpret_cast<const uint16_t*>(src.data_ptr()),
                               reinterpret_cast<uint16_t*>(dst.data_ptr()),
                               reinterpret_cast<const long long*>(table.data_ptr()),
                               (int)table.size(0), (long long)max_elems, cur_stream());
}

// Native zero fill of a dense tensor (the grad arena at every step start: no
// ATen fill kernel).  Deliberately a kernel and not hipMemsetAsync: a captured
// memset node raced with the previous graph replay (csrc/optim.hip zero_fill).
void zero_(Tensor t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_: a contiguous GPU tensor");
  const long long bytes = (long long)t.numel() * t.element_size();
  TORCH_CHECK(bytes % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "zero_: a 16-B aligned tensor of whole dwords");
  dmp::launch_zero_fill(t.data_ptr(), bytes, cur_stream());
}

Tensor conv_dgrad(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t stride, int64_t pad,
                  int64_t cfg, optional<Tensor> wt_pre, optional<Tensor> addend,
                  optional<Tensor> bn_x, optional<Tensor> bn_mask, optional<Tensor> bn_stats,
                  optional<Tensor> bn_part, int64_t bn_relu, bool addend_sub,
                  optional<Tensor> addend_mask) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  check_gpu(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv weight must be bf16 channels_last");
  const int B = (int)dy.size(0);
  auto xshape = at::empty({0}, dy.options());
  ConvGeom g{B, (int)w.size(1), (int)H, (int)W, (int)w.size(0), (int)w.size(2), (int)w.size(3),
             (int)dy.size(2), (int)dy.size(3)};
  TORCH_CHECK(dy.size(1) == g.CO, "dgrad: dy channels mismatch");
  TORCH_CHECK((g.H + 2 * pad - g.R) / stride + 1 == g.OH && (g.W + 2 * pad - g.S) / stride + 1 == g.OW,
              "dgrad: geometry mismatch");
  TORCH_CHECK(g.CI % 64 == 0 && g.CO % 64 == 0, "native dgrad needs CI, CO % 64 == 0");
  Tensor wt;
  if (wt_pre.has_value() && wt_pre->defined()) {
    wt = *wt_pre;   // pre-transposed [CI][R][S][CO] (batched per step by the arena)
    check_gpu(wt, "wt");
    TORCH_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() &&
                    wt.numel() == (int64_t)g.CI * g.R * g.S * g.CO,
                "dgrad: pre-transposed weight must be contiguous bf16 [CI, R, S, CO]");
  } else {
    wt = at::empty({g.CI, g.R, g.S, g.CO}, w.options().memory_format(at::MemoryFormat::Contiguous));
    dmp::launch_conv_weight_transpose(reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                      reinterpret_cast<uint16_t*>(wt.data_ptr()), g.CO, g.R * g.S,
                                      g.CI, cur_stream());
  }
  auto dx = at::empty({B, g.CI, g.H, g.W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const uint16_t* add_ptr = nullptr;
  Tensor add_t;
  if (addend.has_value() && addend->defined()) {
    add_t = addend->contiguous(at::MemoryFormat::ChannelsLast);
    check_nhwc_bf16(add_t, "addend");
    if (addend_sub) {
      // gradient of x[:, :, ::2, ::2] (a 1x1 / stride-2 shortcut's input): added on
      // the stride-2 data gradient's parity class (0, 0)
      TORCH_CHECK(stride == 2, "dgrad: a subsampled addend needs stride 2");
      TORCH_CHECK(add_t.size(0) == B && add_t.size(1) == g.CI && add_t.size(2) == (g.H + 1) / 2 &&
                      add_t.size(3) == (g.W + 1) / 2,
                  "dgrad: subsampled addend must be [B, CI, ceil(H/2), ceil(W/2)]");
    } else {
      TORCH_CHECK(add_t.sizes() == dx.sizes(), "dgrad: addend must have the input's shape");
    }
    add_ptr = reinterpret_cast<const uint16_t*>(add_t.data_ptr());
  }
  // deferred ReLU mask of the addend (the residual BN backward's dres not written)
  const uint8_t* amask = nullptr;
  if (addend_mask.has_value() && addend_mask->defined()) {
    TORCH_CHECK(add_ptr != nullptr, "dgrad: addend_mask without an addend");
    TORCH_CHECK(addend_mask->is_cuda() && addend_mask->scalar_type() == at::kByte &&
                    addend_mask->is_contiguous() && addend_mask->numel() == add_t.numel() / 8,
                "dgrad: addend_mask must be the addend's contiguous uint8 [pixels, C/8] bit mask");
    amask = addend_mask->data_ptr<uint8_t>();
  }
  // fused backward of the BatchNorm(+ReLU) that produced the conv input (bn_relu >= 0)
  dmp::BnBwdFuse bnf{};
  const bool fuse = bn_relu >= 0;
  if (fuse) {
    TORCH_CHECK(bn_relu <= 3 && bn_x.has_value() && bn_stats.has_value() && bn_part.has_value(),
                "dgrad: BN fusion needs bn_x, bn_stats and bn_part");
    check_nhwc_bf16(*bn_x, "bn_x");
    TORCH_CHECK(bn_x->sizes() == dx.sizes(), "dgrad: bn_x must have the input's shape");
    TORCH_CHECK(bn_stats->is_cuda() && bn_stats->scalar_type() == at::kFloat &&
                    bn_stats->is_contiguous() && bn_stats->numel() == 4LL * g.CI,
                "dgrad: bn_stats must be contiguous fp32 [4, C]");
    bn_slots(bn_part, g.CI, dy.options().dtype(at::kFloat));
    if (bn_relu == 1) {
      TORCH_CHECK(bn_mask.has_value(), "dgrad: bn_relu 1 needs bn_mask");
      check_nhwc_bf16(*bn_mask, "bn_mask");
      TORCH_CHECK(bn_mask->sizes() == dx.sizes(), "dgrad: bn_mask must have the input's shape");
      bnf.mask = reinterpret_cast<const uint16_t*>(bn_mask->data_ptr());
    } else if (bn_relu == 3) {
      TORCH_CHECK(bn_mask.has_value() && bn_mask->is_cuda() &&
                      bn_mask->scalar_type() == at::kByte && bn_mask->is_contiguous() &&
                      bn_mask->numel() == dx.numel() / 8,
                  "dgrad: bn_relu 3 needs the uint8 [pixels, C/8] ReLU bit mask");
      bnf.mask = reinterpret_cast<const uint16_t*>(bn_mask->data_ptr());
    }
    bnf.x = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    bnf.stats = bn_stats->data_ptr<float>();
    bnf.part = bn_part->data_ptr<float>();
    bnf.relu = (int)bn_relu;
  }
  dmp::launch_conv_dgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                         reinterpret_cast<const uint16_t*>(wt.data_ptr()),
                         reinterpret_cast<uint16_t*>(dx.data_ptr()), B, g.H, g.W, g.CI, g.OH,
                         g.OW, g.CO, g.R, g.S, (int)stride, (int)pad, (int)cfg, cur_stream(),
                         add_ptr, fuse ? &bnf : nullptr, add_ptr != nullptr && addend_sub,
                         amask);
  return dx;
}

// dx[:, :, ::2, ::2] += xs in place (both channels_last bf16)
void add_subsampled2(Tensor dx, Tensor xs) {
  check_nhwc_bf16(dx, "dx");
  check_nhwc_bf16(xs, "xs");
  TORCH_CHECK(dx.dim() == 4 && dx.size(1) % 8 == 0 && xs.size(0) == dx.size(0) &&
                  xs.size(1) == dx.size(1) && xs.size(2) == (dx.size(2) + 1) / 2 &&
                  xs.size(3) == (dx.size(3) + 1) / 2,
              "add_subsampled2: xs must be [B, C, ceil(H/2), ceil(W/2)] of dx [B, C, H, W]");
  dmp::launch_add_subsampled2(reinterpret_cast<uint16_t*>(dx.data_ptr()),
                              reinterpret_cast<const uint16_t*>(xs.data_ptr()), (int)dx.size(0),
                              (int)dx.size(2), (int)dx.size(3), (int)dx.size(1), cur_stream());
}

// x[:, :, ::2, ::2] of a channels_last bf16 activation, gathered (channels_last out)
Tensor subsample2(Tensor x) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) % 8 == 0, "subsample2: [B, C, H, W] with C % 8 == 0");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto xs = at::empty({B, C, (H + 1) / 2, (W + 1) / 2},
                      x.options().memory_format(at::MemoryFormat::ChannelsLast));
  dmp::launch_subsample2(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                         reinterpret_cast<uint16_t*>(xs.data_ptr()), (int)B, (int)H, (int)W,
                         (int)C, cur_stream());
  return xs;
}

void conv_wgrad(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad, int64_t cfg,
                optional<Tensor> dbias) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  check_nhwc_bf16(x, "x");
  check_gpu(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 4 &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast),
              "dw must be an fp32 channels_last [CO, CI, R, S] tensor");
  auto g = conv_geom(x, dw, stride, pad);
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.CO && dy.size(2) == g.OH && dy.size(3) == g.OW,
              "wgrad: dy shape mismatch");
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == at::kFloat &&
                    dbias->is_contiguous() && dbias->numel() == g.CO,
                "wgrad: dbias must be a contiguous fp32 [CO] GPU tensor");
    db = dbias->data_ptr<float>();
  }
  Tensor ws;   // slab-mode halo cfg: per-split partials, reduced into dw after the kernel
  if (db == nullptr) {
    const long long se = dmp::conv_wgrad_halo_slab_elems((int)cfg, g.B, g.H, g.W, g.CI, g.CO, g.R,
                                                         g.S, (int)stride, (int)pad);
    if (se > 0) ws = at::empty({(int64_t)se}, dw.options().memory_format(at::MemoryFormat::Contiguous));
  }
  dmp::launch_conv_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                         reinterpret_cast<const uint16_t*>(x.data_ptr()), dw.data_ptr<float>(),
                         g.B, g.H, g.W, g.CI, g.OH, g.OW, g.CO, g.R, g.S, (int)stride, (int)pad,
                         (int)cfg, cur_stream(), db, ws.defined() ? ws.data_ptr<float>() : nullptr);
}

// few-input-channel (stem) convolutions: x any dense bf16 4-D layout,
// w bf16 channels_last [CO, CI, R, S] with CO % 64 == 0 and R*S*CI <= 384
struct SmallGeom {
  int B, CI, H, W, CO, R, S, OH, OW;
};

SmallGeom small_geom(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad) {
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "small conv: 4-D tensors expected");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16, "small conv: x must be bf16 GPU");
  TORCH_CHECK(w.size(1) == x.size(1), "small conv: weight/input channel mismatch");
  TORCH_CHECK(stride >= 1 && pad >= 0 && w.size(2) <= 255 && w.size(3) <= 255,
              "small conv: bad geometry");
  TORCH_CHECK(w.size(0) % 64 == 0, "small conv: CO must be a multiple of 64");
  TORCH_CHECK(w.size(1) * w.size(2) * w.size(3) <= dmp::conv_small_max_k(),
              "small conv: R*S*CI too large");
  const int64_t OH = dmp::guard::conv_out(x.size(2), pad, w.size(2), stride);
  const int64_t OW = dmp::guard::conv_out(x.size(3), pad, w.size(3), stride);
  TORCH_CHECK(OH > 0 && OW > 0, "small conv: empty output");
  TORCH_CHECK(dmp::guard::small_conv_ok(x.size(0), OH, OW, w.size(0), x.numel()),
              "small conv: tensor too large for 32-bit indexing");
  SmallGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)w.size(0),
              (int)w.size(2), (int)w.size(3), (int)OH, (int)OW};
  return g;
}

// ImageNet stem (csrc/stem.hip): x [B, 3, H, W] channels_last bf16, w [64, 3, 7, 7]
// channels_last bf16 -> (y [B, 64, H/2, W/2] channels_last, BN slots, xs for the wgrad)
std::vector<Tensor> stem_fwd(Tensor x, Tensor w, bool want_stats, optional<Tensor> slots,
                             optional<Tensor> bias, bool relu) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: x must be a channels_last bf16 [B, 3, H, W] tensor");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == 64 &&
                  w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: w must be a channels_last bf16 [64, 3, 7, 7] tensor");
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(dmp::stem_supported((int)H, (int)W), "stem: unsupported input size ", H, "x", W);
  TORCH_CHECK(dmp::guard::stem_batch_ok(B, H, W), "stem: batch too large");
  auto xs = at::empty({B, H / 2, W / 2, 16}, x.options());
  auto wp = at::empty({64, 256}, w.options());
  auto y = at::empty({B, 64, H / 2, W / 2}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part;
  if (want_stats) part = bn_slots(slots, 64, x.options());
  if (bias) {
    check_gpu(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == 64 && bias->is_contiguous(),
                "stem: bias must be a contiguous fp32 [64] tensor");
  }
  auto st = cur_stream();
  dmp::launch_stem_s2d(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       reinterpret_cast<uint16_t*>(xs.data_ptr()), (int)B, (int)H, (int)W, st);
  dmp::launch_stem_wpack(reinterpret_cast<const uint16_t*>(w.data_ptr()),
                         reinterpret_cast<uint16_t*>(wp.data_ptr()), st);
  dmp::launch_stem_fwd(reinterpret_cast<const uint16_t*>(xs.data_ptr()),
                       reinterpret_cast<const uint16_t*>(wp.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()),
                       want_stats ? part.data_ptr<float>() : nullptr, (int)B, (int)H, (int)W, st,
                       bias ? bias->data_ptr<float>() : nullptr, relu);
  return {y, part, xs};
}

// dw (fp32 [64, 3, 7, 7] channels_last) += stem weight gradient from dY and the s2d input
void stem_wgrad(Tensor dy, Tensor xs, Tensor dw) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  check_gpu(xs, "xs");
  check_gpu(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 4 && dw.size(0) == 64 &&
                  dw.size(1) == 3 && dw.size(2) == 7 && dw.size(3) == 7 &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: dw must be an fp32 channels_last [64, 3, 7, 7] tensor");
  TORCH_CHECK(xs.scalar_type() == at::kBFloat16 && xs.dim() == 4 && xs.size(3) == 16 &&
                  xs.is_contiguous(), "stem: bad s2d input");
  const int64_t B = xs.size(0), H = 2 * xs.size(1), W = 2 * xs.size(2);
  TORCH_CHECK(dy.size(0) == B && dy.size(1) == 64 && dy.size(2) == H / 2 && dy.size(3) == W / 2,
              "stem: dy shape mismatch");
  TORCH_CHECK(dmp::stem_supported((int)H, (int)W), "stem: unsupported input size");
  auto dwp = at::empty({64, 256}, dw.options().memory_format(at::MemoryFormat::Contiguous));
  auto st = cur_stream();
  dmp::launch_stem_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                         reinterpret_cast<const uint16_t*>(xs.data_ptr()), dwp.data_ptr<float>(),
                         (int)B, (int)H, (int)W, st);
  dmp::launch_stem_wfold(dwp.data_ptr<float>(), dw.data_ptr<float>(), st);
}

// 3x3/s1/p1, CI <= 3, CO = 64 stems on MFMA (conv_small.hip stem3_*); DMP_STEM3=0
// keeps the VALU kernels (A/B)
bool stem3_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DMP_STEM3");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

std::vector<Tensor> conv_small_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad,
                                   bool want_stats, optional<Tensor> slots) {
  check_gpu(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv weight must be bf16 channels_last");
  auto g = small_geom(x, w, stride, pad);
  auto y = at::empty({g.B, g.CO, g.OH, g.OW},
                     x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const long long P = (long long)g.B * g.OH * g.OW;
  Tensor part;
  int64_t G = 0;
  if (want_stats) {
    G = dmp::kBnSlots;
    part = bn_slots(slots, g.CO, x.options());
  }
  if (stem3_enabled() && dmp::stem3_supported(g.CI, g.R, g.S, g.CO, (int)stride, (int)pad, g.W)) {
    dmp::launch_stem3_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), (int)(2 * x.numel()),
                          (int)x.stride(0), (int)x.stride(2), (int)x.stride(3), (int)x.stride(1),
                          reinterpret_cast<const uint16_t*>(w.data_ptr()),
                          reinterpret_cast<uint16_t*>(y.data_ptr()),
                          want_stats ? part.data_ptr<float>() : nullptr, g.B, g.H, g.W, g.CI,
                          cur_stream());
    return {y, part, at::scalar_tensor(G, at::kLong)};
  }
  dmp::launch_conv_small_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                             (int)(2 * x.numel()), (int)x.stride(0),
                             (int)x.stride(2), (int)x.stride(3), (int)x.stride(1),
                             reinterpret_cast<const uint16_t*>(w.data_ptr()),
                             reinterpret_cast<uint16_t*>(y.data_ptr()),
                             want_stats ? part.data_ptr<float>() : nullptr, g.B, g.H, g.W, g.CI,
                             g.OH, g.OW, g.CO, g.R, g.S, (int)stride, (int)pad, cur_stream());
  return {y, part, at::scalar_tensor(G, at::kLong)};
}

void conv_small_wgrad(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  check_gpu(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 4 &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast),
              "dw must be an fp32 channels_last [CO, CI, R, S] tensor");
  auto g = small_geom(x, dw, stride, pad);
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.CO && dy.size(2) == g.OH && dy.size(3) == g.OW,
              "small wgrad: dy shape mismatch");
  const long long P = (long long)g.B * g.OH * g.OW;
  if (stem3_enabled() && dmp::stem3_supported(g.CI, g.R, g.S, g.CO, (int)stride, (int)pad, g.W)) {
    dmp::launch_stem3_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                            reinterpret_cast<const uint16_t*>(x.data_ptr()), (int)(2 * x.numel()),
                            (int)x.stride(0), (int)x.stride(2), (int)x.stride(3),
                            (int)x.stride(1), dw.data_ptr<float>(), g.B, g.H, g.W, g.CI,
                            cur_stream());
    return;
  }
  const int G = dmp::conv_small_wgrad_blocks(P, g.CO, g.R, g.S, g.CI);
  auto ws = at::empty({(int64_t)G * g.CO * g.R * g.S * g.CI}, dw.options());
  dmp::launch_conv_small_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                               reinterpret_cast<const uint16_t*>(x.data_ptr()),
                               (int)(2 * x.numel()), (int)x.stride(0),
                               (int)x.stride(2), (int)x.stride(3), (int)x.stride(1),
                               dw.data_ptr<float>(), ws.data_ptr<float>(), g.B,
                               g.H, g.W, g.CI, g.OH, g.OW, g.CO, g.R, g.S, (int)stride, (int)pad,
                               cur_stream());
}

// ------------------------------------------------------- fused attention
// qkv: [B, N, 3*H*64] bf16 rows of the qkv projection ([B, N, 3, H, 64])
void check_attn(const Tensor& qkv, int64_t heads, int64_t& B, int64_t& N, int64_t& D) {
  check_gpu(qkv, "qkv");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.is_contiguous() && qkv.dim() == 3,
              "attention: qkv must be a contiguous bf16 [B, N, 3*D] tensor");
  B = qkv.size(0);
  N = qkv.size(1);
  TORCH_CHECK(qkv.size(2) % 3 == 0, "attention: last dim must be 3*D");
  D = qkv.size(2) / 3;
  TORCH_CHECK(heads > 0 && D % heads == 0 && D / heads == dmp::attention_head_dim(),
              "attention: head dim must be ", dmp::attention_head_dim());
  TORCH_CHECK(N >= 1 && N <= dmp::attention_max_tokens(), "attention: 1 <= N <= ",
              dmp::attention_max_tokens());
}

std::vector<Tensor> attention_fwd(Tensor qkv, int64_t heads) {
  int64_t B, N, D;
  check_attn(qkv, heads, B, N, D);
  auto out = at::empty({B, N, D}, qkv.options());
  auto lse = at::empty({B, heads, N}, qkv.options().dtype(at::kFloat));
  dmp::launch_attention_fwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()),
                            reinterpret_cast<uint16_t*>(out.data_ptr()), lse.data_ptr<float>(),
                            (int)B, (int)N, (int)heads,
                            1.f / std::sqrt((float)dmp::attention_head_dim()), cur_stream());
  return {out, lse};
}

Tensor attention_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, int64_t heads) {
  int64_t B, N, D;
  check_attn(qkv, heads, B, N, D);
  dout = dout.contiguous();
  for (const Tensor* t : {&out, &dout}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->numel() == B * N * D,
                "attention_bwd: out / dout must be contiguous bf16 [B, N, D]");
  }
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.numel() == B * heads * N,
              "attention_bwd: bad lse");
  auto dqkv = at::empty_like(qkv);
  dmp::launch_attention_bwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()),
                            reinterpret_cast<const uint16_t*>(out.data_ptr()),
                            reinterpret_cast<const uint16_t*>(dout.data_ptr()),
                            lse.data_ptr<float>(), reinterpret_cast<uint16_t*>(dqkv.data_ptr()),
                            (int)B, (int)N, (int)heads,
                            1.f / std::sqrt((float)dmp::attention_head_dim()), cur_stream());
  return dqkv;
}

// ----------------------------------------------------------- bias gradients
// out[n] += sum over rows of dy[..., n]; dy: bf16 with the channel dim
// innermost in memory (contiguous [.., N] or channels_last NCHW)
void colsum_acc(Tensor dy, Tensor out, optional<Tensor> slots) {
  check_gpu(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16, "colsum_acc: dy must be bf16");
  int64_t N;
  if (dy.dim() == 4) {
    N = dy.size(1);
    if (!dy.is_contiguous(at::MemoryFormat::ChannelsLast))
      dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  } else {
    N = dy.size(-1);
    dy = dy.contiguous();
  }
  TORCH_CHECK(N % 8 == 0, "colsum_acc: the summed-into dim must be a multiple of 8, got ", N);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() &&
                  out.numel() == N,
              "colsum_acc: out must be a contiguous fp32 [N] GPU tensor");
  const int64_t M = dy.numel() / N;
  if (M == 0) return;
  // per-device persistent zeroed scratch (every call re-zeroes it; calls on one
  // stream are ordered, and a graph replays them in the same order)
  const int64_t need = (int64_t)dmp::colsum_num_slots() * N;
  Tensor sl;
  if (slots.has_value() && slots->defined()) {
    TORCH_CHECK(slots->is_cuda() && slots->scalar_type() == at::kFloat &&
                    slots->is_contiguous() && slots->numel() >= need,
                "colsum_acc: slots must be a zeroed contiguous fp32 GPU tensor of >= ", need);
    sl = *slots;
  } else {
    sl = at::zeros({need}, out.options());
  }
  dmp::launch_colsum_acc(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                         out.data_ptr<float>(), sl.data_ptr<float>(), M, (int)N, cur_stream());
}

// ------------------------------------------------------------------- GEMM
// 2-D operand with a unit inner stride: checked and its row stride returned
int64_t mat_ld(const Tensor& t, at::ScalarType dt, int64_t rows, int64_t cols,
               const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == 2, name, " must be a 2-D ", dt,
              " GPU tensor");
  TORCH_CHECK(t.size(0) == rows && t.size(1) == cols, name, " is ", t.sizes(), ", expected [",
              rows, ", ", cols, "]");
  TORCH_CHECK(t.stride(1) == 1, name, " must have a unit inner stride");
  const int64_t ld = rows <= 1 ? cols : t.stride(0);
  TORCH_CHECK(ld >= cols, name, ": row stride smaller than the row");
  TORCH_CHECK(dmp::guard::rows_bytes_ok(t.element_size(), rows, ld), name,
              " exceeds the 2 GiB 32-bit offset range of the GEMM kernels");
  return ld;
}

// C = epilogue(sum_k A(m, k) B(n, k)); see csrc/gemm.hip.  mode 0: a [M,K], b [N,K];
// mode 1: a [M,K], b [K,N]; mode 2: a [K,M], b [K,N], c fp32 accumulated.
void gemm(int64_t mode, int64_t epi, int64_t cfg, Tensor a, Tensor b, Tensor c,
          optional<Tensor> c2, optional<Tensor> bias, optional<Tensor> aux,
          optional<Tensor> dbias, int64_t splits, bool relu, optional<Tensor> part, bool slab,
          optional<Tensor> auxmask) {
  TORCH_CHECK(!relu || epi == 0, "gemm: relu only with the store epilogue");
  TORCH_CHECK(mode >= 0 && mode <= 2, "gemm: mode must be 0 (fwd), 1 (dgrad) or 2 (wgrad)");
  TORCH_CHECK(c.dim() == 2 && a.dim() == 2 && b.dim() == 2, "gemm: 2-D operands expected");
  TORCH_CHECK((mode == 0 && (epi == 0 || epi == 1)) ||
                  (mode == 1 && (epi == 0 || epi == 2 || epi == 4)) || (mode == 2 && epi == 3),
              "gemm: epilogue ", epi, " not available in mode ", mode);
  TORCH_CHECK(dmp::gemm_config_ok((int)mode, (int)cfg), "gemm: config ", cfg,
              " is not available in mode ", mode);
  const int64_t M = c.size(0), N = c.size(1);
  const int64_t K = mode == 2 ? a.size(0) : a.size(1);
  const int64_t lda = mat_ld(a, at::kBFloat16, mode == 2 ? K : M, mode == 2 ? M : K, "a");
  const int64_t ldb = mat_ld(b, at::kBFloat16, mode == 0 ? N : K, mode == 0 ? K : N, "b");
  const int64_t ldc = mat_ld(c, mode == 2 ? at::kFloat : at::kBFloat16, M, N, "c");
  if (M == 0 || N == 0) return;
  auto same_as_c = [&](const Tensor& t, const char* name) {
    TORCH_CHECK(mat_ld(t, at::kBFloat16, M, N, name) == ldc, name,
                " must have the output's row stride");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
                " must be 16-byte aligned");
  };
  uint16_t* c2p = nullptr;
  if (epi == 1) {
    TORCH_CHECK(c2.has_value() && c2->defined(), "gemm: GELU epilogue needs c2");
    same_as_c(*c2, "c2");
    c2p = reinterpret_cast<uint16_t*>(c2->data_ptr());
  }
  const uint16_t* auxp = nullptr;
  if (aux.has_value() && aux->defined()) {
    TORCH_CHECK(epi == 0 || epi == 2 || epi == 4, "gemm: aux only with epilogues 0 / 2 / 4");
    same_as_c(*aux, "aux");
    auxp = reinterpret_cast<const uint16_t*>(aux->data_ptr());
  }
  // deferred ReLU bit mask of the addend (ops/functional.py deferred residual mask)
  const uint8_t* amp = nullptr;
  if (auxmask.has_value() && auxmask->defined()) {
    TORCH_CHECK(auxp != nullptr && epi == 0 && cfg >= 0,
                "gemm: auxmask needs an addend, the store epilogue and an MFMA tile config");
    TORCH_CHECK(ldc == N && N % 8 == 0, "gemm: auxmask needs a dense output with N % 8 == 0");
    TORCH_CHECK(auxmask->is_cuda() && auxmask->scalar_type() == at::kByte &&
                    auxmask->is_contiguous() && auxmask->numel() == M * N / 8,
                "gemm: auxmask must be a contiguous uint8 [M * N / 8] GPU tensor");
    amp = auxmask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(epi != 2 || auxp != nullptr, "gemm: GELU-backward epilogue needs aux = h");
  TORCH_CHECK(epi != 4 || auxp != nullptr, "gemm: ReLU-backward epilogue needs aux = the input");
  const uint16_t* biasp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(epi == 0 || epi == 1, "gemm: bias only in the forward epilogues");
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 &&
                    bias->is_contiguous() && bias->numel() == N &&
                    reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
                "gemm: bias must be a contiguous 8-byte aligned bf16 [N] GPU tensor");
    biasp = reinterpret_cast<const uint16_t*>(bias->data_ptr());
  }
  float* dbp = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(mode == 2, "gemm: dbias only in wgrad mode");
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == at::kFloat &&
                    dbias->is_contiguous() && dbias->numel() == M,
                "gemm: dbias must be a contiguous fp32 [M] GPU tensor");
    dbp = dbias->data_ptr<float>();
  }
  float* partp = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(epi == 0 && cfg >= 0, "gemm: BN partial sums need the MFMA store epilogue");
    TORCH_CHECK(N % 8 == 0 && ldc % 8 == 0, "gemm: BN partial sums need N % 8 == 0");
    partp = bn_slots(part, N, c.options()).data_ptr<float>();
  }
  if (cfg >= 0) {
    // MFMA tiles: 16-B DMA pieces along k (row-major operand) or along the
    // row (k-strided operand), 8-B bf16x4 output stores
    for (const Tensor* t : {&a, &b})
      TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "gemm: operands must be 16-byte aligned for the MFMA kernels");
    if (mode != 2)   // bf16 output rows are stored as 16-B pieces when ldc allows
      TORCH_CHECK(reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 == 0,
                  "gemm: the bf16 output must be 16-byte aligned");
    TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm: operand row strides must be multiples of 8");
    auto c8 = [](int64_t v) { return (v + 7) / 8 * 8; };
    if (mode == 0) TORCH_CHECK(K % 8 == 0, "gemm: K must be a multiple of 8 (else cfg -1)");
    if (mode == 1)
      TORCH_CHECK(K % 8 == 0 && (N % 8 == 0 || ldb >= c8(N)),
                  "gemm: K must be a multiple of 8, N too unless padded in b's row stride");
    // k-strided operands are fetched in 8-column pieces: a partial last piece
    // may read into the row padding, never past the row stride
    if (mode == 2)
      TORCH_CHECK((M % 8 == 0 || lda >= c8(M)) && (N % 8 == 0 || ldb >= c8(N)),
                  "gemm: wgrad M, N must be multiples of 8 or padded in the row stride");
    // bf16 outputs: 16-B row segments, or element stores when N / ldc are not
    // multiples of 8 (any width)
  }
  // wgrad split-K through a plain-store slab + reduce pass instead of atomics
  Tensor ws;
  if (slab && mode == 2 && cfg >= 0) {
    const int sp = dmp::gemm_effective_splits((int)K, (int)std::max<int64_t>(1, splits));
    if (sp > 1) ws = at::empty({(int64_t)sp * M * N}, c.options().dtype(at::kFloat));
  }
  // fwd / dgrad remainder split-K: per-call fp32 piece workspace + zeroed tickets
  // (caching-allocator memory: safe inside a captured graph)
  Tensor skw, skc;
  if (mode != 2 && cfg >= 0 && splits > 1) {
    long long wf = 0;
    int nc = 0;
    dmp::gemm_sk_sizes((int)cfg, (int)M, (int)N, (int)K, (int)splits, &wf, &nc);
    if (wf > 0 && nc > 0) {
      skw = at::empty({(int64_t)wf}, c.options().dtype(at::kFloat));
      skc = at::zeros({(int64_t)nc}, c.options().dtype(at::kInt));
    }
  }
  dmp::launch_gemm((int)mode, (int)epi, (int)cfg, reinterpret_cast<const uint16_t*>(a.data_ptr()),
                   (int)lda, reinterpret_cast<const uint16_t*>(b.data_ptr()), (int)ldb,
                   c.data_ptr(), (int)ldc, c2p, biasp, auxp, dbp, (int)M, (int)N, (int)K,
                   (int)std::max<int64_t>(1, splits), cur_stream(), relu, partp,
                   ws.defined() ? ws.data_ptr<float>() : nullptr,
                   skw.defined() ? skw.data_ptr<float>() : nullptr,
                   skc.defined() ? skc.data_ptr<int>() : nullptr, amp);
}

std::vector<std::vector<int64_t>> gemm_configs() {
  std::vector<std::vector<int64_t>> out;
  for (int i = 0; i < dmp::gemm_num_configs(); ++i) {
    int info[5];
    dmp::gemm_config_info(i, info);
    out.push_back({i, info[0], info[1], info[2], info[3], info[4]});
  }
  return out;
}

// ------------------------------------------------------------- transformer
void check_rows_bf16(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.is_contiguous(), name,
              " must be a contiguous bf16 tensor");
}

std::vector<Tensor> layernorm_fwd(Tensor x, optional<Tensor> gamma, optional<Tensor> beta,
                                  double eps, optional<Tensor> residual) {
  check_rows_bf16(x, "x");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(dmp::layernorm_supported((int)D),
              "layernorm: D must be a multiple of 8 with D/8 / lanes <= 8, got ", D);
  for (auto* t : {&gamma, &beta})
    if (t->has_value())
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == D &&
                      (*t)->is_contiguous(), "layernorm affine params must be fp32 [D]");
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, fopt), rstd = at::empty({rows}, fopt);
  Tensor r, h;
  const bool fused = residual.has_value() && residual->defined();
  if (fused) {
    r = residual->contiguous();
    check_rows_bf16(r, "residual");
    TORCH_CHECK(r.sizes() == x.sizes(), "layernorm: residual shape mismatch");
    h = at::empty_like(x);
  }
  dmp::launch_layernorm_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                            ptr_or_null<float>(gamma), ptr_or_null<float>(beta),
                            reinterpret_cast<uint16_t*>(y.data_ptr()), mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), rows, (int)D, (float)eps, cur_stream(),
                            fused ? reinterpret_cast<const uint16_t*>(r.data_ptr()) : nullptr,
                            fused ? reinterpret_cast<uint16_t*>(h.data_ptr()) : nullptr);
  if (fused) return {y, mean, rstd, h};
  return {y, mean, rstd};
}

// ViT token assembly: h [B, N+1, D] = cat(cls, tok) + pos (bf16 operands)
// [B, D] gradient of the token-`tok` rows -> the [B, N, D] stream gradient
// (zeros elsewhere), one native pass (models/vit.py class-token head)
Tensor token_row_scatter(Tensor g, int64_t N, int64_t tok) {
  check_gpu(g, "g");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 && g.dim() == 2 && g.is_contiguous(),
              "token_row_scatter: g must be a contiguous bf16 [B, D] GPU tensor");
  const int64_t B = g.size(0), D = g.size(1);
  TORCH_CHECK(D % 8 == 0 && N >= 1 && tok >= 0 && tok < N,
              "token_row_scatter: D % 8 == 0 and 0 <= tok < N");
  TORCH_CHECK(B * N * D < (1LL << 40), "token_row_scatter: tensor too large");
  Tensor out = at::empty({B, N, D}, g.options());
  dmp::launch_token_row_scatter(reinterpret_cast<const uint16_t*>(g.data_ptr()),
                                reinterpret_cast<uint16_t*>(out.data_ptr()), (int)B, (int)N,
                                (int)D, (int)tok, cur_stream());
  return out;
}

Tensor vit_embed_fwd(Tensor tok, Tensor cls, Tensor pos) {
  tok = tok.contiguous();
  check_rows_bf16(tok, "tok");
  TORCH_CHECK(tok.dim() == 3, "vit_embed_fwd: tok must be [B, N, D]");
  const int64_t B = tok.size(0), N = tok.size(1), D = tok.size(2);
  TORCH_CHECK(D % 8 == 0, "vit_embed_fwd: D must be a multiple of 8");
  cls = cls.contiguous();
  pos = pos.contiguous();
  check_rows_bf16(cls, "cls");
  check_rows_bf16(pos, "pos");
  TORCH_CHECK(cls.numel() == D && pos.numel() == (N + 1) * D, "vit_embed_fwd: cls / pos shape");
  Tensor h = at::empty({B, N + 1, D}, tok.options());
  dmp::launch_vit_embed_fwd(reinterpret_cast<const uint16_t*>(tok.data_ptr()),
                            reinterpret_cast<const uint16_t*>(cls.data_ptr()),
                            reinterpret_cast<const uint16_t*>(pos.data_ptr()),
                            reinterpret_cast<uint16_t*>(h.data_ptr()), (int)B, (int)N, (int)D,
                            cur_stream());
  return h;
}

// backward: returns dtok [B, N, D] (bf16) and adds the batch sums into the fp32
// gradients dpos [(N+1) * D] and dcls [D] in place
Tensor vit_embed_bwd(Tensor dh, optional<Tensor> dpos, optional<Tensor> dcls, bool want_dtok) {
  dh = dh.contiguous();
  check_rows_bf16(dh, "dh");
  TORCH_CHECK(dh.dim() == 3, "vit_embed_bwd: dh must be [B, N+1, D]");
  const int64_t B = dh.size(0), N = dh.size(1) - 1, D = dh.size(2);
  TORCH_CHECK(D % 8 == 0 && N >= 0, "vit_embed_bwd: bad shape");
  for (auto* t : {&dpos, &dcls})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->is_contiguous() &&
                      reinterpret_cast<uintptr_t>((*t)->data_ptr()) % 16 == 0,
                  "vit_embed_bwd: fp32 contiguous 16-B aligned parameter gradients");
  if (dpos.has_value() && dpos->defined())
    TORCH_CHECK(dpos->numel() == (N + 1) * D, "vit_embed_bwd: dpos shape");
  if (dcls.has_value() && dcls->defined()) TORCH_CHECK(dcls->numel() == D, "vit_embed_bwd: dcls shape");
  Tensor dtok;
  if (want_dtok) dtok = at::empty({B, N, D}, dh.options());
  dmp::launch_vit_embed_bwd(reinterpret_cast<const uint16_t*>(dh.data_ptr()),
                            want_dtok ? reinterpret_cast<uint16_t*>(dtok.data_ptr()) : nullptr,
                            ptr_or_null<float>(dpos), ptr_or_null<float>(dcls), (int)B, (int)N,
                            (int)D, cur_stream());
  return dtok;
}

Tensor layernorm_bwd(Tensor x, Tensor dy, optional<Tensor> gamma, Tensor mean, Tensor rstd,
                     optional<Tensor> dgamma, optional<Tensor> dbeta, optional<Tensor> slots,
                     optional<Tensor> dres) {
  check_rows_bf16(x, "x");
  dy = dy.contiguous();
  check_rows_bf16(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "layernorm_bwd: dy shape mismatch");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(dmp::layernorm_supported((int)D), "layernorm_bwd: unsupported D ", D);
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd: stats mismatch");
  for (auto* t : {&gamma, &dgamma, &dbeta})
    if (t->has_value())
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == D &&
                      (*t)->is_contiguous(), "layernorm gamma/dgamma/dbeta must be fp32 [D]");
  // [kLnSlots][2][D] fp32 partial-sum slots: a persistent per-layer buffer (zero,
  // re-zeroed by the param-grad kernel) or a fresh zeroed one
  Tensor sl;
  const bool grads = dgamma.has_value() || dbeta.has_value();
  const int64_t nsl = (int64_t)dmp::layernorm_num_slots() * 2 * D;
  if (grads) {
    if (slots.has_value() && slots->defined()) {
      TORCH_CHECK(slots->is_cuda() && slots->scalar_type() == at::kFloat &&
                      slots->is_contiguous() && slots->numel() == nsl,
                  "layernorm slots must be a contiguous fp32 GPU tensor of ", nsl, " elements");
      sl = *slots;
    } else {
      sl = at::zeros({nsl}, x.options().dtype(at::kFloat));
    }
  }
  auto dx = at::empty_like(x);
  Tensor dr;
  if (dres.has_value() && dres->defined()) {
    dr = dres->contiguous();
    check_rows_bf16(dr, "dres");
    TORCH_CHECK(dr.sizes() == x.sizes(), "layernorm_bwd: dres shape mismatch");
  }
  dmp::launch_layernorm_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                            reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                            ptr_or_null<float>(gamma), mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                            ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta),
                            grads ? sl.data_ptr<float>() : nullptr, rows, (int)D, cur_stream(),
                            dr.defined() ? reinterpret_cast<const uint16_t*>(dr.data_ptr())
                                         : nullptr);
  return dx;
}

Tensor gelu_fwd(Tensor x) {
  check_rows_bf16(x, "x");
  TORCH_CHECK(x.numel() % 8 == 0, "gelu: numel % 8 == 0");
  auto y = at::empty_like(x);
  dmp::launch_gelu_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()), x.numel(), cur_stream());
  return y;
}

Tensor gelu_bwd(Tensor x, Tensor dy) {
  check_rows_bf16(x, "x");
  dy = dy.contiguous();
  check_rows_bf16(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes() && x.numel() % 8 == 0, "gelu_bwd: shape");
  auto dx = at::empty_like(x);
  dmp::launch_gelu_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                       reinterpret_cast<uint16_t*>(dx.data_ptr()), x.numel(), cur_stream());
  return dx;
}

Tensor softmax_fwd(Tensor sc, double scale) {
  check_rows_bf16(sc, "scores");
  const int64_t L = sc.size(-1);
  TORCH_CHECK(L <= dmp::softmax_max_len(), "softmax: row length <= ", dmp::softmax_max_len());
  auto p = at::empty_like(sc);
  dmp::launch_softmax_fwd(reinterpret_cast<const uint16_t*>(sc.data_ptr()),
                          reinterpret_cast<uint16_t*>(p.data_ptr()), sc.numel() / L, (int)L,
                          (float)scale, cur_stream());
  return p;
}

Tensor softmax_bwd(Tensor p, Tensor dp, double scale) {
  check_rows_bf16(p, "p");
  dp = dp.contiguous();
  check_rows_bf16(dp, "dp");
  TORCH_CHECK(dp.sizes() == p.sizes(), "softmax_bwd: shape mismatch");
  const int64_t L = p.size(-1);
  auto ds = at::empty_like(p);
  dmp::launch_softmax_bwd(reinterpret_cast<const uint16_t*>(p.data_ptr()),
                          reinterpret_cast<const uint16_t*>(dp.data_ptr()),
                          reinterpret_cast<uint16_t*>(ds.data_ptr()), p.numel() / L, (int)L,
                          (float)scale, cur_stream());
  return ds;
}

// ------------------------------------------------------------------ dropout
// mode 0: element-wise; 1: per (n, c) plane of an NCHW tensor; 2: per (n, c)
// of an NHWC (channels_last) tensor.
std::vector<Tensor> dropout_fwd(Tensor x, double p, int64_t seed, Tensor offset, int64_t mode) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
              "dropout: bf16 or fp32 input");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout: p must be in [0, 1)");
  TORCH_CHECK(offset.is_cuda() && offset.scalar_type() == at::kLong && offset.numel() >= 2 &&
                  offset.is_contiguous(),
              "dropout: offset must be an int64 GPU tensor [offset, ticket] (zeros at creation)");
  TORCH_CHECK(mode >= 0 && mode <= 2, "dropout: bad mode");
  long long inner = 1, nmask = x.numel();
  int C = 1;
  if (mode != 0) {
    TORCH_CHECK(x.dim() >= 3, "channel dropout needs [N, C, ...]");
    C = (int)x.size(1);
    inner = x.numel() / (x.size(0) * C);
    nmask = x.size(0) * C;
    if (mode == 1) {
      TORCH_CHECK(x.is_contiguous(), "mode 1 needs a contiguous NCHW tensor");
    } else {
      TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
                  "mode 2 needs a channels_last tensor");
    }
  } else {
    TORCH_CHECK(x.is_contiguous() || x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "dropout: dense input");
  }
  auto mask = at::empty({nmask}, x.options().dtype(at::kByte));
  auto y = at::empty_like(x);
  // one launch: draw + mask + scaled product; it advances offset[0] itself
  dmp::launch_dropout_fwd_fused(x.data_ptr(), mask.data_ptr<uint8_t>(), y.data_ptr(),
                                x.scalar_type() == at::kBFloat16, x.numel(), (float)p, (int)mode,
                                inner, C, (unsigned long long)seed,
                                reinterpret_cast<long long*>(offset.data_ptr<int64_t>()),
                                cur_stream());
  return {y, mask};
}

Tensor dropout_bwd(Tensor dy, Tensor mask, double p, int64_t mode) {
  check_gpu(dy, "dy");
  long long inner = 1;
  int C = 1;
  if (mode == 2) dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  else if (!(mode == 0 && dy.is_contiguous(at::MemoryFormat::ChannelsLast))) dy = dy.contiguous();
  if (mode != 0) {
    C = (int)dy.size(1);
    inner = dy.numel() / (dy.size(0) * C);
  }
  auto dx = at::empty_like(dy);
  const float scale = (float)(1.0 / (1.0 - p));
  if (dy.scalar_type() == at::kBFloat16)
    dmp::launch_dropout_apply_bf16(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                   mask.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                   dy.numel(), scale, (int)mode, inner, C, cur_stream());
  else
    dmp::launch_dropout_apply_f32(dy.data_ptr<float>(), mask.data_ptr<uint8_t>(), dx.data_ptr<float>(),
                                  dy.numel(), scale, (int)mode, inner, C, cur_stream());
  return dx;
}

std::vector<std::vector<int64_t>> conv_configs() {
  std::vector<std::vector<int64_t>> out;
  for (int c = 0; c < dmp::conv_num_configs(); ++c) {
    int info[5];
    dmp::conv_config_info(c, info);
    out.push_back({c, info[0], info[1], info[2], info[3], info[4]});
  }
  return out;
}

// halo-tile cfg ids applicable to a conv over a [*, C, H, W] input (3x3 / stride 1 / pad 1)
std::vector<int64_t> conv_halo_configs(int64_t H, int64_t W, int64_t C, int64_t R, int64_t S,
                                       int64_t stride, int64_t pad) {
  std::vector<int64_t> out;
  for (int i = 0; i < dmp::conv_num_halo_configs(); ++i) {
    const int c = dmp::conv_halo_base() + i;
    if (dmp::conv_halo_ok(c, (int)H, (int)W, (int)C, (int)R, (int)S, (int)stride, (int)pad))
      out.push_back(c);
  }
  return out;
}

// stride-2 halo dgrad cfg ids applicable to dX [*, CI, H, W] from dY [*, CO, OH, OW]
std::vector<int64_t> conv_dgrad_s2_configs(int64_t H, int64_t W, int64_t OH, int64_t OW,
                                           int64_t CO, int64_t CI, int64_t R, int64_t S,
                                           int64_t stride, int64_t pad) {
  std::vector<int64_t> out;
  for (int i = 0; i < dmp::conv_dgrad_s2_num_configs(); ++i) {
    const int c = dmp::conv_dgrad_s2_base() + i;
    if (dmp::conv_dgrad_s2_ok(c, (int)H, (int)W, (int)OH, (int)OW, (int)CO, (int)CI, (int)R,
                              (int)S, (int)stride, (int)pad))
      out.push_back(c);
  }
  return out;
}

// halo wgrad cfg ids applicable to dW of a conv over [B, CI, H, W] -> CO channels
std::vector<int64_t> conv_wgrad_halo_configs(int64_t B, int64_t H, int64_t W, int64_t CI,
                                             int64_t CO, int64_t R, int64_t S, int64_t stride,
                                             int64_t pad) {
  std::vector<int64_t> out;
  for (int base : {dmp::conv_wgrad_halo_base(), dmp::conv_wgrad_halo_slab_base()}) {
    for (int i = 0; i < dmp::conv_wgrad_num_halo_configs(); ++i) {
      const int c = base + i;
      if (dmp::conv_wgrad_halo_ok(c, (int)B, (int)H, (int)W, (int)CI, (int)CO, (int)R, (int)S,
                                  (int)stride, (int)pad))
        out.push_back(c);
    }
  }
  return out;
}

std::vector<Tensor> bn_fwd_from_partials(Tensor x, Tensor part, int64_t G, optional<Tensor> res,
                                         optional<Tensor> gamma, optional<Tensor> beta,
                                         optional<Tensor> running_mean,
                                         optional<Tensor> running_var, double momentum,
                                         double eps, bool relu, bool want_mask) {
  check_nhwc_bf16(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: bad C");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  G == dmp::kBnSlots && part.numel() == 2 * G * C + dmp::kBnTail,
              "bad BN slot sums");
  if (res) {
    check_nhwc_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
  }
  auto y = at::empty_like(x);
  auto stats = at::empty({4, C}, x.options().dtype(at::kFloat));
  Tensor mask;
  if (want_mask && relu) mask = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  dmp::launch_bn_fwd_partials(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                              res ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr,
                              reinterpret_cast<uint16_t*>(y.data_ptr()), ptr_or_null<float>(gamma),
                              ptr_or_null<float>(beta), ptr_or_null<float>(running_mean),
                              ptr_or_null<float>(running_var), stats.data_ptr<float>(),
                              part.data_ptr<float>(), M, (int)C, (float)momentum,
                              (float)eps, relu, cur_stream(),
                              mask.defined() ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, stats, mask};
}


// BatchNorm with the finalize folded into the apply passes (bn.hip fold kernels).
// part: the forward slot sums (already filled by the producing conv when
// have_partials, else reduced here first); zero_buf: the layer's backward slots,
// zeroed by the apply for the next backward.
std::vector<Tensor> bn_fwd_fold(Tensor x, Tensor part, bool have_partials, optional<Tensor> res,
                                optional<Tensor> gamma, optional<Tensor> beta,
                                optional<Tensor> running_mean, optional<Tensor> running_var,
                                double momentum, double eps, bool relu, bool want_mask,
                                optional<Tensor> zero_buf) {
  check_nhwc_bf16(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: C must be a multiple of 8 and <= 2048, got ", C);
  auto fopt = x.options().dtype(at::kFloat);
  part = bn_slots(part, C, fopt);
  float* zb = nullptr;
  if (zero_buf.has_value() && zero_buf->defined()) {
    zb = bn_slots(zero_buf, C, fopt).data_ptr<float>();
    TORCH_CHECK(zb != part.data_ptr<float>(), "bn fold: zero_buf must not alias part");
  }
  if (res) {
    check_nhwc_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
  }
  for (auto* t : {&gamma, &beta, &running_mean, &running_var}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn affine/running tensors must be contiguous fp32 [C] on the GPU");
    }
  }
  auto y = at::empty_like(x);
  auto stats = at::empty({4, C}, fopt);
  Tensor mask;
  if (want_mask && relu) mask = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  dmp::launch_bn_fwd_fold(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                          res ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr,
                          reinterpret_cast<uint16_t*>(y.data_ptr()), ptr_or_null<float>(gamma),
                          ptr_or_null<float>(beta), ptr_or_null<float>(running_mean),
                          ptr_or_null<float>(running_var), stats.data_ptr<float>(),
                          part.data_ptr<float>(), zb, M, (int)C, (float)momentum, (float)eps,
                          relu, have_partials, cur_stream(),
                          mask.defined() ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, stats, mask};
}

// backward: reduce into `slots` (the layer's backward slots, zero on entry), then
// the folded apply; zero_buf: the forward slot sums this layer's forward read
std::vector<Tensor> bn_bwd_fold(Tensor x, Tensor dy, optional<Tensor> y, optional<Tensor> gamma,
                                Tensor stats, optional<Tensor> dgamma, optional<Tensor> dbeta,
                                bool relu, bool want_dres, Tensor slots, optional<Tensor> mask,
                                optional<Tensor> zero_buf) {
  check_nhwc_bf16(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: bad C");
  if (!dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.dim() == 4)
    dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  const bool have_y = relu && y.has_value() && y->defined();
  if (have_y) {
    check_nhwc_bf16(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes(), "y shape mismatch");
  }
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * C, "bad stats");
  for (auto* t : {&gamma, &dgamma, &dbeta}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn gamma/dgamma/dbeta must be contiguous fp32 [C]");
    }
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto part = bn_slots(slots, C, fopt);
  float* zb = nullptr;
  if (zero_buf.has_value() && zero_buf->defined()) {
    zb = bn_slots(zero_buf, C, fopt).data_ptr<float>();
    TORCH_CHECK(zb != part.data_ptr<float>(), "bn fold: zero_buf must not alias slots");
  }
  auto dx = at::empty_like(x);
  Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  const uint8_t* mptr = nullptr;
  if (relu && mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == M * C / 8,
                "bn: ReLU bit mask must be a contiguous uint8 [M, C/8] GPU tensor");
    mptr = mask->data_ptr<uint8_t>();
  }
  // [3][C] coefficient hand-off of the one-pass kernel (bn.hip bn_bwd_onepass_kernel)
  auto coef = at::empty({3 * C}, fopt);
  dmp::launch_bn_bwd_fold(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                          reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                          have_y ? reinterpret_cast<const uint16_t*>(y->data_ptr()) : nullptr,
                          ptr_or_null<float>(gamma), stats.data_ptr<float>(),
                          ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta),
                          part.data_ptr<float>(), zb, reinterpret_cast<uint16_t*>(dx.data_ptr()),
                          want_dres ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr, M,
                          (int)C, relu, cur_stream(), mptr, coef.data_ptr<float>());
  return {dx, want_dres ? dres : Tensor()};
}

// BN + ReLU + max pool 3x3/s2/p1 with the finalize folded in (bn.hip): x is the
// raw conv output; returns the pooled output, its uint8 argmax taps and stats.
std::vector<Tensor> bn_relu_maxpool_fwd(Tensor x, Tensor part, bool have_partials,
                                        optional<Tensor> gamma, optional<Tensor> beta,
                                        optional<Tensor> running_mean,
                                        optional<Tensor> running_var, double momentum, double eps,
                                        optional<Tensor> zero_buf, int64_t K, int64_t S,
                                        int64_t P) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_relu_maxpool expects 4-D input");
  TORCH_CHECK(dmp::guard::bf16_bytes_ok(x.size(0), x.size(2), x.size(3), x.size(1)),
              "bn_relu_maxpool: x over 2 GiB (32-bit offsets)");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(dmp::bn_maxpool_supported(C, (int)K, (int)S, (int)P),
              "bn_relu_maxpool: needs C % 64 == 0, C <= 2048 and a 3x3/s2/p1 window");
  auto fopt = x.options().dtype(at::kFloat);
  part = bn_slots(part, C, fopt);
  float* zb = nullptr;
  if (zero_buf.has_value() && zero_buf->defined()) {
    zb = bn_slots(zero_buf, C, fopt).data_ptr<float>();
    TORCH_CHECK(zb != part.data_ptr<float>(), "bn fold: zero_buf must not alias part");
  }
  for (auto* t : {&gamma, &beta, &running_mean, &running_var}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn affine/running tensors must be contiguous fp32 [C] on the GPU");
    }
  }
  const int Ho = dmp::maxpool_out(H, (int)K, (int)S, (int)P);
  const int Wo = dmp::maxpool_out(W, (int)K, (int)S, (int)P);
  TORCH_CHECK(Ho > 0 && Wo > 0, "bn_relu_maxpool: window larger than input");
  auto mf = at::MemoryFormat::ChannelsLast;
  auto y = at::empty({N, C, Ho, Wo}, x.options().memory_format(mf));
  auto idx = at::empty({N, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(mf));
  auto xm = at::empty({N, C, Ho, Wo}, x.options().memory_format(mf));
  auto stats = at::empty({4, C}, fopt);
  dmp::launch_bn_relu_maxpool_fold(
      reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
      idx.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(xm.data_ptr()), ptr_or_null<float>(gamma), ptr_or_null<float>(beta),
      ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var), stats.data_ptr<float>(),
      part.data_ptr<float>(), zb, N, H, W, C, (float)momentum, (float)eps, have_partials,
      cur_stream());
  return {y, idx, stats, xm};
}

// backward of bn_relu_maxpool_fwd: dx of the raw conv output from the pooled
// gradient; slots = the layer's backward slots (zero on entry), zero_buf = the
// forward slot sums the forward read
Tensor maxpool_bn_bwd(Tensor x, Tensor dp, Tensor idx, Tensor xm, optional<Tensor> gamma, Tensor stats,
                      optional<Tensor> dgamma, optional<Tensor> dbeta, Tensor slots,
                      optional<Tensor> zero_buf, int64_t K, int64_t S, int64_t P) {
  check_nhwc_bf16(x, "x");
  auto mf = at::MemoryFormat::ChannelsLast;
  dp = dp.contiguous(mf);
  check_nhwc_bf16(dp, "dp");
  TORCH_CHECK(dmp::guard::bf16_bytes_ok(x.size(0), x.size(2), x.size(3), x.size(1)),
              "maxpool_bn_bwd: x over 2 GiB (32-bit offsets)");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(dmp::bn_maxpool_supported(C, (int)K, (int)S, (int)P), "maxpool_bn_bwd: bad window");
  TORCH_CHECK(dp.size(0) == N && dp.size(1) == C &&
                  dp.size(2) == dmp::maxpool_out(H, (int)K, (int)S, (int)P) &&
                  dp.size(3) == dmp::maxpool_out(W, (int)K, (int)S, (int)P),
              "maxpool_bn_bwd: dp shape mismatch");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.sizes() == dp.sizes() &&
                  idx.is_contiguous(mf),
              "maxpool_bn_bwd: idx mismatch");
  check_nhwc_bf16(xm, "xm");
  TORCH_CHECK(xm.sizes() == dp.sizes(), "maxpool_bn_bwd: xm mismatch");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * C, "bad stats");
  for (auto* t : {&gamma, &dgamma, &dbeta}) {
    if (t->has_value()) {
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kFloat && (*t)->numel() == C &&
                      (*t)->is_contiguous(),
                  "bn gamma/dgamma/dbeta must be contiguous fp32 [C]");
    }
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto part = bn_slots(slots, C, fopt);
  float* zb = nullptr;
  if (zero_buf.has_value() && zero_buf->defined()) {
    zb = bn_slots(zero_buf, C, fopt).data_ptr<float>();
    TORCH_CHECK(zb != part.data_ptr<float>(), "bn fold: zero_buf must not alias slots");
  }
  auto dx = at::empty_like(x);
  dmp::launch_maxpool_bn_bwd_fold(
      reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(dp.data_ptr()),
      idx.data_ptr<uint8_t>(), reinterpret_cast<const uint16_t*>(xm.data_ptr()),
      ptr_or_null<float>(gamma), stats.data_ptr<float>(), ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta), part.data_ptr<float>(), zb,
      reinterpret_cast<uint16_t*>(dx.data_ptr()), N, H, W, C, cur_stream());
  return dx;
}
}  // namespace

PYBIND11_MODULE(_native, m) {
  m.def("conv_fwd", &conv_fwd, "NHWC bf16 implicit-GEMM conv forward (+BN partials)",
        py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("want_stats"),
        py::arg("cfg") = -1, py::arg("slots") = py::none(), py::arg("bias") = py::none(),
        py::arg("relu") = false, py::arg("addend") = py::none());
  m.def("bn_fold_weights", &bn_fold_weights,
        "inference-time BatchNorm fold: (bf16 w * s, fp32 shift, bf16 shift)", py::arg("w"),
        py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"),
        py::arg("cbias") = py::none(), py::arg("eps") = 1e-5);
  m.def("conv_dgrad", &conv_dgrad, "NHWC bf16 implicit-GEMM conv data gradient", py::arg("dy"),
        py::arg("w"), py::arg("H"), py::arg("W"), py::arg("stride"), py::arg("pad"),
        py::arg("cfg") = -1, py::arg("wt") = py::none(), py::arg("addend") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(),
        py::arg("bn_stats") = py::none(), py::arg("bn_part") = py::none(),
        py::arg("bn_relu") = -1, py::arg("addend_sub") = false,
        py::arg("addend_mask") = py::none());
  m.def("subsample2", &subsample2, "x[:, :, ::2, ::2] of a channels_last bf16 activation",
        py::arg("x"));
  m.def("add_subsampled2", &add_subsampled2, "dx[:, :, ::2, ::2] += xs in place",
        py::arg("dx"), py::arg("xs"));
  m.def("bn_bwd_from_partials", &bn_bwd_from_partials,
        "BN backward from conv-dgrad-epilogue partials (dz already ReLU-masked)", py::arg("x"),
        py::arg("dz"), py::arg("gamma"), py::arg("stats"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("part"));
  m.def("pad_rows_batched", &pad_rows_batched, "padded-row copies of im2col conv weights");
  m.def("zero_", &zero_, "native zero fill of a dense GPU tensor (a kernel, not a memset)");
  m.def("conv_weight_transpose_batched", &conv_weight_transpose_batched,
        "transpose every conv weight of a flat bf16 shadow in one launch");
  m.def("conv_wgrad", &conv_wgrad, "NHWC bf16 conv weight gradient (fp32 accumulate)",
        py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("stride"), py::arg("pad"),
        py::arg("cfg") = -1, py::arg("dbias") = py::none());
  m.def("conv_configs", &conv_configs, "[(id, BM, BN, BK, threads)] of the compiled conv tiles");
  m.def("conv_wgrad_halo_configs", &conv_wgrad_halo_configs,
        "3x3 stride-1 / stride-2 halo wgrad cfg ids applicable to (B, H, W, CI, CO, R, S, stride, pad)");
  m.def("conv_dgrad_s2_configs", &conv_dgrad_s2_configs,
        "3x3/stride-2 halo data-gradient cfg ids for (H, W, OH, OW, CO, CI, R, S, stride, pad)");
  m.def("conv_halo_configs", &conv_halo_configs,
        "3x3/stride-1 halo-tile cfg ids applicable to (H, W, C, R, S, stride, pad)");
  m.def("bn_fwd_from_partials", &bn_fwd_from_partials, "BN forward from conv-epilogue partials",
        py::arg("x"), py::arg("part"), py::arg("G"), py::arg("res"), py::arg("gamma"),
        py::arg("beta"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"),
        py::arg("eps"), py::arg("relu"), py::arg("want_mask") = false);
  m.def("stem_supported", [](int64_t H, int64_t W) { return dmp::stem_supported((int)H, (int)W); },
        "ImageNet 7x7/2 stem kernel applies to an H x W input");
  m.def("stem_fwd", &stem_fwd, "ImageNet stem conv forward (+BN partials) via space-to-depth",
        py::arg("x"), py::arg("w"), py::arg("want_stats"), py::arg("slots") = py::none(),
        py::arg("bias") = py::none(), py::arg("relu") = false);
  m.def("stem_wgrad", &stem_wgrad, "ImageNet stem conv weight gradient (fp32 +=)", py::arg("dy"),
        py::arg("xs"), py::arg("dw"));
  m.def("conv_small_fwd", &conv_small_fwd, "few-input-channel conv forward (+BN partials)",
        py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("want_stats"),
        py::arg("slots") = py::none());
  m.def("conv_small_wgrad", &conv_small_wgrad, "few-input-channel conv weight gradient (fp32 +=)",
        py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("stride"), py::arg("pad"));
  m.doc() = "gfx950 (MI355X) HIP kernels for distributed_ml_pytorch_amd";
  m.def("asgd_fused_step", &asgd_fused_step, "fused flat ASGD/SGD update");
  m.def("gemm_sk_pieces",
        [](int64_t cfg, int64_t M, int64_t N, int64_t K, int64_t splits) {
          long long wf = 0;
          int nc = 0;
          dmp::gemm_sk_sizes((int)cfg, (int)M, (int)N, (int)K, (int)splits, &wf, &nc);
          return nc > 0 ? wf / std::max<long long>(1, nc) : 0LL;
        },
        "fwd / dgrad remainder split-K: fp32 workspace floats per split tile (0 = no split)");
  m.def("ps_apply", &ps_apply, "parameter-server delta apply", py::arg("shard"), py::arg("delta"),
        py::arg("mirror") = py::none(), py::arg("scale") = 1.0, py::arg("atomic") = false);
  m.def("ps_count", &ps_count, "bump / set a PS applied-count", py::arg("cnt"),
        py::arg("add") = 1, py::arg("set") = false);
  m.def("ps_stamp", &ps_stamp, "copy a PS applied-count into a reply's version element");
  m.def("pull_land", &pull_land, "land a parameter pull into the worker arena");
  m.def("push_handoff", &push_handoff, "snapshot+zero the push accumulator");
  m.def("cast_f32_bf16", &cast_f32_bf16, "flat fp32 -> bf16");
  m.def("sumsq", &sumsq, "sum of squares of a flat fp32 buffer");
  m.def("softmax_xent", &softmax_xent, "fused softmax cross entropy fwd+bwd");
  m.def("bn_fwd_fold", &bn_fwd_fold, "BN forward, finalize folded into the apply",
        py::arg("x"), py::arg("part"), py::arg("have_partials"), py::arg("res") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(),
        py::arg("running_mean") = py::none(), py::arg("running_var") = py::none(),
        py::arg("momentum") = 0.1, py::arg("eps") = 1e-5, py::arg("relu") = false,
        py::arg("want_mask") = false, py::arg("zero_buf") = py::none());
  m.def("bn_bwd_fold", &bn_bwd_fold, "BN backward, finalize folded into the apply",
        py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("gamma"), py::arg("stats"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("relu"), py::arg("want_dres"),
        py::arg("slots"), py::arg("mask") = py::none(), py::arg("zero_buf") = py::none());
  m.def("bn_maxpool_supported",
        [](int64_t C, int64_t K, int64_t S, int64_t P) {
          return dmp::bn_maxpool_supported((int)C, (int)K, (int)S, (int)P);
        },
        "fused BN + ReLU + max pool applies to (C, K, S, P)");
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd,
        "BN + ReLU + max pool forward, finalize folded in -> (y, idx, stats, x at the taps)",
        py::arg("x"),
        py::arg("part"), py::arg("have_partials"), py::arg("gamma"), py::arg("beta"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("zero_buf"), py::arg("K"), py::arg("S"), py::arg("P"));
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd, "backward of bn_relu_maxpool_fwd -> dx", py::arg("x"),
        py::arg("dp"), py::arg("idx"), py::arg("xm"), py::arg("gamma"), py::arg("stats"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("slots"), py::arg("zero_buf"), py::arg("K"), py::arg("S"),
        py::arg("P"));
  m.def("bn_fwd", &bn_fwd, "NHWC batchnorm(+residual)(+relu) forward", py::arg("x"),
        py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("training"),
        py::arg("relu"), py::arg("slots") = py::none(), py::arg("want_mask") = false);
  m.def("bn_bwd", &bn_bwd, "NHWC batchnorm(+residual)(+relu) backward", py::arg("x"),
        py::arg("dy"), py::arg("y"), py::arg("gamma"), py::arg("stats"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("relu"), py::arg("want_dres"), py::arg("slots") = py::none(),
        py::arg("mask") = py::none());
  m.def("token_row_scatter", &token_row_scatter, "gradient of a per-sample token-row select");
  m.def("vit_embed_fwd", &vit_embed_fwd, "ViT token assembly cat(cls, tok) + pos");
  m.def("vit_embed_bwd", &vit_embed_bwd, "ViT token assembly backward (dtok + fp32 batch sums)");
  m.def("layernorm_fwd", &layernorm_fwd,
        "row LayerNorm forward -> (y, mean, rstd[, h = x + residual])", py::arg("x"),
        py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("residual") = py::none());
  m.def("layernorm_bwd", &layernorm_bwd, "row LayerNorm backward (dgamma/dbeta accumulated)",
        py::arg("x"), py::arg("dy"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("slots") = py::none(),
        py::arg("dres") = py::none());
  m.def("layernorm_num_slots", &dmp::layernorm_num_slots, "slot rows of the LayerNorm param grads");
  m.def("colsum_acc", &colsum_acc, "bias gradient: out[n] += sum_m dy[m][n] (bf16 -> fp32)",
        py::arg("dy"), py::arg("out"), py::arg("slots") = py::none());
  m.def("colsum_num_slots", &dmp::colsum_num_slots, "slot rows of the colsum scratch");
  m.def("gemm", &gemm, "bf16 MFMA GEMM (fwd / dgrad / wgrad modes, fused epilogues)",
        py::arg("mode"), py::arg("epi"), py::arg("cfg"), py::arg("a"), py::arg("b"), py::arg("c"),
        py::arg("c2") = py::none(), py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("dbias") = py::none(), py::arg("splits") = 1, py::arg("relu") = false,
        py::arg("part") = py::none(), py::arg("slab") = false, py::arg("auxmask") = py::none());
  m.def("im2col", &im2col, "NHWC patch rows [B*OH*OW, Kp], k = (r, s, ci), zero-padded",
        py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("Kp"));
  m.def("col2im", &col2im, "gather-form inverse of im2col -> channels_last dX", py::arg("dcols"),
        py::arg("B"), py::arg("CI"), py::arg("H"), py::arg("W"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"));
  m.def("relu_bwd", &relu_bwd, "ReLU backward from the saved output", py::arg("dy"), py::arg("y"),
        py::arg("out") = py::none());
  m.def("gemm_config_ok", &dmp::gemm_config_ok, "tile config usable in this mode");
  m.def("gemm_set_xcd_k", &dmp::gemm_set_xcd_k, "split-major XCD deal of wgrad split-K on/off");
  m.def("gemm_configs", &gemm_configs, "[(id, BM, BN, threads, stages, BK)] of the GEMM tiles");
  m.def("attention_fwd", &attention_fwd, "fused MHSA forward on qkv rows -> (out, lse2)");
  m.def("attention_bwd", &attention_bwd, "fused MHSA backward -> dqkv (qkv layout)");
  m.def("attention_max_tokens", &dmp::attention_max_tokens, "max sequence length of the fused path");
  m.def("gelu_fwd", &gelu_fwd, "tanh-GELU forward");
  m.def("gelu_bwd", &gelu_bwd, "tanh-GELU backward");
  m.def("softmax_fwd", &softmax_fwd, "scaled row softmax forward");
  m.def("softmax_bwd", &softmax_bwd, "scaled row softmax backward");
  m.def("dropout_fwd", &dropout_fwd, "Philox dropout forward -> (y, keep mask)");
  m.def("dropout_bwd", &dropout_bwd, "dropout backward from the saved keep mask");
  m.def("gap_fwd", &gap_fwd, "NHWC global average pool forward");
  m.def("gap_linear_fwd", &gap_linear_fwd, "fused NHWC global average pool + Linear forward",
        py::arg("x"), py::arg("w"), py::arg("bias") = py::none());
  m.def("gap_linear_bwd", &gap_linear_bwd, "fused GAP + Linear backward (dx, dW +=, db +=)",
        py::arg("dy"), py::arg("f"), py::arg("w"), py::arg("gw"), py::arg("gb") = py::none(),
        py::arg("H"), py::arg("W"));
  m.def("gap_linear_supported",
        [](int64_t C, int64_t N) { return dmp::gap_linear_supported((int)C, (int)N); },
        "fused GAP + Linear head applies to C channels / N classes");
  m.def("gap_bwd", &gap_bwd, "NHWC global average pool backward");
  m.def("maxpool_fwd", &maxpool_fwd, "NHWC KxK / stride S / pad P max pool forward",
        py::arg("x"), py::arg("K"), py::arg("S") = -1, py::arg("P") = 0,
        py::arg("nchw_out") = false, py::arg("relu_in") = false);
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC KxK / stride S / pad P max pool backward",
        py::arg("dy"), py::arg("idx"), py::arg("H"), py::arg("W"), py::arg("K"),
        py::arg("S") = -1, py::arg("P") = 0);
  m.attr("arch") = "gfx950";
}
