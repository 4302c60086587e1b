// Host-side launch entry points of the gfx950 kernels (raw pointers + stream).
#pragma once
#include <hip/hip_runtime_api.h>

#include "bn_slots.h"
#include <stdint.h>

namespace dmp {

// optim.hip
void launch_asgd_fused_step(const float* g, float* p, float* acc, float* mom, uint16_t* w16,
                            long long n, float lr, float wd, float momentum, float dampening,
                            bool nesterov, hipStream_t s);
void launch_ps_apply_atomic(float* shard, const void* delta, bool bf16, long long n, float scale,
                            hipStream_t s);
void launch_ps_apply_f32(float* shard, const float* delta, uint16_t* mirror, long long n,
                         float scale, hipStream_t s);
void launch_ps_apply_bf16(float* shard, const uint16_t* delta, uint16_t* mirror, long long n,
                          float scale, hipStream_t s);
void launch_ps_count(int* cnt, int add, bool set, hipStream_t s);
void launch_ps_stamp(int* cnt, float* dst, hipStream_t s);
void launch_pull_land_f32(float* p, const float* src, const float* acc, uint16_t* w16,
                          long long n, hipStream_t s);
void launch_pull_land_bf16(float* p, const uint16_t* src, const float* acc, uint16_t* w16,
                           long long n, hipStream_t s);
void launch_push_handoff(float* acc, float* out32, uint16_t* out16, long long n, hipStream_t s);
void launch_cast_f32_bf16(const float* src, uint16_t* dst, long long n, hipStream_t s);
int launch_sumsq_partial(const float* x, float* partial, long long n, hipStream_t s);
void launch_zero_fill(void* p, long long bytes, hipStream_t s);

// xent.hip
void launch_softmax_xent_bf16(const uint16_t* logits, const int64_t* labels, uint16_t* dlogits,
                              float* row_loss, int* row_hit, float* loss_out, int* hits_out,
                              int B, int C, float grad_scale, float smoothing, int ignore_index,
                              hipStream_t s);
void launch_softmax_xent_f32(const float* logits, const int64_t* labels, float* dlogits,
                             float* row_loss, int* row_hit, float* loss_out, int* hits_out, int B,
                             int C, float grad_scale, float smoothing, int ignore_index,
                             hipStream_t s);

// bn.hip
int bn_num_partials(long long M, int C);
// inference-time BN folding into the producing conv (bn.hip): w16 = bf16(w * s),
// b32 / b16 (either may be null) = beta + (conv_bias - running_mean) * s, per output channel
// s = gamma / sqrt(running_var + eps); w is the fp32 [CO][...] master
void launch_bn_fold_weights(const float* w, const float* gamma, const float* beta,
                            const float* rmean, const float* rvar, const float* cbias,
                            uint16_t* w16, float* b32, uint16_t* b16, long long n, int CO,
                            float eps, hipStream_t s);
void launch_bn_fwd(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* gamma,
                   const float* beta, float* running_mean, float* running_var, float* stats,
                   float* part, long long M, int C, float momentum, float eps, bool training,
                   bool relu, hipStream_t s, uint8_t* mask = nullptr);
void launch_bn_bwd_from_partials(const uint16_t* x, const uint16_t* dz, const float* gamma,
                                 const float* stats, float* dgamma, float* dbeta, float* coef,
                                 float* part, uint16_t* dx, long long M, int C, hipStream_t s);
// finalize folded into the apply passes (zero_buf: the other direction's slots)
void launch_bn_fwd_fold(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, float* stats,
                        float* part, float* zero_buf, long long M, int C, float momentum,
                        float eps, bool relu, bool have_partials, hipStream_t s, uint8_t* mask);
void launch_bn_bwd_fold(const uint16_t* x, const uint16_t* dy, const uint16_t* y,
                        const float* gamma, const float* stats, float* dgamma, float* dbeta,
                        float* part, float* zero_buf, uint16_t* dx, uint16_t* dres, long long M,
                        int C, bool relu, hipStream_t s, const uint8_t* mask,
                        float* coef = nullptr);   // [3][C] scratch: one-pass kernel (bn.hip)
// BN + ReLU + max pool 3x3/s2/p1 fused (ImageNet ResNet stem), folded finalize
bool bn_maxpool_supported(int C, int K, int S, int P);
void launch_bn_relu_maxpool_fold(const uint16_t* x, uint16_t* y, uint8_t* idx, uint16_t* xm,
                                 const float* gamma,
                                 const float* beta, float* running_mean, float* running_var,
                                 float* stats, float* part, float* zero_buf, int N, int H, int W,
                                 int C, float momentum, float eps, bool have_partials,
                                 hipStream_t s);
void launch_maxpool_bn_bwd_fold(const uint16_t* x, const uint16_t* dp, const uint8_t* idx,
                                const uint16_t* xm, const float* gamma, const float* stats, float* dgamma,
                                float* dbeta, float* part, float* zero_buf, uint16_t* dx, int N,
                                int H, int W, int C, hipStream_t s);
void launch_bn_bwd(const uint16_t* x, const uint16_t* dy, const uint16_t* y, const float* gamma,
                   const float* stats, float* dgamma, float* dbeta, float* coef, float* part,
                   uint16_t* dx, uint16_t* dres, long long M, int C, bool relu, hipStream_t s,
                   const uint8_t* mask = nullptr);

// pool.hip
void launch_gap_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s);
void launch_gap_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s);
// fused global-average-pool + Linear head (csrc/head.hip)
bool gap_linear_supported(int C, int N);
void launch_gap_linear_fwd(const uint16_t* x, const uint16_t* w, const uint16_t* bias, uint16_t* y,
                           uint16_t* f, int B, int HW, int C, int N, hipStream_t s);
void launch_gap_linear_bwd(const uint16_t* dy, const uint16_t* f, const uint16_t* w, uint16_t* dx,
                           float* gw, float* gb, int B, int HW, int C, int N, hipStream_t s);
int maxpool_out(int H, int K, int S, int P);
void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C,
                        int K, int S, int P, hipStream_t s, bool nchw_out = false,
                        bool relu_in = false);
void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H,
                        int W, int C, int K, int S, int P, hipStream_t s, bool nchw_dy = false);


// transformer.hip: LayerNorm / GELU / softmax (ViT)
bool layernorm_supported(int D);
int layernorm_num_slots();
// radd/hout: fused residual add (h = x + radd written to hout, LayerNorm of h)
void launch_layernorm_fwd(const uint16_t* x, const float* gamma, const float* beta, uint16_t* y,
                          float* mean, float* rstd, long long rows, int D, float eps,
                          hipStream_t s, const uint16_t* radd = nullptr, uint16_t* hout = nullptr);
// dadd: gradient added to dx (the residual stream's direct gradient)
void launch_layernorm_bwd(const uint16_t* x, const uint16_t* dy, const float* gamma,
                          const float* mean, const float* rstd, uint16_t* dx, float* dgamma,
                          float* dbeta, float* slots, long long rows, int D, hipStream_t s,
                          const uint16_t* dadd = nullptr);
void launch_gelu_fwd(const uint16_t* x, uint16_t* y, long long n, hipStream_t s);
void launch_gelu_bwd(const uint16_t* x, const uint16_t* dy, uint16_t* dx, long long n,
                     hipStream_t s);
int softmax_max_len();
void launch_softmax_fwd(const uint16_t* sc, uint16_t* p, long long rows, int L, float scale,
                        hipStream_t s);
void launch_softmax_bwd(const uint16_t* p, const uint16_t* dp, uint16_t* ds, long long rows, int L,
                        float scale, hipStream_t s);
void launch_vit_embed_fwd(const uint16_t* tok, const uint16_t* cls, const uint16_t* pos,
                          uint16_t* h, int B, int N, int D, hipStream_t s);
void launch_token_row_scatter(const uint16_t* g, uint16_t* out, int B, int N, int D, int tok,
                              hipStream_t s);
void launch_vit_embed_bwd(const uint16_t* dh, uint16_t* dtok, float* dpos, float* dcls, int B,
                          int N, int D, hipStream_t s);

// dropout.hip: Philox4x32-10 dropout
void launch_dropout_fwd_fused(const void* x, uint8_t* mask, void* y, bool bf16, long long n,
                              float p, int mode, long long inner, int C, unsigned long long seed,
                              long long* ctr, hipStream_t s);
void launch_dropout_mask(uint8_t* mask, long long nmask, float p, unsigned long long seed,
                         const long long* offset, hipStream_t s);
void launch_dropout_apply_bf16(const uint16_t* x, const uint8_t* mask, uint16_t* y, long long n,
                               float scale, int mode, long long inner, int C, hipStream_t s);
void launch_dropout_apply_f32(const float* x, const uint8_t* mask, float* y, long long n,
                              float scale, int mode, long long inner, int C, hipStream_t s);

// conv.hip
int conv_num_configs();
void conv_config_info(int cfg, int* info);   // {BM, BN, BK, threads, stages}
int conv_default_config(long long M, int CO);
int conv_fwd_num_mblocks(long long M, int CO, int cfg);
// 3x3 / stride-1 halo-tile kernels: cfg ids conv_halo_base() + [0, conv_num_halo_configs())
int conv_num_halo_configs();
// 3x3 / stride-2 halo data-gradient tiles: cfg ids conv_dgrad_s2_base() + [0, num)
bool conv_dgrad_s2_ok(int cfg, int H, int W, int OH, int OW, int K, int N, int R, int S, int stride,
                      int pad);
int conv_dgrad_s2_base();
int conv_dgrad_s2_num_configs();
int conv_halo_base();
bool conv_halo_ok(int cfg, int H, int W, int C, int R, int S, int stride, int pad);
// 3x3 / stride-1 halo wgrad: cfg ids conv_wgrad_halo_base() + [0, conv_wgrad_num_halo_configs())
int conv_wgrad_halo_base();
int conv_wgrad_num_halo_configs();
bool conv_wgrad_halo_ok(int cfg, int B, int H, int W, int CI, int CO, int R, int S, int stride,
                        int pad);
// slab-mode halo wgrad ids: conv_wgrad_halo_slab_base() + the same [0, n) (plain-store
// split-K partials + a reduce pass); fp32 slab elements a cfg needs (0: none)
int conv_wgrad_halo_slab_base();
long long conv_wgrad_halo_slab_elems(int cfg, int B, int H, int W, int CI, int CO, int R, int S,
                                     int stride, int pad);
void launch_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int B, int H,
                     int W, int CI, int OH, int OW, int CO, int R, int S, int stride, int pad,
                     int cfg, hipStream_t s, const float* bias = nullptr, bool relu = false,
                     const uint16_t* addend = nullptr);
// Backward of the BatchNorm(+ReLU) that produced a conv's input, fused into the
// conv's data-gradient epilogue (conv.hip bnb_*): the dgrad stores dz and adds
// sum(dz), sum(dz * xhat) per channel into the BN's backward slot buffer.
struct BnBwdFuse {
  const uint16_t* x;     // BN input [B][H][W][C]
  const uint16_t* mask;  // relu 1: stored BN(+residual)+ReLU output (the conv input);
                         // relu 3: the BN's 1-bit ReLU mask (bytes)
  const float* stats;    // [4][C] mean | invstd | scale | shift
  float* part;           // [2][kBnSlots][C] (+tail) slot sums, zeroed
  int relu;              // 0 none, 1 / 3 mask from `mask`, 2 mask from x and scale/shift
};

void launch_conv_dgrad(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, int B, int H, int W,
                       int CI, int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                       hipStream_t s, const uint16_t* addend = nullptr,
                       const BnBwdFuse* bnf = nullptr, bool addend_sub = false,
                       const uint8_t* addend_mask = nullptr);
// x_sub = x[:, ::2, ::2, :] (NHWC bf16, C % 8 == 0), [B][ceil(H/2)][ceil(W/2)][C]
void launch_subsample2(const uint16_t* x, uint16_t* xs, int B, int H, int W, int C,
                       hipStream_t s);
// dx[:, ::2, ::2, :] += xs in place (NHWC bf16)
void launch_add_subsampled2(uint16_t* dx, const uint16_t* xs, int B, int H, int W, int C,
                            hipStream_t s);
void launch_conv_weight_transpose(const uint16_t* w, uint16_t* wt, int CO, int RS, int CI,
                                  hipStream_t s);
// dbias: optional fp32 [CO] += column sums of dY (gather kernel only; halo cfgs fall back)
void launch_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, int B, int H, int W,
                       int CI, int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                       hipStream_t s, float* dbias = nullptr, float* slab = nullptr);

// conv_small.hip: 3x3/s1/p1 stems with CI <= 3 and CO = 64 on MFMA
bool stem3_supported(int CI, int R, int S, int CO, int stride, int pad, int W);
void launch_stem3_fwd(const uint16_t* x, int xbytes, int sb, int sh, int sw, int sc,
                      const uint16_t* w, uint16_t* y, float* part, int B, int H, int W, int CI,
                      hipStream_t s);
void launch_stem3_wgrad(const uint16_t* dy, const uint16_t* x, int xbytes, int sb, int sh, int sw,
                        int sc, float* dw, int B, int H, int W, int CI, hipStream_t s);
// conv_small.hip: few-input-channel (stem) convolutions, VALU
int conv_small_max_k();
long long conv_small_fwd_blocks(long long P);
void launch_conv_small_fwd(const uint16_t* x, int xbytes, int sb, int sh, int sw, int sc, const uint16_t* w,
                           uint16_t* y, float* part, int B, int H, int W, int CI, int OH, int OW,
                           int CO, int R, int S, int stride, int pad, hipStream_t s);
int conv_small_wgrad_blocks(long long P, int CO, int R, int S, int CI);
// ws: scratch of conv_small_wgrad_blocks(...) * CO * R*S*CI floats
void launch_conv_small_wgrad(const uint16_t* dy, const uint16_t* x, int xbytes, int sb, int sh, int sw, int sc,
                             float* dw, float* ws, int B, int H, int W, int CI, int OH, int OW,
                             int CO, int R, int S, int stride, int pad, hipStream_t s);

// attention.hip: fused MHSA on [B, N, 3, H, 64] qkv rows (ViT)
int attention_max_tokens();
int attention_head_dim();
void launch_attention_fwd(const uint16_t* qkv, uint16_t* out, float* lse2, int B, int N, int H,
                          float scale, hipStream_t s);
void launch_attention_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout,
                          const float* lse2, uint16_t* dqkv, int B, int N, int H, float scale,
                          hipStream_t s);

// linear.hip: bias gradient out[n] += sum_m dy[m][n] (bf16 dy, fp32 out)
int colsum_num_slots();
void launch_colsum_acc(const uint16_t* dy, float* out, float* slots, long long M, int N,
                       hipStream_t s);

// bn.hip: BN forward from conv-epilogue slot sums (finalize + apply)
void launch_bn_fwd_partials(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            float* stats, float* part, long long M, int C,
                            float momentum, float eps, bool relu, hipStream_t s,
                            uint8_t* mask = nullptr);

// gemm.hip: bf16 MFMA GEMM for linear layers.  mode 0 fwd C = A B^T (A [M][K],
// B [N][K]); mode 1 dgrad (A [M][K], B [K][N]); mode 2 wgrad, fp32 C += (A [K][M],
// B [K][N]), split-K over `splits`.  epi: 0 store (+bias, +aux addend),
// 1 GELU (c = h, c2 = gelu(h)), 2 c = acc * gelu'(aux), 3 fp32 accumulate
// (+ dbias row sums).  cfg -1: any-shape fallback kernel.
int gemm_num_configs();
bool gemm_config_ok(int mode, int cfg);   // tile shape usable for this pass
void gemm_config_info(int cfg, int* info);   // {BM, BN, threads, stages, BK}
// split-major XCD deal of the weight-gradient split-K (DMP_GEMM_XCD_K, default on)
void gemm_set_xcd_k(int on);
void launch_gemm(int mode, int epi, int cfg, const uint16_t* a, int lda, const uint16_t* b,
                 int ldb, void* c, int ldc, uint16_t* c2, const uint16_t* bias,
                 const uint16_t* aux, float* dbias, int M, int N, int K, int splits,
                 hipStream_t s, bool relu = false, float* part = nullptr,
                 float* slab = nullptr, float* sk_ws = nullptr, int* sk_cnt = nullptr,
                 const uint8_t* auxmask = nullptr);
// remainder split-K of a fwd / dgrad launch_gemm (splits > 1): fp32 workspace
// floats and ticket counters it needs for (cfg, M, N, K, splits); 0 = not split
void gemm_sk_sizes(int cfg, int M, int N, int K, int splits, long long* ws_floats, int* counters);
// effective split-K count of launch_gemm (mode 2) for K and a requested count
int gemm_effective_splits(int K, int splits);

// im2col.hip: patch matrix [B*OH*OW][Kp] (k = (r, s, ci), zero-padded) and its
// gather-form inverse; ReLU backward from the saved output
void launch_im2col(const uint16_t* x, uint16_t* cols, int B, int H, int W, int CI, int OH, int OW,
                   int R, int S, int stride, int pad, int K, int Kp, hipStream_t st);
void launch_col2im(const uint16_t* dcols, uint16_t* dx, int B, int H, int W, int CI, int OH,
                   int OW, int R, int S, int stride, int pad, int Kp, hipStream_t st);
void launch_pad_rows_batched(const uint16_t* src, uint16_t* dst, const long long* table, int n,
                             long long max_elems, hipStream_t st);
void launch_relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long long n,
                     hipStream_t st);

// conv.hip: every conv weight of a flat bf16 shadow transposed in one launch
void launch_conv_weight_transpose_batched(const uint16_t* src, uint16_t* dst,
                                          const long long* table, int n, long long max_elems,
                                          hipStream_t s);
// stem.hip: ImageNet 7x7/2/3 stem (3 -> 64) as a 4x4 conv over a space-to-depth image
bool stem_supported(int H, int W);
void launch_stem_s2d(const uint16_t* x, uint16_t* xs, int B, int H, int W, hipStream_t s);
void launch_stem_wpack(const uint16_t* w, uint16_t* wp, hipStream_t s);
void launch_stem_wfold(const float* dwp, float* dw, hipStream_t s);
void launch_stem_fwd(const uint16_t* xs, const uint16_t* wp, uint16_t* y, float* part, int B,
                     int H, int W, hipStream_t s, const float* bias = nullptr, bool relu = false);
void launch_stem_wgrad(const uint16_t* dy, const uint16_t* xs, float* dwp, int B, int H, int W,
                       hipStream_t s);

}  // namespace dmp
