// Fused multi-head self-attention for ViT (BASELINE.json config #5, ViT-B/16:
// N = 197 tokens, head dim 64), forward and backward, on gfx950 MFMA
// (v_mfma_f32_16x16x32_bf16).  Not in the reference (no sequence models,
// SURVEY §5.7).
//
// Layout: the qkv projection output is consumed as is, [B, N, 3, H, 64] bf16
// (= the [B*N, 3D] rows of the qkv Linear), the output is written as
// [B, N, H, 64] (= the [B*N, D] input rows of the proj Linear) and the
// backward writes dqkv in the qkv layout: no permute / contiguous copies, no
// zero-filled select-backward buffers, no gradient adds, no materialised
// [B, H, N, N] scores.  One workgroup per (batch, head): the whole key/value
// (or query/dO) set of a head, <= 256 tokens, is staged once in LDS.
//
// MFMA 16x16x32 fragments (lane l, g = l / 16, l16 = l % 16):
//   A (16 x 32): row l16, k = 8g .. 8g+7        B (32 x 16): col l16, k = 8g .. 8g+7
//   D (16 x 16): col l16, rows 4g .. 4g+3 (4 VGPRs)
// A D tile whose ROW index is a reduction index of the next product feeds that
// product directly: two adjacent 16-row D blocks, packed {block0[0..3],
// block1[0..3]}, are the 8 k-values {4g..4g+3, 16+4g..16+4g+3} of a 32-deep
// k-step; the other operand is read from a transposed LDS tile with the same
// k permutation (two 8-B reads).  So every product runs on registers + LDS
// with no shuffles:
//   forward  (query strips):  S^T = K Q^T  ->  softmax  ->  O^T = V^T P^T
//   dQ       (query strips):  S^T, dP^T = V dO^T  ->  dS^T  ->  dQ^T = K^T dS^T
//   dK, dV   (key strips):    S = Q K^T, dP = dO V^T -> dS -> dV^T = dO^T P,
//                             dK^T = Q^T dS
// and every output tile is written as 4 consecutive head-dim values per lane
// (8-B stores).  Softmax statistics are saved as a base-2 log-sum-exp of the
// scaled scores (lse2), so P = exp2(s * scale * log2e - lse2) in the backward.
#include "common.h"

namespace dmp {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kDH = 64;          // head dim
constexpr int kRS = kDH + 8;     // row stride (elements) of row-major [token][64] LDS tiles
constexpr int kMaxKB = 16;       // <= 256 tokens: 16 blocks of 16
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[i] = f2bf(lo[i]);
    r.v[4 + i] = f2bf(hi[i]);
  }
  return r;
}

// k-permuted operand from a transposed tile: 4 values at p, 4 at p + 16
__device__ __forceinline__ bf16x8 ld_perm(const u16* p) {
  bf16x8 r;
  *reinterpret_cast<uint2*>(&r.v[0]) = *reinterpret_cast<const uint2*>(p);
  *reinterpret_cast<uint2*>(&r.v[4]) = *reinterpret_cast<const uint2*>(p + 16);
  return r;
}

__device__ __forceinline__ bf16x8 ld16(const u16* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ void st4(u16* p, const f32x4& v, float s) {
  uint2 w;
  w.x = (u32)f2bf(v[0] * s) | ((u32)f2bf(v[1] * s) << 16);
  w.y = (u32)f2bf(v[2] * s) | ((u32)f2bf(v[3] * s) << 16);
  *reinterpret_cast<uint2*>(p) = w;
}

// Stage token rows [0, NP) of one head's slice t (0 q, 1 k, 2 v) of a
// [B, N, 3, H, 64] tensor (or of a [B, N, H, 64] one with t = -1) into LDS:
// row-major (stride kRS) and/or transposed (stride TS).  Rows >= N are zero.
template <int NT>
__device__ __forceinline__ void stage_head(const u16* __restrict__ src, long long tok0, int N,
                                           int NP, int rowstride, u16* rm, u16* tr, int TS) {
  for (int i = threadIdx.x; i < NP * 8; i += NT) {
    const int n = i >> 3, c = i & 7;
    bf16x8 v;
    if (n < N) {
      v = ld16(src + (tok0 + n) * rowstride + c * 8);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v.v[k] = 0;
    }
    if (rm) *reinterpret_cast<bf16x8*>(rm + n * kRS + c * 8) = v;
    if (tr) {
#pragma unroll
      for (int k = 0; k < 8; ++k) tr[(c * 8 + k) * TS + n] = v.v[k];
    }
  }
}

}  // namespace

// ----------------------------------------------------------------- forward
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_fwd_kernel(const u16* __restrict__ qkv,
                                                          u16* __restrict__ out,
                                                          float* __restrict__ lse2, int N, int H,
                                                          float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int NP = (N + 31) & ~31, TS = NP + 8, D = H * kDH;
  u16* Ks = smem;              // [NP][kRS]
  u16* Vt = smem + NP * kRS;   // [64][TS]
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const long long tok0 = (long long)b * N;
  const u16* base = qkv + h * kDH;
  stage_head<64 * NW>(base + D, tok0, N, NP, 3 * D, Ks, nullptr, TS);
  stage_head<64 * NW>(base + 2 * D, tok0, N, NP, 3 * D, nullptr, Vt, TS);
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  const int nkb = NP / 16, nstrips = (N + 15) / 16;
  for (int qs = wid; qs < nstrips; qs += NW) {
    const int q = qs * 16 + l16, qc = q < N ? q : N - 1;
    const u16* qrow = base + (tok0 + qc) * 3 * D;
    const bf16x8 qf0 = ld16(qrow + 8 * g), qf1 = ld16(qrow + 32 + 8 * g);
    f32x4 s[kMaxKB];
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < kMaxKB; ++kb) {
      if (kb < nkb) {
        const u16* kr = Ks + (kb * 16 + l16) * kRS + 8 * g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = mfma(ld16(kr), qf0, acc);
        acc = mfma(ld16(kr + 32), qf1, acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (kb * 16 + 4 * g + r) < N ? acc[r] * scale_log2 : -INFINITY;
          s[kb][r] = v;
          mx = fmaxf(mx, v);
        }
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < kMaxKB; ++kb) {
      if (kb < nkb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kb][r] = exp2f(s[kb][r] - mx);
          sum += s[kb][r];
        }
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    f32x4 o[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp = 0; kp < kMaxKB / 2; ++kp) {
      if (2 * kp < nkb) {
        const bf16x8 pb = pack8(s[2 * kp], s[2 * kp + 1]);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          o[nb] = mfma(ld_perm(Vt + (nb * 16 + l16) * TS + 32 * kp + 4 * g), pb, o[nb]);
      }
    }
    if (q < N) {
      const float inv = 1.f / sum;
      u16* orow = out + (tok0 + q) * D + h * kDH + 4 * g;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) st4(orow + nb * 16, o[nb], inv);
      if (g == 0) lse2[(long long)bh * N + q] = mx + log2f(sum);
    }
  }
}

// ------------------------------------------------------------- backward: dQ
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dq_kernel(
    const u16* __restrict__ qkv, const u16* __restrict__ out, const u16* __restrict__ dout,
    const float* __restrict__ lse2, u16* __restrict__ dqkv, int N, int H, float scale_log2,
    float scale) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int NP = (N + 31) & ~31, TS = NP + 8, D = H * kDH;
  u16* Ks = smem;                   // [NP][kRS]
  u16* Vs = Ks + NP * kRS;          // [NP][kRS]
  u16* Kt = Vs + NP * kRS;          // [64][TS]
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const long long tok0 = (long long)b * N;
  const u16* base = qkv + h * kDH;
  stage_head<64 * NW>(base + D, tok0, N, NP, 3 * D, Ks, Kt, TS);
  stage_head<64 * NW>(base + 2 * D, tok0, N, NP, 3 * D, Vs, nullptr, TS);
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  const int nkb = NP / 16, nstrips = (N + 15) / 16;
  for (int qs = wid; qs < nstrips; qs += NW) {
    const int q = qs * 16 + l16, qc = q < N ? q : N - 1;
    const u16* qrow = base + (tok0 + qc) * 3 * D;
    const u16* orow = out + (tok0 + qc) * D + h * kDH;
    const u16* drow = dout + (tok0 + qc) * D + h * kDH;
    const bf16x8 qf0 = ld16(qrow + 8 * g), qf1 = ld16(qrow + 32 + 8 * g);
    const bf16x8 df0 = ld16(drow + 8 * g), df1 = ld16(drow + 32 + 8 * g);
    const bf16x8 of0 = ld16(orow + 8 * g), of1 = ld16(orow + 32 + 8 * g);
    float di = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      di += bf2f(df0.v[k]) * bf2f(of0.v[k]) + bf2f(df1.v[k]) * bf2f(of1.v[k]);
    di += __shfl_xor(di, 16, 64);
    di += __shfl_xor(di, 32, 64);
    const float L = lse2[(long long)bh * N + qc];
    f32x4 dq[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) dq[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp = 0; kp < kMaxKB / 2; ++kp) {
      if (2 * kp < nkb) {
        f32x4 ds[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int kb = 2 * kp + hf;
          const u16* kr = Ks + (kb * 16 + l16) * kRS + 8 * g;
          const u16* vr = Vs + (kb * 16 + l16) * kRS + 8 * g;
          f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
          st = mfma(ld16(kr), qf0, st);
          st = mfma(ld16(kr + 32), qf1, st);
          dp = mfma(ld16(vr), df0, dp);
          dp = mfma(ld16(vr + 32), df1, dp);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = (kb * 16 + 4 * g + r) < N ? exp2f(st[r] * scale_log2 - L) : 0.f;
            ds[hf][r] = p * (dp[r] - di);
          }
        }
        const bf16x8 db = pack8(ds[0], ds[1]);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          dq[nb] = mfma(ld_perm(Kt + (nb * 16 + l16) * TS + 32 * kp + 4 * g), db, dq[nb]);
      }
    }
    if (q < N) {
      u16* dst = dqkv + (tok0 + q) * 3 * D + h * kDH + 4 * g;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) st4(dst + nb * 16, dq[nb], scale);
    }
  }
}

// --------------------------------------------------------- backward: dK, dV
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dkv_kernel(
    const u16* __restrict__ qkv, const u16* __restrict__ out, const u16* __restrict__ dout,
    const float* __restrict__ lse2, u16* __restrict__ dqkv, int N, int H, float scale_log2,
    float scale) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int NP = (N + 31) & ~31, TS = NP + 8, D = H * kDH;
  u16* Qs = smem;                   // [NP][kRS]
  u16* Ds = Qs + NP * kRS;          // dO [NP][kRS]
  u16* Qt = Ds + NP * kRS;          // [64][TS]
  u16* Dt = Qt + kDH * TS;          // dO^T [64][TS]
  float* Ls = reinterpret_cast<float*>(Dt + kDH * TS);   // [NP] lse2 (+inf past N)
  float* Di = Ls + NP;                                   // [NP] rowsum(dO * O)
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const long long tok0 = (long long)b * N;
  const u16* base = qkv + h * kDH;
  stage_head<64 * NW>(base, tok0, N, NP, 3 * D, Qs, Qt, TS);
  stage_head<64 * NW>(dout + h * kDH, tok0, N, NP, D, Ds, Dt, TS);
  // Di[q] = dO[q] . O[q]: 8 threads per row, 8 elements each
  for (int i = threadIdx.x; i < NP * 8; i += 64 * NW) {
    const int n = i >> 3, c = i & 7;
    float d = 0.f;
    if (n < N) {
      const bf16x8 ov = ld16(out + (tok0 + n) * D + h * kDH + c * 8);
      const bf16x8 dv = ld16(dout + (tok0 + n) * D + h * kDH + c * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) d += bf2f(ov.v[k]) * bf2f(dv.v[k]);
    }
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    if (c == 0) {
      Di[n] = d;
      Ls[n] = n < N ? lse2[(long long)bh * N + n] : INFINITY;
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  const int nqb = NP / 16, nstrips = (N + 15) / 16;
  for (int ks = wid; ks < nstrips; ks += NW) {
    const int key = ks * 16 + l16, kc = key < N ? key : N - 1;
    const u16* krow = base + (tok0 + kc) * 3 * D + D;
    const bf16x8 kf0 = ld16(krow + 8 * g), kf1 = ld16(krow + 32 + 8 * g);
    const bf16x8 vf0 = ld16(krow + D + 8 * g), vf1 = ld16(krow + D + 32 + 8 * g);
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      dk[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int qp = 0; qp < kMaxKB / 2; ++qp) {
      if (2 * qp < nqb) {
        f32x4 pp[2], ds[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int qb = 2 * qp + hf;
          const u16* qr = Qs + (qb * 16 + l16) * kRS + 8 * g;
          const u16* dr = Ds + (qb * 16 + l16) * kRS + 8 * g;
          f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
          s = mfma(ld16(qr), kf0, s);
          s = mfma(ld16(qr + 32), kf1, s);
          dp = mfma(ld16(dr), vf0, dp);
          dp = mfma(ld16(dr + 32), vf1, dp);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qq = qb * 16 + 4 * g + r;
            const float p = exp2f(s[r] * scale_log2 - Ls[qq]);
            pp[hf][r] = p;
            ds[hf][r] = p * (dp[r] - Di[qq]);
          }
        }
        const bf16x8 pb = pack8(pp[0], pp[1]), db = pack8(ds[0], ds[1]);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int off = (nb * 16 + l16) * TS + 32 * qp + 4 * g;
          dv[nb] = mfma(ld_perm(Dt + off), pb, dv[nb]);
          dk[nb] = mfma(ld_perm(Qt + off), db, dk[nb]);
        }
      }
    }
    if (key < N) {
      u16* dst = dqkv + (tok0 + key) * 3 * D + h * kDH + 4 * g;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        st4(dst + D + nb * 16, dk[nb], scale);
        st4(dst + 2 * D + nb * 16, dv[nb], 1.f);
      }
    }
  }
}

// ---------------------------------------------------------------- launchers
int attention_max_tokens() { return 16 * kMaxKB; }
int attention_head_dim() { return kDH; }

namespace {
constexpr int kFwdWaves = 4, kBwdWaves = 8;
size_t fwd_lds(int N) {
  const int NP = (N + 31) & ~31;
  return ((size_t)NP * kRS + (size_t)kDH * (NP + 8)) * 2;
}
size_t dq_lds(int N) {
  const int NP = (N + 31) & ~31;
  return ((size_t)2 * NP * kRS + (size_t)kDH * (NP + 8)) * 2;
}
size_t dkv_lds(int N) {
  const int NP = (N + 31) & ~31;
  return ((size_t)2 * NP * kRS + (size_t)2 * kDH * (NP + 8)) * 2 + (size_t)2 * NP * 4;
}
template <typename K>
void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
}  // namespace

void launch_attention_fwd(const u16* qkv, u16* out, float* lse2, int B, int N, int H, float scale,
                          hipStream_t s) {
  const size_t lds = fwd_lds(N);
  allow_lds(attn_fwd_kernel<kFwdWaves>, lds);
  hipLaunchKernelGGL(attn_fwd_kernel<kFwdWaves>, dim3(B * H), dim3(64 * kFwdWaves), lds, s, qkv,
                     out, lse2, N, H, scale * 1.4426950408889634f);
}

void launch_attention_bwd(const u16* qkv, const u16* out, const u16* dout, const float* lse2,
                          u16* dqkv, int B, int N, int H, float scale, hipStream_t s) {
  const float sl2 = scale * 1.4426950408889634f;
  const size_t l1 = dkv_lds(N), l2 = dq_lds(N);
  allow_lds(attn_bwd_dkv_kernel<kBwdWaves>, l1);
  allow_lds(attn_bwd_dq_kernel<kBwdWaves>, l2);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<kBwdWaves>, dim3(B * H), dim3(64 * kBwdWaves), l1, s, qkv,
                     out, dout, lse2, dqkv, N, H, sl2, scale);
  hipLaunchKernelGGL(attn_bwd_dq_kernel<kBwdWaves>, dim3(B * H), dim3(64 * kBwdWaves), l2, s, qkv,
                     out, dout, lse2, dqkv, N, H, sl2, scale);
}

}  // namespace dmp
