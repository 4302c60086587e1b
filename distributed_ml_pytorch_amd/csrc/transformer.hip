// Transformer-block kernels for ViT-B/16 (BASELINE.json config #5): LayerNorm
// fwd/bwd, tanh-GELU fwd/bwd and the scaled row softmax fwd/bwd of attention.
// Not in the reference (it has no sequence models); SURVEY §2.3
// lists them as the kernels the ViT target needs.  The attention / MLP GEMMs
// themselves are plain library GEMMs (hipBLASLt through torch.matmul).
//
// Layout: rows of length D (tokens x channels for LayerNorm / GELU, query rows
// of scores for softmax), bf16 storage, fp32 math.  One wave64 per row: each
// lane owns 8-element (16 B) chunks lane, lane+64, ... kept in registers
// between the reduction and the normalisation, so a row is read once.
#include <cstdlib>

#include "common.h"

namespace dmp {

__device__ __forceinline__ void ld8(const u16* p, float v[8]) {
  const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = bf2f(r.v[k]);
}
__device__ __forceinline__ void st8(u16* p, const float v[8]) {
  bf16x8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = f2bf(v[k]);
  *reinterpret_cast<bf16x8*>(p) = r;
}

// ------------------------------------------------------------------ LayerNorm
// A row of D = LR * nc * 8 elements is owned by LR consecutive lanes (a
// power of two <= 64 that divides D / 8), each holding nc <= MAXC 16-B chunks
// in registers: 64 / LR rows per wave, every lane busy (D = 768: 32 lanes x 3
// chunks, 2 rows per wave).  Reductions are LR-lane butterflies.
template <int LR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void ld8f(const float* p, float v[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// y = (x - mean) * rstd * gamma + beta; saves mean, rstd (fp32 per row).
// With radd: the residual add of a pre-norm transformer block is fused in --
// h = bf16(x + radd) is written to hout and normalised (one pass over the
// stream instead of an add kernel plus a LayerNorm read).
template <int LR, int MAXC>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(
    const u16* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    u16* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out, long long rows,
    int D, float eps, const u16* __restrict__ radd, u16* __restrict__ hout) {
  constexpr int RPW = 64 / LR;
  const int lane = threadIdx.x & 63, sub = lane % LR;
  const long long row = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LR;
  const int nc = D / (8 * LR);
  const bool ok = row < rows;
  const u16* xr = x + (ok ? row : 0) * D;
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < nc) {
      ld8(xr + (sub + c * LR) * 8, v[c]);
      if (radd) {
        float t[8];
        ld8(radd + (ok ? row : 0) * D + (sub + c * LR) * 8, t);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[c][k] = bf2f(f2bf(v[c][k] + t[k]));
        if (ok) st8(hout + row * D + (sub + c * LR) * 8, v[c]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[c][k];
    }
  }
  const float invD = 1.f / (float)D;
  const float mean = group_sum<LR>(s) * invD;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < nc) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[c][k] -= mean;
        q += v[c][k] * v[c][k];
      }
    }
  }
  const float rstd = rsqrtf(group_sum<LR>(q) * invD + eps);
  if (!ok) return;
  u16* yr = y + row * D;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < nc) {
      const int e0 = (sub + c * LR) * 8;
      float g[8], b[8], o[8];
      if (gamma) ld8f(gamma + e0, g);
      if (beta) ld8f(beta + e0, b);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        o[k] = v[c][k] * rstd * (gamma ? g[k] : 1.f) + (beta ? b[k] : 0.f);
      st8(yr + e0, o);
    }
  }
  if (sub == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) (+ dadd),  g = dy * gamma.
// dadd: the gradient reaching the residual-stream value h directly (fused
// add-LayerNorm), summed in fp32 before the single bf16 rounding.
// dgamma / dbeta: per-lane partials over the rows the wave visits, folded over
// the wave's row groups (butterfly) and the 4 waves (LDS), then added into
// slot blockIdx % kLnSlots of a persistent [kLnSlots][2][D] buffer (<= 32
// adders per address); layernorm_param_grad_kernel sums the slots into the
// fp32 grad arena and re-zeroes them.  (One atomic per column per block into a
// single row serialises at the memory-side atomic unit once ~1000 blocks add.)
constexpr int kLnSlots = 32;

template <int LR, int MAXC>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, u16* __restrict__ dx,
    float* __restrict__ slots, long long rows, int D, const u16* __restrict__ dadd) {
  constexpr int RPW = 64 / LR;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, sub = lane % LR;
  const int nc = D / (8 * LR);
  float pg[MAXC][8], pb[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) { pg[c][k] = 0.f; pb[c][k] = 0.f; }
  const long long step = (long long)gridDim.x * 4 * RPW;
  // software-pipelined over the wave's rows: the next row group's x / dy / dadd
  // (and mean / rstd) are in flight while this one is reduced and stored
  bf16x8 nx[MAXC], ny[MAXC], na[MAXC];
  float nmean = 0.f, nrstd = 0.f;
  auto fetch = [&](long long row) {
    const long long r = row < rows ? row : 0;
    nmean = mean_in[r];
    nrstd = rstd_in[r];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < nc) {
        const int e0 = (sub + c * LR) * 8;
        nx[c] = *reinterpret_cast<const bf16x8*>(x + r * D + e0);
        ny[c] = *reinterpret_cast<const bf16x8*>(dy + r * D + e0);
        if (dadd) na[c] = *reinterpret_cast<const bf16x8*>(dadd + r * D + e0);
      }
    }
  };
  long long row = ((long long)blockIdx.x * 4 + wid) * RPW + lane / LR;
  if (row - lane / LR < rows) fetch(row);
  for (; row - lane / LR < rows; row += step) {
    const bool ok = row < rows;
    const long long r = ok ? row : 0;
    const float mean = nmean, rstd = nrstd;
    bf16x8 cx[MAXC], cy[MAXC], ad[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) { cx[c] = nx[c]; cy[c] = ny[c]; ad[c] = na[c]; }
    if (row + step - lane / LR < rows) fetch(row + step);
    float xh[MAXC][8], dv[MAXC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < nc) {
        const int e0 = (sub + c * LR) * 8;
        float gm[8];
        if (gamma) ld8f(gamma + e0, gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[c][k] = bf2f(cx[c].v[k]);
          dv[c][k] = ok ? bf2f(cy[c].v[k]) : 0.f;
          xh[c][k] = (xh[c][k] - mean) * rstd;
          const float g = dv[c][k] * (gamma ? gm[k] : 1.f);
          s1 += g;
          s2 += g * xh[c][k];
          pg[c][k] += dv[c][k] * xh[c][k];
          pb[c][k] += dv[c][k];
        }
      }
    }
    const float invD = 1.f / (float)D;
    const float m1 = group_sum<LR>(s1) * invD, m2 = group_sum<LR>(s2) * invD;
    if (ok) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < nc) {
          const int e0 = (sub + c * LR) * 8;
          float gm[8], o[8];
          if (gamma) ld8f(gamma + e0, gm);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            o[k] = rstd * (dv[c][k] * (gamma ? gm[k] : 1.f) - m1 - xh[c][k] * m2);
          if (dadd) {
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] += bf2f(ad[c].v[k]);
          }
          st8(dx + r * D + e0, o);
        }
      }
    }
  }
  if (slots == nullptr) return;
  // fold the RPW row groups of the wave (lanes sub, sub + LR, ...)
#pragma unroll
  for (int o = LR; o < 64; o <<= 1) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        pg[c][k] += __shfl_xor(pg[c][k], o, 64);
        pb[c][k] += __shfl_xor(pb[c][k], o, 64);
      }
  }
  extern __shared__ float red[];   // [4][2][D]
  if (lane < LR) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < nc) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int e = (sub + c * LR) * 8 + k;
          red[(wid * 2 + 0) * D + e] = pg[c][k];
          red[(wid * 2 + 1) * D + e] = pb[c][k];
        }
      }
    }
  }
  __syncthreads();
  float* out = slots + (long long)(blockIdx.x % kLnSlots) * 2 * D;
  for (int e = threadIdx.x; e < 2 * D; e += 256) {
    const float v = red[e] + red[2 * D + e] + red[4 * D + e] + red[6 * D + e];
    atomicAdd(out + e, v);
  }
}

// dgamma[d] += sum_s slots[s][0][d], dbeta[d] += sum_s slots[s][1][d]; slots re-zeroed
__global__ void __launch_bounds__(256) layernorm_param_grad_kernel(float* __restrict__ slots,
                                                                   float* __restrict__ dgamma,
                                                                   float* __restrict__ dbeta,
                                                                   int D) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * D) return;
  float acc = 0.f;
#pragma unroll 8
  for (int sl = 0; sl < kLnSlots; ++sl) {
    float* p = slots + (long long)sl * 2 * D + e;
    acc += *p;
    *p = 0.f;
  }
  float* dst = e < D ? dgamma : dbeta;
  if (dst) dst[e < D ? e : e - D] += acc;
}

// ----------------------------------------------------------------------- GELU
// (gelu_tanh / fast_tanh live in common.h: the GEMM epilogues share them)

__global__ void __launch_bounds__(256) gelu_fwd_kernel(const u16* __restrict__ x,
                                                       u16* __restrict__ y, long long nvec) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float a[8];
    ld8(x + v * 8, a);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = gelu_tanh(a[k], nullptr);
    st8(y + v * 8, a);
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const u16* __restrict__ x,
                                                       const u16* __restrict__ dy,
                                                       u16* __restrict__ dx, long long nvec) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float a[8], g[8];
    ld8(x + v * 8, a);
    ld8(dy + v * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float d;
      gelu_tanh(a[k], &d);
      a[k] = g[k] * d;
    }
    st8(dx + v * 8, a);
  }
}

// -------------------------------------------------------------------- softmax
// P = softmax(scale * S) along rows of length L (scalar loads: L = 197 is not a
// multiple of 8); one wave per row, values held in registers (L <= 64*MAXE)
template <int MAXE>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const u16* __restrict__ s,
                                                          u16* __restrict__ p, long long rows,
                                                          int L, float scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const u16* sr = s + row * L;
  float v[MAXE];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + e * 64;
    v[e] = j < L ? bf2f(sr[j]) * scale : -INFINITY;
    mx = fmaxf(mx, v[e]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    v[e] = (lane + e * 64) < L ? __expf(v[e] - mx) : 0.f;
    sum += v[e];
  }
  const float inv = 1.f / wave_sum(sum);
  u16* pr = p + row * L;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + e * 64;
    if (j < L) pr[j] = f2bf(v[e] * inv);
  }
}

// dS = scale * P * (dP - sum_j P_j dP_j)
template <int MAXE>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const u16* __restrict__ p,
                                                          const u16* __restrict__ dp,
                                                          u16* __restrict__ ds, long long rows,
                                                          int L, float scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float pv[MAXE], gv[MAXE];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + e * 64;
    pv[e] = j < L ? bf2f(p[row * L + j]) : 0.f;
    gv[e] = j < L ? bf2f(dp[row * L + j]) : 0.f;
    dot += pv[e] * gv[e];
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + e * 64;
    if (j < L) ds[row * L + j] = f2bf(scale * pv[e] * (gv[e] - dot));
  }
}

// ------------------------------------------------------------------ launchers
int layernorm_num_slots() { return kLnSlots; }

// lanes per row: the largest power of two <= 64 dividing D/8; chunks per lane <= 8
static int ln_lanes(int D) {
  const int nch = D / 8;
  int lr = 64;
  while (lr > 1 && nch % lr) lr >>= 1;
  while (lr > 1 && nch / lr < 1) lr >>= 1;
  return lr;
}

#define DMP_LN_LAUNCH(KERNEL, LR_, NC_, GRID, LDS, ...)                                         \
  do {                                                                                         \
    if ((NC_) <= 2) hipLaunchKernelGGL((KERNEL<LR_, 2>), GRID, dim3(256), LDS, s, __VA_ARGS__); \
    else if ((NC_) == 3) hipLaunchKernelGGL((KERNEL<LR_, 3>), GRID, dim3(256), LDS, s, __VA_ARGS__); \
    else if ((NC_) <= 4) hipLaunchKernelGGL((KERNEL<LR_, 4>), GRID, dim3(256), LDS, s, __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<LR_, 8>), GRID, dim3(256), LDS, s, __VA_ARGS__);            \
  } while (0)

#define DMP_LN_BY_LR(KERNEL, LR, NC, GRID, LDS, ...)                         \
  do {                                                                     \
    switch (LR) {                                                          \
      case 64: DMP_LN_LAUNCH(KERNEL, 64, NC, GRID, LDS, __VA_ARGS__); break; \
      case 32: DMP_LN_LAUNCH(KERNEL, 32, NC, GRID, LDS, __VA_ARGS__); break; \
      case 16: DMP_LN_LAUNCH(KERNEL, 16, NC, GRID, LDS, __VA_ARGS__); break; \
      case 8: DMP_LN_LAUNCH(KERNEL, 8, NC, GRID, LDS, __VA_ARGS__); break;   \
      case 4: DMP_LN_LAUNCH(KERNEL, 4, NC, GRID, LDS, __VA_ARGS__); break;   \
      case 2: DMP_LN_LAUNCH(KERNEL, 2, NC, GRID, LDS, __VA_ARGS__); break;   \
      default: DMP_LN_LAUNCH(KERNEL, 1, NC, GRID, LDS, __VA_ARGS__); break;  \
    }                                                                      \
  } while (0)

// D % 8 == 0 and at most 8 chunks of 8 per lane
bool layernorm_supported(int D) { return D > 0 && D % 8 == 0 && D / 8 / ln_lanes(D) <= 8; }

void launch_layernorm_fwd(const u16* x, const float* gamma, const float* beta, u16* y,
                          float* mean, float* rstd, long long rows, int D, float eps,
                          hipStream_t s, const u16* radd, u16* hout) {
  const int lr = ln_lanes(D), nc = D / 8 / lr;
  const long long rows_per_block = 4LL * (64 / lr);
  const dim3 grid((unsigned)((rows + rows_per_block - 1) / rows_per_block));
  DMP_LN_BY_LR(layernorm_fwd_kernel, lr, nc, grid, 0, x, gamma, beta, y, mean, rstd, rows, D, eps,
               radd, hout);
}

// slots: [kLnSlots][2][D] fp32, zero on entry and on return (nullptr: no param grads)
void launch_layernorm_bwd(const u16* x, const u16* dy, const float* gamma, const float* mean,
                          const float* rstd, u16* dx, float* dgamma, float* dbeta, float* slots,
                          long long rows, int D, hipStream_t s, const u16* dadd) {
  const int lr = ln_lanes(D), nc = D / 8 / lr;
  const long long rows_per_block = 4LL * (64 / lr);
  long long blocks = (rows + rows_per_block - 1) / rows_per_block;
  // the per-block param-grad epilogue (LDS fold + 2*D slot atomics) costs about
  // as much as a row group, so fewer, longer-lived blocks (ViT-B/16 bs64, 25
  // LayerNorms: 1024 blocks 601 us, 1576 blocks 741 us)
  static const int cap = [] {
    const char* e = std::getenv("DMP_LN_BWD_BLOCKS");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  // (DMP_LN_BWD_BLOCKS sweeps, ViT-B/16 after the row pipelining: 256 / 512 / 768 /
  // 1024 blocks 691 / 553 / 673 / 627 us per step; trip-balanced grids of 394 / 526 /
  // 788 blocks 589 / 727 / 670: two blocks per CU wins, profiles/layernorm_bwd_pipelined_r5.txt)
  if (blocks > cap) blocks = cap;
  const bool grads = slots != nullptr && (dgamma != nullptr || dbeta != nullptr);
  const size_t lds = grads ? (size_t)8 * D * sizeof(float) : 0;
  DMP_LN_BY_LR(layernorm_bwd_kernel, lr, nc, dim3((unsigned)blocks), lds, x, dy, gamma, mean, rstd,
               dx, grads ? slots : nullptr, rows, D, dadd);
  if (grads)
    hipLaunchKernelGGL(layernorm_param_grad_kernel, dim3((2 * D + 255) / 256), dim3(256), 0, s,
                       slots, dgamma, dbeta, D);
}

void launch_gelu_fwd(const u16* x, u16* y, long long n, hipStream_t s) {
  const long long nvec = n / 8;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, x, y, nvec);
}

void launch_gelu_bwd(const u16* x, const u16* dy, u16* dx, long long n, hipStream_t s) {
  const long long nvec = n / 8;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, x, dy, dx,
                     nvec);
}

int softmax_max_len() { return 64 * 16; }

void launch_softmax_fwd(const u16* sc, u16* p, long long rows, int L, float scale, hipStream_t s) {
  const dim3 grid((unsigned)((rows + 3) / 4));
  const int me = (L + 63) / 64;
  if (me <= 2) hipLaunchKernelGGL((softmax_fwd_kernel<2>), grid, dim3(256), 0, s, sc, p, rows, L, scale);
  else if (me <= 4) hipLaunchKernelGGL((softmax_fwd_kernel<4>), grid, dim3(256), 0, s, sc, p, rows, L, scale);
  else if (me <= 8) hipLaunchKernelGGL((softmax_fwd_kernel<8>), grid, dim3(256), 0, s, sc, p, rows, L, scale);
  else hipLaunchKernelGGL((softmax_fwd_kernel<16>), grid, dim3(256), 0, s, sc, p, rows, L, scale);
}

void launch_softmax_bwd(const u16* p, const u16* dp, u16* ds, long long rows, int L, float scale,
                        hipStream_t s) {
  const dim3 grid((unsigned)((rows + 3) / 4));
  const int me = (L + 63) / 64;
  if (me <= 2) hipLaunchKernelGGL((softmax_bwd_kernel<2>), grid, dim3(256), 0, s, p, dp, ds, rows, L, scale);
  else if (me <= 4) hipLaunchKernelGGL((softmax_bwd_kernel<4>), grid, dim3(256), 0, s, p, dp, ds, rows, L, scale);
  else if (me <= 8) hipLaunchKernelGGL((softmax_bwd_kernel<8>), grid, dim3(256), 0, s, p, dp, ds, rows, L, scale);
  else hipLaunchKernelGGL((softmax_bwd_kernel<16>), grid, dim3(256), 0, s, p, dp, ds, rows, L, scale);
}

// ------------------------------------------------------- ViT token assembly
// h[b][0] = cls + pos[0]; h[b][1 + i] = tok[b][i] + pos[1 + i]   (bf16, fp32 add)
// One pass replaces torch.cat([cls.expand(B), tok]) + pos (a concat copy and a
// broadcast add).  8 bf16 per thread, grid-stride over B * (N + 1) * D / 8.
__global__ void __launch_bounds__(256) vit_embed_fwd_kernel(const u16* __restrict__ tok,
                                                            const u16* __restrict__ cls,
                                                            const u16* __restrict__ pos,
                                                            u16* __restrict__ h, int B, int N,
                                                            int D) {
  const int dv = D / 8, T = N + 1;
  const long long nvec = (long long)B * T * dv;
  const long long gs = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += gs) {
    const int d8 = (int)(v % dv);
    const long long bt = v / dv;
    const int t = (int)(bt % T);
    const int b = (int)(bt / T);
    const bf16x8 pv = reinterpret_cast<const bf16x8*>(pos)[(long long)t * dv + d8];
    const bf16x8 xv = t == 0 ? reinterpret_cast<const bf16x8*>(cls)[d8]
                             : reinterpret_cast<const bf16x8*>(tok)[((long long)b * N + t - 1) * dv + d8];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.v[e] = f2bf(bf2f(xv.v[e]) + bf2f(pv.v[e]));
    reinterpret_cast<bf16x8*>(h)[v] = o;
  }
}

// Backward of the token assembly: dtok[b][i] = dh[b][1 + i] (bf16 copy), and the
// batch sums dpos[t] += sum_b dh[b][t], dcls += sum_b dh[b][0] accumulated in
// fp32 straight into the parameters' fp32 gradients (the flat grad arena).
// Block = 32 chunks of 8 columns x 8 batch groups of one token row t; the batch
// groups' partial sums meet in LDS, so every (t, column) is owned by one thread
// at the end (plain read-add-write, no atomics).
__global__ void __launch_bounds__(256) vit_embed_bwd_kernel(const u16* __restrict__ dh,
                                                            u16* __restrict__ dtok,
                                                            float* __restrict__ dpos,
                                                            float* __restrict__ dcls, int B, int N,
                                                            int D) {
  __shared__ float red[8][32 * 8 + 4];
  const int dv = D / 8, T = N + 1;
  const int cx = threadIdx.x & 31, bg = threadIdx.x >> 5;
  const int t = blockIdx.x;
  const int d8 = blockIdx.y * 32 + cx;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (d8 < dv) {
    for (int b = bg; b < B; b += 8) {
      const bf16x8 g = reinterpret_cast<const bf16x8*>(dh)[((long long)b * T + t) * dv + d8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(g.v[e]);
      if (t > 0 && dtok != nullptr)
        reinterpret_cast<bf16x8*>(dtok)[((long long)b * N + t - 1) * dv + d8] = g;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[bg][cx * 8 + e] = acc[e];
  __syncthreads();
  if (bg == 0 && d8 < dv) {
#pragma unroll
    for (int k = 1; k < 8; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += red[k][cx * 8 + e];
    if (dpos != nullptr) {
      float4* pp = reinterpret_cast<float4*>(dpos + (long long)t * D + d8 * 8);
      float4 a0 = pp[0], a1 = pp[1];
      a0.x += acc[0]; a0.y += acc[1]; a0.z += acc[2]; a0.w += acc[3];
      a1.x += acc[4]; a1.y += acc[5]; a1.z += acc[6]; a1.w += acc[7];
      pp[0] = a0;
      pp[1] = a1;
    }
    if (t == 0 && dcls != nullptr) {
      float4* pc = reinterpret_cast<float4*>(dcls + d8 * 8);
      float4 a0 = pc[0], a1 = pc[1];
      a0.x += acc[0]; a0.y += acc[1]; a0.z += acc[2]; a0.w += acc[3];
      a1.x += acc[4]; a1.y += acc[5]; a1.z += acc[6]; a1.w += acc[7];
      pc[0] = a0;
      pc[1] = a1;
    }
  }
}

// Backward of selecting ONE token row per sample (the ViT head reads the class
// token, models/vit.py): out[b][t][:] = t == tok ? g[b][:] : 0 over the whole
// [B][N][D] stream gradient in one 16-B-per-lane pass -- instead of ATen's zero
// fill of the stream gradient plus a strided slice copy (two launches).
__global__ void __launch_bounds__(256) token_row_scatter_kernel(const u16* __restrict__ g,
                                                                u16* __restrict__ out, int N,
                                                                int dv, int tok, long long nvec) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const long long row = i / dv;
    const int d8 = (int)(i - row * dv);
    const long long b = row / N;
    const int t = (int)(row - b * N);
    bf16x8 v;
    if (t == tok) {
      v = reinterpret_cast<const bf16x8*>(g)[b * dv + d8];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v.v[e] = 0;
    }
    reinterpret_cast<bf16x8*>(out)[i] = v;
  }
}

void launch_vit_embed_fwd(const u16* tok, const u16* cls, const u16* pos, u16* h, int B, int N,
                          int D, hipStream_t s) {
  const long long nvec = (long long)B * (N + 1) * (D / 8);
  hipLaunchKernelGGL(vit_embed_fwd_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, tok, cls,
                     pos, h, B, N, D);
}

void launch_token_row_scatter(const u16* g, u16* out, int B, int N, int D, int tok,
                              hipStream_t s) {
  const long long nvec = (long long)B * N * (D / 8);
  if (nvec <= 0) return;
  hipLaunchKernelGGL(token_row_scatter_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, g,
                     out, N, D / 8, tok, nvec);
}

void launch_vit_embed_bwd(const u16* dh, u16* dtok, float* dpos, float* dcls, int B, int N, int D,
                          hipStream_t s) {
  const dim3 grid((unsigned)(N + 1), (unsigned)((D / 8 + 31) / 32));
  hipLaunchKernelGGL(vit_embed_bwd_kernel, grid, dim3(256), 0, s, dh, dtok, dpos, dcls, B, N, D);
}

}  // namespace dmp
