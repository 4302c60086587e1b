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
// y = (x - mean) * rstd * gamma + beta; saves mean, rstd (fp32 per row)
template <int MAXC>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(
    const u16* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    u16* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out, long long rows,
    int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = D >> 3;
  const u16* xr = x + row * D;
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      ld8(xr + ch * 8, v[c]);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[c][k];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[c][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  u16* yr = y + row * D;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int d = ch * 8 + k;
        o[k] = (v[c][k] - mean) * rstd * (gamma ? gamma[d] : 1.f) + (beta ? beta[d] : 0.f);
      }
      st8(yr + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// dgamma += sum_rows dy * xhat, dbeta += sum_rows dy  (fp32 atomics per block)
template <int MAXC>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, u16* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, long long rows, int D) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = D >> 3;
  float pg[MAXC][8], pb[MAXC][8];   // per-lane dgamma / dbeta partials over this wave's rows
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) { pg[c][k] = 0.f; pb[c][k] = 0.f; }
  for (long long row = (long long)blockIdx.x * 4 + wid; row < rows; row += (long long)gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[MAXC][8], g[MAXC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float dv[8];
        ld8(x + row * D + ch * 8, xh[c]);
        ld8(dy + row * D + ch * 8, dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int d = ch * 8 + k;
          xh[c][k] = (xh[c][k] - mean) * rstd;
          g[c][k] = dv[k] * (gamma ? gamma[d] : 1.f);
          s1 += g[c][k];
          s2 += g[c][k] * xh[c][k];
          pg[c][k] += dv[k] * xh[c][k];
          pb[c][k] += dv[k];
        }
      }
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (g[c][k] - m1 - xh[c][k] * m2);
        st8(dx + row * D + ch * 8, o);
      }
    }
  }
  if (dgamma == nullptr && dbeta == nullptr) return;
  // block reduce of the 4 waves' partials through LDS, then one atomic per
  // column per block
  extern __shared__ float red[];   // [2][4][D]
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(0 * 4 + wid) * D + ch * 8 + k] = pg[c][k];
        red[(1 * 4 + wid) * D + ch * 8 + k] = pb[c][k];
      }
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256) {
    const float sg = red[0 * D + d] + red[1 * D + d] + red[2 * D + d] + red[3 * D + d];
    const float sb = red[4 * D + d] + red[5 * D + d] + red[6 * D + d] + red[7 * D + d];
    if (dgamma) atomicAdd(dgamma + d, sg);
    if (dbeta) atomicAdd(dbeta + d, sb);
  }
}

// ----------------------------------------------------------------------- GELU
__device__ __forceinline__ float gelu_tanh(float x, float* dgelu) {
  constexpr float c0 = 0.7978845608028654f, c1 = 0.044715f;
  const float u = c0 * (x + c1 * x * x * x);
  const float t = tanhf(u);
  if (dgelu) {
    const float du = c0 * (1.f + 3.f * c1 * x * x);
    *dgelu = 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
  }
  return 0.5f * x * (1.f + t);
}

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
#define DMP_LN_DISPATCH(MAXC_EXPR, KERNEL, ...)                                      \
  do {                                                                                \
    const int mc_ = (MAXC_EXPR);                                                      \
    if (mc_ <= 1) hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__);                       \
    else if (mc_ <= 2) hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__);                  \
    else if (mc_ <= 4) hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__);                  \
    else hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__);                                \
  } while (0)

int layernorm_max_dim() { return 8 * 64 * 8; }

void launch_layernorm_fwd(const u16* x, const float* gamma, const float* beta, u16* y,
                          float* mean, float* rstd, long long rows, int D, float eps,
                          hipStream_t s) {
  const int chunks = (D / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4));
  DMP_LN_DISPATCH(chunks, layernorm_fwd_kernel, grid, dim3(256), 0, s, x, gamma, beta, y, mean, rstd,
                  rows, D, eps);
}

void launch_layernorm_bwd(const u16* x, const u16* dy, const float* gamma, const float* mean,
                          const float* rstd, u16* dx, float* dgamma, float* dbeta, long long rows,
                          int D, hipStream_t s) {
  const int chunks = (D / 8 + 63) / 64;
  long long blocks = (rows + 3) / 4;
  if (blocks > 256) blocks = 256;   // rows per wave grow; atomics per column = blocks
  const size_t lds = (size_t)8 * D * sizeof(float);
  DMP_LN_DISPATCH(chunks, layernorm_bwd_kernel, dim3((unsigned)blocks), dim3(256), lds, s, x, dy,
                  gamma, mean, rstd, dx, dgamma, dbeta, rows, D);
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

}  // namespace dmp
