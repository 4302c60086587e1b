// NHWC pooling kernels (bf16, 8 channels = 16 B per thread).
//
//  * global average pool  [N,H,W,C] -> [N,C]   (ResNet head, avg_pool2d(4) on CIFAR)
//  * max pool k x k / stride s / padding p (the reference's 2x2/s2 pooling,
//    /root/reference/example/models.py:16-17,29,32,41, and the ImageNet
//    ResNet stem's overlapping 3x3/s2/p1), uint8 argmax indices, gather-form
//    backward.
#include "common.h"

namespace dmp {

// Block = (sample n, 64 channel vectors); its 4 waves split the HW rows (wave w
// takes rows w, w + 4, ...; 4 loads in flight per lane) and meet in LDS.  One
// thread per (n, vector) walking all HW rows serially left ResNet-50's head
// (128 x 49 x 2048) at 0.5 waves per SIMD: 22.5 us for 26 MB.
__global__ void __launch_bounds__(256) gap_fwd_kernel(const u16* __restrict__ x,
                                                      u16* __restrict__ y, int N, int HW, int C) {
  __shared__ float red[4][64][9];
  const int tpr = C >> 3;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x, cg = blockIdx.y * 64 + lane;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cg < tpr) {
    const u16* base = x + (long long)n * HW * C + cg * 8;
    int p = w;
    for (; p + 12 < HW; p += 16) {
      bf16x8 r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = *reinterpret_cast<const bf16x8*>(base + (long long)(p + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += bf2f(r[u].v[k]);
    }
    for (; p < HW; p += 4) {
      const bf16x8 r = *reinterpret_cast<const bf16x8*>(base + (long long)p * C);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += bf2f(r.v[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane][k] = acc[k];
  __syncthreads();
  if (w == 0 && cg < tpr) {
    const float inv = 1.f / (float)HW;
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      o.v[k] = f2bf((red[0][lane][k] + red[1][lane][k] + red[2][lane][k] + red[3][lane][k]) * inv);
    *reinterpret_cast<bf16x8*>(y + (long long)n * C + cg * 8) = o;
  }
}

__global__ void __launch_bounds__(256) gap_bwd_kernel(const u16* __restrict__ dy,
                                                      u16* __restrict__ dx, int N, int HW, int C) {
  const int tpr = C >> 3;
  const long long total = (long long)N * HW * tpr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float inv = 1.f / (float)HW;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int cg = (int)(t % tpr);
    const long long n = t / ((long long)HW * tpr);
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(dy + n * C + cg * 8);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = f2bf(bf2f(r.v[k]) * inv);
    *reinterpret_cast<bf16x8*>(dx + t * 8) = o;
  }
}

// Max pool, window K x K, stride S, zero..K/2 padding (padded taps never win),
// floor mode; the argmax tap (i*K + j, K <= 15) is kept as uint8 per element.
// NCHW_OUT: y is written NCHW-contiguous (a pool feeding a flatten + Linear in
// the reference's (c, h, w) order: LeNet), idx stays NHWC.
template <bool NCHW_OUT>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const u16* __restrict__ x,
                                                          u16* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H,
                                                          int W, int C, int K, int S, int P,
                                                          int Ho, int Wo, int relu_in) {
  const int tpr = C >> 3;
  const long long total = (long long)N * Ho * Wo * tpr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int cg = (int)(t % tpr);
    long long r = t / tpr;
    const int wo = (int)(r % Wo); r /= Wo;
    const int ho = (int)(r % Ho);
    const long long n = r / Ho;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    const int h0 = ho * S - P, w0 = wo * S - P;
    for (int i = 0; i < K; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int j = 0; j < K; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)W) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((n * H + h) * W + w) * C + cg * 8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float f = bf2f(v.v[k]);
          if (f > best[k] || (f != f)) { best[k] = f; bi[k] = (uint8_t)(i * K + j); }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o.v[k] = f2bf(best[k]);
      // a ReLU'd input whose window max is 0: relu' = 0 everywhere in it -> no tap
      if (relu_in && !(best[k] > 0.f)) bi[k] = 255;
    }
    if constexpr (NCHW_OUT) {
#pragma unroll
      for (int k = 0; k < 8; ++k) y[((n * C + cg * 8 + k) * Ho + ho) * Wo + wo] = o.v[k];
    } else {
      *reinterpret_cast<bf16x8*>(y + t * 8) = o;
    }
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((u32)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((u32)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + t * 8) = packed;
  }
}

// Gather form (no atomics, no zero fill): every input element sums dy over the
// outputs whose window covers it and whose saved argmax is this tap.
// NCHW_DY: dy arrives NCHW-contiguous (the gradient of an NCHW_OUT forward)
template <bool NCHW_DY>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const u16* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          u16* __restrict__ dx, int N, int H,
                                                          int W, int C, int K, int S, int P,
                                                          int Ho, int Wo) {
  const int tpr = C >> 3;
  const long long total = (long long)N * H * W * tpr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int cg = (int)(t % tpr);
    long long r = t / tpr;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const long long n = r / H;
    // outputs ho with ho*S - P <= h <= ho*S - P + K - 1
    const int hlo = max(0, (h + P - K + S) / S), hhi = min(Ho - 1, (h + P) / S);
    const int wlo = max(0, (w + P - K + S) / S), whi = min(Wo - 1, (w + P) / S);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ho = hlo; ho <= hhi; ++ho) {
      for (int wo = wlo; wo <= whi; ++wo) {
        const uint8_t me = (uint8_t)((h - (ho * S - P)) * K + (w - (wo * S - P)));
        const long long o = ((n * Ho + ho) * Wo + wo) * C + cg * 8;
        bf16x8 g;
        if constexpr (NCHW_DY) {
#pragma unroll
          for (int k = 0; k < 8; ++k) g.v[k] = dy[((n * C + cg * 8 + k) * Ho + ho) * Wo + wo];
        } else {
          g = *reinterpret_cast<const bf16x8*>(dy + o);
        }
        const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint8_t bi = (uint8_t)(((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xff);
          if (bi == me) acc[k] += bf2f(g.v[k]);
        }
      }
    }
    bf16x8 out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out.v[k] = f2bf(acc[k]);
    *reinterpret_cast<bf16x8*>(dx + t * 8) = out;
  }
}

// Any channel count (C % 8 != 0: LeNet's 6-channel pool): one element per
// lane, same argmax / gather-form semantics as the 8-wide kernels above.
__global__ void __launch_bounds__(256) maxpool_fwd_c1_kernel(const u16* __restrict__ x,
                                                             u16* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int N,
                                                             int H, int W, int C, int K, int S,
                                                             int P, int Ho, int Wo, int relu_in) {
  const long long total = (long long)N * Ho * Wo * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int wo = (int)(r % Wo); r /= Wo;
    const int ho = (int)(r % Ho);
    const long long n = r / Ho;
    float best = -INFINITY;
    uint8_t bi = 0;
    const int h0 = ho * S - P, w0 = wo * S - P;
    for (int i = 0; i < K; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int j = 0; j < K; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)W) continue;
        const float f = bf2f(x[((n * H + h) * W + w) * C + c]);
        if (f > best || (f != f)) { best = f; bi = (uint8_t)(i * K + j); }
      }
    }
    y[t] = f2bf(best);
    idx[t] = (relu_in && !(best > 0.f)) ? (uint8_t)255 : bi;
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_c1_kernel(const u16* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx,
                                                             u16* __restrict__ dx, int N, int H,
                                                             int W, int C, int K, int S, int P,
                                                             int Ho, int Wo) {
  const long long total = (long long)N * H * W * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const long long n = r / H;
    const int hlo = max(0, (h + P - K + S) / S), hhi = min(Ho - 1, (h + P) / S);
    const int wlo = max(0, (w + P - K + S) / S), whi = min(Wo - 1, (w + P) / S);
    float acc = 0.f;
    for (int ho = hlo; ho <= hhi; ++ho)
      for (int wo = wlo; wo <= whi; ++wo) {
        const uint8_t me = (uint8_t)((h - (ho * S - P)) * K + (w - (wo * S - P)));
        const long long o = ((n * Ho + ho) * Wo + wo) * C + c;
        if (idx[o] == me) acc += bf2f(dy[o]);
      }
    dx[t] = f2bf(acc);
  }
}

void launch_gap_fwd(const u16* x, u16* y, int N, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((unsigned)N, (unsigned)((C / 8 + 63) / 64)), dim3(256), 0,
                     s, x, y, N, HW, C);
}

void launch_gap_bwd(const u16* dy, u16* dx, int N, int HW, int C, hipStream_t s) {
  const long long total = (long long)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, dy, dx, N, HW, C);
}

int maxpool_out(int H, int K, int S, int P) { return (H + 2 * P - K) / S + 1; }

void launch_maxpool_fwd(const u16* x, u16* y, uint8_t* idx, int N, int H, int W, int C, int K,
                        int S, int P, hipStream_t s, bool nchw_out, bool relu_in) {
  const int Ho = maxpool_out(H, K, S, P), Wo = maxpool_out(W, K, S, P);
  const int ri = relu_in ? 1 : 0;
  if (C % 8) {
    const long long n1 = (long long)N * Ho * Wo * C;
    hipLaunchKernelGGL(maxpool_fwd_c1_kernel, dim3(stream_grid(n1, 256)), dim3(256), 0, s, x, y,
                       idx, N, H, W, C, K, S, P, Ho, Wo, ri);
    return;
  }
  const long long total = (long long)N * Ho * Wo * (C / 8);
  if (nchw_out)
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(stream_grid(total, 256)), dim3(256), 0, s, x,
                       y, idx, N, H, W, C, K, S, P, Ho, Wo, ri);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(stream_grid(total, 256)), dim3(256), 0, s,
                       x, y, idx, N, H, W, C, K, S, P, Ho, Wo, ri);
}

void launch_maxpool_bwd(const u16* dy, const uint8_t* idx, u16* dx, int N, int H, int W, int C,
                        int K, int S, int P, hipStream_t s, bool nchw_dy) {
  const int Ho = maxpool_out(H, K, S, P), Wo = maxpool_out(W, K, S, P);
  if (C % 8) {
    const long long n1 = (long long)N * H * W * C;
    hipLaunchKernelGGL(maxpool_bwd_c1_kernel, dim3(stream_grid(n1, 256)), dim3(256), 0, s, dy,
                       idx, dx, N, H, W, C, K, S, P, Ho, Wo);
    return;
  }
  const long long total = (long long)N * H * W * (C / 8);
  if (nchw_dy)
    hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(stream_grid(total, 256)), dim3(256), 0, s, dy,
                       idx, dx, N, H, W, C, K, S, P, Ho, Wo);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(stream_grid(total, 256)), dim3(256), 0, s,
                       dy, idx, dx, N, H, W, C, K, S, P, Ho, Wo);
}

}  // namespace dmp
