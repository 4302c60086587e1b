// im2col / col2im for NHWC bf16 convolutions that the implicit-GEMM / halo
// kernels (conv.hip) do not take: few input or output channels, any window and
// stride -- AlexNet's 11x11/s4 CI=3 stem, both LeNet convs (CO = 6 / 16,
// /root/reference/example/models.py:8-9,29), the ResNet-50 7x7/s2 stem.
// The patch matrix feeds the native MFMA GEMM (gemm.hip) for all three passes:
//   fwd   Y[m][co]      = cols[m][:] . W[co][:]        (bias / ReLU epilogue)
//   wgrad dW[co][k]    += sum_m dY[m][co] cols[m][k]
//   dgrad dcols[m][k]   = sum_co dY[m][co] W[co][k]  -> col2im (gather) -> dX
// m = (b, oh, ow); k = (r, s, ci) with ci fastest, which is exactly the
// channels_last weight's [CO][R][S][CI] memory order, zero-padded to Kp (a
// multiple of 8) so every GEMM operand row is whole 16-B pieces.
#include "common.h"

#include <algorithm>

namespace dmp {

// one lane = 8 consecutive k of one row m (one 16-B store); the (r, s, ci)
// decode is done once per lane and stepped, taps outside the image read 0
__global__ void __launch_bounds__(256) im2col_kernel(const u16* __restrict__ x,
                                                     u16* __restrict__ cols, int H, int W, int CI,
                                                     int OH, int OW, int S, int stride, int pad,
                                                     int K, int Kp, long long chunks) {
  const int cpr = Kp >> 3;
  const long long gs = (long long)gridDim.x * blockDim.x;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < chunks; q += gs) {
    const long long m = q / cpr;
    const int k0 = (int)(q - m * cpr) * 8;
    const int ow = (int)(m % OW);
    const long long t = m / OW;
    const int oh = (int)(t % OH);
    const long long b = t / OH;
    int ci = k0 % CI;
    int rs = k0 / CI;
    int s = rs % S, r = rs / S;
    if ((CI & 7) == 0) {
      // every 8-chunk is 8 consecutive channels of ONE tap: a 16-B load (the
      // 64+-channel ResNet convs on the im2col weight-gradient route)
      const int ih = oh * stride - pad + r, iw = ow * stride - pad + s;
      bf16x8 v{};
      if (k0 < K && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        v = *reinterpret_cast<const bf16x8*>(x + ((b * H + ih) * W + iw) * CI + ci);
      *reinterpret_cast<bf16x8*>(cols + q * 8) = v;
      continue;
    }
    bf16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      u16 v = 0;
      if (k0 + e < K) {
        const int ih = oh * stride - pad + r, iw = ow * stride - pad + s;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          v = x[((b * H + ih) * W + iw) * CI + ci];
      }
      out.v[e] = v;
      if (++ci == CI) {
        ci = 0;
        if (++s == S) { s = 0; ++r; }
      }
    }
    *reinterpret_cast<bf16x8*>(cols + q * 8) = out;
  }
}

// gather form (no atomics): input element (b, h, w, ci) sums the patch
// entries of every output pixel whose window covers it
__global__ void __launch_bounds__(256) col2im_kernel(const u16* __restrict__ dcols,
                                                     u16* __restrict__ dx, int H, int W, int CI,
                                                     int OH, int OW, int R, int S, int stride,
                                                     int pad, int Kp, long long total) {
  const long long gs = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int ci = (int)(i % CI);
    long long t = i / CI;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const long long b = t / H;
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
      const int hn = h + pad - r;
      if (hn < 0 || hn % stride) continue;
      const int oh = hn / stride;
      if (oh >= OH) continue;
      for (int s = 0; s < S; ++s) {
        const int wn = w + pad - s;
        if (wn < 0 || wn % stride) continue;
        const int ow = wn / stride;
        if (ow >= OW) continue;
        acc += bf2f(dcols[((b * OH + oh) * OW + ow) * Kp + (r * S + s) * CI + ci]);
      }
    }
    dx[i] = f2bf(acc);
  }
}

// ReLU backward from the saved output: dx = y > 0 ? dy : 0 (in place allowed)
__global__ void __launch_bounds__(256) relu_bwd_kernel(const u16* __restrict__ dy,
                                                       const u16* __restrict__ y,
                                                       u16* __restrict__ dx, long long n) {
  const long long gs = (long long)gridDim.x * blockDim.x;
  const long long nv = n >> 3;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gs) {
    const bf16x8 g = reinterpret_cast<const bf16x8*>(dy)[v];
    const bf16x8 a = reinterpret_cast<const bf16x8*>(y)[v];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.v[e] = (a.v[e] & 0x8000u) || a.v[e] == 0 ? 0 : g.v[e];
    reinterpret_cast<bf16x8*>(dx)[v] = o;
  }
  for (long long i = (nv << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs)
    dx[i] = (y[i] & 0x8000u) || y[i] == 0 ? 0 : dy[i];
}

void launch_im2col(const u16* x, u16* cols, int B, int H, int W, int CI, int OH, int OW, int R,
                   int S, int stride, int pad, int K, int Kp, hipStream_t st) {
  (void)R;
  const long long chunks = (long long)B * OH * OW * (Kp / 8);
  hipLaunchKernelGGL(im2col_kernel, dim3(stream_grid(chunks, 256)), dim3(256), 0, st, x, cols, H,
                     W, CI, OH, OW, S, stride, pad, K, Kp, chunks);
}

void launch_col2im(const u16* dcols, u16* dx, int B, int H, int W, int CI, int OH, int OW, int R,
                   int S, int stride, int pad, int Kp, hipStream_t st) {
  const long long total = (long long)B * H * W * CI;
  hipLaunchKernelGGL(col2im_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, dcols, dx, H,
                     W, CI, OH, OW, R, S, stride, pad, Kp, total);
}

void launch_relu_bwd(const u16* dy, const u16* y, u16* dx, long long n, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(stream_grid((n + 7) / 8, 256)), dim3(256), 0, st, dy, y,
                     dx, n);
}

// All padded-row weight copies of a model in ONE launch: table[i] = {src_off,
// dst_off, rows, K, Kp}; dst[dst_off + r*Kp + k] = src[src_off + r*K + k] for
// k < K (the pad columns were zeroed once at allocation and are never
// written).  The im2col GEMMs read a conv weight [CO][R*S*CI] whose row length
// is not a multiple of 8 (LeNet: 75 / 150) from this padded image.
__global__ void __launch_bounds__(256) pad_rows_batched_kernel(const u16* __restrict__ src,
                                                               u16* __restrict__ dst,
                                                               const long long* __restrict__ tab) {
  const long long* t = tab + 5 * blockIdx.y;
  const long long so = t[0], d_o = t[1], rows = t[2], K = t[3], Kp = t[4];
  const long long n = rows * K;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / K, k = e - r * K;
    dst[d_o + r * Kp + k] = src[so + e];
  }
}

void launch_pad_rows_batched(const u16* src, u16* dst, const long long* table, int n,
                             long long max_elems, hipStream_t st) {
  if (n <= 0) return;
  const dim3 grid((unsigned)std::min<long long>((max_elems + 255) / 256, 64), (unsigned)n);
  hipLaunchKernelGGL(pad_rows_batched_kernel, grid, dim3(256), 0, st, src, dst, table);
}

}  // namespace dmp
