// Fused classifier head of the ResNets: global average pool + Linear, forward
// and backward, each in ONE launch (the reference's models end in a pooled
// Linear, /root/reference/example/models.py; the CIFAR ResNet-18 bench head is
// 512 -> 10).  Unfused, the head of a ResNet-18 bs512 step was six latency-bound
// launches -- gap_fwd 6.8, a one-tile GEMM 14.7, the two backward GEMMs 8.7 +
// 15.2 and gap_bwd 6.6 us (profiles/resnet18_step_dispatches_r4.txt) -- around
// 8 MB of pooled-activation traffic that takes ~2 us at HBM rate.
//
//   forward   f[b][c] = mean_hw x[b][hw][c]          (x channels-last bf16)
//             y[b][n] = sum_c W[n][c] f[b][c] + bias[n]
//   backward  dx[b][hw][c] = (sum_n dy[b][n] W[n][c]) / HW
//             dW[n][c] += sum_b dy[b][n] f[b][c]      (fp32, the grad arena)
//             db[n]    += sum_b dy[b][n]
//
// One wave per sample: lane l owns channels 8l + 512k (16-B vectors), so the
// pooling reads and the dx writes are whole 1-KiB rows per wave instruction.
// The N <= kHeadN class dot products are lane partials reduced by shuffles.
// The backward block (4 waves x SPW samples) sums its samples' dW / db
// contributions in registers, then through LDS across its waves, and adds them
// to the fp32 gradient with one atomic per (n, c) per block.
#include "common.h"

namespace dmp {

constexpr int kHeadN = 16;      // classes per launch (more: the unfused path)
constexpr int kHeadCV = 4;      // 16-B channel vectors per lane: C <= 64 * 8 * 4 = 2048

__global__ void __launch_bounds__(256) gap_linear_fwd_kernel(
    const u16* __restrict__ x, const u16* __restrict__ w, const u16* __restrict__ bias,
    u16* __restrict__ y, u16* __restrict__ f, int B, int HW, int C, int N) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float inv = 1.f / (float)HW;
  float part[kHeadN];
#pragma unroll
  for (int n = 0; n < kHeadN; ++n) part[n] = 0.f;
#pragma unroll
  for (int k = 0; k < kHeadCV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c >= C) break;
    bf16x8 wv[kHeadN];                       // issued ahead of the pooling loads
#pragma unroll
    for (int n = 0; n < kHeadN; ++n)
      if (n < N) wv[n] = *reinterpret_cast<const bf16x8*>(w + (long long)n * C + c);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const u16* px = x + (long long)b * HW * C + c;
    int p = 0;
    for (; p + 4 <= HW; p += 4) {            // four rows in flight
      bf16x8 r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = *reinterpret_cast<const bf16x8*>(px + (long long)(p + u) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(r[u].v[e]);
    }
    for (; p < HW; ++p) {
      const bf16x8 r = *reinterpret_cast<const bf16x8*>(px + (long long)p * C);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(r.v[e]);
    }
    bf16x8 fo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] *= inv;
      fo.v[e] = f2bf(acc[e]);
    }
    *reinterpret_cast<bf16x8*>(f + (long long)b * C + c) = fo;
#pragma unroll
    for (int n = 0; n < kHeadN; ++n) {
      if (n < N) {
#pragma unroll
        for (int e = 0; e < 8; ++e) part[n] += bf2f(wv[n].v[e]) * acc[e];
      }
    }
  }
#pragma unroll
  for (int n = 0; n < kHeadN; ++n) {
    if (n < N) {
      const float s = wave_sum(part[n]);
      if (lane == n) y[(long long)b * N + n] = f2bf(s + (bias != nullptr ? bf2f(bias[n]) : 0.f));
    }
  }
}

// SPW samples per wave, 4 waves per block
template <int SPW>
__global__ void __launch_bounds__(256) gap_linear_bwd_kernel(
    const u16* __restrict__ dy, const u16* __restrict__ f, const u16* __restrict__ w,
    u16* __restrict__ dx, float* __restrict__ gw, float* __restrict__ gb, int B, int HW, int C,
    int N) {
  __shared__ float red[4][64 * 8];   // one class's dW partials of a channel slice, per wave
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * 4 + wid) * SPW;
  const float inv = 1.f / (float)HW;
  float dbp[kHeadN];
#pragma unroll
  for (int n = 0; n < kHeadN; ++n) dbp[n] = 0.f;
#pragma unroll
  for (int k = 0; k < kHeadCV; ++k) {
    if (k * 512 >= C) break;                 // uniform
    const int c = (k * 64 + lane) * 8;
    const bool con = c < C;
    float gwp[kHeadN][8];
#pragma unroll
    for (int n = 0; n < kHeadN; ++n)
#pragma unroll
      for (int e = 0; e < 8; ++e) gwp[n][e] = 0.f;
    bf16x8 wv[kHeadN];
#pragma unroll
    for (int n = 0; n < kHeadN; ++n)
      if (n < N && con) wv[n] = *reinterpret_cast<const bf16x8*>(w + (long long)n * C + c);
    for (int s = 0; s < SPW; ++s) {
      const int b = b0 + s;
      if (b >= B) break;
      float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      float fv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (con) {
        const bf16x8 fr = *reinterpret_cast<const bf16x8*>(f + (long long)b * C + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) fv[e] = bf2f(fr.v[e]);
      }
      float dv[kHeadN];
#pragma unroll
      for (int n = 0; n < kHeadN; ++n) dv[n] = n < N ? bf2f(dy[(long long)b * N + n]) : 0.f;
#pragma unroll
      for (int n = 0; n < kHeadN; ++n) {
        if (n < N) {
          const float d = dv[n];
          if (k == 0) dbp[n] += d;
          if (con) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              g[e] += d * bf2f(wv[n].v[e]);
              gwp[n][e] += d * fv[e];
            }
          }
        }
      }
      if (con) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = f2bf(g[e] * inv);
        u16* pd = dx + (long long)b * HW * C + c;
#pragma unroll 4
        for (int p = 0; p < HW; ++p) *reinterpret_cast<bf16x8*>(pd + (long long)p * C) = o;
      }
    }
    // the block's 4 waves hold partials of the same channels: sum them through
    // LDS, one class at a time, and let wave 0 add them (one atomic per (n, c))
#pragma unroll
    for (int n = 0; n < kHeadN; ++n) {
      if (n < N) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8; ++e) red[wid][lane * 8 + e] = gwp[n][e];
        __syncthreads();
        if (wid == 0 && con) {
          float* dst = gw + (long long)n * C + c;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            atomicAdd(dst + e, red[0][lane * 8 + e] + red[1][lane * 8 + e] +
                                   red[2][lane * 8 + e] + red[3][lane * 8 + e]);
        }
      }
    }
  }
  // db: every lane of a wave summed the same dy values; one atomic per class per wave
  if (gb != nullptr && lane < N) {
    float v = 0.f;
#pragma unroll
    for (int n = 0; n < kHeadN; ++n) v = n == lane ? dbp[n] : v;
    atomicAdd(gb + lane, v);
  }
}

bool gap_linear_supported(int C, int N) { return N >= 1 && N <= kHeadN && C % 8 == 0 && C <= 64 * 8 * kHeadCV; }

void launch_gap_linear_fwd(const u16* x, const u16* w, const u16* bias, u16* y, u16* f, int B, int HW,
                           int C, int N, hipStream_t s) {
  hipLaunchKernelGGL(gap_linear_fwd_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, x, w,
                     bias, y, f, B, HW, C, N);
}

void launch_gap_linear_bwd(const u16* dy, const u16* f, const u16* w, u16* dx, float* gw, float* gb,
                           int B, int HW, int C, int N, hipStream_t s) {
  constexpr int SPW = 2;
  hipLaunchKernelGGL(gap_linear_bwd_kernel<SPW>, dim3((unsigned)((B + 4 * SPW - 1) / (4 * SPW))),
                     dim3(256), 0, s, dy, f, w, dx, gw, gb, B, HW, C, N);
}

}  // namespace dmp
