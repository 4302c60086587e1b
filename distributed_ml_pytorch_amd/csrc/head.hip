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
// The backward grid has a dx role (one wave per sample) and a weight-gradient
// role (one block per 64-channel slice, all samples, owned outputs).
#include "common.h"

namespace dmp {

constexpr int kHeadN = 16;      // classes per launch (more: the unfused path)
constexpr int kHeadCV = 4;      // 16-B channel vectors per lane: C <= 64 * 8 * 4 = 2048
constexpr int kHeadKS = 4;      // sample chunks of the weight-gradient role
constexpr int kHeadU = 4;       // samples per thread with their loads in flight together

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

// Two block roles in one grid.  Blocks [0, nbx): dx, one wave per sample (4 per
// block).  Blocks [nbx, nbx + (C / 64) * kHeadKS): the weight gradient of one
// 64-channel slice over one of kHeadKS sample chunks (one atomic per (n, c) per
// dx block measured 34 us: 64 adds per address serialise; one block per slice
// over ALL samples 36 us: a serial 16-deep load chain per thread).  dW role:
// thread t takes channel vector t % 8 of the slice and samples t / 8 + 32 i of
// its chunk, loads issued together; the 32 sample groups are summed through LDS
// one class at a time and added with kHeadKS atomics per (n, c).
__global__ void __launch_bounds__(256) gap_linear_bwd_kernel(
    const u16* __restrict__ dy, const u16* __restrict__ f, const u16* __restrict__ w,
    u16* __restrict__ dx, float* __restrict__ gw, float* __restrict__ gb, int B, int HW, int C,
    int N, int nbx) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < nbx) {
    const int lane = tid & 63;
    const int b = blockIdx.x * 4 + (tid >> 6);
    if (b >= B) return;
    const float inv = 1.f / (float)HW;
    float dv[kHeadN];
#pragma unroll
    for (int n = 0; n < kHeadN; ++n) dv[n] = n < N ? bf2f(dy[(long long)b * N + n]) : 0.f;
#pragma unroll
    for (int k = 0; k < kHeadCV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c >= C) break;
      float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < kHeadN; ++n) {
        if (n < N) {
          const bf16x8 wr = *reinterpret_cast<const bf16x8*>(w + (long long)n * C + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] += dv[n] * bf2f(wr.v[e]);
        }
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.v[e] = f2bf(g[e] * inv);
      u16* pd = dx + (long long)b * HW * C + c;
#pragma unroll 4
      for (int p = 0; p < HW; ++p) *reinterpret_cast<bf16x8*>(pd + (long long)p * C) = o;
    }
    return;
  }
  __shared__ float red[32][64];                 // [sample group][channel of the slice]
  const int role = blockIdx.x - nbx, slice = role / kHeadKS, chunk = role % kHeadKS;
  const int cv = tid & 7, sg = tid >> 3;
  const int c = slice * 64 + cv * 8;
  const int per = (B + kHeadKS - 1) / kHeadKS;
  const int bbeg = chunk * per, bend = min(B, bbeg + per);
  float gwp[kHeadN][8];
#pragma unroll
  for (int n = 0; n < kHeadN; ++n)
#pragma unroll
    for (int e = 0; e < 8; ++e) gwp[n][e] = 0.f;
  float dbp[kHeadN];
#pragma unroll
  for (int n = 0; n < kHeadN; ++n) dbp[n] = 0.f;
  for (int b = bbeg + sg; b < bend; b += 32 * kHeadU) {
    bf16x8 fr[kHeadU];
    float dv[kHeadU][kHeadN];
#pragma unroll
    for (int u = 0; u < kHeadU; ++u) {       // every load of kHeadU samples in flight
      const int bu = b + 32 * u;
      const bool ok = bu < bend;
      fr[u] = ok ? *reinterpret_cast<const bf16x8*>(f + (long long)bu * C + c) : bf16x8{};
#pragma unroll
      for (int n = 0; n < kHeadN; ++n) dv[u][n] = ok && n < N ? bf2f(dy[(long long)bu * N + n]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kHeadU; ++u)
#pragma unroll
      for (int n = 0; n < kHeadN; ++n) {
        if (n < N) {
          dbp[n] += dv[u][n];
#pragma unroll
          for (int e = 0; e < 8; ++e) gwp[n][e] += dv[u][n] * bf2f(fr[u].v[e]);
        }
      }
  }
#pragma unroll
  for (int n = 0; n < kHeadN; ++n) {
    if (n < N) {
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[sg][cv * 8 + e] = gwp[n][e];
      __syncthreads();
      if (tid < 64) {
        float v = 0.f;
#pragma unroll 8
        for (int q = 0; q < 32; ++q) v += red[q][tid];
        atomicAdd(gw + (long long)n * C + slice * 64 + tid, v);
      }
    }
  }
  if (slice == 0 && gb != nullptr) {
    // every channel-vector lane of a sample group summed the same dy: take cv 0's
#pragma unroll
    for (int n = 0; n < kHeadN; ++n) {
      if (n < N) {
        __syncthreads();
        if (cv == 0) red[sg][0] = dbp[n];
        __syncthreads();
        if (tid == 0) {
          float v = 0.f;
          for (int q = 0; q < 32; ++q) v += red[q][0];
          atomicAdd(gb + n, v);
        }
      }
    }
  }
}

bool gap_linear_supported(int C, int N) {
  return N >= 1 && N <= kHeadN && C % 64 == 0 && C <= 64 * 8 * kHeadCV;
}

void launch_gap_linear_fwd(const u16* x, const u16* w, const u16* bias, u16* y, u16* f, int B, int HW,
                           int C, int N, hipStream_t s) {
  hipLaunchKernelGGL(gap_linear_fwd_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, x, w,
                     bias, y, f, B, HW, C, N);
}

void launch_gap_linear_bwd(const u16* dy, const u16* f, const u16* w, u16* dx, float* gw, float* gb,
                           int B, int HW, int C, int N, hipStream_t s) {
  const int nbx = (B + 3) / 4;
  hipLaunchKernelGGL(gap_linear_bwd_kernel, dim3((unsigned)(nbx + C / 64 * kHeadKS)), dim3(256), 0, s, dy, f,
                     w, dx, gw, gb, B, HW, C, N, nbx);
}

}  // namespace dmp
