// Bias gradients of linear / conv layers: out[n] += sum_m dy[m][n].
//
// dy is a bf16 [M, N] row-major activation gradient (a Linear's output grad,
// or an NHWC conv output grad with N = channels); out is the layer's fp32
// bias gradient, usually a view into the flat grad arena.  Replaces
// `dy.sum(0, dtype=float32)` + `grad.add_(col)` (two launches, a [N] fp32
// temporary; 24 us per ViT-B/16 linear at M = 12608, N = 768 in
// gpurun_out/mprof/steady_vit_b16.txt) with one streaming pass over dy plus a
// tiny fold: a thread owns 8 columns (16-B loads, 4 rows in flight), the
// 256/(N/8) row lanes of a block meet in LDS, and each block adds its N partial
// sums into slot row blockIdx % kColSlots of a zeroed fp32 scratch (<= 32
// adders per address: one row shared by ~500 blocks measured 19 us per call,
// the memory-side atomic unit serialising same-address adds);
// colsum_fold_kernel adds the slot rows into `out` and re-zeroes them.
#include "common.h"

namespace dmp {

constexpr int kColSlots = 16;

__global__ void __launch_bounds__(256) colsum_acc_kernel(const u16* __restrict__ dy,
                                                         float* __restrict__ slots, long long M,
                                                         int N, long long rows_per_block) {
  extern __shared__ float red[];   // [rpi][8 * min(tpr, 256)]
  const int tpr = N >> 3;
  const int t = threadIdx.x;
  const int cw = tpr < 256 ? tpr : 256;    // column chunks per pass
  const int rpi = 256 / cw;                // row lanes
  const int cl = t % cw, rl = t / cw;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  for (int cb = 0; cb < tpr; cb += cw) {
    const int cg = cb + cl;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (rl < rpi && cg < tpr) {
      const u16* p = dy + cg * 8;
      long long r = r0 + rl;
      for (; r + 3 * rpi < r1; r += 4 * rpi) {
        bf16x8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u] = *reinterpret_cast<const bf16x8*>(p + (r + u * rpi) * N);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += bf2f(v[u].v[k]);
      }
      for (; r < r1; r += rpi) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(p + r * N);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += bf2f(v.v[k]);
      }
    }
    __syncthreads();
    if (rl < rpi) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[rl * cw * 8 + cl * 8 + k] = acc[k];
    }
    __syncthreads();
    for (int e = t; e < cw * 8; e += 256) {
      const int col = cb * 8 + e;
      if (col < N) {
        float s = 0.f;
        for (int q = 0; q < rpi; ++q) s += red[q * cw * 8 + e];
        atomicAdd(slots + (long long)(blockIdx.x % kColSlots) * N + col, s);
      }
    }
  }
}

__global__ void __launch_bounds__(256) colsum_fold_kernel(float* __restrict__ slots,
                                                          float* __restrict__ out, int N) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < kColSlots; ++k) {
    acc += slots[(long long)k * N + c];
    slots[(long long)k * N + c] = 0.f;
  }
  out[c] += acc;
}

int colsum_num_slots() { return kColSlots; }

// slots: zeroed fp32 scratch of colsum_num_slots() * N floats, zero again on return
void launch_colsum_acc(const u16* dy, float* out, float* slots, long long M, int N,
                       hipStream_t s) {
  const int tpr = N / 8;
  const int cw = tpr < 256 ? tpr : 256;
  const int rpi = 256 / cw;
  long long blocks = (M + 4 * rpi - 1) / (4 * rpi);   // >= 4 rows per row lane
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  const long long rpb = (M + blocks - 1) / blocks;
  const size_t lds = (size_t)rpi * cw * 8 * sizeof(float);
  hipLaunchKernelGGL(colsum_acc_kernel, dim3((unsigned)blocks), dim3(256), lds, s, dy, slots, M, N,
                     rpb);
  hipLaunchKernelGGL(colsum_fold_kernel, dim3((N + 255) / 256), dim3(256), 0, s, slots, out, N);
}

}  // namespace dmp
