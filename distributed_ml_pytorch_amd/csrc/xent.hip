// Fused softmax-cross-entropy: forward loss + backward dlogits + top-1 hits in
// ONE pass over the logits (one wave per row, 64-lane shuffle reductions).
//
// Replaces the ATen chain _log_softmax -> nll_loss_forward -> nll_loss_backward
// -> _log_softmax_backward_data -> max that the reference runs per iteration
// (/root/reference/example/main.py:71-75; op trace in SURVEY.md §2.3).
//
// dlogits = (softmax(x) - onehot(y)) * grad_scale  where grad_scale = 1/#valid
// rows (grad_scale <= 0: counted on device) for the loss averaged over the
// rows whose label is not ignore_index; the autograd wrapper rescales by the
// incoming grad_output.
#include "common.h"

namespace dmp {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<u16>(const u16* p, long long i) { return bf2f(p[i]); }

template <typename T>
__device__ __forceinline__ void st(T* p, long long i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, long long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<u16>(u16* p, long long i, float v) { p[i] = f2bf(v); }

// Labels outside [0, C) are treated like ignore_index (no out-of-bounds read).
__device__ __forceinline__ bool label_ok(long long y, int C, int ignore_index) {
  return y != ignore_index && y >= 0 && y < C;
}

// 1 / (number of non-ignored labels), counted by every block over all B labels
// (B <= a few thousand int64: cheaper than a separate pass): the gradient of a
// mean over the valid rows, exactly as F.cross_entropy(ignore_index=...).
__device__ float valid_grad_scale(const int64_t* __restrict__ labels, int B, int C,
                                  int ignore_index) {
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  int c = 0;
  for (int r = threadIdx.x; r < B; r += blockDim.x) c += label_ok(labels[r], C, ignore_index);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&cnt, c);
  __syncthreads();
  return 1.f / (float)max(cnt, 1);
}

// Phase 1: rows [blockIdx.x*rows_per_block, ...). Each wave owns one row at a time.
// If `fused_finalize` (grid == 1) the same block reduces the row results.
// MAXE > 0: the row (C <= 64 * MAXE) is read ONCE into registers and the max,
// sum-exp and gradient passes run on them (ImageNet heads, C = 1000: 16 values
// per lane); MAXE = 0 streams the row three times from memory.
template <typename T, int MAXE>
__global__ void __launch_bounds__(1024) softmax_xent_kernel(
    const T* __restrict__ logits, const int64_t* __restrict__ labels, T* __restrict__ dlogits,
    float* __restrict__ row_loss, int* __restrict__ row_hit, float* __restrict__ loss_out,
    int* __restrict__ hits_out, int B, int C, float grad_scale, float label_smoothing,
    int ignore_index, int rows_per_block, int fused_finalize) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const int r_begin = blockIdx.x * rows_per_block;
  const int r_end = min(B, r_begin + rows_per_block);
  if (grad_scale <= 0.f) grad_scale = valid_grad_scale(labels, B, C, ignore_index);
  float my_loss = 0.f;
  int my_hit = 0, my_valid = 0;
  for (int r = r_begin + wid; r < r_end; r += nw) {
    const T* x = logits + (long long)r * C;
    const long long y = labels[r];
    const bool valid = label_ok(y, C, ignore_index);
    constexpr int NE = MAXE > 0 ? MAXE : 1;
    float cv[NE];
    if constexpr (MAXE > 0) {
#pragma unroll
      for (int e = 0; e < MAXE; ++e) {
        const int j = lane + 64 * e;
        cv[e] = j < C ? ld(x, j) : -INFINITY;
      }
    }
    // pass 1: max + argmax
    float m = -INFINITY;
    int am = 0x7fffffff;
    if constexpr (MAXE > 0) {
#pragma unroll
      for (int e = 0; e < MAXE; ++e) {
        const int j = lane + 64 * e;
        if (cv[e] > m) { m = cv[e]; am = j; }   // ascending j: first max wins
      }
    } else {
      for (int j = lane; j < C; j += 64) {
        const float v = ld(x, j);
        if (v > m || (v == m && j < am)) { m = v; am = j; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > m || (om == m && oa < am)) { m = om; am = oa; }
    }
    // pass 2: sum exp and sum of logits (for label smoothing)
    float s = 0.f, sx = 0.f;
    if constexpr (MAXE > 0) {
#pragma unroll
      for (int e = 0; e < MAXE; ++e) {
        if (lane + 64 * e < C) {
          s += __expf(cv[e] - m);
          sx += cv[e];
        }
      }
    } else {
      for (int j = lane; j < C; j += 64) {
        const float v = ld(x, j);
        s += __expf(v - m);
        sx += v;
      }
    }
    s = wave_sum(s);
    sx = wave_sum(sx);
    const float lse = m + __logf(s);
    const float xy = valid ? ld(x, y) : 0.f;
    // loss = (1-eps) * (lse - x_y) + eps * (lse - mean(x))
    const float eps = label_smoothing;
    const float loss = valid ? ((1.f - eps) * (lse - xy) + eps * (lse - sx / (float)C)) : 0.f;
    // pass 3: gradient
    if (dlogits) {
      T* d = dlogits + (long long)r * C;
      const float inv_s = 1.f / s;
      const float smooth = eps / (float)C;
      if constexpr (MAXE > 0) {
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
          const int j = lane + 64 * e;
          if (j < C) {
            float g = 0.f;
            if (valid) {
              const float p = __expf(cv[e] - m) * inv_s;
              g = (p - smooth - (j == y ? (1.f - eps) : 0.f)) * grad_scale;
            }
            st(d, j, g);
          }
        }
      } else {
        for (int j = lane; j < C; j += 64) {
          float g = 0.f;
          if (valid) {
            const float p = __expf(ld(x, j) - m) * inv_s;
            g = (p - smooth - (j == y ? (1.f - eps) : 0.f)) * grad_scale;
          }
          st(d, j, g);
        }
      }
    }
    if (lane == 0) {
      if (row_loss) row_loss[r] = loss;
      if (row_hit) row_hit[r] = (valid && am == y) ? 1 : 0;
      my_loss += loss;
      my_hit += (valid && am == y) ? 1 : 0;
      my_valid += valid ? 1 : 0;
    }
  }
  if (!fused_finalize) return;
  __shared__ float sl[16];
  __shared__ int sh[16];
  __shared__ int sv[16];
  if (lane == 0) { sl[wid] = my_loss; sh[wid] = my_hit; sv[wid] = my_valid; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tl = 0.f; int th = 0, tv = 0;
    for (int w = 0; w < nw; ++w) { tl += sl[w]; th += sh[w]; tv += sv[w]; }
    loss_out[0] = tl / (float)max(tv, 1);
    hits_out[0] = th;
  }
}

// Narrow heads (C <= 32: every CIFAR/MNIST classifier): one ROW per THREAD, the
// whole row in registers, one block with the fused finalize.  The wave-per-row
// kernel above leaves 54 of 64 lanes idle at C = 10 and walks the rows 16 at a
// time through dependent shuffle chains (62 us at B = 512); here all rows of a
// 1024-row chunk are in flight at once.
template <typename T>
__global__ void __launch_bounds__(1024) softmax_xent_narrow_kernel(
    const T* __restrict__ logits, const int64_t* __restrict__ labels, T* __restrict__ dlogits,
    float* __restrict__ row_loss, int* __restrict__ row_hit, float* __restrict__ loss_out,
    int* __restrict__ hits_out, int B, int C, float grad_scale, float label_smoothing,
    int ignore_index) {
  constexpr int CMAX = 32;
  const float eps = label_smoothing, smooth = eps / (float)C;
  if (grad_scale <= 0.f) grad_scale = valid_grad_scale(labels, B, C, ignore_index);
  float my_loss = 0.f;
  int my_hit = 0, my_valid = 0;
  for (int r = threadIdx.x; r < B; r += blockDim.x) {
    const T* x = logits + (long long)r * C;
    const long long y = labels[r];
    const bool valid = label_ok(y, C, ignore_index);
    float v[CMAX];
#pragma unroll
    for (int j = 0; j < CMAX; ++j) v[j] = j < C ? ld(x, j) : -INFINITY;
    float m = v[0];
    int am = 0;
#pragma unroll
    for (int j = 1; j < CMAX; ++j)
      if (v[j] > m) { m = v[j]; am = j; }
    float se = 0.f, sx = 0.f, xy = 0.f;
#pragma unroll
    for (int j = 0; j < CMAX; ++j) {
      if (j < C) {
        v[j] -= m;
        sx += v[j];
        if (j == y) xy = v[j];
        v[j] = __expf(v[j]);
        se += v[j];
      }
    }
    const float lse = __logf(se);   // shifted by m, like xy and sx
    const float loss = valid ? ((1.f - eps) * (lse - xy) + eps * (lse - sx / (float)C)) : 0.f;
    if (dlogits) {
      T* d = dlogits + (long long)r * C;
      const float inv = 1.f / se;
#pragma unroll
      for (int j = 0; j < CMAX; ++j)
        if (j < C)
          st(d, j, valid ? (v[j] * inv - smooth - (j == y ? (1.f - eps) : 0.f)) * grad_scale : 0.f);
    }
    const int hit = (valid && am == y) ? 1 : 0;
    if (row_loss) row_loss[r] = loss;
    if (row_hit) row_hit[r] = hit;
    my_loss += loss;
    my_hit += hit;
    my_valid += valid ? 1 : 0;
  }
  __shared__ float sl[16];
  __shared__ int sh[16], sv[16];
  my_loss = wave_sum(my_loss);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    my_hit += __shfl_xor(my_hit, o, 64);
    my_valid += __shfl_xor(my_valid, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sl[wid] = my_loss; sh[wid] = my_hit; sv[wid] = my_valid; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tl = 0.f; int th = 0, tv = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { tl += sl[w]; th += sh[w]; tv += sv[w]; }
    loss_out[0] = tl / (float)max(tv, 1);
    hits_out[0] = th;
  }
}

// Phase 2 for the multi-block path: one block reduces the per-row results.
__global__ void __launch_bounds__(1024) xent_finalize_kernel(
    const float* __restrict__ row_loss, const int* __restrict__ row_hit,
    const int64_t* __restrict__ labels, float* __restrict__ loss_out, int* __restrict__ hits_out,
    int B, int C, int ignore_index) {
  __shared__ float sl[16];
  __shared__ int sh[16], sv[16];
  float l = 0.f; int h = 0, v = 0;
  for (int r = threadIdx.x; r < B; r += blockDim.x) {
    l += row_loss[r]; h += row_hit[r]; v += label_ok(labels[r], C, ignore_index) ? 1 : 0;
  }
  l = wave_sum(l);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { h += __shfl_xor(h, o, 64); v += __shfl_xor(v, o, 64); }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sl[wid] = l; sh[wid] = h; sv[wid] = v; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tl = 0.f; int th = 0, tv = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { tl += sl[w]; th += sh[w]; tv += sv[w]; }
    loss_out[0] = tl / (float)max(tv, 1);
    hits_out[0] = th;
  }
}

template <typename T>
void launch_xent_t(const T* logits, const int64_t* labels, T* dlogits, float* row_loss,
                   int* row_hit, float* loss_out, int* hits_out, int B, int C, float grad_scale,
                   float smoothing, int ignore_index, hipStream_t s) {
  if (C <= 32 && B <= (1 << 16)) {
    hipLaunchKernelGGL(softmax_xent_narrow_kernel<T>, dim3(1), dim3(1024), 0, s, logits, labels,
                       dlogits, row_loss, row_hit, loss_out, hits_out, B, C, grad_scale,
                       smoothing, ignore_index);
    return;
  }
  // Small problems: one block, fused finalize.  (A single block walking 128
  // ImageNet rows, C = 1000, 8 rows per wave in series took 122 us in the
  // ResNet-50 step: wide heads take the multi-block path, one row per wave.)
  const long long work = (long long)B * C;
  const bool cached = C <= 1024;
  if (work <= (1 << 14) || (B <= 16 && !cached)) {
    if (cached)
      hipLaunchKernelGGL((softmax_xent_kernel<T, 16>), dim3(1), dim3(1024), 0, s, logits, labels,
                         dlogits, row_loss, row_hit, loss_out, hits_out, B, C, grad_scale,
                         smoothing, ignore_index, B, 1);
    else
      hipLaunchKernelGGL((softmax_xent_kernel<T, 0>), dim3(1), dim3(1024), 0, s, logits, labels,
                         dlogits, row_loss, row_hit, loss_out, hits_out, B, C, grad_scale,
                         smoothing, ignore_index, B, 1);
    return;
  }
  const int rows_per_block = 16;   // one row per wave
  const int grid = (B + rows_per_block - 1) / rows_per_block;
  if (cached)
    hipLaunchKernelGGL((softmax_xent_kernel<T, 16>), dim3(grid), dim3(1024), 0, s, logits, labels,
                       dlogits, row_loss, row_hit, loss_out, hits_out, B, C, grad_scale,
                       smoothing, ignore_index, rows_per_block, 0);
  else
    hipLaunchKernelGGL((softmax_xent_kernel<T, 0>), dim3(grid), dim3(1024), 0, s, logits, labels,
                       dlogits, row_loss, row_hit, loss_out, hits_out, B, C, grad_scale,
                       smoothing, ignore_index, rows_per_block, 0);
  hipLaunchKernelGGL(xent_finalize_kernel, dim3(1), dim3(1024), 0, s, row_loss, row_hit, labels,
                     loss_out, hits_out, B, C, ignore_index);
}

void launch_softmax_xent_bf16(const u16* logits, const int64_t* labels, u16* dlogits,
                              float* row_loss, int* row_hit, float* loss_out, int* hits_out,
                              int B, int C, float grad_scale, float smoothing, int ignore_index,
                              hipStream_t s) {
  launch_xent_t<u16>(logits, labels, dlogits, row_loss, row_hit, loss_out, hits_out, B, C,
                     grad_scale, smoothing, ignore_index, s);
}

void launch_softmax_xent_f32(const float* logits, const int64_t* labels, float* dlogits,
                             float* row_loss, int* row_hit, float* loss_out, int* hits_out, int B,
                             int C, float grad_scale, float smoothing, int ignore_index,
                             hipStream_t s) {
  launch_xent_t<float>(logits, labels, dlogits, row_loss, row_hit, loss_out, hits_out, B, C,
                       grad_scale, smoothing, ignore_index, s);
}

}  // namespace dmp
