// Dropout / Dropout2d with a counter-based Philox4x32-10 generator.
//
// Reference: LeNet's nn.Dropout2d + F.dropout (/root/reference/example/models.py:10,17,20),
// SURVEY §2.3 "Philox RNG dropout kernel, fused mask-multiply".
//
// The random stream is a pure function of (seed, offset, element index): one
// Philox call yields four 32-bit draws, one per element of a 4-element group.
// The offset is read from device memory (a per-layer int64 counter), so a step
// captured in a hipGraph draws fresh masks on every replay.  The forward is ONE
// kernel: draw, keep mask (1 byte per mask element, reused by the backward) and
// the scaled product, and the launch advances its own offset -- the last block
// to finish (an arrival ticket next to the counter) adds 1, after every block
// has read the old value at its start.
//
// Mask granularity: element-wise (Dropout), or one draw per (n, c) plane
// (Dropout2d) for NCHW (`inner` = H*W) or NHWC (`inner` = 1 with channel
// stride C) activations.
#include "common.h"

namespace dmp {

__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
  constexpr u32 M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const u32 hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const u32 hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

// mask index of element i
__device__ __forceinline__ long long mask_index(long long i, int mode, long long inner, int C) {
  if (mode == 0) return i;                       // element-wise
  if (mode == 1) return i / inner;               // NCHW planes: i / (H*W) = n*C + c
  const long long pix = i / C;                   // NHWC: (n*HW + hw)*C + c
  return (pix / inner) * C + (i - pix * C);      // inner = H*W here
}

// one thread = 4 consecutive mask elements = one Philox call
__global__ void __launch_bounds__(256) dropout_mask_kernel(u8* __restrict__ mask, long long nmask,
                                                           u32 threshold, unsigned long long seed,
                                                           const long long* __restrict__ offset) {
  const unsigned long long off = (unsigned long long)offset[0];
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g * 4 < nmask; g += stride) {
    const uint4 r = philox4x32_10(
        make_uint4((u32)g, (u32)(g >> 32), (u32)off, (u32)(off >> 32)),
        make_uint2((u32)seed, (u32)(seed >> 32)));
    const u32 d[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long i = g * 4 + k;
      if (i < nmask) mask[i] = d[k] >= threshold ? 1 : 0;
    }
  }
}

// y = x * mask * scale (forward) or dx = dy * mask * scale (backward); 8 elements / thread
template <typename T>
__global__ void __launch_bounds__(256) dropout_apply_kernel(const T* __restrict__ x,
                                                            const u8* __restrict__ mask,
                                                            T* __restrict__ y, long long n,
                                                            float scale, int mode,
                                                            long long inner, int C) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v * 8 < n; v += stride) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long long i = v * 8 + k;
      if (i >= n) break;
      const float m = mask[mask_index(i, mode, inner, C)] ? scale : 0.f;
      if constexpr (sizeof(T) == 2) {
        y[i] = f2bf(bf2f(x[i]) * m);
      } else {
        y[i] = x[i] * m;
      }
    }
  }
}

void launch_dropout_mask(u8* mask, long long nmask, float p, unsigned long long seed,
                         const long long* offset, hipStream_t s) {
  double t = (double)p * 4294967296.0;
  if (t > 4294967295.0) t = 4294967295.0;
  const u32 threshold = (u32)t;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(stream_grid((nmask + 3) / 4, 256)), dim3(256), 0,
                     s, mask, nmask, threshold, seed, offset);
}

void launch_dropout_apply_bf16(const u16* x, const u8* mask, u16* y, long long n, float scale,
                               int mode, long long inner, int C, hipStream_t s) {
  hipLaunchKernelGGL((dropout_apply_kernel<u16>), dim3(stream_grid((n + 7) / 8, 256)), dim3(256),
                     0, s, x, mask, y, n, scale, mode, inner, C);
}

void launch_dropout_apply_f32(const float* x, const u8* mask, float* y, long long n, float scale,
                              int mode, long long inner, int C, hipStream_t s) {
  hipLaunchKernelGGL((dropout_apply_kernel<float>), dim3(stream_grid((n + 7) / 8, 256)),
                     dim3(256), 0, s, x, mask, y, n, scale, mode, inner, C);
}

// Fused forward: y = x * keep * scale and the keep mask, 8 elements per thread;
// ctr[0] = Philox offset (advanced by the launch's last block), ctr[1] = ticket.
template <typename T>
__global__ void __launch_bounds__(256) dropout_fwd_fused_kernel(
    const T* __restrict__ x, u8* __restrict__ mask, T* __restrict__ y, long long n, u32 threshold,
    float scale, int mode, long long inner, int C, unsigned long long seed,
    long long* __restrict__ ctr) {
  const unsigned long long off = (unsigned long long)ctr[0];
  const uint2 key = make_uint2((u32)seed, (u32)(seed >> 32));
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v * 8 < n; v += stride) {
    long long gcur = -1;
    u32 d[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long long i = v * 8 + k;
      if (i >= n) break;
      const long long mi = mask_index(i, mode, inner, C);
      const long long g = mi >> 2;
      if (g != gcur) {                 // one Philox call per 4-mask-element group
        const uint4 r = philox4x32_10(
            make_uint4((u32)g, (u32)(g >> 32), (u32)off, (u32)(off >> 32)), key);
        d[0] = r.x; d[1] = r.y; d[2] = r.z; d[3] = r.w;
        gcur = g;
      }
      const bool keep = d[mi & 3] >= threshold;
      mask[mi] = keep ? 1 : 0;         // planes: every element of the plane writes the same byte
      const float m = keep ? scale : 0.f;
      if constexpr (sizeof(T) == 2) y[i] = f2bf(bf2f(x[i]) * m);
      else y[i] = x[i] * m;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = __hip_atomic_fetch_add(
        reinterpret_cast<unsigned long long*>(ctr + 1), 1ull, __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {          // every block has read ctr[0]: advance it
      ctr[0] = (long long)(off + 1);
      ctr[1] = 0;
    }
  }
}

void launch_dropout_fwd_fused(const void* x, u8* mask, void* y, bool bf16, long long n, float p,
                              int mode, long long inner, int C, unsigned long long seed,
                              long long* ctr, hipStream_t s) {
  double t = (double)p * 4294967296.0;
  if (t > 4294967295.0) t = 4294967295.0;
  const u32 threshold = (u32)t;
  const float scale = 1.f / (1.f - p);
  const dim3 grid(stream_grid((n + 7) / 8, 256));
  if (bf16)
    hipLaunchKernelGGL((dropout_fwd_fused_kernel<u16>), grid, dim3(256), 0, s,
                       static_cast<const u16*>(x), mask, static_cast<u16*>(y), n, threshold, scale,
                       mode, inner, C, seed, ctr);
  else
    hipLaunchKernelGGL((dropout_fwd_fused_kernel<float>), grid, dim3(256), 0, s,
                       static_cast<const float*>(x), mask, static_cast<float*>(y), n, threshold,
                       scale, mode, inner, C, seed, ctr);
}

}  // namespace dmp
