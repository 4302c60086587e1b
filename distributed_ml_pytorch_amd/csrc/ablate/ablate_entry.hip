// C entry points of the roofline-ablation library (scripts/conv_roofline.py):
// conv.hip and conv_wgrad.hip compiled again with -DDMP_ABLATE=N next to this
// file, loaded with ctypes.  Never part of the extension.
#include "../common.h"
#include "../launchers.h"

extern "C" {

int abl_conv_fwd(const void* x, const void* w, void* y, float* part, int B, int H, int W, int CI,
                 int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                 void* stream) {
  dmp::launch_conv_fwd(static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w),
                       static_cast<uint16_t*>(y), part, B, H, W, CI, OH, OW, CO, R, S, stride,
                       pad, cfg, static_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}

int abl_conv_dgrad(const void* dy, const void* wt, void* dx, int B, int H, int W, int CI, int OH,
                   int OW, int CO, int R, int S, int stride, int pad, int cfg, void* stream) {
  dmp::launch_conv_dgrad(static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(wt),
                         static_cast<uint16_t*>(dx), B, H, W, CI, OH, OW, CO, R, S, stride, pad,
                         cfg, static_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}

int abl_conv_wgrad(const void* dy, const void* x, float* dw, int B, int H, int W, int CI, int OH,
                   int OW, int CO, int R, int S, int stride, int pad, int cfg, float* slab,
                   void* stream) {
  dmp::launch_conv_wgrad(static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x), dw, B,
                         H, W, CI, OH, OW, CO, R, S, stride, pad, cfg,
                         static_cast<hipStream_t>(stream), nullptr, slab);
  return (int)hipGetLastError();
}

long long abl_wgrad_slab_elems(int cfg, int B, int H, int W, int CI, int CO, int R, int S,
                               int stride, int pad) {
  return dmp::conv_wgrad_halo_slab_elems(cfg, B, H, W, CI, CO, R, S, stride, pad);
}

}  // extern "C"

// ------------------------------------------------------------------ fill ceiling
// Global -> LDS DMA rate with nothing else running: every block (one per CU: the
// LDS size forces it) has NW waves each keeping INF 1-KiB buffer_load ... lds
// pieces in flight from a power-of-two source window (L2-resident when small,
// HBM-streamed when large), `iters` rounds of INF pieces per wave.
namespace {

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, unsigned voff, uint16_t* lds) {
  const unsigned m0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "{m0}"(m0));
}

template <int NW, int INF>
__global__ void __launch_bounds__(64 * NW) dma_ceiling_kernel(const uint16_t* src, unsigned mask,
                                                              int iters, int* sink) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)(mask + 1), 0x00020000);
  unsigned off = ((unsigned)(blockIdx.x * NW + wid) * (INF * 1024u) + lane * 16u) & mask;
  const unsigned step = (unsigned)gridDim.x * NW * INF * 1024u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < INF; ++j)
      dma16(rs, (off + j * 1024u) & mask, lds + (wid * INF + j) * 512);
    off = (off + step) & mask;
    __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0): the round landed
  }
  __syncthreads();
  if (lds[threadIdx.x * 8] == 0x7fff && sink != nullptr) sink[0] = 1;   // keep the loads live
}

}  // namespace

extern "C" int abl_dma_ceiling(const void* src, unsigned long long window_bytes, int blocks, int nw,
                               int inflight, int iters, int* sink, void* stream) {
  const unsigned mask = (unsigned)(window_bytes - 1);
  const size_t lds = (size_t)nw * inflight * 1024;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * nw), lds, static_cast<hipStream_t>(stream),
                       static_cast<const uint16_t*>(src), mask, iters, sink);
  };
  if (nw == 4 && inflight == 8) go(dma_ceiling_kernel<4, 8>);
  else if (nw == 4 && inflight == 16) go(dma_ceiling_kernel<4, 16>);
  else if (nw == 8 && inflight == 8) go(dma_ceiling_kernel<8, 8>);
  else if (nw == 8 && inflight == 16) go(dma_ceiling_kernel<8, 16>);
  else return -1;
  return (int)hipGetLastError();
}
