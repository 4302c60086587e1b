// Few-input-channel convolutions (network stems: CIFAR ResNet 3x3x3, ImageNet
// ResNet 7x7x3, AlexNet 11x11x3) on gfx950.
//
// K = R*S*CI is tiny (27 .. 363), so the implicit GEMM has nothing to feed the
// matrix cores with and MIOpen spends its time in layout shuffles and
// zero-fills around a K=27 GEMM.  These are VALU kernels shaped so that most
// per-FMA operand traffic is an LDS broadcast:
//
//   forward  lane = 4 consecutive output pixels, wave = 16 of the 64 output
//            channels of the tile (64 fp32 accumulators per lane).  The weight
//            tile [K][64] sits in LDS as fp32; all lanes of a wave read the same
//            row (broadcast ds_read_b128), so 4 LDS reads feed 64 FMAs.  Patch
//            taps are gathered 8 at a time through an LDS tap table (no integer
//            division in the loop).  Epilogue: bf16 NHWC store + per-channel BN
//            partial sums (recursive-halving butterfly over the lanes, lane l
//            ends up owning channel l & 15), added into the same
//            [2][kBnSlots][CO] slot sums as the implicit-GEMM epilogue.
//   wgrad    dW[co][k] = sum_p dY[p][co] * patch_p[k]: a block owns a chunk of
//            P, a 64-channel x 32-tap output tile; 64-pixel slabs of dY and of
//            the patches are staged to LDS as fp32, each lane accumulates a 4 x 8
//            outer product per pixel, the 4 waves split the slab rows and are
//            summed through LDS, then fp32 atomics into the arena gradient.
// The input image is read with explicit element strides (any dense layout of
// the bf16 activations).
#include <cstdlib>

#include "common.h"

namespace dmp {

struct SmallConvArgs {
  const u16* x;     // input, element strides below (bf16)
  const u16* w;     // [CO][R][S][CI] bf16
  const u16* dy;    // [P][CO] bf16 (wgrad)
  u16* y;           // [P][CO] bf16 (forward)
  float* part;      // [2][kBnSlots][CO] BN slot sums (forward, optional, accumulated)
  float* dw;        // [CO][R][S][CI] fp32 (wgrad, accumulated)
  float* ws;        // wgrad: [G][CO][K] per-block partial tiles
  int sb, sh, sw, sc;           // input strides in elements (input < 2^30 elements)
  int xbytes;                   // input extent in bytes (buffer descriptor bound)
  int B, H, W, CI, OH, OW, CO, R, S, stride, pad, K;
  long long P;
  int chunk;        // wgrad: pixels per block
};

// tap table entry: r | s << 8 | ci << 16 (k >= K -> -1)
__device__ __forceinline__ int tap_of(const SmallConvArgs& a, int k) {
  if (k >= a.K) return -1;
  const int ci = k % a.CI, rs = k / a.CI;
  return (rs / a.S) | ((rs % a.S) << 8) | (ci << 16);
}

// raw buffer descriptor over the input image (gfx9 dword3); a load whose
// offset is past num_records returns 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc(const SmallConvArgs& a) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
}

// boff = b * sb (element offset of the image).  Padding / masked taps get an
// out-of-range offset and read 0 from the buffer unit: no branch per tap, so a
// thread's gathers issue back to back and retire under one wait.
__device__ __forceinline__ float load_tap(const SmallConvArgs& a, __amdgpu_buffer_rsrc_t rs,
                                          int tap, int boff, int ih0, int iw0) {
  const int ih = ih0 + (tap & 255), iw = iw0 + ((tap >> 8) & 255), ci = tap >> 16;
  const bool ok = tap >= 0 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
  const int off = ok ? 2 * (boff + ih * a.sh + iw * a.sw + ci * a.sc) : 0x7ffffff0;
  return bf2f(__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
}

// output pixel p (< 2^31) -> {b * sb, oh * stride - pad, ow * stride - pad}
__device__ __forceinline__ int3 decode_pixel(const SmallConvArgs& a, int p) {
  const int ow = p % a.OW, t = p / a.OW;
  const int oh = t % a.OH, b = t / a.OH;
  return make_int3(b * a.sb, oh * a.stride - a.pad, ow * a.stride - a.pad);
}

// v[0..2H) -> v[0..H): lanes with bit H set keep the upper half
template <int H>
__device__ __forceinline__ void halve(float* v, int lane) {
  const bool up = lane & H;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float send = up ? v[i] : v[i + H];
    const float keep = up ? v[i + H] : v[i];
    v[i] = keep + __shfl_xor(send, H, 64);
  }
}
// forward: lane = 4 consecutive output pixels, wave = 16 output channels of the
// 64-channel tile -> each broadcast weight read (4 x ds_read_b128) feeds 64 FMAs
constexpr int kOutPitch = 72;   // bf16 per staged output row (144 B: 16-B aligned, odd x 16 B)
__global__ void __launch_bounds__(256) conv_small_fwd_kernel(SmallConvArgs a) {
  constexpr int TC = 8;                          // taps gathered per pass
  extern __shared__ float smem[];
  float* wl = smem;                              // [K][64] fp32
  const int K = a.K, Kp = (K + TC - 1) / TC * TC;
  int* taps = reinterpret_cast<int*>(smem + K * 64);   // [Kp]
  u16* ot = reinterpret_cast<u16*>(smem + ((K * 64 + Kp + 3) & ~3));   // [256][kOutPitch]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co0 = blockIdx.y * 64;
  for (int i = tid; i < K * 64; i += 256) {
    const int k = i >> 6, c = i & 63;
    wl[i] = bf2f(a.w[(long long)(co0 + c) * K + k]);
  }
  for (int k = tid; k < Kp; k += 256) taps[k] = tap_of(a, k);
  __syncthreads();

  const int pbase = blockIdx.x * 256 + lane * 4;
  int pb[4], ph[4], pw[4];
  bool pv_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pv_ok[i] = pbase + i < a.P;
    const int3 d = decode_pixel(a, pv_ok[i] ? pbase + i : 0);
    pb[i] = d.x;
    ph[i] = d.y;
    pw[i] = d.z;
  }
  float acc[4][16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[i][c] = 0.f;
  const float* wcol = wl + wid * 16;
  const __amdgpu_buffer_rsrc_t rs = image_rsrc(a);
  for (int k0 = 0; k0 < K; k0 += TC) {
    float pv[4][TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int tap = taps[k0 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i][j] = load_tap(a, rs, pv_ok[i] ? tap : -1, pb[i], ph[i], pw[i]);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      if (k0 + j < K) {
        const float4* wr = reinterpret_cast<const float4*>(wcol + (k0 + j) * 64);
        float wv[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 w4 = wr[q];
          wv[4 * q] = w4.x; wv[4 * q + 1] = w4.y; wv[4 * q + 2] = w4.z; wv[4 * q + 3] = w4.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int c = 0; c < 16; ++c) acc[i][c] += pv[i][j] * wv[c];
      }
    }
  }
  // round to the stored bf16 values (BN statistics describe what is stored)
  float s1[16], s2[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) { s1[c] = 0.f; s2[c] = 0.f; }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32 packed[8];
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      const u16 lo = f2bf(acc[i][c]), hi = f2bf(acc[i][c + 1]);
      packed[c / 2] = (u32)lo | ((u32)hi << 16);
      if (pv_ok[i]) {
        const float flo = bf2f(lo), fhi = bf2f(hi);
        s1[c] += flo; s2[c] += flo * flo;
        s1[c + 1] += fhi; s2[c + 1] += fhi * fhi;
      }
    }
    // stage the block's [256 px][64 ch] bf16 tile in LDS: a lane's own pixels are
    // 4 rows apart in the output, so direct 16-B stores would scatter
    uint4* t = reinterpret_cast<uint4*>(ot + (lane * 4 + i) * kOutPitch + wid * 16);
    t[0] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    t[1] = make_uint4(packed[4], packed[5], packed[6], packed[7]);
  }
  __syncthreads();
  // coalesced write-out: 8 threads per 128-B pixel row
#pragma unroll
  for (int pass = 0; pass < 8; ++pass) {
    const int idx = pass * 256 + tid;
    const int row = idx >> 3, ch = idx & 7;
    const int p = blockIdx.x * 256 + row;
    if (p < a.P)
      *reinterpret_cast<uint4*>(a.y + (long long)p * a.CO + co0 + ch * 8) =
          *reinterpret_cast<const uint4*>(ot + row * kOutPitch + ch * 8);
  }
  if (a.part == nullptr) return;
  // 16 channels x 64 lanes: halve over lane bits 3..0 (lane ends up owning
  // channel lane & 15), then fold lane bits 4, 5
  halve<8>(s1, lane); halve<4>(s1, lane); halve<2>(s1, lane); halve<1>(s1, lane);
  halve<8>(s2, lane); halve<4>(s2, lane); halve<2>(s2, lane); halve<1>(s2, lane);
  float t1 = s1[0], t2 = s2[0];
  t1 += __shfl_xor(t1, 16, 64); t2 += __shfl_xor(t2, 16, 64);
  t1 += __shfl_xor(t1, 32, 64); t2 += __shfl_xor(t2, 32, 64);
  if (lane < 16) {
    const int c = co0 + wid * 16 + lane;
    const int slot = blockIdx.x % kBnSlots;
    atomicAdd(a.part + (long long)slot * a.CO + c, t1);
    atomicAdd(a.part + (long long)(kBnSlots + slot) * a.CO + c, t2);
  }
}

// wgrad: blockIdx.z = 32-tap pass.  Lane = (co quad cq = lane & 15, tap octet
// ko = lane >> 4) -> 4 x 8 outputs per lane, 32 FMAs per (float4 dY + 2 float4
// patch) LDS reads; the 4 waves split each 64-pixel slab's rows and are summed
// through LDS.  Each block stores its [64][32] tile to ws[blockIdx.x] (plain
// stores); conv_small_wgrad_reduce then adds the G tiles into dW -- every
// block hitting the same 1.7k addresses with fp32 atomics serialises at the
// memory-side atomic units.
__global__ void __launch_bounds__(256) conv_small_wgrad_kernel(SmallConvArgs a) {
  constexpr int SLAB = 64, KT = 32;
  // [SLAB][64] dY slab + [SLAB][KT] patch slab; afterwards the same 24 KiB
  // hold waves 1..3's [64][KT] tiles for the cross-wave sum
  __shared__ __attribute__((aligned(16))) float smem[SLAB * 64 + SLAB * KT];
  static_assert(3 * 64 * KT == SLAB * 64 + SLAB * KT, "reduction tile reuses the slabs");
  __shared__ int taps[KT];
  __shared__ int4 rows[2][SLAB];   // pixel decode of slab s in rows[s & 1]
  float* dyl = smem;
  float* pl = smem + SLAB * 64;
  float* red = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co0 = blockIdx.y * 64, k0 = blockIdx.z * KT;
  const int cq = lane & 15, ko = lane >> 4;
  const __amdgpu_buffer_rsrc_t rs = image_rsrc(a);
  const int p_begin = blockIdx.x * a.chunk;
  const int p_end = min((int)a.P, p_begin + a.chunk);
  const int nslab = (p_end - p_begin + SLAB - 1) / SLAB;
  auto fill_rows = [&](int sl) {       // threads 0..63, slab sl
    const int p = p_begin + sl * SLAB + tid;
    const bool ok = sl < nslab && p < p_end;
    const int3 d = decode_pixel(a, ok ? p : p_begin);
    rows[sl & 1][tid] = make_int4(d.x, d.y, d.z, ok);
  };
  // slab operands in registers: this thread's 16 dY values and 8 patch taps
  uint4 rdy0, rdy1;
  float rg[SLAB * KT / 256];
  auto load_slab = [&](int sl) {
    {
      const int r = tid >> 2, c = (tid & 3) * 16;
      const int p = p_begin + sl * SLAB + r;
      if (sl < nslab && p < p_end) {
        const uint4* src = reinterpret_cast<const uint4*>(a.dy + (long long)p * a.CO + co0 + c);
        rdy0 = src[0];
        rdy1 = src[1];
      } else {
        rdy0 = rdy1 = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < SLAB * KT / 256; ++it) {
      const int i = it * 256 + tid;
      const int r = i / KT, k = i % KT;
      const int4 e = rows[sl & 1][r];
      rg[it] = load_tap(a, rs, e.w ? taps[k] : -1, e.x, e.y, e.z);
    }
  };
  auto store_slab = [&]() {
    const int r = tid >> 2, c = (tid & 3) * 16;
    float4* d = reinterpret_cast<float4*>(dyl + r * 64 + c);
    const u32 u[8] = {rdy0.x, rdy0.y, rdy0.z, rdy0.w, rdy1.x, rdy1.y, rdy1.z, rdy1.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[q] = make_float4(bf2f((u16)(u[2 * q] & 0xffff)), bf2f((u16)(u[2 * q] >> 16)),
                         bf2f((u16)(u[2 * q + 1] & 0xffff)), bf2f((u16)(u[2 * q + 1] >> 16)));
#pragma unroll
    for (int it = 0; it < SLAB * KT / 256; ++it) pl[it * 256 + tid] = rg[it];
  };

  float acc[4][8];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  // prologue: tables for slabs 0 and 1, slab 0 staged
  if (tid < KT) taps[tid] = tap_of(a, k0 + tid);
  if (tid < SLAB) fill_rows(0);
  __syncthreads();
  load_slab(0);
  store_slab();
  if (tid < SLAB) fill_rows(1);
  __syncthreads();
  for (int sl = 0; sl < nslab; ++sl) {
    // next slab's global loads fly while this one is consumed from LDS
    if (sl + 1 < nslab) load_slab(sl + 1);
#pragma unroll 4
    for (int rr = 0; rr < SLAB / 4; ++rr) {
      const int r = rr * 4 + wid;
      const float4 d = *reinterpret_cast<const float4*>(dyl + r * 64 + cq * 4);
      const float4 v0 = *reinterpret_cast<const float4*>(pl + r * KT + ko * 8);
      const float4 v1 = *reinterpret_cast<const float4*>(pl + r * KT + ko * 8 + 4);
      const float dv[4] = {d.x, d.y, d.z, d.w};
      const float pv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] += dv[c] * pv[j];
    }
    __syncthreads();   // slab sl consumed; its row table slot is free
    if (sl + 1 < nslab) {
      store_slab();
      if (tid < SLAB) fill_rows(sl + 2);
    }
    __syncthreads();
  }
  // sum the 4 waves: waves 1..3 park their tiles, wave 0 adds and stores
  __syncthreads();
  if (wid > 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[((wid - 1) * 64 + cq * 4 + c) * KT + ko * 8 + j] = acc[c][j];
  }
  __syncthreads();
  if (wid == 0) {
    float* tile = a.ws + (long long)blockIdx.x * a.CO * a.K;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int co = co0 + cq * 4 + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kl = ko * 8 + j;
        float v = acc[c][j];
#pragma unroll
        for (int w = 0; w < 3; ++w) v += red[(w * 64 + cq * 4 + c) * KT + kl];
        if (k0 + kl < a.K) tile[(long long)co * a.K + k0 + kl] = v;
      }
    }
  }
}

// dw[i] += sum_g ws[g][i]: block (x, y) sums outputs [64x, 64x+64) over the
// y-th 1/16 of the G tiles (4 waves split it), one fp32 atomic per output
__global__ void __launch_bounds__(256) conv_small_wgrad_reduce(const float* __restrict__ ws,
                                                               float* __restrict__ dw, int n,
                                                               int G) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int g0 = (int)((long long)G * blockIdx.y / gridDim.y);
  const int g1 = (int)((long long)G * (blockIdx.y + 1) / gridDim.y);
  __shared__ float red[4][64];
  float v0 = 0.f, v1 = 0.f;
  if (i < n) {
    int g = g0 + w;
    for (; g + 4 < g1; g += 8) {
      v0 += ws[(long long)g * n + i];
      v1 += ws[(long long)(g + 4) * n + i];
    }
    for (; g < g1; g += 4) v0 += ws[(long long)g * n + i];
  }
  red[w][threadIdx.x & 63] = v0 + v1;
  __syncthreads();
  if (threadIdx.x < 64 && i < n)
    atomicAdd(dw + i, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                          red[3][threadIdx.x]);
}

static SmallConvArgs small_args(const u16* x, int xbytes, int sb, int sh, int sw, int sc, int B, int H, int W, int CI, int OH, int OW, int CO,
                                int R, int S, int stride, int pad) {
  SmallConvArgs a{};
  a.x = x;
  a.xbytes = xbytes;
  a.sb = sb; a.sh = sh; a.sw = sw; a.sc = sc;
  a.B = B; a.H = H; a.W = W; a.CI = CI; a.OH = OH; a.OW = OW; a.CO = CO;
  a.R = R; a.S = S; a.stride = stride; a.pad = pad; a.K = R * S * CI;
  a.P = (long long)B * OH * OW;
  return a;
}

int conv_small_max_k() { return 384; }   // forward weight tile [K][64] fp32 must fit LDS

long long conv_small_fwd_blocks(long long P) { return (P + 255) / 256; }

void launch_conv_small_fwd(const u16* x, int xbytes, int sb, int sh, int sw, int sc,
                           const u16* w, u16* y, float* part, int B, int H, int W, int CI, int OH,
                           int OW, int CO, int R, int S, int stride, int pad, hipStream_t s) {
  SmallConvArgs a = small_args(x, xbytes, sb, sh, sw, sc, B, H, W, CI, OH, OW, CO, R, S, stride, pad);
  a.w = w;
  a.y = y;
  a.part = part;
  const int Kp = (a.K + 7) / 8 * 8;
  const size_t lds = (size_t)((a.K * 64 + Kp + 3) & ~3) * 4 + 256 * kOutPitch * 2;
  const dim3 grid((unsigned)conv_small_fwd_blocks(a.P), (unsigned)(CO / 64));
  hipLaunchKernelGGL(conv_small_fwd_kernel, grid, dim3(256), lds, s, a);
}

int conv_small_wgrad_blocks(long long P, int CO, int R, int S, int CI) {
  (void)CO; (void)R; (void)S; (void)CI;
  // ~4 blocks (16 waves) per CU: one 4-wave block per CU leaves every SIMD a
  // single wave and the LDS -> FMA chains unhidden; whole 64-pixel slabs
  long long chunk = (P + 1023) / 1024;
  chunk = (chunk + 63) / 64 * 64;
  if (chunk < 256) chunk = 256;
  return (int)((P + chunk - 1) / chunk);
}

void launch_conv_small_wgrad(const u16* dy, const u16* x, int xbytes, int sb, int sh, int sw, int sc,
                             float* dw, float* ws, int B, int H, int W, int CI, int OH, int OW,
                             int CO, int R, int S, int stride, int pad, hipStream_t s) {
  SmallConvArgs a = small_args(x, xbytes, sb, sh, sw, sc, B, H, W, CI, OH, OW, CO, R, S, stride, pad);
  a.dy = dy;
  a.dw = dw;
  a.ws = ws;
  const int G = conv_small_wgrad_blocks(a.P, CO, R, S, CI);
  a.chunk = (int)((a.P + G - 1) / G);
  a.chunk = (a.chunk + 63) / 64 * 64;
  const dim3 grid((unsigned)G, (unsigned)(CO / 64), (unsigned)((a.K + 31) / 32));
  hipLaunchKernelGGL(conv_small_wgrad_kernel, grid, dim3(256), 0, s, a);
  const int n = CO * a.K;
  hipLaunchKernelGGL(conv_small_wgrad_reduce, dim3((n + 63) / 64, 16), dim3(256), 0, s, ws, dw, n,
                     G);
}


// ------------------------------------------------------------------------------
// CIFAR-style stem on the matrix cores: 3x3, stride 1, pad 1, CI <= 3 (K = 9*CI
// <= 27 padded to one 32-deep MFMA k-step), CO = 64.  The VALU kernels above spend
// ~60 us per ResNet-18 bs512 step in each direction on 1.8 GFLOP; here both
// passes are a handful of v_mfma_f32_16x16x32_bf16 per 16 / 32 pixels and run at
// the output / dY streaming rate.
//
// forward: D[co][px] = W[co][k] X[k][px].  The four 16-row weight fragments (all
//   64 output channels) live in registers for the whole block; a lane gathers its
//   B fragment (8 taps k = 8*(lane>>4)+i of pixel lane & 15) straight from the
//   L2-resident input through the buffer unit (padding taps read 0 via an
//   out-of-range offset).  The D layout gives a lane 4 consecutive channels of one
//   pixel: 8-B stores, and the BN partial sums of the stored (bf16-rounded)
//   values accumulate in registers, reduced once per block over the 16 pixel
//   lanes (xor shuffles) and the 4 waves (LDS) into slot blockIdx % kBnSlots.
// wgrad: D[co][k] = dY^T[co][px] X[px][k] over 32-pixel k-steps.  dY[32 px][64]
//   is staged row-major into a [32][128] LDS image (chunk-swizzled like the GEMM's
//   transposed operands, gemm.hip toff) and read with ds_read_b64_tr_b16, which
//   hands a lane 8 consecutive pixels of one channel; X fragments (8 consecutive
//   pixels of one tap: one image row when W % 8 == 0) are gathered from L2.  Each
//   wave owns a 32-pixel slice of a 128-pixel step, 8 MFMAs; the 4 waves' 64 x 32
//   tiles are summed in LDS and flushed with one fp32 atomic per weight per block.
typedef __bf16 bf16x8_t_ __attribute__((ext_vector_type(8)));
typedef short s16x4_t_ __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 s3_mfma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t_, a),
                                                 __builtin_bit_cast(bf16x8_t_, b), c, 0, 0, 0);
}

struct Stem3Args {
  const u16* x;
  const u16* w;     // [64][3][3][CI] bf16
  const u16* dy;    // [P][64]
  u16* y;           // [P][64]
  float* part;      // [2][kBnSlots][64]
  float* dw;        // [64][K] fp32 (+=)
  int sb, sh, sw, sc, xbytes;
  int H, W, CI, K;
  long long P;
  int groups;       // forward: 16-pixel groups per wave; wgrad: 128-pixel steps per block
};

// per-lane tap table for k = 8*(lane>>4) + i: (dr, ds) in [-1, 1], ci; invalid k -> r = 9
__device__ __forceinline__ void s3_taps(int CI, int K, int kg, int dr[8], int ds[8], int ci[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k = kg * 8 + i;
    const int c = k % CI, rs = k / CI;
    dr[i] = k < K ? rs / 3 - 1 : 9;
    ds[i] = rs % 3 - 1;
    ci[i] = c;
  }
}

__global__ void __launch_bounds__(256) stem3_fwd_kernel(Stem3Args a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
  // weight fragments: row co = 16j + col, k = 8kg..8kg+7
  bf16x8 wf[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = kg * 8 + i;
      wf[j].v[i] = k < a.K ? a.w[(16 * j + col) * a.K + k] : (u16)0;
    }
  int dr[8], ds[8], ci[8];
  s3_taps(a.CI, a.K, kg, dr, ds, ci);
  float s[4][4], q[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s[j][r] = 0.f; q[j][r] = 0.f; }
  const long long base = ((long long)blockIdx.x * 4 + wid) * a.groups * 16;
  __shared__ __attribute__((aligned(16))) u16 stg[4][16][72];   // per wave: 16 pixels x 64 ch (+pad)
  // the 8-tap gather of group gi+1 is issued before group gi's MFMAs and stores:
  // one dependent L2 round trip per group otherwise set the kernel time (a wave
  // walks its groups in sequence at 2 waves / SIMD)
  auto gather = [&](int gi, bf16x8& xf) {
    const long long px = base + gi * 16 + col;
    const bool pv = px < a.P;
    const int p32 = pv ? (int)px : 0;
    const int ow = p32 % a.W, t = p32 / a.W;
    const int oh = t % a.H, b = t / a.H;
    const int boff = b * a.sb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ih = oh + dr[i], iw = ow + ds[i];
      const bool ok = pv && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const int off = ok ? 2 * (boff + ih * a.sh + iw * a.sw + ci[i] * a.sc) : 0x7ffffff0;
      xf.v[i] = __builtin_bit_cast(u16, __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
    }
  };
  bf16x8 xnext;
  gather(0, xnext);
  for (int gi = 0; gi < a.groups; ++gi) {
    const long long px = base + gi * 16 + col;
    const bool pv = px < a.P;
    const bf16x8 xf = xnext;
    if (gi + 1 < a.groups) gather(gi + 1, xnext);
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = s3_mfma(wf[j], xf, f32x4{0.f, 0.f, 0.f, 0.f});
    // D: lane holds channels 16j + 4kg + r of pixel `col`... of THIS group's pixel px
    // (D row = co, D col = pixel: lane = (row block kg, col))
    // the D fragments (8 B per lane: 16 pixels x 32 B per store instruction) go
    // through a wave-private LDS tile and leave as whole 128-B pixel rows (16 B
    // per lane, 8 pixels per instruction); LDS ops of one wave complete in order
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        o.v[r] = f2bf(acc[j][r]);
        const float v = pv ? bf2f(o.v[r]) : 0.f;
        s[j][r] += v;
        q[j][r] += v * v;
      }
      *reinterpret_cast<bf16x4*>(&stg[wid][col][16 * j + 4 * kg]) = o;
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int pr = hh * 8 + (lane >> 3), ck = lane & 7;
      const long long pxo = base + gi * 16 + pr;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stg[wid][pr][ck * 8]);
      if (pxo < a.P) *reinterpret_cast<bf16x8*>(a.y + pxo * 64 + ck * 8) = v;
    }
  }
  if (a.part == nullptr) return;
  // reduce over the 16 pixel lanes sharing kg
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s[j][r] += __shfl_xor(s[j][r], o, 64);
        q[j][r] += __shfl_xor(q[j][r], o, 64);
      }
  __shared__ float red[4][2][64];
  if (col == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wid][0][16 * j + 4 * kg + r] = s[j][r];
        red[wid][1][16 * j + 4 * kg + r] = q[j][r];
      }
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = threadIdx.x & 63, h = threadIdx.x >> 6;
    const float v = red[0][h][c] + red[1][h][c] + red[2][h][c] + red[3][h][c];
    const int slot = blockIdx.x % kBnSlots;
    atomicAdd(a.part + (long long)(h * kBnSlots + slot) * 64 + c, v);
  }
}

// [32][128] bf16 transposed-read image: 32-B granule u of row r holds logical
// granule u ^ tf(r) (gemm.hip toff<128>)
__device__ __forceinline__ int s3_tf(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }
__device__ __forceinline__ int s3_toff(int row, int col) {
  return row * 128 + (((col >> 4) ^ s3_tf(row)) << 4) + (col & 15);
}

__global__ void __launch_bounds__(256) stem3_wgrad_kernel(Stem3Args a) {
  __shared__ __attribute__((aligned(16))) u16 img[4][32 * 128];
  __shared__ float tile[64][33];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
  // this lane's two B columns: taps 16t + col, t = 0, 1
  int tdr[2], tds[2], tci[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = 16 * t + col;
    tdr[t] = k < a.K ? (k / a.CI) / 3 - 1 : 9;
    tds[t] = (k / a.CI) % 3 - 1;
    tci[t] = k % a.CI;
  }
  f32x4 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) { acc[j][0] = f32x4{0.f, 0.f, 0.f, 0.f}; acc[j][1] = acc[j][0]; }
  u16* im = img[wid];
  const long long blk0 = (long long)blockIdx.x * a.groups * 128;
  // step st+1's dY chunks and X taps are loaded into registers before step st's
  // LDS image write and MFMAs (each step was one dependent round trip)
  auto load_step = [&](int st, bf16x8 (&dv)[4], bf16x8 (&xf)[2]) {
    const long long p0 = blk0 + (long long)st * 128 + wid * 32;   // this wave's 32 pixels
    // dY[p0 .. p0+32)[0..64) : 256 real 16-B chunks per wave image, 4 per lane
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * 64 + lane;              // logical chunk: row e >> 3, cols (e & 7) * 8
      const int row = e >> 3, c0 = (e & 7) * 8;
      const long long p = p0 + row;
      if (p < a.P) dv[u] = *reinterpret_cast<const bf16x8*>(a.dy + p * 64 + c0);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) dv[u].v[i] = 0;
      }
    }
    // X fragments: pixels p0 + 8kg + i (one image row when W % 8 == 0), taps 16t + col
    {
      const long long pb = p0 + 8 * kg;
      const bool pv = pb < a.P;
      const int p32 = pv ? (int)pb : 0;
      const int ow0 = p32 % a.W, t0 = p32 / a.W;
      const int oh = t0 % a.H, b = t0 / a.H;
      const int boff = b * a.sb;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ih = oh + tdr[t];
        const bool rok = pv && (unsigned)ih < (unsigned)a.H;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int iw = ow0 + i + tds[t];
          const bool ok = rok && (unsigned)iw < (unsigned)a.W && pb + i < a.P;
          const int off = ok ? 2 * (boff + ih * a.sh + iw * a.sw + tci[t] * a.sc) : 0x7ffffff0;
          xf[t].v[i] = __builtin_bit_cast(u16, __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
        }
      }
    }
  };
  bf16x8 dnext[4], xnext[2];
  load_step(0, dnext, xnext);
  for (int st = 0; st < a.groups; ++st) {
    bf16x8 dcur[4], xf[2];
#pragma unroll
    for (int u = 0; u < 4; ++u) dcur[u] = dnext[u];
    xf[0] = xnext[0];
    xf[1] = xnext[1];
    if (st + 1 < a.groups) load_step(st + 1, dnext, xnext);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * 64 + lane;
      *reinterpret_cast<bf16x8*>(im + s3_toff(e >> 3, (e & 7) * 8)) = dcur[u];   // 8 cols stay in one granule
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS image writes landed
    __builtin_amdgcn_wave_barrier();
    // A fragments (co tile j): lane row co = 16j + col... read transposed: 8 consecutive
    // pixels (k) 8kg..8kg+7 of channel column
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
      const int row = 8 * g + qq;
      const s16x4_t_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4_t_*)(im + s3_toff(row, 16 * j + 4 * pp)));
      const s16x4_t_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4_t_*)(im + s3_toff(row + 4, 16 * j + 4 * pp)));
      const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      acc[j][0] = s3_mfma(af, xf[0], acc[j][0]);
      acc[j][1] = s3_mfma(af, xf[1], acc[j][1]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // sum the 4 waves' [64 co][32 k] tiles, one atomic per weight per block
  // D: lane holds rows co = 16j + 4kg + r, column k = 16t + col
  for (int w = 0; w < 4; ++w) {
    if (wid == w) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float& d = tile[16 * j + 4 * kg + r][16 * t + col];
            d = (w == 0 ? 0.f : d) + acc[j][t][r];
          }
    }
    __syncthreads();
  }
  for (int e = tid; e < 64 * a.K; e += 256) {
    const int co = e / a.K, k = e % a.K;
    atomicAdd(a.dw + e, tile[co][k]);
  }
}

bool stem3_supported(int CI, int R, int S, int CO, int stride, int pad, int W) {
  return CI >= 1 && CI <= 3 && R == 3 && S == 3 && CO == 64 && stride == 1 && pad == 1 &&
         W % 8 == 0;
}

void launch_stem3_fwd(const u16* x, int xbytes, int sb, int sh, int sw, int sc, const u16* w,
                      u16* y, float* part, int B, int H, int W, int CI, hipStream_t s) {
  Stem3Args a{};
  a.x = x; a.w = w; a.y = y; a.part = part;
  a.sb = sb; a.sh = sh; a.sw = sw; a.sc = sc; a.xbytes = xbytes;
  a.H = H; a.W = W; a.CI = CI; a.K = 9 * CI;
  a.P = (long long)B * H * W;
  // 16 groups of 16 pixels per wave (1024 pixels per block) unless that leaves
  // fewer than ~2 blocks per CU
  static const int gmax = [] {
    const char* e = getenv("DMP_STEM3_GROUPS");   // A/B knob: max groups per wave
    return e ? atoi(e) : 16;
  }();
  int groups = gmax > 0 ? gmax : 16;
  while (groups > 1 && (a.P + 64LL * groups - 1) / (64LL * groups) < 512) groups >>= 1;
  a.groups = groups;
  const long long nb = (a.P + 64LL * groups - 1) / (64LL * groups);
  hipLaunchKernelGGL(stem3_fwd_kernel, dim3((unsigned)nb), dim3(256), 0, s, a);
}

void launch_stem3_wgrad(const u16* dy, const u16* x, int xbytes, int sb, int sh, int sw, int sc,
                        float* dw, int B, int H, int W, int CI, hipStream_t s) {
  Stem3Args a{};
  a.x = x; a.dy = dy; a.dw = dw;
  a.sb = sb; a.sh = sh; a.sw = sw; a.sc = sc; a.xbytes = xbytes;
  a.H = H; a.W = W; a.CI = CI; a.K = 9 * CI;
  a.P = (long long)B * H * W;
  // ~512 blocks: 128-pixel steps per block
  static const long long target = [] {
    const char* e = getenv("DMP_STEM3_WG_BLOCKS");   // A/B knob: target block count
    const long long v = e ? atoll(e) : 512;
    return v > 0 ? v : 512;
  }();
  const long long steps = (a.P + 127) / 128;
  long long per = (steps + target - 1) / target;
  // >= 4 steps per block: at the reference batch (512 steps) 128 blocks beat 512 --
  // a quarter of the per-block atomic flushes (ResNet-18 bs64 -0.75 %,
  // profiles/stem3_wgrad_grid_r6.txt); batches >= 256 already run >= 4 per block
  if (per < 4) per = 4;
  a.groups = (int)per;
  const long long nb = (steps + per - 1) / per;
  hipLaunchKernelGGL(stem3_wgrad_kernel, dim3((unsigned)nb), dim3(256), 0, s, a);
}

}  // namespace dmp
