// ImageNet stem convolution (ResNet-50: 7x7 / stride 2 / pad 3, 3 -> 64
// channels) on MFMA without a patch matrix.
//
// The patch-matrix route (im2col.hip + gemm.hip) writes and re-reads a
// 1.6M x 152 bf16 matrix (488 MB at batch 128) and ran the stem at 686 us per
// step, behind MIOpen's 369.  Here the input is re-laid out once as a
// space-to-depth image (2x2 pixels x 4 channels, the 4th zero):
//   xs[b][i][j][(dy*2+dx)*4 + c] = x[b][2i+dy][2j+dx][c]        (H/2 x W/2 x 16)
// and the stride-2 7x7 conv becomes a stride-1 4x4 conv over xs with padding
// 2 before / 1 after and the packed weight
//   Wp[co][(r'*4+s')*16 + (dy*2+dx)*4 + c] = W[co][2r'+dy-1][2s'+dx-1][c]
// (zero where the original tap or channel does not exist): K = 256 instead of
// 147, every 8-value MFMA fragment a 16-B piece of one staged xs pixel.
//
// Forward: persistent blocks, the whole packed weight (32 KB) resident in LDS,
// tiles of 4 output rows (one per wave) streamed through an LDS-DMA ring of
// halo images (7 x (W/2 + 3) xs pixels); BN partial sums of the stored output
// reduced once per block.  Weight gradient: dWp[co][k] += dY^T xs_gather over
// 2-row tiles (dY rows and the xs halo staged per tile, both read transposed
// with ds_read_b64_tr_b16), fp32 atomics once per block, then folded back to
// the 64 x 7 x 7 x 3 layout in the grad arena.  The stem's input is data: no
// data gradient.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace dmp {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr unsigned kOOBs = 0x80000000u;
constexpr int kSCO = 64, kSK = 256;   // output channels, packed reduction length
constexpr int kSAPW = 8;              // max halo DMA pieces per wave per tile

__device__ __forceinline__ f32x4 smfma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// LDS DMA from inline asm, completion counted by hand (see conv.hip)
__device__ __forceinline__ void sdma16(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                       u16* lds_wave_base) {
  const unsigned m0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave_base;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "{m0}"(m0));
}

template <int N>
__device__ __forceinline__ void swait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}

// vmcnt wait with a launch-time (wave-uniform) count
__device__ __forceinline__ void swait_vm_n(int n) {
  switch (n) {
#define DMP_SWV(k) \
  case k:          \
    swait_vm<k>(); \
    break;
    DMP_SWV(1) DMP_SWV(2) DMP_SWV(3) DMP_SWV(4) DMP_SWV(5) DMP_SWV(6) DMP_SWV(7) DMP_SWV(8)
    DMP_SWV(9) DMP_SWV(10) DMP_SWV(11) DMP_SWV(12) DMP_SWV(13) DMP_SWV(14) DMP_SWV(15) DMP_SWV(16)
    DMP_SWV(17) DMP_SWV(18) DMP_SWV(19) DMP_SWV(20) DMP_SWV(21) DMP_SWV(22) DMP_SWV(23) DMP_SWV(24)
#undef DMP_SWV
    default:
      swait_vm<0>();
  }
}

__device__ __forceinline__ float srow_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// 32-B granule swizzle of the [pixel][64] dY rows read transposed (as the
// weight-gradient kernels of conv_wgrad.hip)
__device__ __forceinline__ int sg_off(int row, int col) {
  const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return row * 64 + ((((col >> 4) ^ f)) << 4) + (col & 15);
}

}  // namespace

// --------------------------------------------------------------- re-layouts
__global__ void __launch_bounds__(256) stem_s2d_kernel(const u16* __restrict__ x,
                                                       u16* __restrict__ xs, int B, int H, int W) {
  const int OH = H / 2, OW = W / 2;
  const long long total = (long long)B * OH * OW;
  const long long gs = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gs) {
    const int j = (int)(p % OW);
    const long long t = p / OW;
    const int i = (int)(t % OH);
    const long long b = t / OH;
    bf16x8 lo, hi;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1, dx = d & 1;
      const u16* src = x + ((b * H + 2 * i + dy) * W + 2 * j + dx) * 3;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const u16 v = c < 3 ? src[c] : (u16)0;
        if (d < 2) lo.v[d * 4 + c] = v;
        else hi.v[(d - 2) * 4 + c] = v;
      }
    }
    reinterpret_cast<bf16x8*>(xs + p * 16)[0] = lo;
    reinterpret_cast<bf16x8*>(xs + p * 16)[1] = hi;
  }
}

// W [64][7][7][3] (channels_last [co][r][s][c]) -> Wp [64][256]
__global__ void __launch_bounds__(256) stem_wpack_kernel(const u16* __restrict__ w,
                                                         u16* __restrict__ wp) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= kSCO * kSK) return;
  const int co = idx / kSK, k = idx % kSK;
  const int t = k >> 4, rem = k & 15;
  const int rp = t >> 2, sp = t & 3, d = rem >> 2, c = rem & 3;
  const int r = 2 * rp + (d >> 1) - 1, s = 2 * sp + (d & 1) - 1;
  wp[idx] = (c < 3 && r >= 0 && r < 7 && s >= 0 && s < 7) ? w[((co * 7 + r) * 7 + s) * 3 + c]
                                                           : (u16)0;
}

// dW [64][7][7][3] fp32 += the matching entries of dWp [64][256]
__global__ void __launch_bounds__(256) stem_wfold_kernel(const float* __restrict__ dwp,
                                                         float* __restrict__ dw) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= kSCO * 147) return;
  const int co = idx / 147, rem = idx % 147;
  const int r = rem / 21, s = (rem / 3) % 7, c = rem % 3;
  const int rp = (r + 1) >> 1, dy = (r + 1) & 1, sp = (s + 1) >> 1, dx = (s + 1) & 1;
  dw[idx] += dwp[co * kSK + (rp * 4 + sp) * 16 + (dy * 2 + dx) * 4 + c];
}

// ------------------------------------------------------------------ forward
struct StemGeom {
  int OH, OW, TH, APW, ntiles;
};

// bias (fp32 [64], may be null) and relu: the inference-time BatchNorm fold
// (ops/eval_fold.py) -- the eval forward's stem is then ONE launch instead of
// im2col + GEMM
template <int TM, int NS, bool STATS>
__global__ void __launch_bounds__(256) stem_fwd_kernel(const u16* __restrict__ xs,
                                                       const u16* __restrict__ wp,
                                                       u16* __restrict__ y, float* __restrict__ part,
                                                       int B, StemGeom sg,
                                                       const float* __restrict__ bias, int relu) {
  constexpr int NW = 4, TN = kSCO / 16, NSTEP = kSK / 32;
  constexpr int OW = TM * 16, W2 = OW + 3;
  extern __shared__ __attribute__((aligned(16))) u16 lds_s[];
  u16* Ws = lds_s;                         // [64][256] (16-B chunks XOR co & 15)
  u16* Hs = lds_s + kSCO * kSK;            // NS x [APW*NW*32 pixels][16]
  const int APW = sg.APW, OH = sg.OH;
  const int STAGE = APW * NW * 512;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, ntiles = sg.ntiles;
  const int nt = (ntiles - (int)blockIdx.x + G - 1) / G;
  if (nt <= 0) return;
  const int tpi = OH / NW;                 // 4-row tiles per image
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xs, 0, (int)(2LL * B * OH * OW * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wp, 0, 2 * kSCO * kSK, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)y, 0, (int)(2LL * B * OH * OW * kSCO), 0x00020000);

  // resident weights: 32 pieces of 1 KiB, 8 per wave; source-side chunk swizzle
#pragma unroll
  for (int j = 0; j < kSCO * kSK / 512 / NW; ++j) {
    const int ins = wid + j * NW;
    const int e = ins * 512 + lane * 8;
    const int co = e / kSK, cp = (e % kSK) >> 3;
    sdma16(rsW, 2u * (unsigned)(co * kSK + ((cp ^ (co & 15)) << 3)), Ws + ins * 512);
  }
  // halo slots: staged pixel q (32 per piece, 2 lanes per pixel) -> offset from the
  // tile's first output-row pixel + {valid, source row - oh0}
  int x_off[kSAPW];
  unsigned x_inf[kSAPW];
#pragma unroll
  for (int j = 0; j < kSAPW; ++j) {
    x_off[j] = 0;
    x_inf[j] = 0;
    if (j < APW) {
      const int q = (wid + j * NW) * 32 + (lane >> 1), half = lane & 1;
      const int hr = q / W2, hc = q - hr * W2;
      const int dh = hr - 2, w = hc - 2;
      const bool ok = hr < NW + 3 && (unsigned)w < (unsigned)OW;
      x_off[j] = (dh * OW + w) * 16 + half * 8;
      x_inf[j] = (ok ? 0x80000000u : 0u) | ((unsigned)(dh + 64) << 8);
    }
  }
  auto tile_of = [&](int k) { return (int)blockIdx.x + k * G; };
  auto stage = [&](int buf, int k) {
    u16* As = Hs + buf * STAGE;
    const int t = tile_of(k);
    const bool live = k < nt;
    const int b = t / tpi, oh0 = (t - b * tpi) * NW;
    const int m0 = (b * OH + oh0) * OW;
#pragma unroll
    for (int j = 0; j < kSAPW; ++j) {
      if (j < APW) {
        const unsigned inf = x_inf[j];
        const int dh = (int)((inf >> 8) & 255) - 64;
        const bool ok = live && (inf >> 31) && (unsigned)(oh0 + dh) < (unsigned)OH;
        sdma16(rsX, ok ? 2u * (unsigned)(m0 * 16 + x_off[j]) : kOOBs, As + (wid + j * NW) * 512);
      }
    }
  };

  const int l16 = lane & 15, kg = lane >> 4;
  f32x4 acc[TM][TN];
  auto compute = [&](int buf) {
    const u16* As = Hs + buf * STAGE;
    bf16x8 af[2][TM], bw[2][TN];
    auto load = [&](int st, int slot) {
      const int t = 2 * st + (kg >> 1), rp = t >> 2, sp = t & 3, half = kg & 1;
      const int prow = (wid + rp) * W2 + sp + l16;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[slot][i] = *reinterpret_cast<const bf16x8*>(As + (prow + i * 16) * 16 + half * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = j * 16 + l16, c = st * 4 + kg;
        bw[slot][j] = *reinterpret_cast<const bf16x8*>(Ws + co * kSK + ((c ^ (co & 15)) << 3));
      }
    };
    load(0, 0);
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      if (st + 1 < NSTEP) load(st + 1, (st + 1) & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = smfma(bw[st & 1][j], af[st & 1][i], acc[i][j]);
    }
  };

  float s_sum[TN][4], s_sq[TN][4], bj[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s_sum[j][r] = 0.f;
      s_sq[j][r] = 0.f;
      bj[j][r] = bias != nullptr ? bias[j * 16 + 4 * kg + r] : 0.f;
    }
  // The D fragments (8 B per lane: a store instruction wrote 16 pixels x 32 B)
  // go through a wave-private LDS tile and leave as whole 128-B pixel rows,
  // 16 B per lane, 8 rows per instruction (LDS ops of one wave complete in
  // order).  DMP_STEM_ROWSTORE=0 at build time: the direct fragment stores.
#ifndef DMP_STEM_ROWSTORE
#define DMP_STEM_ROWSTORE 1
#endif
  __shared__ __attribute__((aligned(16))) u16 stg[NW][16][kSCO + 8];
  auto epilogue = [&](int k) {
    const int t = tile_of(k);
    const int b = t / tpi, oh0 = (t - b * tpi) * NW;
    const int mrow = (b * OH + oh0 + wid) * OW;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned rowoff = 2u * (unsigned)((mrow + i * 16 + l16) * kSCO);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + 4 * kg;
        u16 hv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[i][j][r] + bj[j][r];
          if (relu) t = fmaxf(t, 0.f);
          hv[r] = f2bf(t);
          if (STATS) {
            const float v = bf2f(hv[r]);
            s_sum[j][r] += v;
            s_sq[j][r] += v * v;
          }
        }
        const u32x2_t packed = {(u32)hv[0] | ((u32)hv[1] << 16), (u32)hv[2] | ((u32)hv[3] << 16)};
        if constexpr (DMP_STEM_ROWSTORE)
          *reinterpret_cast<u32x2_t*>(&stg[wid][l16][n]) = packed;
        else
          __builtin_amdgcn_raw_buffer_store_b64(packed, rsY, rowoff + 2u * n, 0, 0);
      }
      if constexpr (DMP_STEM_ROWSTORE) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int pr = hh * 8 + (lane >> 3), ck = lane & 7;
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(&stg[wid][pr][ck * 8]);
          __builtin_amdgcn_raw_buffer_store_b128(
              v, rsY, 2u * (unsigned)((mrow + i * 16 + pr) * kSCO + ck * 8), 0, 0);
        }
      }
    }
  };

  // weights first, then the ring; the first stage's wait also covers the weights
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage(s, s);
  for (int k = 0; k < nt; ++k) {
    // tile k (and, at k = 0, the weights) landed: later loads are only the
    // (NS-2) younger stages' pieces (epilogue stores may retire in any order)
    if constexpr (NS == 2) swait_vm<0>();
    else swait_vm_n((NS - 2) * APW);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stage((k + NS - 1) % NS, k + NS - 1);
    if (k > 0) epilogue(k - 1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    compute(k % NS);
  }
  epilogue(nt - 1);
  if (STATS) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s_sum[j][r] = srow_sum16(s_sum[j][r]);
        s_sq[j][r] = srow_sum16(s_sq[j][r]);
      }
    swait_vm<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(Hs);
    if (l16 == 15) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = j * 16 + 4 * kg + r;
          red[wid * kSCO + nl] = s_sum[j][r];
          red[NW * kSCO + wid * kSCO + nl] = s_sq[j][r];
        }
    }
    __syncthreads();
    if (tid < kSCO) {
      float ss = 0.f, qq = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) { ss += red[w * kSCO + tid]; qq += red[NW * kSCO + w * kSCO + tid]; }
      const int slot = blockIdx.x % kBnSlots;
      atomicAdd(part + (long long)slot * kSCO + tid, ss);
      atomicAdd(part + (long long)(kBnSlots + slot) * kSCO + tid, qq);
    }
  }
}

// ----------------------------------------------------------- weight gradient
// Tile = 2 output rows (2*OW pixels).  Wave w owns tap row r' = w: the 4 taps
// (w, s') x all 64 output channels, acc[co tile][s'].
template <int TM, int NS>
__global__ void __launch_bounds__(256) stem_wgrad_kernel(const u16* __restrict__ dy,
                                                         const u16* __restrict__ xs,
                                                         float* __restrict__ dwp, int B,
                                                         StemGeom sg) {
  constexpr int NW = 4, TH = 2, OW = TM * 16, W2 = OW + 3, BM = TH * OW;
  constexpr int D_INS = BM * kSCO / 512;               // dY pieces per tile
  static_assert(D_INS % NW == 0, "dY pieces per wave");
  constexpr int D_PW = D_INS / NW, NPK = BM / 32;
  extern __shared__ __attribute__((aligned(16))) u16 lds_s[];
  const int APW = sg.APW, OH = sg.OH;
  const int STAGE = D_INS * 512 + APW * NW * 512;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, ntiles = sg.ntiles;
  const int nt = (ntiles - (int)blockIdx.x + G - 1) / G;
  if (nt <= 0) return;
  const int tpi = OH / TH;
  const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy, 0, (int)(2LL * B * OH * OW * kSCO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xs, 0, (int)(2LL * B * OH * OW * 16), 0x00020000);

  int d_off[D_PW];
#pragma unroll
  for (int j = 0; j < D_PW; ++j) {
    const int row = (wid + j * NW) * 8 + lane / 8, pch = lane % 8;
    const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    d_off[j] = row * kSCO + (((pch >> 1) ^ f) * 16) + (pch & 1) * 8;
  }
  int x_off[kSAPW];
  unsigned x_inf[kSAPW];
#pragma unroll
  for (int j = 0; j < kSAPW; ++j) {
    x_off[j] = 0;
    x_inf[j] = 0;
    if (j < APW) {
      const int q = (wid + j * NW) * 32 + (lane >> 1), half = lane & 1;
      const int hr = q / W2, hc = q - hr * W2;
      const int dh = hr - 2, w = hc - 2;
      const bool ok = hr < TH + 3 && (unsigned)w < (unsigned)OW;
      x_off[j] = (dh * OW + w) * 16 + half * 8;
      x_inf[j] = (ok ? 0x80000000u : 0u) | ((unsigned)(dh + 64) << 8);
    }
  }
  auto tile_of = [&](int k) { return (int)blockIdx.x + k * G; };
  auto stage = [&](int buf, int k) {
    u16* Ds = lds_s + buf * STAGE;
    u16* Xs = Ds + D_INS * 512;
    const int t = tile_of(k);
    const bool live = k < nt;
    const int b = t / tpi, oh0 = (t - b * tpi) * TH;
    const int m0 = (b * OH + oh0) * OW;
#pragma unroll
    for (int j = 0; j < D_PW; ++j)
      sdma16(rsD, live ? 2u * (unsigned)(m0 * kSCO + d_off[j]) : kOOBs, Ds + (wid + j * NW) * 512);
#pragma unroll
    for (int j = 0; j < kSAPW; ++j) {
      if (j < APW) {
        const unsigned inf = x_inf[j];
        const int dh = (int)((inf >> 8) & 255) - 64;
        const bool ok = live && (inf >> 31) && (unsigned)(oh0 + dh) < (unsigned)OH;
        sdma16(rsX, ok ? 2u * (unsigned)(m0 * 16 + x_off[j]) : kOOBs, Xs + (wid + j * NW) * 512);
      }
    }
  };

  // lane (g = lane>>4, li = lane&15, q = li>>2, pc = li&3): reduction rows
  // pk*32 + 8g + q and +4; staged halo pixel of those rows at tap (w, 0)
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pc = li & 3;
  int xr_lo[NPK], xr_hi[NPK];
#pragma unroll
  for (int pk = 0; pk < NPK; ++pk) {
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int pl = pk * 32 + 8 * g + q + 4 * hs;
      const int th = pl / OW, tw = pl - th * OW;
      const int xr = (th + wid) * W2 + tw;
      if (hs) xr_hi[pk] = xr; else xr_lo[pk] = xr;
    }
  }
  auto trd = [&](const u16* img, int row, int col) -> s16x4_t {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + sg_off(row, col)));
  };
  auto trx = [&](const u16* img, int px) -> s16x4_t {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + px * 16 + 4 * pc));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[i][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    const u16* Ds = lds_s + buf * STAGE;
    const u16* Xs = Ds + D_INS * 512;
#pragma unroll
    for (int pk = 0; pk < NPK; ++pk) {
      bf16x8 af[4], bx[4];
      const int drow = pk * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x4_t lo = trd(Ds, drow, i * 16 + 4 * pc), hi = trd(Ds, drow + 4, i * 16 + 4 * pc);
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const s16x4_t lo = trx(Xs, xr_lo[pk] + s), hi = trx(Xs, xr_hi[pk] + s);
        bx[s] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][s] = smfma(af[i], bx[s], acc[i][s]);
    }
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage(s, s);
  for (int k = 0; k < nt; ++k) {
    if constexpr (NS == 2) swait_vm<0>();
    else swait_vm_n((NS - 2) * (D_PW + APW));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stage((k + NS - 1) % NS, k + NS - 1);
    compute(k % NS);
  }
  swait_vm<0>();
  // D layout: lane holds rows co = 4*(lane>>4)+rr of column ci = lane & 15
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = i * 16 + 4 * g + rr;
        atomicAdd(dwp + co * kSK + (wid * 4 + s) * 16 + li, acc[i][s][rr]);
      }
}

// ---------------------------------------------------------------- launchers
namespace {
int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}
template <typename K>
void allow_lds160(K kernel) {
  static bool done = false;
  if (!done) {
    // the dynamic cap excludes the kernel's static LDS (stem_fwd's store tile)
    hipFuncAttributes fa{};
    const int stat = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kernel)) == hipSuccess
                         ? (int)fa.sharedSizeBytes
                         : 0;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - stat);
    done = true;
  }
}
}  // namespace

// the s2d stem applies to 7x7 / 2 / 3 convs, 3 -> 64 channels, with H % 8 == 0
// and W / 2 == 16 * 7 (the 224 x 224 ImageNet input: 112-pixel output rows)
bool stem_supported(int H, int W) { return H % 8 == 0 && W == 224; }

void launch_stem_s2d(const u16* x, u16* xs, int B, int H, int W, hipStream_t s) {
  const long long total = (long long)B * (H / 2) * (W / 2);
  hipLaunchKernelGGL(stem_s2d_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, x, xs, B, H,
                     W);
}

void launch_stem_wpack(const u16* w, u16* wp, hipStream_t s) {
  hipLaunchKernelGGL(stem_wpack_kernel, dim3(kSCO * kSK / 256), dim3(256), 0, s, w, wp);
}

void launch_stem_wfold(const float* dwp, float* dw, hipStream_t s) {
  hipLaunchKernelGGL(stem_wfold_kernel, dim3((kSCO * 147 + 255) / 256), dim3(256), 0, s, dwp, dw);
}

void launch_stem_fwd(const u16* xs, const u16* wp, u16* y, float* part, int B, int H, int W,
                     hipStream_t s, const float* bias, bool relu) {
  constexpr int TM = 7, NS = 3;
  StemGeom g{};
  g.OH = H / 2;
  g.OW = W / 2;
  g.TH = 4;
  const int pieces = ((g.TH + 3) * (g.OW + 3) + 31) / 32;
  g.APW = (pieces + 3) / 4;
  g.ntiles = B * (g.OH / g.TH);
  const size_t lds = 2 * ((size_t)kSCO * kSK + (size_t)NS * g.APW * 4 * 512);
  const int grid = std::min(g.ntiles, num_cus());
  if (part) {
    allow_lds160(stem_fwd_kernel<TM, NS, true>);
    hipLaunchKernelGGL((stem_fwd_kernel<TM, NS, true>), dim3(grid), dim3(256), lds, s, xs, wp, y,
                       part, B, g, bias, relu ? 1 : 0);
  } else {
    allow_lds160(stem_fwd_kernel<TM, NS, false>);
    hipLaunchKernelGGL((stem_fwd_kernel<TM, NS, false>), dim3(grid), dim3(256), lds, s, xs, wp, y,
                       part, B, g, bias, relu ? 1 : 0);
  }
}

// dwp: fp32 [64][256], zeroed here then accumulated
void launch_stem_wgrad(const u16* dy, const u16* xs, float* dwp, int B, int H, int W,
                       hipStream_t s) {
  constexpr int TM = 7, NS = 3;
  StemGeom g{};
  g.OH = H / 2;
  g.OW = W / 2;
  g.TH = 2;
  const int pieces = ((g.TH + 3) * (g.OW + 3) + 31) / 32;
  g.APW = (pieces + 3) / 4;
  g.ntiles = B * (g.OH / g.TH);
  const size_t lds = 2 * (size_t)NS * (2 * 112 * kSCO + (size_t)g.APW * 4 * 512);
  // a native fill kernel, not hipMemsetAsync: a memset node captured into the step's
  // graph raced with the previous replay (optim.hip zero_fill), and it is no dmp:: kernel
  launch_zero_fill(dwp, (long long)sizeof(float) * kSCO * kSK, s);
  const int grid = std::min(g.ntiles, num_cus());
  allow_lds160(stem_wgrad_kernel<TM, NS>);
  hipLaunchKernelGGL((stem_wgrad_kernel<TM, NS>), dim3(grid), dim3(256), lds, s, dy, xs, dwp, B, g);
}

}  // namespace dmp
