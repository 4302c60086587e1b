// NHWC bf16 convolution as implicit GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Not a translation of anything in the reference (it only calls torch.nn.Conv2d,
// /root/reference/example/models.py:8-9,28-38); these kernels replace the
// ATen/MIOpen `convolution` + `convolution_backward` rows of SURVEY §2.3.
//
//   fwd   : Y[m][co]  = sum_k  X_gather[m][k] * W[co][k]     k = (r, s, ci), ci fastest
//   dgrad : dX[m][ci] = sum_k dY_tgather[m][k] * Wt[ci][k]    k = (r, s, co), Wt = W^T per tap
//           ("transposed gather": th = h + pad - r must be a multiple of stride)
//   wgrad : dW[co][k] += sum_p dY[p][co] * X_gather[p][k]     split over p, fp32 atomics
//           straight into the flat fp32 grad arena (channels_last weight layout).
//
// Tiles are staged through LDS with an XOR swizzle that makes the 16-lane
// ds_read_b128 operand fetches bank-conflict free (derivation in the comments at
// swz()).  fwd/dgrad compute D^T = W * X^T so each lane ends up owning 4
// consecutive output channels of one pixel (8-byte NHWC stores), and can fold
// per-channel BatchNorm partial sums into the epilogue (no extra pass over Y).
// wgrad reads both [p][*] tiles with ds_read_b64_tr_b16 (hardware transpose).
#include "common.h"

namespace dmp {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

struct ConvArgs {
  const u16* x;     // gathered operand, NHWC [B][GH][GW][CI]
  const u16* w;     // [CO][R][S][CI]
  u16* y;           // [B][OH][OW][CO]
  float* part;      // optional BN partials [2][gridDim.x][CO]
  int B, GH, GW, CI, OH, OW, CO, R, S, stride, pad;
  long long M;      // B*OH*OW
};

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// 16-byte chunk swizzle for a row-major [rows][BK] bf16 LDS tile.
//  BK=64 (128-B rows, 2 rows per 256-B bank row): chunk ^= (row>>1)&7
//  BK=32 ( 64-B rows, 4 rows per bank row):       chunk ^= (-(row>>2))&3
// Both make each ds_read_b128 lane group (rows l&15, chunk c + (l>>4)) hit 16
// distinct 16-B slots.
template <int BK>
__device__ __forceinline__ int swz(int row, int c) {
  if constexpr (BK == 64) return c ^ ((row >> 1) & 7);
  else return c ^ ((-(row >> 2)) & 3);
}

template <int BM, int BN, int BK, int WM, int WN, bool TRANS, bool STATS>
__global__ void __launch_bounds__(64 * WM * WN) conv_igemm_kernel(ConvArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int CPR = BK / 8;
  constexpr int ROWSTEP = NT / CPR;
  constexpr int A_PER = BM / ROWSTEP;
  constexpr int B_PER = (BN + ROWSTEP - 1) / ROWSTEP;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(BM % ROWSTEP == 0, "A tile must split evenly over threads");
  __shared__ __attribute__((aligned(16))) u16 lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ch = tid % CPR, r0 = tid / CPR;
  const int GH = a.GH, GW = a.GW, CI = a.CI, st = a.stride;

  // per-thread A rows: pixel base and the (h, w) origin of its receptive field
  int a_pix[A_PER], a_h[A_PER], a_w[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const long long m = m0 + r0 + i * ROWSTEP;
    a_ok[i] = m < a.M;
    const long long mm = a_ok[i] ? m : 0;
    const int ow = (int)(mm % a.OW);
    const long long t = mm / a.OW;
    const int oh = (int)(t % a.OH);
    const int b = (int)(t / a.OH);
    a_pix[i] = b * GH * GW;
    if (!TRANS) { a_h[i] = oh * st - a.pad; a_w[i] = ow * st - a.pad; }
    else        { a_h[i] = oh + a.pad;      a_w[i] = ow + a.pad; }
  }
  const long long K = (long long)a.R * a.S * CI;
  const u16* b_row[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int row = r0 + i * ROWSTEP;
    const int n = n0 + row;
    b_ok[i] = row < BN && n < a.CO;
    b_row[i] = a.w + (long long)(b_ok[i] ? n : 0) * K + ch * 8;
  }

  const int kpr = CI / BK;          // k-tiles per (r, s) tap
  const int KT = a.R * a.S * kpr;
  bf16x8 ra[A_PER], rb[B_PER];
  const bf16x8 zero = {};

  auto load = [&](int kt) {
    const int rs = kt / kpr;
    const int cb = (kt - rs * kpr) * BK + ch * 8;
    const int r = rs / a.S, s = rs - r * a.S;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int ih, iw;
      bool ok = a_ok[i];
      if (!TRANS) {
        ih = a_h[i] + r;
        iw = a_w[i] + s;
      } else {
        const int th = a_h[i] - r, tw = a_w[i] - s;
        ok = ok && th >= 0 && tw >= 0;
        if (st == 1) { ih = th; iw = tw; }
        else {
          ok = ok && (th % st) == 0 && (tw % st) == 0;
          ih = th / st;
          iw = tw / st;
        }
      }
      ok = ok && (unsigned)ih < (unsigned)GH && (unsigned)iw < (unsigned)GW;
      ra[i] = ok ? *reinterpret_cast<const bf16x8*>(
                       a.x + ((long long)a_pix[i] + ih * GW + iw) * CI + cb)
                 : zero;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      rb[i] = b_ok[i] ? *reinterpret_cast<const bf16x8*>(b_row[i] + (long long)kt * BK) : zero;
  };

  auto store = [&](int buf) {
    u16* As = lds + buf * STAGE;
    u16* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = r0 + i * ROWSTEP;
      *reinterpret_cast<bf16x8*>(As + row * BK + swz<BK>(row, ch) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = r0 + i * ROWSTEP;
      if (row < BN) *reinterpret_cast<bf16x8*>(Bs + row * BK + swz<BK>(row, ch) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      bf16x8 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * BK + swz<BK>(row, c) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + swz<BK>(row, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bw[j], af[i], acc[i][j]);
    }
  };

  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load(kt + 1);
    compute(cur);
    if (kt + 1 < KT) store(cur ^ 1);
    __syncthreads();
  }

  // epilogue: D^T layout -> lane owns channels n..n+3 of pixel m
  float s_sum[TN][4], s_sq[TN][4];
  if (STATS) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s_sum[j][r] = 0.f; s_sq[j][r] = 0.f; }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long long m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o.v[r] = f2bf(acc[i][j][r]);
      if (m < a.M && n < a.CO) {
        *reinterpret_cast<bf16x4*>(a.y + m * a.CO + n) = o;
        if (STATS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f(o.v[r]);
            s_sum[j][r] += v;
            s_sq[j][r] += v * v;
          }
        }
      }
    }
  }
  if (STATS) {
    // reduce over the 16 pixels (lane & 15) that share a channel quad
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s_sum[j][r] += __shfl_xor(s_sum[j][r], o, 64);
          s_sq[j][r] += __shfl_xor(s_sq[j][r], o, 64);
        }
      }
    // then over the WM waves of the block (lds is free after the last barrier)
    float* red = reinterpret_cast<float*>(lds);   // [WM][BN] sums, then [WM][BN] squares
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn * (BN / WN) + j * 16 + 4 * (lane >> 4) + r;
          red[wm * BN + nl] = s_sum[j][r];
          red[WM * BN + wm * BN + nl] = s_sq[j][r];
        }
    }
    __syncthreads();
    for (int nl = tid; nl < BN; nl += NT) {
      const int n = n0 + nl;
      if (n < a.CO) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { ss += red[w * BN + nl]; qq += red[WM * BN + w * BN + nl]; }
        a.part[(long long)blockIdx.x * a.CO + n] = ss;
        a.part[(long long)(gridDim.x + blockIdx.x) * a.CO + n] = qq;
      }
    }
  }
}

// ------------------------------------------------------------------- wgrad
struct WgradArgs {
  const u16* dy;    // [P][CO]  (P = B*OH*OW)
  const u16* x;     // [B][GH][GW][CI]
  float* dw;        // [CO][R][S][CI] fp32, accumulated
  int B, GH, GW, CI, OH, OW, CO, R, S, stride, pad;
  long long P;
  int p_chunk;      // rows of P per block (multiple of BP)
};

// 32-B granule swizzle for the [p][64] bf16 images read with ds_read_b64_tr_b16:
// a half-wave's transposed read touches rows {8g+q, g=0,1, q=0..3} (+4 for the
// second read) at one 32-B granule; granule ^= f(row>>1) with
// f(j) = (j&1) | ((j>>1)&2) puts those 8 rows in 8 distinct bank granules.
__device__ __forceinline__ int wg_off(int row, int col) {
  const int j = row >> 1;
  const int f = (j & 1) | ((j >> 1) & 2);
  return row * 64 + ((((col >> 4) ^ f) & 3) << 4) + (col & 15);
}

// D[co][k] += sum_p dY[p][co] * Xg[p][k]. Block tile BMW (co) x BNW (k) over a
// chunk of P; both operands staged as swizzled [p][64] images.
template <int BMW, int BNW, int BP, int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN) conv_wgrad_kernel(WgradArgs a) {
  static_assert(BMW == 64 && BNW == 64, "wg_off swizzle assumes 64-wide images");
  constexpr int NT = 64 * WM * WN;
  constexpr int LDA = BMW;
  constexpr int LDB = BNW;
  constexpr int ACH = BMW / 8, BCH = BNW / 8;    // 16-B chunks per row
  constexpr int A_PER = BP * ACH / NT;
  constexpr int B_PER = BP * BCH / NT;
  constexpr int TM = BMW / WM / 16, TN = BNW / WN / 16;
  constexpr int STAGE = BP * (LDA + LDB);
  static_assert(BP * ACH % NT == 0 && BP * BCH % NT == 0, "tile/thread mismatch");
  __shared__ __attribute__((aligned(16))) u16 lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int kx0 = blockIdx.x * BNW;            // column in K = (r, s, ci)
  const int co0 = blockIdx.y * BMW;
  const long long p_begin = (long long)blockIdx.z * a.p_chunk;
  const long long p_end = min(a.P, p_begin + a.p_chunk);
  const int rs = kx0 / a.CI;
  const int ci0 = kx0 - rs * a.CI;
  const int r = rs / a.S, s = rs - (rs / a.S) * a.S;
  const int GH = a.GH, GW = a.GW, CI = a.CI;

  bf16x8 ra[A_PER], rb[B_PER];
  const bf16x8 zero = {};
  auto load = [&](long long pb) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / ACH, c = idx - row * ACH;
      const long long p = pb + row;
      ra[i] = (p < p_end) ? *reinterpret_cast<const bf16x8*>(a.dy + p * a.CO + co0 + c * 8) : zero;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / BCH, c = idx - row * BCH;
      const long long p = pb + row;
      bool ok = p < p_end;
      const long long pp = ok ? p : 0;
      const int ow = (int)(pp % a.OW);
      const long long t = pp / a.OW;
      const int oh = (int)(t % a.OH);
      const int b = (int)(t / a.OH);
      const int ih = oh * a.stride - a.pad + r, iw = ow * a.stride - a.pad + s;
      ok = ok && (unsigned)ih < (unsigned)GH && (unsigned)iw < (unsigned)GW;
      rb[i] = ok ? *reinterpret_cast<const bf16x8*>(
                       a.x + (((long long)b * GH + ih) * GW + iw) * CI + ci0 + c * 8)
                 : zero;
    }
  };
  auto store = [&](int buf) {
    u16* As = lds + buf * STAGE;
    u16* Bs = As + BP * LDA;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / ACH, c = idx - row * ACH;
      *reinterpret_cast<bf16x8*>(As + wg_off(row, c * 8)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / BCH, c = idx - row * BCH;
      *reinterpret_cast<bf16x8*>(Bs + wg_off(row, c * 8)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed operand fetch: lane (g = lane>>4, i = lane&15) gets column
  // col0 + i of rows pk + 8g .. 8g+7 as 8 consecutive k elements.
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pc = li & 3;
  auto tr8 = [&](const u16* base, int ld, int pk, int col0) -> bf16x8 {
    (void)ld;
    const int row = pk + 8 * g + q;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(base + wg_off(row, col0 + 4 * pc)));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(base + wg_off(row + 4, col0 + 4 * pc)));
    const s16x8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  };
  auto compute = [&](int buf) {
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + BP * LDA;
#pragma unroll
    for (int pk = 0; pk < BP; pk += 32) {
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr8(As, LDA, pk, wm * (BMW / WM) + i * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = tr8(Bs, LDB, pk, wn * (BNW / WN) + j * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
  };

  const int nsteps = (int)((p_end - p_begin + BP - 1) / BP);
  if (nsteps <= 0) return;
  load(p_begin);
  store(0);
  __syncthreads();
  for (int it = 0; it < nsteps; ++it) {
    const int cur = it & 1;
    if (it + 1 < nsteps) load(p_begin + (long long)(it + 1) * BP);
    compute(cur);
    if (it + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }
  // D layout: lane holds rows co = 4*(lane>>4)+r, column k = lane & 15
  const long long K = (long long)a.R * a.S * a.CI;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int kk = kx0 + wn * (BNW / WN) + j * 16 + (lane & 15);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + wm * (BMW / WM) + i * 16 + 4 * (lane >> 4) + rr;
        atomicAdd(a.dw + (long long)co * K + kk, acc[i][j][rr]);
      }
    }
}

// W[co][r][s][ci] -> Wt[ci][r][s][co]  (bf16)
__global__ void __launch_bounds__(256) conv_weight_transpose_kernel(
    const u16* __restrict__ w, u16* __restrict__ wt, int CO, int RS, int CI) {
  const long long total = (long long)CO * RS * CI;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ci = (int)(i % CI);
    const long long t = i / CI;
    const int rs = (int)(t % RS);
    const int co = (int)(t / RS);
    wt[((long long)ci * RS + rs) * CO + co] = w[i];
  }
}

// ---------------------------------------------------------------- launchers
template <int BM, int BN, int BK, int WM, int WN, bool TRANS>
static void launch_igemm(const ConvArgs& a, bool stats, hipStream_t s) {
  const dim3 grid((unsigned)((a.M + BM - 1) / BM), (unsigned)((a.CO + BN - 1) / BN));
  const dim3 block(64 * WM * WN);
  if (stats)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, WM, WN, TRANS, true>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, WM, WN, TRANS, false>), grid, block, 0, s, a);
}

// Tile choice: the widest N tile that the output channels fill, then the
// tallest M tile that still gives >= ~2 blocks per CU on 256 CUs.
int conv_tile_m(long long M, int CO) {
  const int bn = CO >= 128 ? 128 : 64;
  const long long nb = (CO + bn - 1) / bn;
  if ((M + 255) / 256 * nb >= 512) return 256;
  if ((M + 127) / 128 * nb >= 256) return 128;
  return 64;
}

template <bool TRANS>
static void dispatch_igemm(const ConvArgs& a, bool stats, hipStream_t s) {
  const int bm = conv_tile_m(a.M, a.CO);
  const bool bk64 = (a.CI % 64) == 0;
  if (a.CO >= 128) {
    if (bm == 256) { if (bk64) launch_igemm<256, 128, 64, 2, 2, TRANS>(a, stats, s); else launch_igemm<256, 128, 32, 2, 2, TRANS>(a, stats, s); }
    else if (bm == 128) { if (bk64) launch_igemm<128, 128, 64, 2, 2, TRANS>(a, stats, s); else launch_igemm<128, 128, 32, 2, 2, TRANS>(a, stats, s); }
    else { if (bk64) launch_igemm<64, 128, 64, 1, 4, TRANS>(a, stats, s); else launch_igemm<64, 128, 32, 1, 4, TRANS>(a, stats, s); }
  } else {
    if (bm == 256) { if (bk64) launch_igemm<256, 64, 64, 4, 1, TRANS>(a, stats, s); else launch_igemm<256, 64, 32, 4, 1, TRANS>(a, stats, s); }
    else if (bm == 128) { if (bk64) launch_igemm<128, 64, 64, 2, 2, TRANS>(a, stats, s); else launch_igemm<128, 64, 32, 2, 2, TRANS>(a, stats, s); }
    else { if (bk64) launch_igemm<64, 64, 64, 2, 2, TRANS>(a, stats, s); else launch_igemm<64, 64, 32, 2, 2, TRANS>(a, stats, s); }
  }
}

int conv_fwd_num_mblocks(long long M, int CO) {
  const int bm = conv_tile_m(M, CO);
  return (int)((M + bm - 1) / bm);
}

void launch_conv_fwd(const u16* x, const u16* w, u16* y, float* part, int B, int H, int W,
                     int CI, int OH, int OW, int CO, int R, int S, int stride, int pad,
                     hipStream_t s) {
  ConvArgs a{x, w, y, part, B, H, W, CI, OH, OW, CO, R, S, stride, pad,
             (long long)B * OH * OW};
  dispatch_igemm<false>(a, part != nullptr, s);
}

// dX (B,H,W,CI) from dY (B,OH,OW,CO) and Wt [CI][R][S][CO]
void launch_conv_dgrad(const u16* dy, const u16* wt, u16* dx, int B, int H, int W, int CI,
                       int OH, int OW, int CO, int R, int S, int stride, int pad,
                       hipStream_t s) {
  ConvArgs a{dy, wt, dx, nullptr, B, OH, OW, CO, H, W, CI, R, S, stride, pad,
             (long long)B * H * W};
  dispatch_igemm<true>(a, false, s);
}

void launch_conv_weight_transpose(const u16* w, u16* wt, int CO, int RS, int CI, hipStream_t s) {
  const long long total = (long long)CO * RS * CI;
  hipLaunchKernelGGL(conv_weight_transpose_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s,
                     w, wt, CO, RS, CI);
}

void launch_conv_wgrad(const u16* dy, const u16* x, float* dw, int B, int H, int W, int CI,
                       int OH, int OW, int CO, int R, int S, int stride, int pad,
                       hipStream_t s) {
  constexpr int BMW = 64, BNW = 64, BP = 64;
  WgradArgs a{dy, x, dw, B, H, W, CI, OH, OW, CO, R, S, stride, pad, (long long)B * OH * OW, 0};
  const long long K = (long long)R * S * CI;
  const long long tiles = (K / BNW) * (CO / BMW);
  // enough P-splits for >= ~1024 blocks, but >= 1024 rows of P per block so the
  // fp32 atomics stay a small fraction of the traffic
  long long splits = (1024 + tiles - 1) / tiles;
  long long chunk = (a.P + splits - 1) / splits;
  if (chunk < 1024) chunk = 1024;
  chunk = (chunk + BP - 1) / BP * BP;
  splits = (a.P + chunk - 1) / chunk;
  a.p_chunk = (int)chunk;
  const dim3 grid((unsigned)(K / BNW), (unsigned)(CO / BMW), (unsigned)splits);
  hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, BP, 2, 2>), grid, dim3(256), 0, s, a);
}

}  // namespace dmp
