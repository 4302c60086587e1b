// Convolution weight gradient on gfx950 MFMA:
//
//   dW[co][k] += sum_p dY[p][co] * X_gather[p][k]     k = (r, s, ci), p = (b, oh, ow)
//
// The reduction runs over p, which is the SLOW index of both NHWC operands, so
// both tiles are staged as [p][*] row-major images (buffer_load ... lds DMA,
// 16 B per lane, swizzle applied on the source side) and read back transposed with
// ds_read_b64_tr_b16: a lane receives 8 consecutive p of one column, exactly
// the v_mfma_f32_16x16x32_bf16 operand layout.  P is split over blocks and each
// block adds its fp32 tile into the flat fp32 grad arena with atomics (no
// zero-fill or second reduction pass; the arena is zeroed once per step).
//
// Compile-time variants (host tuner picks per shape, ops/tuner.py):
//   BNW  - k columns per block (64 / 128 / 192; a 192 tile spans three taps so
//          dY is re-read K/192 times instead of once per tap)
//   WM x WN wave layout over the 64 x BNW tile: the LDS-read : MFMA ratio of a
//          wave tile TM x TN is (TM+TN)*2 tr-reads per TM*TN MFMAs; the CU does
//          ~2 tr-reads per MFMA slot, so thin 64x16 wave tiles are LDS-bound
//          while 64x48 ones are MFMA-bound
//   BP   - reduction rows per stage (32 / 64)
//   NS   - pipeline depth: NS-1 stages of DMA in flight, retired with a
//          counted s_waitcnt vmcnt(N) before one raw s_barrier per stage.
#include "common.h"

namespace dmp {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));


struct WgradArgs {
  const u16* dy;    // [P][CO]  (P = B*OH*OW)
  const u16* x;     // [B][GH][GW][CI]
  float* dw;        // [CO][R][S][CI] fp32, accumulated
  int B, GH, GW, CI, OH, OW, CO, R, S, stride, pad;
  long long P;
  int p_chunk;      // rows of P per block (multiple of BP)
};

__device__ __forceinline__ f32x4 mfma16w(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// LDS DMA (buffer_load_dwordx4 ... lds) issued from inline asm on purpose: the
// compiler models the builtin as an LDS store it cannot disambiguate from the
// ring buffer being read, and inserts s_waitcnt vmcnt(0) in front of the very
// next ds_read -- serialising every stage's DMA with the MFMA work.
// Completion is tracked by hand (wait_vm below).  32-bit byte offsets into a
// buffer descriptor; offsets past its bound read zeros (padding taps, rows
// past the end of P).
constexpr unsigned kOOBw = 0x80000000u;
__device__ __forceinline__ void bdma16w(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                        u16* lds_wave_base) {
  const unsigned m0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave_base;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "{m0}"(m0));
}

// wait until at most N vector-memory ops (our DMAs) of this wave are outstanding,
// and for all of this wave's LDS ops (row-table writes) to complete
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}

// 32-B granule swizzle (an involution) for [p][ROWE] bf16 images read by
// ds_read_b64_tr_b16.  A transposed read of one half-wave touches rows
// {8g+q : g=0,1, q=0..3} (and +4 for the second read) in one granule.  Row
// strides of 128/384 B put rows of equal parity on one bank offset -> f spreads
// rows {0,2,8,10} over 4 granules; 256-B rows put every row on one offset -> f
// spreads all 8 rows.
template <int ROWE>
__device__ __forceinline__ int wg_f(int row) {
  if constexpr (ROWE == 128) return (row & 3) | (((row >> 3) & 1) << 2);
  else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}
template <int ROWE>
__device__ __forceinline__ int wg_off(int row, int col) {
  return row * ROWE + ((((col >> 4) ^ wg_f<ROWE>(row))) << 4) + (col & 15);
}

template <int BNW, int WM, int WN, int BP, int NS>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  constexpr int BMW = 64, NW = 4;
  static_assert(WM * WN == NW, "4 waves");
  constexpr int TM = BMW / WM / 16, TN = BNW / WN / 16;
  constexpr int A_EL = BP * BMW, B_EL = BP * BNW;
  constexpr int A_INS = A_EL / 512, B_INS = B_EL / 512;     // 1 KiB per glds instruction
  constexpr int A_PW = A_INS / NW, B_PW = B_INS / NW;
  constexpr int INS_PW = A_PW + B_PW;                       // DMAs per wave per stage
  constexpr int STAGE = A_EL + B_EL;
  static_assert(A_INS % NW == 0 && B_INS % NW == 0, "instruction split");
  static_assert(NS >= 2 && (NS - 2) * INS_PW < 64, "pipeline depth");
  // [NS][STAGE] staging, then the [NS][BP] row table (int4 per row)
  __shared__ __attribute__((aligned(16))) u16 lds[NS * STAGE + NS * BP * 8];
  int4* rowtab = reinterpret_cast<int4*>(lds + NS * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int kx0 = blockIdx.x * BNW;            // first column in K = (r, s, ci)
  const int co0 = blockIdx.y * BMW;
  const long long p_begin = (long long)blockIdx.z * a.p_chunk;
  const long long p_end = min(a.P, p_begin + a.p_chunk);
  const int GH = a.GH, GW = a.GW, CI = a.CI;
  const int nsteps = (int)((p_end - p_begin + BP - 1) / BP);
  if (nsteps <= 0) return;

  // per-lane DMA slots (fixed across stages): A = dY rows, B = X rows x tap columns
  int a_row[A_PW], a_col[A_PW];
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int e = (wid + j * NW) * 512 + lane * 8;       // element index in the A image
    const int row = e / BMW, pch = (e % BMW) / 8;
    const int u = (pch >> 1) ^ wg_f<BMW>(row);
    a_row[j] = row;
    a_col[j] = co0 + u * 16 + (pch & 1) * 8;
  }
  int b_row[B_PW], b_r[B_PW], b_s[B_PW], b_ci[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int e = (wid + j * NW) * 512 + lane * 8;
    const int row = e / BNW, pch = (e % BNW) / 8;
    const int u = (pch >> 1) ^ wg_f<BNW>(row);
    const int kc = kx0 + u * 16 + (pch & 1) * 8;
    const int rs = kc / CI;
    b_row[j] = row;
    b_ci[j] = kc - rs * CI;
    b_r[j] = rs / a.S;
    b_s[j] = rs - b_r[j] * a.S;
  }
  // row table for stage `stg`: {pixel base, oh*stride-pad, ow*stride-pad, valid}
  auto fill_rows = [&](int stg) {
    if (tid < BP) {
      const int p = (int)p_begin + stg * BP + tid;
      int4 e = make_int4(0, -(1 << 20), -(1 << 20), 0);
      if (stg < nsteps && p < (int)p_end) {
        const int ow = p % a.OW, t = p / a.OW;
        const int oh = t % a.OH, b = t / a.OH;
        e = make_int4(b * GH * GW, oh * a.stride - a.pad, ow * a.stride - a.pad, 1);
      }
      rowtab[(stg % NS) * BP + tid] = e;
    }
  };
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.dy, 0, (int)(2 * a.P * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * a.B * GH * GW * CI), 0x00020000);
  auto stage = [&](int stg) {
    const int buf = stg % NS;
    const int pb = (int)p_begin + stg * BP;
    u16* As = lds + buf * STAGE;
    u16* Bs = As + A_EL;
#pragma unroll
    for (int j = 0; j < A_PW; ++j) {
      const int p = pb + a_row[j];
      const bool ok = stg < nsteps && p < (int)p_end;
      bdma16w(rsA, ok ? 2u * (unsigned)(p * a.CO + a_col[j]) : kOOBw, As + (wid + j * NW) * 512);
    }
    const int4* tb = rowtab + buf * BP;
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int4 e = tb[b_row[j]];
      const int ih = e.y + b_r[j], iw = e.z + b_s[j];
      const bool ok = e.w && (unsigned)ih < (unsigned)GH && (unsigned)iw < (unsigned)GW;
      bdma16w(rsB, ok ? 2u * (unsigned)((e.x + ih * GW + iw) * CI + b_ci[j]) : kOOBw,
              Bs + (wid + j * NW) * 512);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // lane (g = lane>>4, li = lane&15) receives column col0+li of rows
  // pk+8g .. pk+8g+7 = 8 consecutive reduction elements (two tr reads).
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pc = li & 3;
  auto trA = [&](const u16* img, int pk, int col0) -> bf16x8 {
    const int row = pk + 8 * g + q;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + wg_off<BMW>(row, col0 + 4 * pc)));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + wg_off<BMW>(row + 4, col0 + 4 * pc)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto trB = [&](const u16* img, int pk, int col0) -> bf16x8 {
    const int row = pk + 8 * g + q;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + wg_off<BNW>(row, col0 + 4 * pc)));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + wg_off<BNW>(row + 4, col0 + 4 * pc)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int buf) {
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + A_EL;
#pragma unroll
    for (int pk = 0; pk < BP; pk += 32) {
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = trA(As, pk, wm * (BMW / WM) + i * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = trB(Bs, pk, wn * (BNW / WN) + j * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16w(af[i], bf[j], acc[i][j]);
    }
  };

  // prologue: tables for stages 0..NS-1, DMA for stages 0..NS-2
#pragma unroll
  for (int s = 0; s < NS; ++s) fill_rows(s);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage(s);
  for (int it = 0; it < nsteps; ++it) {
    // stage `it` landed (this wave's DMAs; younger stages may still fly) ...
    wait_vm<(NS - 2) * INS_PW>();
    // ... for every wave; and everyone finished compute(it-1), freeing its buffer
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stage(it + NS - 1);                 // reuses buffer (it-1) % NS; zero-page past the end
    compute(it % NS);
    fill_rows(it + NS);                 // table slot it % NS: stage `it` already issued
  }
  wait_vm<0>();
  // D layout: lane holds rows co = 4*(lane>>4)+r of column k = lane & 15
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

// cfg bits: [1:0] BNW (0 auto, 1 -> 64, 2 -> 128, 3 -> 192), [2] BP (0 -> 64, 1 -> 32),
// [3] NS (0 -> 2, 1 -> 3), [7:4] minimum rows of P per block in units of 512 (0 auto).
template <int BNW, int WM, int WN>
static void launch_wgrad_variant(const WgradArgs& a, dim3 grid, int bp, int ns, hipStream_t s) {
  if (bp == 32) {
    if (ns == 3) hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 32, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 32, 2>), grid, dim3(256), 0, s, a);
  } else {
    if (ns == 3) hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 64, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 64, 2>), grid, dim3(256), 0, s, a);
  }
}

void launch_conv_wgrad(const u16* dy, const u16* x, float* dw, int B, int H, int W, int CI,
                       int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                       hipStream_t s) {
  WgradArgs a{dy, x, dw, B, H, W, CI, OH, OW, CO, R, S, stride, pad, (long long)B * OH * OW, 0};
  const long long K = (long long)R * S * CI;
  const int sel = cfg < 0 ? 0 : (cfg & 3);
  int bnw = sel == 1 ? 64 : (sel == 2 ? 128 : (sel == 3 ? 192 : 0));
  if (bnw == 0) bnw = (K % 192 == 0) ? 192 : (K % 128 == 0 ? 128 : 64);
  if (K % bnw != 0) bnw = 64;
  const int bp = (cfg >= 0 && (cfg & 4)) ? 32 : 64;
  const int ns = (cfg >= 0 && (cfg & 8)) ? 3 : 2;
  const long long tiles = (K / bnw) * (CO / 64);
  long long min_chunk = cfg < 0 ? 0 : (long long)((cfg >> 4) & 15) * 512;
  if (min_chunk <= 0) min_chunk = 2048;
  long long splits = (768 + tiles - 1) / tiles;
  long long chunk = (a.P + splits - 1) / splits;
  if (chunk < min_chunk) chunk = min_chunk;
  chunk = (chunk + bp - 1) / bp * bp;
  splits = (a.P + chunk - 1) / chunk;
  a.p_chunk = (int)chunk;
  const dim3 grid((unsigned)(K / bnw), (unsigned)(CO / 64), (unsigned)splits);
  if (bnw == 192) launch_wgrad_variant<192, 1, 4>(a, grid, bp, ns, s);
  else if (bnw == 128) launch_wgrad_variant<128, 2, 2>(a, grid, bp, ns, s);
  else launch_wgrad_variant<64, 2, 2>(a, grid, bp, ns, s);
}

}  // namespace dmp
