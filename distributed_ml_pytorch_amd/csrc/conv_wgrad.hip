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
//   BMW  - output channels per block (64, or 128 for wide 1x1 GEMMs such as the
//          ViT linear layers: half the dY re-reads, 20 tr-reads per 24 MFMAs)
//   WM x WN wave layout over the BMW x BNW tile: the LDS-read : MFMA ratio of a
//          wave tile TM x TN is (TM+TN)*2 tr-reads per TM*TN MFMAs; the CU does
//          ~2 tr-reads per MFMA slot, so thin 64x16 wave tiles are LDS-bound
//          while 64x48 ones are MFMA-bound
//   BP   - reduction rows per stage (32 / 64)
//   NS   - pipeline depth: NS-1 stages of DMA in flight, retired with a
//          counted s_waitcnt vmcnt(N) before one raw s_barrier per stage.
#include "common.h"

#ifndef DMP_ABLATE
#define DMP_ABLATE 0   // roofline ablations: see conv.hip
#endif

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
  float* dbias;     // optional fp32 [CO] += sum_p dY[p][co] (linear / conv bias grad)
  float* slab;      // halo wgrad, slab mode: per-split partials [splits][CO][R][S][CI]
  int xcd;          // gather wgrad: XCD-aware deal of the blocks (cfg bit 512)
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

// Halo wgrad X image (128-B rows; staged row = X row hx of image tb of the tile,
// column c of W2 = W + 2).  A half-wave's tr read touches the tap-shifted rows of
// pixels {p..p+3} and {p+8..p+11}: stride 1, 4 consecutive columns (alternating
// row parity) and 8 pixels later (same row at W >= 16, next row at W = 8, next
// image / two rows at W = 4); stride 2, columns c, c+2, c+4, c+6 (one parity).
// Keyed on the column and on bit 3 of the pixel-like index (tb * TH + hx) * W + c,
// every (parity, granule) pair of the 8 rows is distinct at any W -- wg_f<64> of
// the row NUMBER collides for W2 = 10 / 6 (22 % / 9.5 % LDS bank conflicts on the
// 8x8 / 4x4 layers, profiles/pmc_r5.txt); stride 2 keeps the unavoidable 2-way
// (8 rows of one parity over 4 granules).
#ifndef DMP_WGX_SWZ
#define DMP_WGX_SWZ 1
#endif
template <bool S2>
__device__ __forceinline__ int wgx_f(int c, int pidx) {
  if constexpr (S2) return (c >> 1) & 3;
  else return ((c >> 1) & 1) | (((pidx >> 3) & 1) << 1);
}

template <int BNW, int WM, int WN, int BP, int NS, int BMW>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  constexpr int NW = 4;
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
  // XCD-aware bijective remap (a.xcd): consecutive logical blocks -- the (k, co)
  // tiles of one pixel split, which read the same dY / X rows -- land on one XCD
  // under round-robin dispatch instead of being spread over all eight L2s
  const int nx = gridDim.x, ny = gridDim.y, G = nx * ny * gridDim.z;
  const int bid = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int lid = a.xcd ? (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3)
                        : bid;
  const int bx = lid % nx, by = (lid / nx) % ny, bz = lid / (nx * ny);
  const int kx0 = bx * BNW;            // first column in K = (r, s, ci)
  const int co0 = by * BMW;
  const long long p_begin = (long long)bz * a.p_chunk;
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
  // bias gradient from the dY tiles already staged for the weight gradient:
  // one extra MFMA per fragment with an all-ones B operand (column sums), by
  // the wn == 0 waves of the blocks of the first k tile only
  const bool do_bias = a.dbias != nullptr && bx == 0 && wn == 0;
  f32x4 accb[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones.v[k] = 0x3f80;   // bf16 1.0
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
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < TM; ++i) accb[i] = mfma16w(af[i], ones, accb[i]);
      }
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
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        atomicAdd(a.dbias + co0 + wm * (BMW / WM) + i * 16 + 4 * (lane >> 4) + rr, accb[i][rr]);
  }
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

// ------------------------------------------------- 3x3 stride-1 halo wgrad
// dW[co][r][s][ci] += sum_p dY[p][co] * X[p shifted by (r-1, s-1)][ci] for 3x3 /
// stride 1 / pad 1.  The gather kernel above fetches X once per tap column
// tile; here a block owns a 64 x 64 (co, ci) tile and TR tap rows (TR = 1: one
// row r, grid.y enumerates r; TR = 3: all nine taps) and walks a run of
// BM-pixel tiles (whole image rows / whole images, as the forward halo kernel).
// Per tile it stages dY [BM][64] plus the input rows those tap rows read,
// X[h - 1 + r][-1 .. W] (W + 2 columns, zero outside the image), ONCE: the
// taps are the same staged rows offset by r * (W + 2) + s.  Both images are
// [row][64] with the 32-B granule swizzle and read with ds_read_b64_tr_b16; a
// lane supplies its own row address per tr read, so the shifted pixel -> row
// map needs no layout change.  4 waves, wave w: all 64 co x ci 16w..16w+15 x
// 3*TR taps (12 or 36 accumulator tiles).
//
// Tiles stream through an NS-deep ring of LDS-DMA stages (counted vmcnt + one
// raw s_barrier per tile): every wave issues the same D_PW + XPW DMAs per stage
// (padding rows past the staged image read zeros), so "stage t landed" is
// vmcnt <= (NS - 2) * (D_PW + XPW).  With NS = 2 one tile of compute (~0.3 us
// at BM 128, TR 1) had to cover a whole HBM round trip.
// Blocks are mapped XCD-aware: the tiles of one pixel split share an XCD's L2.
// Partial sums go to dW with fp32 atomics, or plain read-add-write when one
// block owns the tile (splits == 1).
// MV: pixels per tile (= BM, or TB * H * W < BM for padded whole-image tiles on
// 14x14 / 7x7 maps: the dY rows past MV stage zeros, so they add nothing)
struct WgradHaloGeom {
  int TH, TB, THX, XROWS, XPW, ntiles, tiles_per_split, MV;
};

constexpr int kWhXPW = 12;   // max X-row DMA instructions per wave per stage

// vmcnt wait with a launch-time (wave-uniform) count
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
#define DMP_WV(k) \
  case k:         \
    wait_vm<k>(); \
    break;
    DMP_WV(1) DMP_WV(2) DMP_WV(3) DMP_WV(4) DMP_WV(5) DMP_WV(6) DMP_WV(7) DMP_WV(8) DMP_WV(9)
    DMP_WV(10) DMP_WV(11) DMP_WV(12) DMP_WV(13) DMP_WV(14) DMP_WV(15) DMP_WV(16) DMP_WV(17)
    DMP_WV(18) DMP_WV(19) DMP_WV(20) DMP_WV(21) DMP_WV(22) DMP_WV(23) DMP_WV(24) DMP_WV(25)
    DMP_WV(26) DMP_WV(27) DMP_WV(28) DMP_WV(29) DMP_WV(30) DMP_WV(31) DMP_WV(32) DMP_WV(33)
    DMP_WV(34) DMP_WV(35) DMP_WV(36) DMP_WV(37) DMP_WV(38) DMP_WV(39) DMP_WV(40)
#undef DMP_WV
    default:
      wait_vm<0>();
  }
}

// PG = 2: 8 waves in two pixel groups.  Group g (waves 4g..4g+3) owns the
// same 64 x 16-column slices as the 4-wave block but only pk steps
// [g * NPK / 2, (g+1) * NPK / 2) of every tile; at the end group 1 parks its
// accumulators in LDS and group 0 adds them before the single atomic flush.
// One such block per CU replaces two 4-wave blocks: the same two waves per
// SIMD, half the fp32 partials through the memory-side atomic units (~1.3
// TB/s chip-wide, ~25 % of the 4-wave kernel's time: profiles/conv_kernels_r2.txt).
//
// S2: the 3x3 / stride-2 / pad-1 weight gradient (TR = 1).  Tiles are dY pixels
// (OH x OW); for tap row r0 the block stages, per output row th of the tile, the
// ONE input row 2 (h0 + th) - 1 + r0 (W + 2 columns), and output pixel (th, tw)
// reads tap s at staged column 2 tw + s: the same DMA slots and transposing
// reads as stride 1, with the pixel -> staged-row map doubled along w (the
// implicit-GEMM gather ran these at 345-420 TF/s, profiles/resnet18_steady_state_r4.txt).
template <int BM, int NS, int TR, int PG = 1, bool S2 = false>
__global__ void __launch_bounds__(256 * PG) conv_wgrad_halo_kernel(WgradArgs a, WgradHaloGeom hg,
                                                                   int atomic) {
  static_assert(!S2 || TR == 1, "stride-2 halo wgrad: one tap row per block");
  constexpr int NW = 4 * PG, CW = 64;             // 64-channel rows (128 B)
  constexpr int D_PW = BM / 8 / NW;               // dY DMA instructions per wave per tile
  constexpr int NT = 3 * TR;                      // taps per block
  extern __shared__ __attribute__((aligned(16))) u16 lds_w[];
  const int XPW = hg.XPW;
  const int D_EL = BM * CW;
  const int STAGE = D_EL + XPW * NW * 512;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid & 3, grp = wid >> 2;         // column slice, pixel group
  // XCD-aware bijective remap: consecutive logical blocks (the (ci, co, r)
  // tiles of one pixel split) land on one XCD under round-robin dispatch
  const int nx = gridDim.x, ny = gridDim.y, G = nx * ny * gridDim.z;
  const int bid = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int bx = lid % nx, by = (lid / nx) % ny, bz = lid / (nx * ny);
  const int ci0 = bx * CW;
  const int co0 = (TR == 3 ? by : by / 3) * CW, r0 = TR == 3 ? 0 : by % 3;
  const int t_begin = bz * hg.tiles_per_split;
  const int t_end = min(hg.ntiles, t_begin + hg.tiles_per_split);
  if (t_begin >= t_end) return;
  const int H = a.GH, W = a.GW, C = a.CI, CO = a.CO, TH = hg.TH, THX = hg.THX, W2 = W + 2;
  const int img = H * W;                           // input (X) image
  const int OHd = S2 ? a.OH : H, OWd = S2 ? a.OW : W, imgd = OHd * OWd;   // dY image
  const int P = (int)a.P;
  const int MV = hg.MV;

  // DMA slots, fixed per lane: byte offsets RELATIVE to the tile's first pixel.
  // dY: row of the tile + swizzled source column.  X: staged row -> (image in
  // tile tb, source row dh relative to the tile's first row h0, column w); a
  // row that is outside the image for every tile (column halo, rows past the
  // staged image, and with whole-image tiles the row halo) holds kOOBw, and
  // the halo row above the tile wraps below 0 (correct modulo 2^32 once the
  // tile's base offset is added).  Interior tiles then issue every piece with
  // ONE v_add (kOOBw + base stays >= 2^31, past the descriptor's bound); only
  // tiles touching an image edge or the end of P test rows per lane.  (Per-tile
  // integer divisions and the per-piece decode/compare chain were ~2/3 of the
  // kernel's VALU: 4.1 VALU per MFMA, issue-bound, profiles/conv_kernels_r2.txt.)
  int d_row[D_PW];
  unsigned d_rel[D_PW];
#pragma unroll
  for (int j = 0; j < D_PW; ++j) {
    const int row = (wid + j * NW) * 8 + lane / 8, pch = lane % 8;
    d_row[j] = row;
    d_rel[j] = row < MV ? 2u * (unsigned)(row * CO + co0 + (((pch >> 1) ^ wg_f<CW>(row)) * 16) +
                                          (pch & 1) * 8)
                        : kOOBw;   // padded tile: zeros
  }
  const bool whole_img = TH == OHd;   // tiles of whole images: h0 == 0 for every tile
  unsigned x_rel[kWhXPW];
  int x_dh[kWhXPW], x_tb[kWhXPW];
#pragma unroll
  for (int j = 0; j < kWhXPW; ++j) {
    x_rel[j] = kOOBw;
    x_dh[j] = 0;
    x_tb[j] = 0;
    if (j < XPW) {
      const int row = (wid + j * NW) * 8 + lane / 8, pch = lane % 8;
      const int tb = row / (THX * W2), rem = row - tb * THX * W2;
      const int th = rem / W2, w = rem - th * W2 - 1;
      const int dh = (S2 ? 2 * th : th) - 1 + r0;   // relative to the tile's first X row
      const bool ok = row < hg.XROWS && tb < hg.TB && (unsigned)w < (unsigned)W &&
                      (!whole_img || (unsigned)dh < (unsigned)H);
      const int fx = DMP_WGX_SWZ ? wgx_f<S2>(w + 1, (tb * TH + th) * W + w + 1) : wg_f<CW>(row);
      if (ok)
        x_rel[j] = 2u * (unsigned)((tb * img + dh * W + w) * C + ci0 +
                                   (((pch >> 1) ^ fx) * 16) + (pch & 1) * 8);
      x_dh[j] = dh;
      x_tb[j] = tb;
    }
  }
  const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.dy, 0, (int)(2LL * P * CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * a.B * img * C), 0x00020000);

  // tile cursor (image b0, first row h0 of the tile stage() issues next): the
  // stages are issued for consecutive tiles, so it advances by one tile per
  // call instead of dividing per tile
  int cb0 = (t_begin * MV) / imgd;
  int ch0 = (t_begin * MV - cb0 * imgd) / OWd;
  // staged X rows relative to the tile's first X row (h0, or 2 h0 for S2)
  const int lo_dh = r0 - 1, hi_dh = S2 ? 2 * (TH - 1) - 1 + r0 : THX - 2 + r0;

  // issue stage `t` into ring slot `buf`; a tile past the run loads zeros so
  // every wave's DMA count per stage stays D_PW + XPW
  auto stage = [&](int buf, int t) {
    u16* Ds = lds_w + buf * STAGE;
    u16* Xs = Ds + D_EL;
    const bool live = t < t_end;
    const int m0 = t * MV;
    const int b0 = cb0, h0 = ch0;
    if (whole_img) {
      cb0 += hg.TB;
    } else {
      ch0 += TH;
      if (ch0 >= OHd) { ch0 = 0; cb0 += 1; }
    }
    const int hx0 = S2 ? 2 * h0 : h0;   // the tile's first X row
    const unsigned dbase = 2u * (unsigned)(m0 * CO);
    const unsigned xbase = S2 ? 2u * (unsigned)((b0 * img + hx0 * W) * C) : 2u * (unsigned)(m0 * C);
    const bool interior = live && m0 + MV <= P && b0 + hg.TB <= a.B &&
                          (whole_img || (hx0 + lo_dh >= 0 && hx0 + hi_dh < H));
    if (interior) {
#pragma unroll
      for (int j = 0; j < D_PW; ++j) bdma16w(rsD, d_rel[j] + dbase, Ds + (wid + j * NW) * 512);
#pragma unroll
      for (int j = 0; j < kWhXPW; ++j)
        if (j < XPW) bdma16w(rsX, x_rel[j] + xbase, Xs + (wid + j * NW) * 512);
    } else {
#pragma unroll
      for (int j = 0; j < D_PW; ++j) {
        const bool ok = live && m0 + d_row[j] < P;
        bdma16w(rsD, ok ? d_rel[j] + dbase : kOOBw, Ds + (wid + j * NW) * 512);
      }
#pragma unroll
      for (int j = 0; j < kWhXPW; ++j) {
        if (j < XPW) {
          const bool ok = live && x_rel[j] != kOOBw && b0 + x_tb[j] < a.B &&
                          (whole_img || (unsigned)(hx0 + x_dh[j]) < (unsigned)H);
          bdma16w(rsX, ok ? x_rel[j] + xbase : kOOBw, Xs + (wid + j * NW) * 512);
        }
      }
    }
  };

  // staged X row of the lane's reduction rows (pixels pk*32 + 8g + q and +4), tap (0, 0)
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pc = li & 3;
  int xr_lo[BM / 32 / PG], xr_hi[BM / 32 / PG];
  int xk_lo[BM / 32 / PG], xk_hi[BM / 32 / PG];   // X-image swizzle keys (wgx_f)
#pragma unroll
  for (int pk = 0; pk < BM / 32 / PG; ++pk) {
#pragma unroll
    for (int hsel = 0; hsel < 2; ++hsel) {
      int pl = (grp * (BM / 32 / PG) + pk) * 32 + 8 * g + q + 4 * hsel;
      if (pl >= MV) pl = 0;   // padded tile: its dY row is zero, read any staged X row
      const int tb = pl / (TH * OWd), r2 = pl - tb * TH * OWd;
      const int th = r2 / OWd, tw = r2 - th * OWd;
      const int xr = (tb * THX + th) * W2 + (S2 ? 2 * tw : tw);
      // swizzle keys of the 3 * TR taps, 2 bits each: column c0 + s, pixel-like
      // index of image row th + r (stride 2: one staged row per output row, TR = 1)
      const int c0 = S2 ? 2 * tw : tw, p0 = (tb * TH + th) * W + c0;
      int xk = 0;
#pragma unroll
      for (int r = 0; r < TR; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) xk |= wgx_f<S2>(c0 + s, p0 + r * W + s) << (2 * (r * 3 + s));
      if (hsel) { xr_hi[pk] = xr; xk_hi[pk] = xk; } else { xr_lo[pk] = xr; xk_lo[pk] = xk; }
    }
  }
  auto tr = [&](const u16* img_, int row, int col) -> s16x4_t {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img_ + wg_off<CW>(row, col)));
  };
  // X image read of tap (r, s) for the lane's pixel (row xr, key xk)
  auto trx = [&](const u16* img_, int xr, int xk, int r, int s, int col) -> s16x4_t {
    const int row = xr + r * W2 + s;
    const int f = DMP_WGX_SWZ ? (xk >> (2 * (r * 3 + s))) & 3 : wg_f<CW>(row);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(
        img_ + row * CW + (((col >> 4) ^ f) << 4) + (col & 15)));
  };

  f32x4 acc[NT][4];
#pragma unroll
  for (int s = 0; s < NT; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[s][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // pk steps with the fragments double-buffered in registers and the reads of
  // step pk+1 pinned between step pk's MFMAs (sched_group_barrier): the
  // scheduler otherwise sinks every read next to its first use and each step
  // waits out its own LDS latency
  auto compute = [&](int buf) {
    const u16* Ds = lds_w + buf * STAGE;
    const u16* Xs = Ds + D_EL;
    constexpr int NPK = BM / 32 / PG, NRD = 8 + 6 * TR, NMF = 12 * TR;
    bf16x8 af[2][4], bx[2][3 * TR];
    auto load = [&](int pkl, int slot) {
      const int pk = grp * NPK + pkl;   // this group's share of the tile
      const int drow = pk * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x4_t lo = tr(Ds, drow, i * 16 + 4 * pc), hi = tr(Ds, drow + 4, i * 16 + 4 * pc);
        af[slot][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int r = 0; r < TR; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const s16x4_t lo = trx(Xs, xr_lo[pkl], xk_lo[pkl], r, s, wc * 16 + 4 * pc);
          const s16x4_t hi = trx(Xs, xr_hi[pkl], xk_hi[pkl], r, s, wc * 16 + 4 * pc);
          bx[slot][r * 3 + s] =
              __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    };
    load(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
#pragma unroll
    for (int pk = 0; pk < NPK; ++pk) {
      if (pk + 1 < NPK) load(pk + 1, (pk + 1) & 1);
#pragma unroll
      for (int t = 0; t < 3 * TR; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = mfma16w(af[pk & 1][i], bx[pk & 1][t], acc[t][i]);
      if (pk + 1 < NPK) {
        // one read of step pk+1 after each MFMA of step pk, the rest at the end
#pragma unroll
        for (int m = 0; m < NMF; ++m) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (m < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (NRD > NMF) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NMF, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      }
    }
  };

  const int nt = t_end - t_begin;
  const int vm_wait = (NS - 2) * (D_PW + XPW);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage(s, t_begin + s);
  for (int it = 0; it < nt; ++it) {
    if (NS == 2) wait_vm<0>();
    else wait_vm_rt(vm_wait);           // tile `it` landed (this wave's DMAs) ...
    __builtin_amdgcn_s_barrier();       // ... for every wave; slot (it-1) % NS is free
    asm volatile("" ::: "memory");
    if (DMP_ABLATE != 2) stage((it + NS - 1) % NS, t_begin + it + NS - 1);
    if (DMP_ABLATE != 1) compute(DMP_ABLATE == 2 ? 0 : it % NS);
  }
  wait_vm<0>();
  if constexpr (PG == 2) {
    // group 1 parks its partial sums in LDS (the staging ring is drained and
    // every wave is past its last read after the barrier), group 0 adds them
    __syncthreads();
    float* park = reinterpret_cast<float*>(lds_w);   // [4 waves][NT*4][64 lanes] f32x4
    if (grp == 1) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<f32x4*>(park + ((wc * NT * 4 + t * 4 + i) * 64 + lane) * 4) = acc[t][i];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[t][i] += *reinterpret_cast<const f32x4*>(park + ((wc * NT * 4 + t * 4 + i) * 64 + lane) * 4);
  }
  // D layout: lane holds rows co = 4*(lane>>4)+rr of column ci = lane & 15
  const long long K = 9LL * C;
  const int ci = ci0 + wc * 16 + (lane & 15);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + i * 16 + 4 * (lane >> 4) + rr;
        float* dst = a.dw + (long long)co * K + ((r0 + t / 3) * 3 + t % 3) * C + ci;
        if (atomic == 1) atomicAdd(dst, acc[t][i][rr]);
        else if (atomic == 0) *dst += acc[t][i][rr];
        else if (atomic == 3) a.slab[(long long)bz * CO * K + (dst - a.dw)] = acc[t][i][rr];
        else *dst = acc[t][i][rr];   // timing diagnostic only (DMP_WGRAD_HALO_DIAG=store)
      }
}

// halo wgrad cfg ids: kWhBase + variant * 12 + bm_sel * 4 + spl; BM = 64 << bm_sel,
// target block count 128 << spl; variant -> (NS, TR) below (ids 1000..1011 are
// the round-1 kernel's configs: NS 2, one tap row per block)
constexpr int kWhBase = 1000;
// variants 6-7: BM fixed at 224 = 4 rows of 56 (ImageNet ResNet stage 1, where no
// power-of-two tile is a whole number of rows); only bm_sel 0 is valid there
constexpr int kWhVariants = 8;
constexpr int kWhNS[kWhVariants] = {2, 3, 4, 2, 3, 2, 2, 3};
constexpr int kWhTR[kWhVariants] = {1, 1, 1, 3, 3, 1, 1, 1};
constexpr int kWhPG[kWhVariants] = {1, 1, 1, 1, 1, 2, 1, 1};   // pixel groups (8 waves when 2)
constexpr int kWhBM[kWhVariants] = {0, 0, 0, 0, 0, 0, 224, 224};   // 0: 64 << bm_sel

// slab mode (ids kWhSlabBase + i = halo config kWhBase + i): the split-K partials
// go to a [splits][dW] fp32 slab with plain stores (~6 TB/s chip-wide) and one
// streaming pass adds them into dW, instead of fp32 atomics (~1.3 TB/s of added
// bytes, ~25 % of the 64-channel wgrad: profiles/conv_kernels_r2.txt); offered
// for the NS-2 one-tap-row variants when the geometry splits K
constexpr int kWhSlabBase = 3000;
constexpr bool wh_slab_variant(int var) { return var == 0 || var == 5 || var == 6; }

static bool wgrad_halo_geom(int cfg, int B, int H, int W, int CI, int CO, int R, int S, int stride,
                            int pad, WgradHaloGeom* g, int* bm_out, int* ns_out, int* tr_out,
                            int* pg_out, size_t* lds, int* splits) {
  if (cfg >= kWhSlabBase) cfg -= kWhSlabBase - kWhBase;
  const int id = cfg - kWhBase;
  if (id < 0 || id >= 12 * kWhVariants) return false;
  const int var = id / 12, rest = id % 12;
  if (kWhBM[var] != 0 && rest / 4 != 0) return false;
  const int bm = kWhBM[var] != 0 ? kWhBM[var] : 64 << (rest / 4), target = 128 << (rest % 4);
  const int ns = kWhNS[var], tr = kWhTR[var], pg = kWhPG[var];
  if (pg == 2 && bm < 128) return false;
  if (R != 3 || S != 3 || pad != 1 || CI % 64 || CO % 64) return false;
  const bool s2 = stride == 2;
  if (stride != 1 && !(s2 && tr == 1 && H % 2 == 0 && W % 2 == 0 && ns <= 3 && kWhBM[var] == 0))
    return false;
  if (tr == 3 && bm > 128) return false;   // 36 accumulator tiles + hoisted addresses spill
  const int XW = W;                        // staged X row width - 2 (input columns)
  if (s2) { H /= 2; W /= 2; }              // tiles run over the dY (output) geometry
  const int img = H * W;
  WgradHaloGeom h{};
  h.MV = bm;
  if (bm <= img) {
    h.TH = bm / W;
    h.TB = 1;
    if (bm % W != 0 || img % bm != 0) {
      // padded row tiles: the most whole rows that tile the image, at most 1/8 idle
      // (ImageNet 28x28: 7 rows = 196 pixels in 224; 56x56: 4 rows in 256)
      while (h.TH > 0 && img % (h.TH * W) != 0) --h.TH;
      if (h.TH == 0) return false;
      h.MV = h.TH * W;
      if (8 * (bm - h.MV) > bm) return false;
    }
  } else {
    h.TH = H;
    h.TB = bm / img;
    if (bm % img != 0) {   // padded whole-image tiles: at most 1/8 of the rows idle
      h.MV = h.TB * img;
      if (8 * (bm - h.MV) > bm) return false;
    }
  }
  h.THX = h.TH + tr - 1;
  h.XROWS = h.TB * h.THX * (XW + 2);
  h.XPW = ((h.XROWS + 7) / 8 + 4 * pg - 1) / (4 * pg);
  if (h.XPW > kWhXPW || h.THX + 1 > 127 || h.TB > 0x7fff) return false;
  if ((ns - 2) * (bm / 32 + h.XPW) > 40) return false;
  const long long M = (long long)B * img;
  if (2LL * M * (CO > CI ? CO : CI) * (s2 ? 4 : 1) >= (1LL << 31)) return false;
  h.ntiles = (int)((M + h.MV - 1) / h.MV);
  const int per = (CI / 64) * (CO / 64) * (3 / tr);
  int sp = target / per;
  if (sp < 1) sp = 1;
  if (sp > h.ntiles) sp = h.ntiles;
  h.tiles_per_split = (h.ntiles + sp - 1) / sp;
  sp = (h.ntiles + h.tiles_per_split - 1) / h.tiles_per_split;
  const size_t stage = (size_t)bm * 64 + (size_t)h.XPW * 4 * pg * 512;
  *lds = (size_t)ns * stage * 2;
  if (*lds > 160 * 1024) return false;
  *g = h;
  *bm_out = bm;
  *ns_out = ns;
  *tr_out = tr;
  *pg_out = pg;
  *splits = sp;
  return true;
}

bool conv_wgrad_halo_ok(int cfg, int B, int H, int W, int CI, int CO, int R, int S, int stride,
                        int pad) {
  WgradHaloGeom g;
  int bm, ns, tr, pg, sp;
  size_t lds;
  if (!wgrad_halo_geom(cfg, B, H, W, CI, CO, R, S, stride, pad, &g, &bm, &ns, &tr, &pg, &lds, &sp))
    return false;
  if (cfg >= kWhSlabBase) return sp > 1 && wh_slab_variant((cfg - kWhSlabBase) / 12);
  return true;
}
// fp32 elements of the slab a slab-mode cfg needs (0: not a slab cfg / no split)
long long conv_wgrad_halo_slab_elems(int cfg, int B, int H, int W, int CI, int CO, int R, int S,
                                     int stride, int pad) {
  if (cfg < kWhSlabBase || !conv_wgrad_halo_ok(cfg, B, H, W, CI, CO, R, S, stride, pad)) return 0;
  WgradHaloGeom g;
  int bm, ns, tr, pg, sp;
  size_t lds;
  wgrad_halo_geom(cfg, B, H, W, CI, CO, R, S, stride, pad, &g, &bm, &ns, &tr, &pg, &lds, &sp);
  return (long long)sp * CO * R * S * CI;
}
int conv_wgrad_halo_base() { return kWhBase; }
int conv_wgrad_halo_slab_base() { return kWhSlabBase; }
int conv_wgrad_num_halo_configs() { return 12 * kWhVariants; }

// dW[e] += sum_s slab[s][e]: a block = 16 float4 columns x 16 split lanes (the
// split count runs to the hundreds on the 64-channel layers: a thread per
// column walking every split was latency-bound), LDS reduce over the lanes
__global__ void __launch_bounds__(256) wgrad_slab_reduce_kernel(const float* __restrict__ slab,
                                                                float* __restrict__ dw,
                                                                long long n4, int splits) {
  __shared__ float4 red[16][16];
  const int lx = threadIdx.x & 15, ly = threadIdx.x >> 4;
  const long long v = (long long)blockIdx.x * 16 + lx;
  const float4* s4 = reinterpret_cast<const float4*>(slab);
  float4 t = {0.f, 0.f, 0.f, 0.f};
  if (v < n4) {
    int sp = ly;
#pragma unroll 4
    for (; sp < splits; sp += 16) {
      const float4 u = s4[sp * n4 + v];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
  }
  red[ly][lx] = t;
  __syncthreads();
  if (ly == 0 && v < n4) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      const float4 u = red[k][lx];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    float4 d = reinterpret_cast<float4*>(dw)[v];
    d.x += t.x; d.y += t.y; d.z += t.z; d.w += t.w;
    reinterpret_cast<float4*>(dw)[v] = d;
  }
}

template <int BM, int NS, int TR, int PG = 1, bool S2 = false>
static void launch_wgrad_halo_t(const WgradArgs& a, const WgradHaloGeom& g, size_t lds, int splits,
                                hipStream_t s) {
  static bool attr = false;
  static int diag = -1;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv_wgrad_halo_kernel<BM, NS, TR, PG, S2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (diag < 0) {
    const char* e = getenv("DMP_WGRAD_HALO_DIAG");
    diag = (e && e[0] == 's') ? 1 : 0;
  }
  const dim3 grid((unsigned)(a.CI / 64), (unsigned)(a.CO / 64 * (3 / TR)), (unsigned)splits);
  const int mode = diag ? 2 : (splits > 1 ? (a.slab != nullptr ? 3 : 1) : 0);
  hipLaunchKernelGGL((conv_wgrad_halo_kernel<BM, NS, TR, PG, S2>), grid, dim3(256 * PG), lds, s, a,
                     g, mode);
  if (mode == 3) {
    const long long n4 = (long long)a.CO * 9 * a.CI / 4;
    hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0,
                       s, a.slab, a.dw, n4, splits);
  }
}

template <int NS, int TR>
static void launch_wgrad_halo_bm(int bm, const WgradArgs& a, const WgradHaloGeom& g, size_t lds,
                                 int sp, hipStream_t s) {
  if constexpr (TR == 1) {
    if (bm == 224) {
      launch_wgrad_halo_t<224, NS, 1>(a, g, lds, sp, s);
      return;
    }
  }
  if (bm == 64) launch_wgrad_halo_t<64, NS, TR>(a, g, lds, sp, s);
  else if (TR == 3 || bm == 128) launch_wgrad_halo_t<128, NS, TR>(a, g, lds, sp, s);
  else launch_wgrad_halo_t<(TR == 3 ? 128 : 256), NS, TR>(a, g, lds, sp, s);   // TR 3: BM <= 128
}

// cfg bits: [1:0] BNW (0 auto, 1 -> 64, 2 -> 128, 3 -> 192), [2] BP (0 -> 64, 1 -> 32),
// [3] NS (0 -> 2, 1 -> 3), [7:4] minimum rows of P per block in units of 512 (0 auto),
// [8] BMW 128 (CO % 128 == 0).
template <int BNW, int WM, int WN, int BMW = 64>
static void launch_wgrad_variant(const WgradArgs& a, dim3 grid, int bp, int ns, hipStream_t s) {
  if (bp == 32) {
    if (ns == 3) hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 32, 3, BMW>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 32, 2, BMW>), grid, dim3(256), 0, s, a);
  } else {
    if (ns == 3) hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 64, 3, BMW>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<BNW, WM, WN, 64, 2, BMW>), grid, dim3(256), 0, s, a);
  }
}

void launch_conv_wgrad(const u16* dy, const u16* x, float* dw, int B, int H, int W, int CI,
                       int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                       hipStream_t s, float* dbias, float* slab) {
  WgradArgs a{dy, x, dw, B, H, W, CI, OH, OW, CO, R, S, stride, pad, (long long)B * OH * OW, 0,
              dbias, nullptr};
  if (cfg >= kWhSlabBase) {
    if (slab != nullptr) a.slab = slab;
    else cfg -= kWhSlabBase - kWhBase;   // no slab given: the atomic variant
  }
  if (cfg >= kWhBase && dbias == nullptr) {
    WgradHaloGeom g;
    int bm, ns, tr, pg, sp;
    size_t lds;
    if (wgrad_halo_geom(cfg, B, H, W, CI, CO, R, S, stride, pad, &g, &bm, &ns, &tr, &pg, &lds,
                        &sp)) {
      if (stride == 2) {   // (geometry: TR 1, NS 2-3, BM 64 / 128 / 256)
        if (pg == 2) {
          if (bm == 128) launch_wgrad_halo_t<128, 2, 1, 2, true>(a, g, lds, sp, s);
          else launch_wgrad_halo_t<256, 2, 1, 2, true>(a, g, lds, sp, s);
        } else if (ns == 2) {
          if (bm == 64) launch_wgrad_halo_t<64, 2, 1, 1, true>(a, g, lds, sp, s);
          else if (bm == 128) launch_wgrad_halo_t<128, 2, 1, 1, true>(a, g, lds, sp, s);
          else launch_wgrad_halo_t<256, 2, 1, 1, true>(a, g, lds, sp, s);
        } else {
          if (bm == 64) launch_wgrad_halo_t<64, 3, 1, 1, true>(a, g, lds, sp, s);
          else if (bm == 128) launch_wgrad_halo_t<128, 3, 1, 1, true>(a, g, lds, sp, s);
          else launch_wgrad_halo_t<256, 3, 1, 1, true>(a, g, lds, sp, s);
        }
        return;
      }
      if (pg == 2) {
        if (bm == 128) launch_wgrad_halo_t<128, 2, 1, 2>(a, g, lds, sp, s);
        else launch_wgrad_halo_t<256, 2, 1, 2>(a, g, lds, sp, s);
      } else if (tr == 3) {
        if (ns == 2) launch_wgrad_halo_bm<2, 3>(bm, a, g, lds, sp, s);
        else launch_wgrad_halo_bm<3, 3>(bm, a, g, lds, sp, s);
      } else {
        if (ns == 2) launch_wgrad_halo_bm<2, 1>(bm, a, g, lds, sp, s);
        else if (ns == 3) launch_wgrad_halo_bm<3, 1>(bm, a, g, lds, sp, s);
        else launch_wgrad_halo_bm<4, 1>(bm, a, g, lds, sp, s);
      }
      return;
    }
    cfg = -1;   // not applicable: gather kernel, heuristic variant
  }
  if (cfg >= kWhBase) cfg = -1;   // halo cfg with a bias gradient: gather kernel
  const long long K = (long long)R * S * CI;
  const int sel = cfg < 0 ? 0 : (cfg & 3);
  int bnw = sel == 1 ? 64 : (sel == 2 ? 128 : (sel == 3 ? 192 : 0));
  if (bnw == 0) bnw = (K % 192 == 0) ? 192 : (K % 128 == 0 ? 128 : 64);
  if (K % bnw != 0) bnw = 64;
  const int bp = (cfg >= 0 && (cfg & 4)) ? 32 : 64;
  const int ns = (cfg >= 0 && (cfg & 8)) ? 3 : 2;
  const int bmw = (cfg >= 0 && (cfg & 256) && CO % 128 == 0) ? 128 : 64;
  const long long tiles = (K / bnw) * (CO / bmw);
  long long min_chunk = cfg < 0 ? 0 : (long long)((cfg >> 4) & 15) * 512;
  if (min_chunk <= 0) min_chunk = 2048;
  long long splits = (768 + tiles - 1) / tiles;
  long long chunk = (a.P + splits - 1) / splits;
  if (chunk < min_chunk) chunk = min_chunk;
  chunk = (chunk + bp - 1) / bp * bp;
  splits = (a.P + chunk - 1) / chunk;
  a.p_chunk = (int)chunk;
  // cfg bit 512: XCD-aware deal (a tuner choice: it wins where one pixel split's
  // tiles share few operand panels, loses where they span a many-MB working set)
  a.xcd = (cfg >= 0 && (cfg & 512)) ? 1 : 0;
  const dim3 grid((unsigned)(K / bnw), (unsigned)(CO / bmw), (unsigned)splits);
  if (bmw == 128) {
    if (bnw == 192) launch_wgrad_variant<192, 2, 2, 128>(a, grid, bp, ns, s);
    else if (bnw == 128) launch_wgrad_variant<128, 2, 2, 128>(a, grid, bp, ns, s);
    else launch_wgrad_variant<64, 2, 2, 128>(a, grid, bp, ns, s);
    return;
  }
  if (bnw == 192) launch_wgrad_variant<192, 1, 4>(a, grid, bp, ns, s);
  else if (bnw == 128) launch_wgrad_variant<128, 2, 2>(a, grid, bp, ns, s);
  else launch_wgrad_variant<64, 2, 2>(a, grid, bp, ns, s);
}

}  // namespace dmp
