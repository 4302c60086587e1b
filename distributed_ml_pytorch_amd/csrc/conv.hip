// NHWC bf16 convolution as implicit GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Not a translation of anything in the reference (it only calls torch.nn.Conv2d,
// /root/reference/example/models.py:8-9,28-38); these kernels replace the
// ATen/MIOpen `convolution` + `convolution_backward` rows of SURVEY §2.3.
//
//   fwd   : Y[m][co]  = sum_k X_gather[m][k] * W[co][k]       k = (r, s, ci), ci fastest
//   dgrad : dX = sum over the taps that actually reach each input pixel.  For
//           stride st the input pixels split into st*st parity classes
//           (h % st, w % st); class (ph, pw) is reached only by taps
//           r = (ph+pad) mod st + i*st (same for s), so each class is a dense
//           implicit GEMM over its own pixels with K = taps(class) * CO and no
//           wasted MFMA work (blockIdx.z = class).  Wt[ci][r][s][co] = W^T per tap.
//   wgrad : dW[co][k] += sum_p dY[p][co] * X_gather[p][k]       split over p, fp32
//           atomics straight into the flat fp32 grad arena (channels_last layout).
//           One block covers up to 3 taps (192 k-columns) so dY is re-read
//           K/192 times, not once per tap.
//
// Staging: every operand tile is fetched with global_load_lds_dwordx4 (LDS DMA,
// 16 B per lane, no VGPR round trip).  The LDS image is lane-linear, so the
// bank-conflict swizzle is applied on the per-lane SOURCE address (the read side
// applies the same involution), and gather lanes whose tap falls in the zero
// padding fetch from a zeroed 16-B page instead of branching.  This keeps the
// VALU work per MFMA low: the first register-staged version of these kernels
// measured ~10 VALU instructions per MFMA (SQ_INSTS_VALU / SQ_INSTS_MFMA) and
// was issue-bound.
//
// fwd/dgrad compute D^T = W * X^T so a lane owns 4 consecutive output channels of
// one pixel (8-byte NHWC stores) and the fwd epilogue can reduce per-channel
// BatchNorm partial sums (no extra pass over Y).  Several tile configurations are
// compiled; the host side times them per shape on first use (ops/tuner.py).
#include <cstdlib>

#include "common.h"

// cache policy (buffer aux bits) of the conv output stores: 0 default, 2 = nt
// (streaming); compile-time A/B knobs (scripts/conv_ab.py build-defines).  Measured
// per kernel family (profiles/conv_store_policy_r6.txt): the halo tiles' epilogues
// (fwd / dgrad, row-staged or not) -2.7..-4.3 % with nt on the 16x16 / 8x8 layers;
// the persistent 64-channel kernel +8 % slower with nt (dgrad): kept at the default
#ifndef DMP_CONV_STORE_AUX
#define DMP_CONV_STORE_AUX 0
#endif
#ifndef DMP_HALO_STORE_AUX
#define DMP_HALO_STORE_AUX 2
#endif
#include "launchers.h"

// Roofline ablations (scripts/conv_roofline.py builds a separate library with
// -DDMP_ABLATE=N; the extension itself is always built with 0):
//   1 = staging only (every global->LDS DMA, no MFMA work),
//   2 = MFMA only (the first stage is staged, later ones re-read it),
//   3 = no epilogue (accumulators kept live, nothing stored),
//   4 = no fragment reads after a stage's first steps (MFMAs on stale
//       registers: the LDS read path removed from the MFMA loop).
#ifndef DMP_ABLATE
#define DMP_ABLATE 0
#endif

namespace dmp {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));


struct ConvArgs {
  const u16* x;     // gathered operand NHWC [B][GH][GW][CI]   (fwd: X, dgrad: dY)
  const u16* w;     // [CO][R][S][CI]                           (fwd: W, dgrad: Wt)
  u16* y;           // output NHWC [B][OH][OW][CO]              (fwd: Y, dgrad: dX)
  float* part;      // optional BN slot sums [2][kBnSlots][CO] (atomically accumulated)
  int B, GH, GW, CI, OH, OW, CO, R, S, stride, pad;
  long long M;      // fwd: B*OH*OW; dgrad: rows of the largest parity class
  const float* bias;   // optional fp32 [CO] added in the fwd epilogue
  const u16* addend;   // dgrad: optional [B][H][W][CI] bf16 added to dX in the epilogue
  int relu;            // fwd: max(0, .) in the epilogue (conv -> ReLU, AlexNet)
  // dgrad with STATS: backward of the BatchNorm(+ReLU) that produced this conv's
  // input, fused into the epilogue (see bnb_* below)
  const u16* bnx;       // the BN's input x [B][H][W][CI]
  const u16* bnmask;    // bnrelu 1: the stored ReLU output (this conv's own input);
                        // bnrelu 3: bn.hip's 1-bit ReLU mask [pixels][CI/8] bytes
  const float* bnstat;  // the BN's [4][CI] mean | invstd | scale | shift
  int bnrelu;           // 0 no ReLU, 1 / 3 mask from bnmask, 2 mask recomputed from bnx
  // dgrad, stride 2: the addend is the gradient of the stride-2 SUBSAMPLED input
  // [B][ceil(H/2)][ceil(W/2)][CI] (a 1x1 / stride-2 shortcut that read x[::2, ::2]):
  // it lands on parity class (0, 0) only, indexed by the class-local row
  int addend_sub;
  // dgrad: optional 1-bit mask of the addend ([pixels][CI/8] bytes, bn.hip's ReLU
  // bit mask): addend element e counts only where its bit is set.  The residual
  // BatchNorm's backward then hands its UNMASKED dY over as the residual gradient
  // instead of writing dres = dY * relu' (ops/functional.py _BNAct, deferred dres)
  const uint8_t* addmask;
};


// Data-gradient epilogue fused with the backward of the BatchNorm(+ReLU) whose
// output the conv consumed (dgrad kernels instantiated with STATS): the kernel
// stores dz = dX * relu'(.) instead of dX, and the two BN-backward reductions
// sum(dz) and sum(dz * (x - mean)) leave through the same per-block slot sums
// as the forward statistics (the second scaled by invstd at the block
// reduction: sum(dz * xhat)).  That removes bn.hip's reduce pass (dY, x and y
// re-read) and the ReLU-mask input of its apply pass.  The mask is the stored
// ReLU output > 0 (bnrelu 1: BN + residual + ReLU, whose output is this conv's
// own input) or is recomputed from x and the folded scale/shift exactly as
// bn.hip relu_mask_from_x (bnrelu 2).
__device__ __forceinline__ float bnb_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bnb_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// relu'(.) of the BN output: stored output mk (bnrelu 1) or recomputed from the
// BN input xb and the folded scale/shift (bnrelu 2, rounded as the stored y)
__device__ __forceinline__ bool bnb_on(int bnrelu, float xb, float mk, float sc, float sh) {
  if (bnrelu == 1 || bnrelu == 3) return mk > 0.f;
  if (bnrelu == 2) return bf2f(f2bf(fmaxf(__fmaf_rn(xb, sc, sh), 0.f))) > 0.f;
  return true;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// LDS DMA (buffer_load_dwordx4 ... lds, 16 B per lane into a lane-linear 1 KiB
// wave slice at m0) from inline asm: with the builtin the compiler cannot tell
// the ring slot being filled from the one being read and puts s_waitcnt
// vmcnt(0) before the next ds_read, serialising the pipeline.  Completion is
// tracked by hand (wait_vm), counted per wave.  Offsets >= the descriptor's
// num_records read as zeros: that is how padding taps are fetched.
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                       u16* lds_wave_base) {
  const unsigned m0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave_base;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "{m0}"(m0));
}

// addend channels n..n+3 at byte offset `boff` (= 2 * element offset) of the
// addend, with the deferred ReLU mask applied when a.addmask is set
__device__ __forceinline__ void masked_addend4(const ConvArgs& a, __amdgpu_buffer_rsrc_t rsAdd,
                                               __amdgpu_buffer_rsrc_t rsAm, unsigned boff, bool ok,
                                               int n, float (&ad)[4]) {
  typedef unsigned int u32x2_m __attribute__((ext_vector_type(2)));
  const u32x2_m av = __builtin_amdgcn_raw_buffer_load_b64(rsAdd, ok ? boff : kOOB, 0, 0);
  ad[0] = __uint_as_float(av.x << 16);
  ad[1] = __uint_as_float(av.x & 0xffff0000u);
  ad[2] = __uint_as_float(av.y << 16);
  ad[3] = __uint_as_float(av.y & 0xffff0000u);
  if (a.addmask != nullptr) {
    // byte (element offset / 8); channels n..n+3 are its bits (n & 4) .. +3
    const unsigned bits = __builtin_amdgcn_raw_buffer_load_b8(rsAm, ok ? boff >> 4 : kOOB, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) ad[r] = (bits >> ((n & 4) + r)) & 1u ? ad[r] : 0.f;
  }
}

// q = n / d, r = n % d for 0 <= n < 2^24 with a float reciprocal (one
// correction step); replaces the ~30-instruction integer division sequence in
// per-lane index math whose dividend is a small in-tile offset
__device__ __forceinline__ void small_divmod(int n, int d, float rcp, int& q, int& r) {
  q = (int)((float)n * rcp);
  r = n - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
}

// sum of v over the 16 lanes of each DPP row, valid in lane 15 of the row:
// four v_add_f32_dpp row_shr steps (bound_ctrl zero-fills lanes shifted in
// from outside the row) instead of four ds_bpermute round trips
__device__ __forceinline__ float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// wait until at most N of this wave's vector-memory ops are outstanding (and
// all of its LDS ops have completed)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}

// 16-byte chunk swizzle (an involution) for a row-major [rows][BK] bf16 tile.
//  BK=64 (128-B rows, 2 rows per 256-B bank row): chunk ^= ((row>>1)&3) << 1
//  BK=32 ( 64-B rows, 4 rows per bank row):       chunk ^= ((row>>2)&1) << 1
// A ds_read_b128 fragment read (lane l: row p + (l&15), chunk c + (l>>4)) is
// serviced in lane groups {0-3,12-15,20-27} / {4-11,16-19,28-31} (+32): rows
// p..p+3 and p+12..p+15 at one chunk, p+4..p+11 at the next.  These XORs give
// 16 distinct 16-B slots per group for ANY start row p, not only p % 16 == 0:
// the halo kernels read fragments at row offsets of +1, +2, W+2, ... (one per
// tap), where the previous (row>>1)&7 / (-(row>>2))&3 forms conflicted (34 %
// extra LDS cycles measured on the 64-channel halo forward,
// profiles/halo_pmc_r1.txt).  Rows r and r+16 share the XOR, so fragment rows
// 16 apart differ by a constant offset (folded into ds_read immediates).
template <int BK>
__device__ __forceinline__ int swz(int row, int c) {
  if constexpr (BK == 64) return c ^ (((row >> 1) & 3) << 1);
  else return c ^ (((row >> 2) & 1) << 1);
}

// MODE 0: forward conv.  MODE 1: data gradient, one parity class per blockIdx.z.
// NS-stage LDS-DMA ring: NS-1 k-tiles in flight while one is consumed.  (A
// register-staged variant -- global_load into VGPRs, ds_write_b128 -- measured
// 2-4x slower on every ResNet-18 shape: profiles/igemm_ablate_r1.txt.)
template <int BM, int BN, int WM, int WN, bool FLIP, bool STATS, int TM, int TN>
__device__ __forceinline__ void halo_epilogue_rows(const ConvArgs& a, f32x4 (&acc)[TM][TN],
                                                   long long m0, int n0, int wm, int wn, int tid,
                                                   int lane, u16* lds_h, int mv);

// ROWS: the row-staged epilogue of the halo kernels (16-B row segments out of
// an LDS block tile) instead of the D^T register stores -- for the store-bound
// 1x1 convs (K = 64 input channels, 4x the output bytes).  Forward tiles, and
// stride-1 data-gradient tiles without the fused BN backward (output row m =
// dX pixel m there too; the launcher checks).
template <int BM, int BN, int BK, int WM, int WN, int MODE, bool STATS, int NS, bool ROWS = false>
__global__ void __launch_bounds__(64 * WM * WN) conv_igemm_kernel(ConvArgs a) {
  constexpr int NW = WM * WN;
  constexpr int CPR = BK / 8;                 // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;               // tile rows per glds wave-instruction (1 KiB)
  constexpr int A_INS = BM / RPI;
  constexpr int B_INS = (BN + RPI - 1) / RPI;
  constexpr int A_PW = (A_INS + NW - 1) / NW;
  constexpr int B_PW = (B_INS + NW - 1) / NW;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int A_EL = BM * BK, B_EL = B_INS * RPI * BK;
  constexpr int STAGE = A_EL + B_EL;
  // DMAs every wave has issued per stage (a wave may issue more; waiting on
  // the minimum is conservative for it)
  constexpr int INS_MIN = A_INS / NW + B_INS / NW;
  static_assert(NS >= 2 && (NS - 2) * INS_MIN < 64, "pipeline depth");
  static_assert(!ROWS || MODE == 0 || !STATS, "row-staged epilogue: no fused BN backward");
  constexpr int LDS_EL = (ROWS && BM * (BN + 8) > NS * STAGE) ? BM * (BN + 8) : NS * STAGE;
  __shared__ __attribute__((aligned(16))) u16 lds[LDS_EL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int GH = a.GH, GW = a.GW, CI = a.CI, st = a.stride;

  // class geometry (MODE 1) -------------------------------------------------
  int ph = 0, pw = 0, r0h = 0, r0w = 0, nth = a.R, ntw = a.S, RH = a.OH, RW = a.OW;
  long long Mc = a.M;
  if (MODE == 1) {
    ph = (int)blockIdx.z / st;
    pw = (int)blockIdx.z - ph * st;
    r0h = (ph + a.pad) % st;
    r0w = (pw + a.pad) % st;
    nth = a.R > r0h ? (a.R - r0h + st - 1) / st : 0;
    ntw = a.S > r0w ? (a.S - r0w + st - 1) / st : 0;
    RH = (a.OH - ph + st - 1) / st;    // output rows of this parity
    RW = (a.OW - pw + st - 1) / st;
    Mc = (long long)a.B * RH * RW;
    if (m0 >= Mc) return;
  }

  // per-lane gather state for the A tile (lane's row in each DMA piece), all
  // 32-bit: byte offsets into the operand buffers; a padded / out-of-range
  // fetch gets an offset past the descriptor's bound and the buffer unit
  // returns zeros (no branch, no zero page, no 64-bit address math per piece)
  int a_h[A_PW], a_w[A_PW];
  unsigned a_base[A_PW];
  bool a_ok[A_PW];
  // the tile's first row decoded once (scalar), lanes step from it with small
  // float-reciprocal divisions
  const int m0i = (int)m0;
  const int ow0 = m0i % RW, t0 = m0i / RW;
  const int oh0 = t0 % RH, b0 = t0 / RH;
  const float rcpW = 1.f / (float)RW, rcpH = 1.f / (float)RH;
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    const int a_c = swz<BK>(row, lane % CPR) * 8;      // logical chunk this lane fetches
    const int m = m0i + row;
    a_ok[j] = ins < A_INS && m < (int)Mc;
    int q1, ow, q2, oh;
    small_divmod(ow0 + (a_ok[j] ? row : 0), RW, rcpW, q1, ow);
    small_divmod(oh0 + q1, RH, rcpH, q2, oh);
    const int b = b0 + q2;
    if (MODE == 0) { a_h[j] = oh * st - a.pad; a_w[j] = ow * st - a.pad; }
    else           { a_h[j] = oh;              a_w[j] = ow; }
    // may wrap for a padded (negative) origin; only used when the tap is in range
    a_base[j] = 2u * (unsigned)(((b * GH + a_h[j]) * GW + a_w[j]) * CI + a_c);
  }
  const int K = a.R * a.S * CI;
  unsigned b_base[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    const int n = n0 + row;
    const bool ok = ins < B_INS && row < BN && n < a.CO;
    b_base[j] = ok ? 2u * (unsigned)(n * K + swz<BK>(row, lane % CPR) * 8) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * a.B * GH * GW * CI), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, 0, (int)(2LL * a.CO * K), 0x00020000);

  const int kpr = CI / BK;          // k-tiles per tap
  const int KT = nth * ntw * kpr;

  auto stage = [&](int buf, int kt) {
    const int t = kt / kpr;
    const int cb = (kt - t * kpr) * BK;
    int r, s, dh, dw;
    if (MODE == 0) {
      r = t / a.S; s = t - r * a.S; dh = r; dw = s;
    } else {
      const int ti = t / ntw, tj = t - ti * ntw;
      r = r0h + ti * st; s = r0w + tj * st;
      dh = (ph + a.pad - r) / st;        // exact: (ph + pad - r) is a multiple of st
      dw = (pw + a.pad - s) / st;
    }
    u16* As = lds + buf * STAGE;
    u16* Bs = As + A_EL;
    const unsigned adelta = 2u * (unsigned)((dh * GW + dw) * CI + cb);   // wave-uniform
#pragma unroll
    for (int j = 0; j < A_PW; ++j) {
      const int ins = wid + j * NW;
      if (A_INS % NW == 0 || ins < A_INS) {
        const int ih = a_h[j] + dh, iw = a_w[j] + dw;
        const bool ok = a_ok[j] && (unsigned)ih < (unsigned)GH && (unsigned)iw < (unsigned)GW;
        bdma16(rsA, ok ? a_base[j] + adelta : kOOB, As + ins * (RPI * BK));
      }
    }
    const unsigned wdelta = 2u * (unsigned)((r * a.S + s) * CI + cb);
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int ins = wid + j * NW;
      if (B_INS % NW == 0 || ins < B_INS)
        bdma16(rsB, b_base[j] == kOOB ? kOOB : b_base[j] + wdelta, Bs + ins * (RPI * BK));
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment offsets (elements) for k-step 0/1; rows 16 apart add 16*BK
  int offA[BK / 32], offB[BK / 32];
  {
    const int ra = wm * (BM / WM) + (lane & 15);
    const int rb = wn * (BN / WN) + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      offA[ks] = ra * BK + swz<BK>(ra, c) * 8;
      offB[ks] = A_EL + rb * BK + swz<BK>(rb, c) * 8;
    }
  }
  auto compute = [&](int buf) {
    const u16* base = lds + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(base + offA[ks] + i * 16 * BK);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[j] = *reinterpret_cast<const bf16x8*>(base + offB[ks] + j * 16 * BK);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bw[j], af[i], acc[i][j]);
    }
  };

  if (KT > 0) {
    {
#pragma unroll
      for (int st0 = 0; st0 < NS - 1; ++st0)
        if (st0 < KT) stage(st0, st0);
      for (int kt = 0; kt < KT; ++kt) {
        // k-tile kt landed for this wave (younger tiles may still fly) ...
        if (kt + NS - 2 < KT) wait_vm<(NS - 2) * INS_MIN>();
        else wait_vm<0>();
        // ... and for every wave; everyone is done with tile kt-1's slot
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + NS - 1 < KT) stage((kt + NS - 1) % NS, kt + NS - 1);
        compute(kt % NS);
      }
    }
  }
  __syncthreads();   // all ring reads done before the epilogue reuses LDS
  if constexpr (ROWS) {
    halo_epilogue_rows<BM, BN, WM, WN, MODE == 1, MODE == 0 && STATS, TM, TN>(
        a, acc, m0, n0, wm, wn, tid, lane, lds, BM);
    return;
  }

  // epilogue: D^T layout -> lane owns channels n..n+3 of output row m.
  // Stores go through a buffer descriptor with 32-bit offsets; rows past M and
  // channels past CO get an out-of-range offset and are dropped by the buffer
  // unit (no per-tile branch).  Bias (fwd) is fetched once per column tile.
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.y, 0, (int)(2LL * a.B * a.OH * a.OW * a.CO), 0x00020000);
  // dgrad accumulate: dX = dgrad + addend (the residual branch's gradient of the
  // same input, fused here instead of an autograd add over the whole tensor);
  // forward: the residual of an inference-time BatchNorm fold, before the ReLU
  const bool add_in = a.addend != nullptr && (MODE == 0 || !a.addend_sub || blockIdx.z == 0);
  const __amdgpu_buffer_rsrc_t rsAdd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in ? a.addend : a.y), 0, (int)(2LL * a.B * a.OH * a.OW * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsAm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in && a.addmask ? (const void*)a.addmask : (const void*)a.y), 0,
      (int)(a.B * a.OH * a.OW * (long long)a.CO / 8), 0x00020000);
  constexpr bool BNB = MODE == 1 && STATS;   // fused BN(+ReLU) backward
  const __amdgpu_buffer_rsrc_t rsBx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNB ? a.bnx : a.y), 0, (int)(2LL * a.B * a.OH * a.OW * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsBm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNB && (a.bnrelu == 1 || a.bnrelu == 3) ? a.bnmask : a.y), 0,
      (int)((a.bnrelu == 3 ? 1LL : 16LL) * a.B * a.OH * a.OW * a.CO / 8), 0x00020000);
  float bj[TN][4];
  bool nok[TN];
  // BNB: per-channel mean | scale | shift of the BN (channels n..n+3 of tile j)
  float bmu[BNB ? TN : 1][4], bsc[BNB ? TN : 1][4], bsh[BNB ? TN : 1][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
    nok[j] = n < a.CO;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bj[j][r] = (MODE == 0 && a.bias != nullptr && n + r < a.CO) ? a.bias[n + r] : 0.f;
      if constexpr (BNB) {
        const int ch = nok[j] ? n + r : 0;
        bmu[j][r] = a.bnstat[ch];
        bsc[j][r] = a.bnrelu == 2 ? a.bnstat[2 * a.CO + ch] : 0.f;
        bsh[j][r] = a.bnrelu == 2 ? a.bnstat[3 * a.CO + ch] : 0.f;
      }
    }
  }
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
    const bool mok = m < Mc;
    long long pix = m;
    if (MODE == 1) {
      const int rloc = mok ? (int)(m - m0) : 0;
      int q1, j, q2, ii;
      small_divmod(ow0 + rloc, RW, rcpW, q1, j);
      small_divmod(oh0 + q1, RH, rcpH, q2, ii);
      const long long b = b0 + q2;
      pix = (b * a.OH + (long long)ii * st + ph) * a.OW + (long long)j * st + pw;
    }
    const unsigned rowoff = 2u * (unsigned)(pix * a.CO);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
      typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
      const bool ok = mok && nok[j];
      float ad[4] = {0.f, 0.f, 0.f, 0.f};
      if (add_in) {
        const unsigned aoff = a.addend_sub ? 2u * (unsigned)(m * a.CO) : rowoff;
        masked_addend4(a, rsAdd, rsAm, aoff + 2u * n, ok, n, ad);
      }
      float xb[4] = {0.f, 0.f, 0.f, 0.f}, mk[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BNB) {
        const u32x2_t xv = __builtin_amdgcn_raw_buffer_load_b64(rsBx, ok ? rowoff + 2u * n : kOOB, 0, 0);
        xb[0] = bnb_lo(xv.x); xb[1] = bnb_hi(xv.x); xb[2] = bnb_lo(xv.y); xb[3] = bnb_hi(xv.y);
        if (a.bnrelu == 1) {
          const u32x2_t mv =
              __builtin_amdgcn_raw_buffer_load_b64(rsBm, ok ? rowoff + 2u * n : kOOB, 0, 0);
          mk[0] = bnb_lo(mv.x); mk[1] = bnb_hi(mv.x); mk[2] = bnb_lo(mv.y); mk[3] = bnb_hi(mv.y);
        } else if (a.bnrelu == 3) {
          // byte (pixel, n / 8) of the bit mask; bits (n & 4) .. +3 are channels n .. n+3
          const unsigned bits = __builtin_amdgcn_raw_buffer_load_b8(
              rsBm, ok ? (rowoff >> 4) + (unsigned)(n >> 3) : kOOB, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) mk[r] = (bits >> ((n & 4) + r)) & 1u ? 1.f : 0.f;
        }
      }
      u16 h[4];
      float v[4], t[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[r] = acc[i][j][r] + bj[j][r] + ad[r];
        if (MODE == 0 && a.relu) t[r] = fmaxf(t[r], 0.f);
        if constexpr (BNB)
          t[r] = bnb_on(a.bnrelu, xb[r], mk[r], bsc[j][r], bsh[j][r]) ? t[r] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = f2bf(t[r]);
        v[r] = bf2f(h[r]);   // statistics of the stored (rounded) values
      }
      const u32x2_t packed = {(u32)h[0] | ((u32)h[1] << 16), (u32)h[2] | ((u32)h[3] << 16)};
      __builtin_amdgcn_raw_buffer_store_b64(packed, rsY, ok ? rowoff + 2u * n : kOOB, 0, DMP_CONV_STORE_AUX);
      if (STATS) {
        const float keep = ok ? 1.f : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = v[r] * keep;
          s_sum[j][r] += x;
          if constexpr (BNB) s_sq[j][r] += x * (xb[r] - bmu[j][r]);
          else s_sq[j][r] += x * x;
        }
      }
    }
  }
  if (STATS) {
    // sum over the 16 rows of each lane group with DPP row shifts (lane 15 of
    // every 16-lane row ends up with the row total)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s_sum[j][r] = row_sum16(s_sum[j][r]);
        s_sq[j][r] = row_sum16(s_sq[j][r]);
      }
    float* red = reinterpret_cast<float*>(lds);   // [WM][BN] sums, then [WM][BN] squares
    if ((lane & 15) == 15) {
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
    for (int nl = tid; nl < BN; nl += 64 * NW) {
      const int n = n0 + nl;
      if (n < a.CO) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { ss += red[w * BN + nl]; qq += red[WM * BN + w * BN + nl]; }
        if (BNB) qq *= a.bnstat[a.CO + n];   // sum dz * (x - mean) -> sum dz * xhat
        const int slot = (blockIdx.x + blockIdx.z * gridDim.x) % kBnSlots;
        atomicAdd(a.part + (long long)slot * a.CO + n, ss);
        atomicAdd(a.part + (long long)(kBnSlots + slot) * a.CO + n, qq);
      }
    }
  }
}

// ------------------------------------------------ 3x3 stride-1 halo tiles
// The implicit GEMM above gathers its A operand once per tap: a 3x3 conv
// pulls every input pixel through L2 / the Infinity Cache nine times, and on
// the 32x32 / 16x16 ResNet-18 layers that traffic (not the MFMA work) sets the
// kernel time (~7.8 TB/s measured on 64->64 32x32, the Infinity-Cache gather
// rate).  For 3x3 / stride 1 / pad 1 this kernel instead stages, per 32-channel
// chunk, the block's input pixels ONCE with their one-pixel halo -- a tile of
// TB images x (TH+2) rows x (W+2) columns, out-of-image positions fetched as
// zeros through the buffer descriptor -- plus all 9 taps of the weight chunk,
// and runs the nine tap products out of LDS by offsetting the pixel row
// (tap (r, s) of output pixel (th, tw) = halo row (th + r) * (W+2) + tw + s).
// The block's BM output pixels are whole image rows (TB = 1, TH = BM / W) or
// whole images (TH = H, TB = BM / (H*W)), so they are a contiguous range of
// NHWC rows and the epilogue is the forward one.  FLIP runs the stride-1 data
// gradient: the same conv over dY with Wt[ci][r][s][co] and the taps mirrored.
// NS = 2: two LDS stages (halo + 9 weight tiles each), one barrier per chunk;
// NS = 1: one stage, more resident blocks per CU.
// MV: output pixels per tile.  = BM, except for "padded whole-image" tiles
// (ImageNet ResNet 14x14 / 7x7 maps, where no multiple of 16 is a whole number
// of images): TB images (MV = TB * H * W < BM) in a BM-row tile whose last
// BM - MV rows read a valid staged row and are dropped by the epilogue.
struct HaloGeom {
  int TH, TB, HROWS, A_INS, MV;
  // conv_halo_kernel staging: staged row width W2 (W + 2, or W + 4 with PSW),
  // rows per image block PI ((TH + 2) * W2 [+ pad]), PSW: swizzle keyed on the
  // pixel-like index (see conv_halo_kernel)
  int W2, PI, PSW;
};

constexpr int kHaloAPW = 8;   // max halo DMA instructions per wave per stage

// Epilogue of the halo tiles (forward layout: output row m = pixel m): bias
// (fwd), residual gradient addend (FLIP), BN partial sums (STATS) -- as
// conv_igemm_kernel.  Wave (wm, wn) holds TM x TN 16x16 D^T fragments; the
// LDS at lds_h is free (the caller synchronised after its last stage read).
// S2: the stride-2 data gradient's parity class `cls` (conv_dgrad_s2_kernel): row
// m of the class grid (dY geometry GH x GW) is dX pixel (2i + ph, 2j + pw); a
// subsampled addend (addend_sub) lands on class 0 only, indexed by m.
template <int BM, int BN, int WM, int WN, bool FLIP, bool STATS, int TM, int TN, bool S2 = false>
__device__ __forceinline__ void halo_epilogue(const ConvArgs& a, f32x4 (&acc)[TM][TN], long long m0,
                                              int n0, int wm, int wn, int tid, int lane,
                                              u16* lds_h, int cls = 0, int mv = BM) {
  constexpr int NW = WM * WN;
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  const long long Mtot = (long long)a.B * a.OH * a.OW;
  const long long Mrows = S2 ? (long long)a.B * a.GH * a.GW : Mtot;
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.y, 0, (int)(2LL * Mtot * a.CO), 0x00020000);
  // the training forward that feeds a BatchNorm (STATS, not FLIP) takes no
  // bias, ReLU or addend (launch_halo routes such a conv elsewhere): compiled out
  constexpr bool PLAIN = STATS && !FLIP;
  const bool add_in = !PLAIN && (S2 ? (a.addend != nullptr && (!a.addend_sub || cls == 0))
                                    : (a.addend != nullptr));   // dgrad residual grad / fwd BN-fold residual
  const __amdgpu_buffer_rsrc_t rsAdd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in ? a.addend : a.y), 0, (int)(2LL * Mtot * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsAm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in && a.addmask ? (const void*)a.addmask : (const void*)a.y), 0,
      (int)(Mtot * a.CO / 8), 0x00020000);
  constexpr bool BNB = FLIP && STATS;   // fused BN(+ReLU) backward
  const __amdgpu_buffer_rsrc_t rsBx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNB ? a.bnx : a.y), 0, (int)(2LL * Mtot * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsBm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNB && (a.bnrelu == 1 || a.bnrelu == 3) ? a.bnmask : a.y), 0,
      (int)((a.bnrelu == 3 ? 1LL : 16LL) * Mtot * a.CO / 8), 0x00020000);
  float bj[TN][4];
  bool nok[TN];
  // BNB: per-channel mean | scale | shift of the BN (channels n..n+3 of tile j)
  float bmu[BNB ? TN : 1][4], bsc[BNB ? TN : 1][4], bsh[BNB ? TN : 1][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
    nok[j] = n < a.CO;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bj[j][r] = (!FLIP && !PLAIN && a.bias != nullptr && n + r < a.CO) ? a.bias[n + r] : 0.f;
      if constexpr (BNB) {
        const int ch = nok[j] ? n + r : 0;
        bmu[j][r] = a.bnstat[ch];
        bsc[j][r] = a.bnrelu == 2 ? a.bnstat[2 * a.CO + ch] : 0.f;
        bsh[j][r] = a.bnrelu == 2 ? a.bnstat[3 * a.CO + ch] : 0.f;
      }
    }
  }
  float s_sum[TN][4], s_sq[TN][4];
  if (STATS) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s_sum[j][r] = 0.f; s_sq[j][r] = 0.f; }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wm * (BM / WM) + i * 16 + (lane & 15);
    const long long m = m0 + ml;
    const bool mok = ml < mv && m < Mrows;
    long long pix = m;
    if constexpr (S2) {
      const int mi = (int)m, gi = a.GH * a.GW;
      const int b = mi / gi, rem = mi - b * gi, ii = rem / a.GW, jj = rem - ii * a.GW;
      pix = ((long long)b * a.OH + 2 * ii + (cls >> 1)) * a.OW + 2 * jj + (cls & 1);
    }
    const unsigned rowoff = 2u * (unsigned)(pix * a.CO);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
      const bool ok = mok && nok[j];
      float ad[4] = {0.f, 0.f, 0.f, 0.f};
      if (add_in) {
        const unsigned aoff = a.addend_sub ? 2u * (unsigned)(m * a.CO) : rowoff;
        masked_addend4(a, rsAdd, rsAm, aoff + 2u * n, ok, n, ad);
      }
      float xb[4] = {0.f, 0.f, 0.f, 0.f}, mk[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BNB) {
        const u32x2_t xv = __builtin_amdgcn_raw_buffer_load_b64(rsBx, ok ? rowoff + 2u * n : kOOB, 0, 0);
        xb[0] = bnb_lo(xv.x); xb[1] = bnb_hi(xv.x); xb[2] = bnb_lo(xv.y); xb[3] = bnb_hi(xv.y);
        if (a.bnrelu == 1) {
          const u32x2_t mv =
              __builtin_amdgcn_raw_buffer_load_b64(rsBm, ok ? rowoff + 2u * n : kOOB, 0, 0);
          mk[0] = bnb_lo(mv.x); mk[1] = bnb_hi(mv.x); mk[2] = bnb_lo(mv.y); mk[3] = bnb_hi(mv.y);
        } else if (a.bnrelu == 3) {
          // byte (pixel, n / 8) of the bit mask; bits (n & 4) .. +3 are channels n .. n+3
          const unsigned bits = __builtin_amdgcn_raw_buffer_load_b8(
              rsBm, ok ? (rowoff >> 4) + (unsigned)(n >> 3) : kOOB, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) mk[r] = (bits >> ((n & 4) + r)) & 1u ? 1.f : 0.f;
        }
      }
      u16 hv[4];
      float v[4], t[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[r] = PLAIN ? acc[i][j][r] : acc[i][j][r] + bj[j][r] + ad[r];
        if (!FLIP && !PLAIN && a.relu) t[r] = fmaxf(t[r], 0.f);
        if constexpr (BNB)
          t[r] = bnb_on(a.bnrelu, xb[r], mk[r], bsc[j][r], bsh[j][r]) ? t[r] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[r] = f2bf(t[r]);
        v[r] = bf2f(hv[r]);
      }
      const u32x2_t packed = {(u32)hv[0] | ((u32)hv[1] << 16), (u32)hv[2] | ((u32)hv[3] << 16)};
      // (the stride-2 data gradient scatters every other pixel: default policy, its
      // half-line writes merge in L2)
      __builtin_amdgcn_raw_buffer_store_b64(packed, rsY, ok ? rowoff + 2u * n : kOOB, 0,
                                            S2 ? 0 : DMP_HALO_STORE_AUX);
      if (STATS) {
        const float keep = ok ? 1.f : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = v[r] * keep;
          s_sum[j][r] += x;
          if constexpr (BNB) s_sq[j][r] += x * (xb[r] - bmu[j][r]);
          else s_sq[j][r] += x * x;
        }
      }
    }
  }
  if (STATS) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s_sum[j][r] = row_sum16(s_sum[j][r]);
        s_sq[j][r] = row_sum16(s_sq[j][r]);
      }
    float* red = reinterpret_cast<float*>(lds_h);   // [WM][BN] sums, then [WM][BN] squares
    if ((lane & 15) == 15) {
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
    for (int nl = tid; nl < BN; nl += 64 * NW) {
      const int n = n0 + nl;
      if (n < a.CO) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { ss += red[w * BN + nl]; qq += red[WM * BN + w * BN + nl]; }
        if (BNB) qq *= a.bnstat[a.CO + n];   // sum dz * (x - mean) -> sum dz * xhat
        const int slot = (blockIdx.x + blockIdx.z * gridDim.x) % kBnSlots;
        atomicAdd(a.part + (long long)slot * a.CO + n, ss);
        atomicAdd(a.part + (long long)(kBnSlots + slot) * a.CO + n, qq);
      }
    }
  }
}

#ifndef DMP_HALO_EPI_LDS
#define DMP_HALO_EPI_LDS 0
#endif


// Row-staged variant of halo_epilogue (no S2, no fused BN backward): the D^T
// fragments (lane: 4 channels of one pixel -> 16 rows x 32-B pieces per store
// instruction) are staged through the free LDS as a [BM][BN + 8] bf16 block
// tile, then every wave moves whole 16-B row segments: 8 channels of one pixel
// per lane, a pixel's BN channels contiguous -- the stores (and the residual
// addend loads) go out as full 128-B lines (BN = 64) instead of 32-B pieces.
// fp32 math before the staging: acc + bias (+ ReLU when no addend follows);
// with an addend the staged bf16 value gets the addend, then the ReLU, in the
// row phase.  BN partial sums (STATS) of the stored values: per lane over its
// rows, shuffle-reduced over the lanes of one channel chunk, LDS across waves,
// one atomic pair per channel per block (slot blockIdx % kBnSlots).
template <int BM, int BN, int WM, int WN, bool FLIP, bool STATS, int TM, int TN>
__device__ __forceinline__ void halo_epilogue_rows(const ConvArgs& a, f32x4 (&acc)[TM][TN],
                                                   long long m0, int n0, int wm, int wn, int tid,
                                                   int lane, u16* lds_h, int mv) {
  constexpr int NW = WM * WN, PITCH = BN + 8, CPR = BN / 8, RPI = 64 / CPR;
  static_assert(BN % 8 == 0 && 64 % CPR == 0, "row segments of 8 channels");
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  const long long Mtot = (long long)a.B * a.OH * a.OW;
  // statistics forward (feeds a BatchNorm): no bias / ReLU / addend, compiled out
  // (launch_cfg sends such a conv with any of them to the plain epilogue)
  constexpr bool PLAIN = STATS && !FLIP;
  const bool add_in = !PLAIN && a.addend != nullptr;
  const bool relu = !FLIP && !PLAIN && a.relu;
  // phase 1: fp32 epilogue math that needs no addend, bf16, into the block tile
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
    float bj[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bj[r] = (!FLIP && !PLAIN && a.bias != nullptr && n0 + nl + r < a.CO) ? a.bias[n0 + nl + r] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / WM) + i * 16 + (lane & 15);
      float t[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[r] = acc[i][j][r] + bj[r];
        if (relu && !add_in) t[r] = fmaxf(t[r], 0.f);
      }
      uint2 pk;
      pk.x = (u32)f2bf(t[0]) | ((u32)f2bf(t[1]) << 16);
      pk.y = (u32)f2bf(t[2]) | ((u32)f2bf(t[3]) << 16);
      *reinterpret_cast<uint2*>(lds_h + ml * PITCH + nl) = pk;
    }
  }
  __syncthreads();
  // phase 2: row segments; wave w takes rows w*RPI + k*NW*RPI + lane/CPR
  const int wid = tid >> 6, lr = lane / CPR, ch = lane - lr * CPR;
  const int n = n0 + ch * 8;
  const bool nok = n < a.CO;
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.y, 0, (int)(2LL * Mtot * a.CO), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsAdd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in ? a.addend : a.y), 0, (int)(2LL * Mtot * a.CO), 0x00020000);
  // deferred ReLU mask of the addend (ConvArgs::addmask): one byte = this lane's 8 channels
  const bool add_mask = add_in && a.addmask != nullptr;
  const __amdgpu_buffer_rsrc_t rsAm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_mask ? (const void*)a.addmask : (const void*)a.y), 0, (int)(Mtot * a.CO / 8),
      0x00020000);
  constexpr int NR = (BM + NW * RPI - 1) / (NW * RPI);
  unsigned off[NR], amb[NR];
  u32x4_t xa[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    const int ml = (q * NW + wid) * RPI + lr;
    const long long m = m0 + ml;
    off[q] = (ml < mv && m < Mtot && nok) ? 2u * (unsigned)(m * a.CO + n) : kOOB;
    if (add_in) xa[q] = __builtin_amdgcn_raw_buffer_load_b128(rsAdd, off[q], 0, 0);
    amb[q] = add_mask ? __builtin_amdgcn_raw_buffer_load_b8(rsAm, off[q] != kOOB ? off[q] >> 4 : kOOB,
                                                             0, 0)
                      : 0xffu;
  }
  float s_sum[8], s_sq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s_sum[e] = 0.f; s_sq[e] = 0.f; }
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    const int ml = min((q * NW + wid) * RPI + lr, BM - 1);
    bf16x8 v = *reinterpret_cast<const bf16x8*>(lds_h + ml * PITCH + ch * 8);
    if (add_in) {
      const bf16x8 xv = __builtin_bit_cast(bf16x8, xa[q]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = bf2f(v.v[e]) + ((amb[q] >> e) & 1u ? bf2f(xv.v[e]) : 0.f);
        if (relu) t = fmaxf(t, 0.f);
        v.v[e] = f2bf(t);
      }
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rsY, off[q], 0, DMP_HALO_STORE_AUX);
    if (STATS && off[q] != kOOB) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float yv = bf2f(v.v[e]);
        s_sum[e] += yv;
        s_sq[e] += yv * yv;
      }
    }
  }
  if constexpr (STATS) {
    // lanes of one channel chunk differ in the bits above CPR
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s_sum[e] += __shfl_xor(s_sum[e], o, 64);
        s_sq[e] += __shfl_xor(s_sq[e], o, 64);
      }
    __syncthreads();                                  // every row segment read the tile
    float* red = reinterpret_cast<float*>(lds_h);     // [NW][BN] sums, then [NW][BN] squares
    if (lr == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid * BN + ch * 8 + e] = s_sum[e];
        red[NW * BN + wid * BN + ch * 8 + e] = s_sq[e];
      }
    }
    __syncthreads();
    for (int nl = tid; nl < BN; nl += 64 * NW) {
      if (n0 + nl < a.CO) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) { ss += red[w * BN + nl]; qq += red[NW * BN + w * BN + nl]; }
        const int slot = blockIdx.x % kBnSlots;
        atomicAdd(a.part + (long long)slot * a.CO + n0 + nl, ss);
        atomicAdd(a.part + (long long)(kBnSlots + slot) * a.CO + n0 + nl, qq);
      }
    }
  }
}

template <int BM, int BN, int BK, int WM, int WN, int NS, bool FLIP, bool STATS>
__global__ void __launch_bounds__(64 * WM * WN) conv_halo_kernel(ConvArgs a, HaloGeom hg) {
  constexpr int NW = WM * WN;
  constexpr int CPR = BK / 8, RPI = 64 / CPR;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int B_ROWS = 9 * BN, B_INS = B_ROWS / RPI, B_PW = (B_INS + NW - 1) / NW;
  static_assert(B_ROWS % RPI == 0, "weight tile rows");
  extern __shared__ __attribute__((aligned(16))) u16 lds_h[];
  const int A_EL = hg.A_INS * RPI * BK;
  const int STAGE = A_EL + B_ROWS * BK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int MV = hg.MV;
  const long long m0 = (long long)blockIdx.x * MV;
  const int n0 = blockIdx.y * BN;
  const int H = a.GH, W = a.GW, C = a.CI, TH = hg.TH, HW2 = hg.W2;
  const int img = H * W;
  // (32-bit: M * C < 2^31 by the host checks; a 64-bit division is ~100 instructions)
  const int b0 = (int)m0 / img, h0 = ((int)m0 - b0 * img) / W;
  const int per_img = hg.PI;
  // in-tile index math by float reciprocal (small_divmod): the integer
  // division sequences were ~2/3 of the ~500-VALU per-block prologue
  const float rcp_pi = 1.f / (float)per_img, rcp_w2 = 1.f / (float)HW2;
  const float rcp_tw = 1.f / (float)(TH * W), rcp_w = 1.f / (float)W;

  // Halo-image chunk swizzle.  A 16-pixel fragment on an image of width W <= 8
  // spans 16 / W image rows whose staged rows are W2 = W + 2 apart, not 16
  // consecutive rows: the row-bit swizzle of swz<32> then maps half of each
  // ds_read_b128 lane group onto the other half's slots (2 LDS cycles per read
  // on the 8 x 8 and 4 x 4 ResNet-18 stages, 40 % bank-conflict cycles measured
  // by PMC).  There the XOR key is the parity of the staged image row (row / W2)
  // instead -- conflict-free for every fragment and tap of those tiles (checked
  // exhaustively over the lane groups of gfx950's b128 reads); W >= 16 keeps
  // swz<32>.  qrow = row / W2 of the staged row.
  //
  // A fragment that wraps an image row at any other width (ImageNet 56 / 28 / 14 /
  // 7) skips the 2 halo columns, which unbalances the staged rows' 64-B quarters
  // of a lane group -- no chunk XOR can fix that (24-40 % conflict cycles,
  // profiles/lds_conflict_census_r5.txt).  There (hg.PSW) the host stages rows
  // W2 = W + 4 wide with (-2W) mod 4 pad rows per image, so every staged row is
  // congruent mod 4 to its pixel-like index pidx = (tb * TH + hx) * W + c, which
  // runs consecutively along every fragment and tap; keyed on pidx, swz<32> then
  // sees 16 consecutive rows.
  const bool qsw = BK == 32 && W <= 8 && 16 % W == 0;
  const bool psw = BK == 32 && hg.PSW;
  auto hswz = [&](int row, int qrow, int c, int pidx) {
    return psw ? swz<BK>(pidx, c) : qsw ? c ^ ((qrow & 1) << 1) : swz<BK>(row, c);
  };
  // halo DMA slots: lane's row of each 1-KiB piece -> (image, h, w) of the
  // source pixel; positions outside the image (or past the batch) read zeros
  unsigned a_base[kHaloAPW];
#pragma unroll
  for (int j = 0; j < kHaloAPW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    int tb, rem, hh, ww;
    small_divmod(row, per_img, rcp_pi, tb, rem);
    small_divmod(rem, HW2, rcp_w2, hh, ww);
    const int b = b0 + tb, h = h0 - 1 + hh, w = ww - 1;
    const bool ok = ins < hg.A_INS && row < hg.HROWS && b < a.B && hh < TH + 2 &&
                    (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    a_base[j] = ok ? 2u * (unsigned)(((b * H + h) * W + w) * C +
                                     hswz(row, tb * (TH + 2) + hh, lane % CPR,
                                          (tb * TH + hh) * W + ww) * 8)
                   : kOOB;
  }
  // weight DMA slots: row = tap * BN + output channel
  unsigned b_base[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    const int t = row / BN, co = row - t * BN;
    const bool ok = ins < B_INS && n0 + co < a.CO;
    b_base[j] = ok ? 2u * (unsigned)(((n0 + co) * 9 + t) * C + swz<BK>(row, lane % CPR) * 8) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * a.B * H * W * C), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, 0, (int)(2LL * a.CO * 9 * C), 0x00020000);

  auto stage = [&](int buf, int c) {
    u16* As = lds_h + buf * STAGE;
    u16* Bs = As + A_EL;
    const unsigned cd = 2u * (unsigned)(c * BK);
#pragma unroll
    for (int j = 0; j < kHaloAPW; ++j) {
      const int ins = wid + j * NW;
      if (ins < hg.A_INS)
        bdma16(rsA, a_base[j] == kOOB ? kOOB : a_base[j] + cd, As + ins * (RPI * BK));
    }
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int ins = wid + j * NW;
      if (B_INS % NW == 0 || ins < B_INS)
        bdma16(rsB, b_base[j] == kOOB ? kOOB : b_base[j] + cd, Bs + ins * (RPI * BK));
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS element offset of each A fragment read, per (fragment, tap), computed
  // once (k-step 0; BK = 32 has one): the staged row of the lane's output pixel
  // at tap (0, 0) plus the tap's row / column shift, swizzled (hswz)
  static_assert(BK == 32, "conv_halo_kernel: one 32-deep k-step per tap");
  int aoff[TM][9];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int ml = wm * (BM / WM) + i * 16 + (lane & 15);
    if (ml >= MV) ml = 0;   // padded tile: a valid staged row, the epilogue drops it
    int tb, r2, th, tw;
    small_divmod(ml, TH * W, rcp_tw, tb, r2);
    small_divmod(r2, W, rcp_w, th, tw);
    const int q0 = tb * (TH + 2) + th, hrow = tb * per_img + th * HW2 + tw;
    const int p0 = (tb * TH + th) * W + tw;   // pixel-like index of tap (0, 0)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int row = hrow + (t / 3) * HW2 + t % 3;
      aoff[i][t] = row * BK + hswz(row, q0 + t / 3, lane >> 4, p0 + (t / 3) * W + t % 3) * 8;
    }
  }
  int offB[BK / 32];
  {
    const int rb = wn * (BN / WN) + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) offB[ks] = rb * BK + swz<BK>(rb, ks * 4 + (lane >> 4)) * 8;
  }
  // (tap, k-step) steps with the fragments double-buffered in registers: the
  // reads of step st+1 are issued ahead of step st's MFMAs, so each step's LDS
  // latency hides behind the previous step's TM*TN MFMAs (reading each step's
  // operands just before its MFMAs left ~3 exposed lgkmcnt waits per tap)
  auto compute = [&](int buf) {
    const u16* As = lds_h + buf * STAGE;
    const u16* Bs = As + A_EL;
    constexpr int KS = BK / 32, NSTEP = 9 * KS;
    bf16x8 af[2][TM], bw[2][TN];
    auto load = [&](int st, int slot) {
      if (DMP_ABLATE == 4 && st >= 2) return;
      const int t = st / KS, ks = st % KS;
      const int wt = FLIP ? 8 - t : t;
#pragma unroll
      for (int i = 0; i < TM; ++i) af[slot][i] = *reinterpret_cast<const bf16x8*>(As + aoff[i][t]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + wt * BN * BK + offB[ks] + j * 16 * BK);
    };
    load(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);   // step 0's reads first
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      if (st + 1 < NSTEP) load(st + 1, (st + 1) & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bw[st & 1][j], af[st & 1][i], acc[i][j]);
      // pin the schedule: step st+1's reads interleaved one per MFMA of step st
      // (the scheduler otherwise sinks each read next to its first use)
      if (st + 1 < NSTEP) {
#pragma unroll
        for (int k = 0; k < TM + TN && k < TM * TN; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if (TM * TN > TM + TN) __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - (TM + TN), 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
      }
    }
  };

  // 8-wave tiles: waves 4-7 at priority 1 (s4 fwd / dgrad -1.8 / -2.1 %,
  // profiles/prio_young_half_r5.txt)
  if (NW == 8) prio_young_half(wid);
  const int KC = C / BK;
  if constexpr (NS == 2) {
    stage(0, 0);
    for (int c = 0; c < KC; ++c) {
      wait_vm<0>();                       // chunk c landed (this wave's DMAs) ...
      __builtin_amdgcn_s_barrier();       // ... for every wave; chunk c-1's slot is free
      asm volatile("" ::: "memory");
      if (c + 1 < KC && DMP_ABLATE != 2) stage((c + 1) & 1, c + 1);
      if (DMP_ABLATE != 1) compute(DMP_ABLATE == 2 ? 0 : c & 1);
    }
  } else {
    // one stage: half the LDS, so two or three blocks share a CU and one
    // block's load / epilogue overlaps another's MFMA work
    for (int c = 0; c < KC; ++c) {
      if (c > 0) __syncthreads();         // everyone done reading chunk c-1
      if (c == 0 || DMP_ABLATE != 2) stage(0, c);
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (DMP_ABLATE != 1) compute(0);
    }
  }
  __syncthreads();   // all stage reads done before the epilogue reuses LDS
  if constexpr (DMP_ABLATE == 3) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // the data gradient stores through the row-staged epilogue (-5..-9 % on the
  // 128 / 256-channel layers, no change on the forward, whose BN sums cost
  // more in the row layout: profiles/conv_roofline_r4.txt)
  if constexpr ((DMP_HALO_EPI_LDS || FLIP) && !(FLIP && STATS))
    halo_epilogue_rows<BM, BN, WM, WN, FLIP, STATS, TM, TN>(a, acc, m0, n0, wm, wn, tid, lane, lds_h,
                                                            MV);
  else
    halo_epilogue<BM, BN, WM, WN, FLIP, STATS>(a, acc, m0, n0, wm, wn, tid, lane, lds_h, 0, MV);
}

// ------------------------------- 3x3 stride-2 data gradient, halo tiles
// dX of a 3x3 / stride-2 / pad-1 conv splits into the parity classes (h % 2,
// w % 2) of dX (top of this file).  Class (ph, pw) is a small STRIDE-1 conv over
// dY: dX[2i+ph][2j+pw] = sum dY[i+u][j+v] Wt[r][s] with r = 1 (ph = 0) or r in
// {2 at u = 0, 0 at u = 1} (ph = 1), s likewise: every tap (r, s) belongs to
// exactly one class.  conv_igemm_kernel runs the classes as implicit GEMMs that
// gather dY once per tap (330-460 TF/s, profiles/conv_layers_bs512_r2.txt).
// Here a block stages its dY tile ONCE per 32-channel chunk with a one-row /
// one-column halo below / right (zeros past the image) plus all nine weight
// taps, and runs the nine taps out of LDS into FOUR accumulator sets, one per
// class -- the fill per MFMA of the stride-1 halo kernel.  (A tile per class
// measured no faster than the implicit GEMM: classes of 1 and 2 taps re-stage
// the same dY tile for a few MFMAs.)  A block's BM pixels are whole rows (or
// whole images) of the class grid = the dY grid for even H, W; halo_epilogue<S2>
// scatters each class's tile to its dX pixels.  Wave tile TM x 16 pixels x
// TN x 16 channels per class (4 x TM x TN accumulators).
template <int BM, int BN, int WM, int WN, int NS>
__global__ void __launch_bounds__(64 * WM * WN) conv_dgrad_s2_kernel(ConvArgs a, HaloGeom hg) {
  constexpr int NW = WM * WN, BK = 32, CPR = BK / 8, RPI = 64 / CPR;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int B_ROWS = 9 * BN, B_INS = B_ROWS / RPI, B_PW = (B_INS + NW - 1) / NW;
  static_assert(B_ROWS % RPI == 0, "weight tile rows");
  extern __shared__ __attribute__((aligned(16))) u16 lds_h[];
  const int A_EL = hg.A_INS * RPI * BK;
  const int STAGE = A_EL + B_ROWS * BK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int H = a.GH, W = a.GW, C = a.CI, TH = hg.TH, W1 = W + 1;
  const int img = H * W;
  const int b0 = (int)m0 / img, h0 = ((int)m0 - b0 * img) / W;
  const int per_img = (TH + 1) * W1;
  const float rcp_pi = 1.f / (float)per_img, rcp_w1 = 1.f / (float)W1;
  const float rcp_tw = 1.f / (float)(TH * W), rcp_w = 1.f / (float)W;

  // dY tile + halo: staged row (tb, hh, jj) = dY[b0 + tb][h0 + hh][jj], hh <= TH,
  // jj <= W; the bottom / right halo past the image reads zeros
  unsigned a_base[kHaloAPW];
#pragma unroll
  for (int j = 0; j < kHaloAPW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    int tb, rem, hh, jj;
    small_divmod(row, per_img, rcp_pi, tb, rem);
    small_divmod(rem, W1, rcp_w1, hh, jj);
    const int b = b0 + tb, h = h0 + hh;
    const bool ok = ins < hg.A_INS && row < hg.HROWS && b < a.B && h < H && jj < W;
    a_base[j] = ok ? 2u * (unsigned)(((b * H + h) * W + jj) * C + swz<BK>(row, lane % CPR) * 8)
                   : kOOB;
  }
  // weight rows: t * BN + n <- Wt[n0 + n][t][chunk]   (t = r * 3 + s)
  unsigned b_base[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / CPR;
    const int t = row / BN, n = row - t * BN;
    const bool ok = ins < B_INS && n0 + n < a.CO;
    b_base[j] = ok ? 2u * (unsigned)(((n0 + n) * 9 + t) * C + swz<BK>(row, lane % CPR) * 8) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * a.B * H * W * C), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, 0, (int)(2LL * a.CO * 9 * C), 0x00020000);
  auto stage = [&](int buf, int c) {
    u16* As = lds_h + buf * STAGE;
    u16* Bs = As + A_EL;
    const unsigned cd = 2u * (unsigned)(c * BK);
#pragma unroll
    for (int j = 0; j < kHaloAPW; ++j) {
      const int ins = wid + j * NW;
      if (ins < hg.A_INS) bdma16(rsA, a_base[j] == kOOB ? kOOB : a_base[j] + cd, As + ins * (RPI * BK));
    }
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int ins = wid + j * NW;
      if (B_INS % NW == 0 || ins < B_INS)
        bdma16(rsB, b_base[j] == kOOB ? kOOB : b_base[j] + cd, Bs + ins * (RPI * BK));
    }
  };

  f32x4 acc[4][TM][TN];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int hrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wm * (BM / WM) + i * 16 + (lane & 15);
    int tb, r2, th, tw;
    small_divmod(ml, TH * W, rcp_tw, tb, r2);
    small_divmod(r2, W, rcp_w, th, tw);
    hrow[i] = (tb * (TH + 1) + th) * W1 + tw;
  }
  int offB;
  {
    const int rb = wn * (BN / WN) + (lane & 15);
    offB = rb * BK + swz<BK>(rb, lane >> 4) * 8;
  }
  // tap t = (r, s): class (r != 1, s != 1), dY offset (r == 0, s == 0)
  auto compute = [&](int buf) {
    const u16* As = lds_h + buf * STAGE;
    const u16* Bs = As + A_EL;
    bf16x8 af[2][TM], bw[2][TN];
    auto load = [&](int t, int slot) {
      const int r = t / 3, sc = t % 3;
      const int rowoff = (r == 0 ? W1 : 0) + (sc == 0 ? 1 : 0);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = hrow[i] + rowoff;
        af[slot][i] = *reinterpret_cast<const bf16x8*>(As + row * BK + swz<BK>(row, lane >> 4) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + t * BN * BK + offB + j * 16 * BK);
    };
    load(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int q = (t / 3 != 1 ? 2 : 0) + (t % 3 != 1 ? 1 : 0);
      if (t + 1 < 9) load(t + 1, (t + 1) & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[q][i][j] = mfma16(bw[t & 1][j], af[t & 1][i], acc[q][i][j]);
      if (t + 1 < 9) {
#pragma unroll
        for (int k = 0; k < TM + TN && k < TM * TN; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if (TM * TN > TM + TN) __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - (TM + TN), 0);
        if (TM * TN < TM + TN) __builtin_amdgcn_sched_group_barrier(0x100, TM + TN - TM * TN, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
      }
    }
  };
  const int KC = C / BK;
  if constexpr (NS == 2) {
    // two stages: chunk c+1's DMA in flight under chunk c's MFMAs (an 8-wave
    // block holds the CU's register file alone, so no second block hides the fill)
    stage(0, 0);
    for (int c = 0; c < KC; ++c) {
      wait_vm<0>();                       // chunk c landed (this wave's DMAs) ...
      __builtin_amdgcn_s_barrier();       // ... for every wave; chunk c-1's slot is free
      asm volatile("" ::: "memory");
      if (c + 1 < KC) stage((c + 1) & 1, c + 1);
      compute(c & 1);
    }
  } else {
    // one stage (several blocks per CU overlap each other's fill and MFMAs)
    for (int c = 0; c < KC; ++c) {
      if (c > 0) __syncthreads();         // everyone done reading chunk c-1
      stage(0, c);
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      compute(0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q)
    halo_epilogue<BM, BN, WM, WN, true, false, TM, TN, true>(a, acc[q], m0, n0, wm, wn, tid, lane,
                                                             lds_h, q);
}

// ------------------------------------ persistent 3x3 halo tiles, 64 channels
// The 64-channel layers (ResNet-18 CIFAR stage 1: 32x32 x 64 -> 64) run the
// halo kernel above with only C/32 = 2 chunks per block, and every block
// re-stages all nine 64x32 weight taps per chunk: 72 KB of weights DMA'd per
// 256 output pixels beside 43 KB of halo input.  These kernels are bound by the
// global->LDS fill rate (~10-15 B/clk/CU, profiles/conv_kernels_r2.txt), so
// here the whole 9 x 64 x 64 weight tensor stays RESIDENT in LDS (72 KB,
// fetched once per block) and a persistent block streams BM-pixel halo tiles
// with all 64 input channels (128-B rows) through an NS-deep LDS-DMA ring:
// the fill traffic per pixel drops ~2.7x.  4 waves, wave = 64 pixels x 64
// output channels (TM = BM / 64 fragments of 16 pixels, TN = 4).
// Per tile the epilogue of the PREVIOUS tile runs after the next stage's DMA
// is issued, so its stores drain under this tile's MFMAs; the ring wait then
// counts only DMA pieces (vmcnt <= (NS-2) * APW also covers those stores,
// whatever order loads and stores retire in).  BN partial sums accumulate in
// registers over all of a block's tiles (one slot reduction per block).
// FLIP = stride-1 data gradient (dY, Wt, mirrored taps); no residual addend
// (the host routes addend dgrads to conv_halo_kernel).
struct HaloPGeom {
  int TH, TB, HROWS, APW, AINS, ntiles;   // APW: pieces per wave (>= AINS / NW), AINS: exact
  // DIAGNOSTIC (DMP_HALO64P_XFORM=1, forward only): the cost of applying a
  // per-channel BatchNorm scale / shift + clamp to the staged input tile in LDS
  // ("apply-in-consumer"): every wave rewrites its own landed halo pieces,
  // x -> max(x * xs + xh, xlo), before the tile's barrier.  Run with the
  // identity (xs 1, xh 0, xlo -inf: outputs unchanged, the work is not
  // foldable: runtime values) to price the transform against the BN apply
  // pass it would replace (profiles/bn_consumer_fusion_r3.txt).
  int xform;
  float xs, xh, xlo;
  // 8-wave blocks: waves 4-7 (the SIMD partners of waves 0-3) run each tile as
  // compute(k) -> epilogue(k) instead of epilogue(k-1) -> compute(k), so one
  // wave's epilogue VALU and stores overlap its partner's MFMAs instead of both
  // waves of a SIMD storing at once after the tile barrier (MI355X_MICROARCH.md,
  // "Two waves per SIMD" item 9: split roles by wave number >= 4)
  int stagger;
};

constexpr int kHpAPW = 12;   // max halo DMA pieces per wave per tile
// 8-wave blocks need at most 8 (BM 256 on 32 x 32 / 64 x 64 maps: 6 / 7): the
// smaller bound frees 8 VGPRs of slot offsets in the register-capped kernel
constexpr int hp_apw_max(int nw) { return nw == 8 ? 8 : kHpAPW; }

__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
#define DMP_WV(k) \
  case k:         \
    wait_vm<k>(); \
    break;
    DMP_WV(1) DMP_WV(2) DMP_WV(3) DMP_WV(4) DMP_WV(5) DMP_WV(6) DMP_WV(7) DMP_WV(8) DMP_WV(9)
    DMP_WV(10) DMP_WV(11) DMP_WV(12) DMP_WV(13) DMP_WV(14) DMP_WV(15) DMP_WV(16) DMP_WV(17)
    DMP_WV(18) DMP_WV(19) DMP_WV(20) DMP_WV(21) DMP_WV(22) DMP_WV(23) DMP_WV(24)
#undef DMP_WV
    default:
      wait_vm<0>();
  }
}

template <int BM, int NS, int NW, bool FLIP, bool STATS>
__global__ void __launch_bounds__(64 * NW) conv_halo64p_kernel(ConvArgs a, HaloPGeom hg) {
  constexpr int BK = 64, BN = 64, RPI = 8;
  constexpr int TM = BM / NW / 16, TN = BN / 16, KS = BK / 32, NSTEP = 9 * KS;
  constexpr int W_EL = 9 * BN * BK;
  constexpr int APWMAX = hp_apw_max(NW);
  extern __shared__ __attribute__((aligned(16))) u16 lds_p[];
  const int APW = hg.APW;
  // NS = 2 drains the ring every tile (vmcnt(0)), so waves may issue unequal
  // piece counts and the stage holds exactly AINS pieces; deeper rings count
  // pieces per wave and pad every wave to APW
  const int STAGE = (NS == 2 ? hg.AINS : APW * NW) * RPI * BK;
  u16* Ws = lds_p;
  u16* Hs = lds_p + W_EL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.y * BN;
  const int H = a.GH, W = a.GW, C = a.CI, TH = hg.TH, W2 = W + 2;
  const int img = H * W;
  const int P = a.B * img;
  const int G = gridDim.x, ntiles = hg.ntiles;
  const int nt = (ntiles - (int)blockIdx.x + G - 1) / G;
  if (nt <= 0) return;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, 0, (int)(2LL * P * C), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, 0, (int)(2LL * a.CO * 9 * C), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.y, 0, (int)(2LL * P * a.CO), 0x00020000);

  // resident weights: row = tap * 64 + output channel, 72 pieces (18 per wave)
#pragma unroll
  for (int j = 0; j < 9 * BN / RPI / NW; ++j) {
    const int ins = wid + j * NW;
    const int row = ins * RPI + lane / 8;
    const int t = row / BN, co = row - t * BN;
    const bool ok = n0 + co < a.CO;
    bdma16(rsB, ok ? 2u * (unsigned)(((n0 + co) * 9 + t) * C + swz<BK>(row, lane % 8) * 8) : kOOB,
           Ws + ins * (RPI * BK));
  }
  // halo DMA slots: staged row -> element offset from the tile's first pixel +
  // {valid, image in tile, source row - h0}
  int x_off[APWMAX];
  unsigned x_inf[APWMAX];
  const int per_img = (TH + 2) * W2;
#pragma unroll
  for (int j = 0; j < APWMAX; ++j) {
    x_off[j] = 0;
    x_inf[j] = 0;
    if (j < APW) {
      const int row = (wid + j * NW) * RPI + lane / 8;
      const int tb = row / per_img, rem = row - tb * per_img;
      const int hh = rem / W2, w = rem - hh * W2 - 1, dh = hh - 1;
      const bool ok = row < hg.HROWS && tb < hg.TB && (unsigned)w < (unsigned)W;
      x_off[j] = (tb * img + dh * W + w) * C + swz<BK>(row, lane % 8) * 8;
      x_inf[j] = (ok ? 0x80000000u : 0u) | ((unsigned)tb << 16) | ((unsigned)(dh + 64) << 8);
    }
  }
  auto tile_of = [&](int k) { return (int)blockIdx.x + k * G; };
  auto stage = [&](int buf, int k) {
    u16* As = Hs + buf * STAGE;
    const int t = tile_of(k);
    const bool live = k < nt;
    const int m0 = t * BM;
    const int b0 = m0 / img, h0 = (m0 - b0 * img) / W;
#pragma unroll
    for (int j = 0; j < APWMAX; ++j) {
      if (j < APW && (NS != 2 || wid + j * NW < hg.AINS)) {
        const unsigned inf = x_inf[j];
        const int tb = (int)((inf >> 16) & 0x7fff), dh = (int)((inf >> 8) & 255) - 64;
        const bool ok = live && (inf >> 31) && b0 + tb < a.B && (unsigned)(h0 + dh) < (unsigned)H;
        bdma16(rsA, ok ? 2u * (unsigned)(m0 * C + x_off[j]) : kOOB, As + (wid + j * NW) * 512);
      }
    }
  };

  // per-lane LDS element offsets of every A fragment read at k-step 0, one per
  // (fragment, tap): tile-invariant, computed ONCE.  (Recomputing row -> swizzled
  // address per read was ~1.5 VALU per MFMA of this VALU-issue-heavy kernel:
  // profiles/pmc_r5.txt.)  k-step 1 is the same offset with 16-B chunk bit 2
  // flipped: (4 + g) ^ t == 4 ^ (g ^ t) for the BK = 64 swizzle, i.e. element ^ 32.
  int aoff[TM][9];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wid * (BM / NW) + i * 16 + (lane & 15);
    const int tb = ml / (TH * W), r2 = ml - tb * TH * W;
    const int th = r2 / W, tw = r2 - th * W;
    const int hrow = (tb * (TH + 2) + th) * W2 + tw;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int row = hrow + (t / 3) * W2 + (t % 3);
      aoff[i][t] = row * BK + swz<BK>(row, lane >> 4) * 8;
    }
  }
  const int rb = lane & 15;
  f32x4 acc[TM][TN];
  auto compute = [&](int buf, f32x4 (&dst)[TM][TN]) {
    const u16* As = Hs + buf * STAGE;
    // fragments prefetched PD steps ahead (PD = 2 when a step has <= 8 MFMAs:
    // one step's MFMAs alone do not cover an LDS read round trip at 1 wave/SIMD)
    constexpr int PD = (TM * TN <= 8 && NW == 4) ? 2 : 1, NB = PD + 1;
    bf16x8 af[NB][TM], bw[NB][TN];
    static_assert(BK == 64 && KS == 2, "tap table: k-step 1 = element offset ^ 32");
    auto load = [&](int st, int slot) {
      if (DMP_ABLATE == 4 && st >= PD) return;
      const int t = st / KS, ks = st % KS;
      const int wt = FLIP ? 8 - t : t;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[slot][i] = *reinterpret_cast<const bf16x8*>(As + (ks ? aoff[i][t] ^ 32 : aoff[i][t]));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[slot][j] = *reinterpret_cast<const bf16x8*>(
            Ws + (wt * BN + j * 16 + rb) * BK + swz<BK>(rb, ks * 4 + (lane >> 4)) * 8);
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load(p, p);
    __builtin_amdgcn_sched_group_barrier(0x100, PD * (TM + TN), 0);
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      if (st + PD < NSTEP) load(st + PD, (st + PD) % NB);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          dst[i][j] = mfma16(bw[st % NB][j], af[st % NB][i], dst[i][j]);
      if (st + PD < NSTEP) {
#pragma unroll
        for (int k = 0; k < TM + TN && k < TM * TN; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if (TM * TN > TM + TN) __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - (TM + TN), 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
      }
    }
  };

  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  // conv bias: forward without BN statistics only (the eval-mode BN fold);
  // the training forward (STATS) feeds a BatchNorm and has none -- the
  // launcher routes a biased STATS conv elsewhere -- which frees 16 VGPRs of
  // this register-capped kernel for the tap address table below
  constexpr bool HAS_BIAS = !FLIP && !STATS;
  float bj[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + j * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bj[j][r] = (HAS_BIAS && a.bias != nullptr && n + r < a.CO) ? a.bias[n + r] : 0.f;
  }
  float s_sum[TN][4], s_sq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s_sum[j][r] = 0.f; s_sq[j][r] = 0.f; }
  // residual-gradient addend of the data gradient (FLIP): its rows of tile k are
  // loaded (inline asm, counted by hand) BEFORE the next tile's DMA is issued,
  // so the deferred epilogue waits only for them, never for that DMA
  typedef unsigned int u32x2_a __attribute__((ext_vector_type(2)));
  // (the statistics forward feeds a BatchNorm: no addend / ReLU, compiled out)
  constexpr bool PLAIN = STATS && !FLIP;
  const bool add_in = a.addend != nullptr;   // dgrad residual grad / fwd BN-fold residual
  const __amdgpu_buffer_rsrc_t rsAdd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_in ? a.addend : a.y), 0, (int)(2LL * P * a.CO), 0x00020000);
  u32x2_a ad[TM][TN];
  // deferred ReLU mask of the addend (ConvArgs::addmask): the 64 bits of the
  // block's 64 channels of pixel m, one dwordx2 per fragment row i
  const bool add_mask = add_in && a.addmask != nullptr;
  const __amdgpu_buffer_rsrc_t rsAm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(add_mask ? (const void*)a.addmask : (const void*)a.y), 0, (int)((long long)P * a.CO / 8),
      0x00020000);
  u32x2_a am[TM];
  auto aload = [&](int k) {
    const int m0 = tile_of(k) * BM;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wid * (BM / NW) + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 16 + 4 * (lane >> 4);
        const unsigned off = (m < P && n < a.CO) ? 2u * (unsigned)(m * a.CO + n) : kOOB;
        asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(ad[i][j]) : "v"(off), "s"(rsAdd)
                     : "memory");
      }
      if (add_mask) {   // counted with the addend loads (issued before the next DMA)
        const unsigned moff = m < P ? (unsigned)((m * a.CO + n0) >> 3) : kOOB;
        asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(am[i]) : "v"(moff), "s"(rsAm)
                     : "memory");
      } else {
        am[i] = u32x2_a{0xffffffffu, 0xffffffffu};
      }
    }
  };
  // this wave's DMA pieces per stage (issued after the addend loads)
  int dma_pw = 0;
#pragma unroll
  for (int j = 0; j < APWMAX; ++j)
    if (j < APW && (NS != 2 || wid + j * NW < hg.AINS)) ++dma_pw;
  // the store of one 16 x 16 fragment (i, j) of tile k from accumulators `src`
  auto epi_one = [&](int k, f32x4 (&src)[TM][TN], int i, int j) {
    const int m0 = tile_of(k) * BM;
    const int m = m0 + wid * (BM / NW) + i * 16 + (lane & 15);
    const bool mok = m < P;
    const unsigned rowoff = 2u * (unsigned)(m * a.CO);
    const int n = n0 + j * 16 + 4 * (lane >> 4);
    const bool ok = mok && n < a.CO;
    float av[4] = {0.f, 0.f, 0.f, 0.f};
    if (add_in) {
      av[0] = __uint_as_float(ad[i][j].x << 16);
      av[1] = __uint_as_float(ad[i][j].x & 0xffff0000u);
      av[2] = __uint_as_float(ad[i][j].y << 16);
      av[3] = __uint_as_float(ad[i][j].y & 0xffff0000u);
      // mask bits of channels n..n+3: bit (n - n0) of the pixel's 64-bit word
      const int nb = j * 16 + 4 * (lane >> 4);
      const unsigned bits = (nb < 32 ? am[i].x >> nb : am[i].y >> (nb - 32)) & 0xfu;
#pragma unroll
      for (int r = 0; r < 4; ++r) av[r] = (bits >> r) & 1u ? av[r] : 0.f;
    }
    u16 hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t = src[i][j][r] + (HAS_BIAS ? bj[j][r] : 0.f) + av[r];
      if (!FLIP && !PLAIN && a.relu) t = fmaxf(t, 0.f);
      hv[r] = f2bf(t);
      if (STATS) {
        const float v = ok ? bf2f(hv[r]) : 0.f;
        s_sum[j][r] += v;
        s_sq[j][r] += v * v;
      }
    }
    const u32x2_t packed = {(u32)hv[0] | ((u32)hv[1] << 16), (u32)hv[2] | ((u32)hv[3] << 16)};
    __builtin_amdgcn_raw_buffer_store_b64(packed, rsY, ok ? rowoff + 2u * n : kOOB, 0, DMP_CONV_STORE_AUX);
  };
  // addend rows of the tile being stored have landed (they were issued BEFORE
  // the next stage's DMA: wait until only those dma_pw pieces may be in flight)
  auto addend_wait = [&](bool last) {
    if (add_in) {
      if (last) wait_vm<0>();
      else wait_vm_n(dma_pw);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(ad[i][j]));
        asm volatile("" : "+v"(am[i]));
      }
    }
  };
  auto epilogue = [&](int k, bool last) {
    addend_wait(last);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) epi_one(k, acc, i, j);
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage(s, s);
  const int vm_wait = (NS - 2) * APW;
  // diagnostic transform of this wave's own landed pieces of tile k (see HaloPGeom)
  auto xform_tile = [&](int k) {
    u16* As = Hs + (k % NS) * STAGE;
    const int t = tile_of(k);
    const int m0 = t * BM;
    const int b0 = m0 / img, h0 = (m0 - b0 * img) / W;
#pragma unroll
    for (int j = 0; j < APWMAX; ++j) {
      if (j < APW && (NS != 2 || wid + j * NW < hg.AINS)) {
        const unsigned inf = x_inf[j];
        const int tb = (int)((inf >> 16) & 0x7fff), dh = (int)((inf >> 8) & 255) - 64;
        const bool ok = (inf >> 31) && b0 + tb < a.B && (unsigned)(h0 + dh) < (unsigned)H;
        if (ok) {   // halo / padding positions stay exactly zero
          bf16x8* q = reinterpret_cast<bf16x8*>(As + (wid + j * NW) * 512 + lane * 8);
          bf16x8 v = *q;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v.v[e] = f2bf(fmaxf(__fmaf_rn(bf2f(v.v[e]), hg.xs, hg.xh), hg.xlo));
          *q = v;
        }
      }
    }
  };
  // waves 4-7 of an 8-wave block: each tile's own stores right after its MFMAs
  const bool late = NS == 2 && NW == 8 && DMP_ABLATE == 0 && hg.stagger && !add_in &&
                    !hg.xform && wid >= 4;
  // (no static priority for waves 4-7 here: s1 dgrad +3 %, fwd +0.4 %,
  // profiles/prio_young_half_r5.txt -- the stagger already orders the halves)
  if (late) {
    for (int k = 0; k < nt; ++k) {
      // tile k landed; the TM*TN youngest ops (tile k-1's stores, issued after
      // tile k's DMA) may still be in flight (vmcnt retires in issue order)
      if (k >= 1) wait_vm<TM * TN>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      stage((k + 1) % 2, k + 1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      compute(k % 2, acc);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) epi_one(k, acc, i, j);
    }
  } else {
    for (int k = 0; k < nt; ++k) {
      if (NS == 2) wait_vm<0>();
      else wait_vm_n(vm_wait);            // tile k (and, at k = 0, the weights) landed ...
      if (!FLIP && hg.xform) xform_tile(k);
      __builtin_amdgcn_s_barrier();       // ... for every wave; slot (k-1) % NS is free
      asm volatile("" ::: "memory");
      if (k > 0 && add_in) aload(k - 1);
      if (DMP_ABLATE != 2) stage((k + NS - 1) % NS, k + NS - 1);
      if (DMP_ABLATE == 3) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
      } else if (k > 0) {
        epilogue(k - 1, false);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (DMP_ABLATE != 1) compute(DMP_ABLATE == 2 ? 0 : k % NS, acc);
    }
    if (add_in) aload(nt - 1);
    if (DMP_ABLATE != 3) epilogue(nt - 1, true);
  }
  if (STATS) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s_sum[j][r] = row_sum16(s_sum[j][r]);
        s_sq[j][r] = row_sum16(s_sq[j][r]);
      }
    wait_vm<0>();                        // the ring's trailing (zero) DMAs have landed
    __syncthreads();
    float* red = reinterpret_cast<float*>(Hs);   // [NW][BN] sums, then [NW][BN] squares
    if ((lane & 15) == 15) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = j * 16 + 4 * (lane >> 4) + r;
          red[wid * BN + nl] = s_sum[j][r];
          red[NW * BN + wid * BN + nl] = s_sq[j][r];
        }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.CO) {
      float ss = 0.f, qq = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) { ss += red[w * BN + tid]; qq += red[NW * BN + w * BN + tid]; }
      const int slot = blockIdx.x % kBnSlots;
      atomicAdd(a.part + (long long)slot * a.CO + n0 + tid, ss);
      atomicAdd(a.part + (long long)(kBnSlots + slot) * a.CO + n0 + tid, qq);
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
// Tile configurations (BM, BN, BK, WM, WN, NS).  Index = the `cfg` id used by
// the host-side tuner; -1 selects the heuristic default.
#define DMP_CONV_CONFIGS(X)      \
  X(0, 256, 64, 64, 4, 1, 2)     \
  X(1, 256, 64, 32, 4, 2, 2)     \
  X(2, 128, 64, 64, 2, 2, 2)     \
  X(3, 128, 64, 32, 2, 2, 2)     \
  X(4, 64, 64, 64, 2, 2, 2)      \
  X(5, 64, 64, 32, 2, 2, 2)      \
  X(6, 256, 128, 64, 2, 2, 2)    \
  X(7, 256, 128, 32, 4, 2, 2)    \
  X(8, 128, 128, 64, 2, 2, 2)    \
  X(9, 128, 128, 32, 2, 4, 2)    \
  X(10, 64, 128, 64, 1, 4, 2)    \
  X(11, 128, 64, 32, 4, 2, 2)    \
  X(12, 256, 64, 64, 4, 2, 2)    \
  X(13, 128, 128, 64, 2, 4, 2)   \
  X(14, 256, 64, 32, 4, 2, 4)    \
  X(15, 256, 64, 64, 4, 2, 3)    \
  X(16, 128, 128, 32, 2, 4, 4)   \
  X(17, 128, 128, 64, 2, 4, 3)   \
  X(18, 64, 64, 64, 2, 2, 4)     \
  X(19, 128, 64, 32, 2, 2, 4)    \
  X(20, 64, 128, 64, 1, 4, 3)    \
  X(21, 128, 64, 64, 2, 2, 3)    \
  X(22, 64, 64, 32, 2, 2, 4)     \
  X(23, 128, 128, 32, 2, 2, 4)
// 24-27: tiles with the row-staged epilogue (conv_igemm_kernel<ROWS>): forward,
// and stride-1 data gradients without the fused BN backward; otherwise they run
// the plain epilogue of the same geometry
#define DMP_CONV_CONFIGS_ROWS(X) \
  X(24, 128, 128, 32, 2, 4, 2)   \
  X(25, 128, 128, 64, 2, 4, 2)   \
  X(26, 256, 128, 32, 4, 2, 2)   \
  X(27, 128, 64, 32, 2, 2, 4)

constexpr int kNumConvConfigs = 28;

static int config_bm(int cfg) {
  switch (cfg) {
#define X(id, BM, BN, BK, WM, WN, NS) case id: return BM;
    DMP_CONV_CONFIGS(X)
    DMP_CONV_CONFIGS_ROWS(X)
#undef X
  }
  return 128;
}

int conv_num_configs() { return kNumConvConfigs; }

void conv_config_info(int cfg, int* info) {
  switch (cfg) {
#define X(id, BM, BN, BK, WM, WN, NS) \
  case id: info[0] = BM; info[1] = BN; info[2] = BK; info[3] = 64 * WM * WN; info[4] = NS; return;
    DMP_CONV_CONFIGS(X)
    DMP_CONV_CONFIGS_ROWS(X)
#undef X
  }
  info[0] = info[1] = info[2] = info[3] = info[4] = 0;
}

// heuristic default: widest N tile the channels fill, tallest M tile that
// still yields >= ~2 blocks per CU.
int conv_default_config(long long M, int CO) {
  if (CO >= 128) {
    const long long nb = CO / 128;
    if ((M + 255) / 256 * nb >= 512) return 7;
    if ((M + 127) / 128 * nb >= 256) return 9;
    return 10;
  }
  if ((M + 255) / 256 >= 512) return 1;
  if ((M + 127) / 128 >= 256) return 11;
  return 5;
}

template <int BM, int BN, int BK, int WM, int WN, int NS, int MODE, bool STATS, bool ROWS = false>
static void launch_cfg(const ConvArgs& a, int classes, hipStream_t s) {
  const dim3 grid((unsigned)((a.M + BM - 1) / BM), (unsigned)((a.CO + BN - 1) / BN),
                  (unsigned)classes);
  // row-staged epilogue: forward, or a stride-1 data gradient without the fused BN
  // backward (one parity class, output row = dX pixel); otherwise the plain tile
  constexpr bool R = ROWS && (MODE == 0 || !STATS);
  // (the row epilogue of a statistics forward has no bias / ReLU / addend: PLAIN)
  const bool plain_ok = !(MODE == 0 && STATS) || (a.bias == nullptr && !a.relu && a.addend == nullptr);
  if (R && plain_ok && (MODE == 0 || (a.stride == 1 && !a.addend_sub)))
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, WM, WN, MODE, STATS, NS, R>), grid,
                       dim3(64 * WM * WN), 0, s, a);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, WM, WN, MODE, STATS, NS, false>), grid,
                       dim3(64 * WM * WN), 0, s, a);
}

template <int MODE, bool STATS>
static void dispatch(const ConvArgs& a, int cfg, int classes, hipStream_t s) {
  switch (cfg) {
#define X(id, BM, BN, BK, WM, WN, NS) \
  case id: launch_cfg<BM, BN, BK, WM, WN, NS, MODE, STATS>(a, classes, s); return;
    DMP_CONV_CONFIGS(X)
#undef X
#define X(id, BM, BN, BK, WM, WN, NS) \
  case id: launch_cfg<BM, BN, BK, WM, WN, NS, MODE, STATS, true>(a, classes, s); return;
    DMP_CONV_CONFIGS_ROWS(X)
#undef X
  }
}

// Halo-tile configurations (BM, BN, BK, WM, WN), cfg ids kHaloBase + i; only for
// 3x3 / stride 1 / pad 1 and block tiles of whole rows or whole images.
#define DMP_HALO_CONFIGS(X)   \
  X(0, 256, 64, 32, 4, 2, 2)  \
  X(1, 128, 64, 32, 2, 2, 2)  \
  X(2, 64, 64, 32, 2, 2, 2)   \
  X(3, 128, 64, 32, 4, 2, 2)  \
  X(4, 256, 64, 32, 2, 2, 2)  \
  X(5, 128, 64, 32, 2, 2, 1)  \
  X(6, 256, 64, 32, 4, 2, 1)  \
  X(7, 64, 64, 32, 2, 2, 1)   \
  X(8, 128, 64, 32, 4, 2, 1)   \
  X(9, 256, 64, 32, 4, 1, 1)   \
  X(10, 256, 64, 32, 4, 1, 2)  \
  X(11, 128, 64, 32, 2, 1, 1)  \
  X(12, 128, 128, 32, 2, 2, 1) \
  X(13, 256, 128, 32, 4, 2, 1) \
  X(14, 512, 64, 32, 8, 1, 1)  \
  X(18, 224, 64, 32, 2, 2, 1)  \
  X(19, 224, 64, 32, 2, 1, 1)  \
  X(20, 112, 64, 32, 1, 2, 1)  \
  X(21, 112, 128, 32, 1, 4, 1) \
  X(22, 112, 128, 32, 1, 2, 1) \
  X(23, 448, 64, 32, 4, 2, 1)  \
  X(24, 224, 64, 32, 2, 2, 2)  \
  X(25, 112, 128, 32, 1, 4, 2)
// 18-25: whole-row tiles of 7 x 16 pixels for the ImageNet ResNet widths (56-
// and 28-pixel rows: 4 / 2 / 8 rows of 56, 4 rows of 28), where none of the
// power-of-two tiles above is a whole number of rows.  Ids 15-17 are the
// persistent kernels below (kept: ids are cached by the tuner).

constexpr int kHaloBase = 100, kNumHaloConfigs = 26;   // ids kHaloBase + [0, 26)
// persistent 64-channel halo kernels (conv_halo64p_kernel): ids 115-117
constexpr int kHaloPBase = kHaloBase + 15, kNumHaloPConfigs = 3;
__host__ __device__ constexpr bool is_halop(int cfg) {
  return cfg >= kHaloPBase && cfg < kHaloPBase + kNumHaloPConfigs;
}

static bool halo_cfg(int cfg, int* bm, int* bn, int* bk, int* nw, int* ns) {
  switch (cfg - kHaloBase) {
#define X(i, BM, BN, BK, WM, WN, NS) \
  case i: *bm = BM; *bn = BN; *bk = BK; *nw = WM * WN; *ns = NS; return true;
    DMP_HALO_CONFIGS(X)
#undef X
  }
  return false;
}

// geometry of a halo config on a (B, H, W, C) input; false when it does not apply
static bool halo_geom(int cfg, int H, int W, int C, int R, int S, int stride, int pad,
                      HaloGeom* g, size_t* lds) {
  int bm, bn, bk, nw, ns;
  if (!halo_cfg(cfg, &bm, &bn, &bk, &nw, &ns)) return false;
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || C % bk != 0) return false;
  const int img = H * W;
  HaloGeom h{};
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
    // padded whole-image tiles: at most 1/8 of the tile's rows idle
    if (bm % img != 0) {
      h.MV = h.TB * img;
      if (8 * (bm - h.MV) > bm) return false;
    }
  }
  const int rpi = 64 / (bk / 8);
  // fragments wrapping image rows (W not a multiple of 16, not the <= 8 widths the
  // row-parity key covers): the W + 4-wide staging of conv_halo_kernel (PSW)
  static const bool psw_on = [] {
    const char* e = std::getenv("DMP_HALO_PSW");
    return e == nullptr || e[0] != '0';
  }();
  h.PSW = psw_on && bk == 32 && W % 16 != 0 && !(W <= 8 && 16 % W == 0);
  h.W2 = h.PSW ? W + 4 : W + 2;
  h.PI = (h.TH + 2) * h.W2;
  if (h.PSW) h.PI += (((h.TH * W - h.PI) % 4) + 4) % 4;   // PI == TH * W (mod 4)
  h.HROWS = h.TB * h.PI;
  h.A_INS = (h.HROWS + rpi - 1) / rpi;
  if (h.A_INS > kHaloAPW * nw) return false;
  const size_t stage = (size_t)h.A_INS * rpi * bk + (size_t)9 * bn * bk;
  size_t bytes = (size_t)ns * stage * 2;
  if (bytes < (size_t)bm * (bn + 8) * 2) bytes = (size_t)bm * (bn + 8) * 2;   // row epilogue tile
  if (bytes > 160 * 1024) return false;
  *g = h;
  *lds = bytes;
  return true;
}

// persistent 64-channel halo ids kHaloPBase + i -> (BM, NS, waves)
static const int kHaloP[3][3] = {{256, 2, 4}, {128, 3, 4}, {256, 2, 8}};

static bool halop_geom(int cfg, int B, int H, int W, int C, int R, int S, int stride, int pad,
                       HaloPGeom* g, int* bm_out, int* ns_out, int* nw_out, size_t* lds) {
  const int id = cfg - kHaloPBase;
  if (id < 0 || id >= kNumHaloPConfigs) return false;
  const int bm = kHaloP[id][0], ns = kHaloP[id][1], nw = kHaloP[id][2];
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || C != 64) return false;
  const int img = H * W;
  HaloPGeom h{};
  if (bm <= img) {
    if (bm % W != 0 || img % bm != 0) return false;
    h.TH = bm / W;
    h.TB = 1;
  } else {
    if (bm % img != 0) return false;
    h.TH = H;
    h.TB = bm / img;
  }
  h.HROWS = h.TB * (h.TH + 2) * (W + 2);
  h.AINS = (h.HROWS + 7) / 8;
  h.APW = (h.AINS + nw - 1) / nw;
  if (h.APW > hp_apw_max(nw) || (ns - 2) * h.APW > 24) return false;
  const long long P = (long long)B * img;
  if (2LL * P * 64 >= (1LL << 31)) return false;
  h.ntiles = (int)((P + bm - 1) / bm);
  const size_t pieces = ns == 2 ? (size_t)h.AINS : (size_t)h.APW * nw;
  const size_t bytes = 2 * ((size_t)9 * 64 * 64 + (size_t)ns * pieces * 8 * 64);
  if (bytes > 160 * 1024) return false;
  *g = h;
  *bm_out = bm;
  *ns_out = ns;
  *nw_out = nw;
  *lds = bytes;
  return true;
}

bool conv_halo_ok(int cfg, int H, int W, int C, int R, int S, int stride, int pad) {
  if (is_halop(cfg)) {
    HaloPGeom g;
    int bm, ns, nw;
    size_t lds;
    return halop_geom(cfg, 1, H, W, C, R, S, stride, pad, &g, &bm, &ns, &nw, &lds);
  }
  HaloGeom g;
  size_t lds;
  return halo_geom(cfg, H, W, C, R, S, stride, pad, &g, &lds);
}

int conv_num_halo_configs() { return kNumHaloConfigs; }
int conv_halo_base() { return kHaloBase; }

template <int BM, int BN, int BK, int WM, int WN, int NS, bool FLIP, bool STATS>
static void launch_halo_t(const ConvArgs& a, const HaloGeom& g, size_t lds, hipStream_t s) {
  auto kern = conv_halo_kernel<BM, BN, BK, WM, WN, NS, FLIP, STATS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const long long M = (long long)a.B * a.OH * a.OW;
  const dim3 grid((unsigned)((M + g.MV - 1) / g.MV), (unsigned)((a.CO + BN - 1) / BN));
  hipLaunchKernelGGL(kern, grid, dim3(64 * WM * WN), lds, s, a, g);
}

template <int BM, int NS, int NW, bool FLIP, bool STATS>
static void launch_halop_t(const ConvArgs& a, const HaloPGeom& g, size_t lds, hipStream_t s) {
  auto kern = conv_halo64p_kernel<BM, NS, NW, FLIP, STATS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  // persistent: one block per CU (the resident weights + ring fill the LDS)
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ny = (a.CO + 63) / 64;
  int gx = (cus + ny - 1) / ny;
  if (gx > g.ntiles) gx = g.ntiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)gx, (unsigned)ny), dim3(64 * NW), lds, s, a, g);
}

// true if launched (cfg is a halo config that applies to this geometry)
template <bool FLIP, bool STATS>
static bool launch_halo(const ConvArgs& a, int cfg, hipStream_t s) {
  HaloGeom g;
  size_t lds;
  if (a.GH != a.OH || a.GW != a.OW) return false;
  if (is_halop(cfg)) {
    HaloPGeom pg;
    int bm, ns, nw;
    size_t plds;
    // the BN-backward epilogue is not fused in the persistent kernel (its
    // deferred epilogue runs with the next tile's DMA in flight): take the 4-wave
    // halo tile for those dgrads instead (a residual addend is fused: loaded ahead
    // of the DMA, see conv_halo64p_kernel)
    // the persistent kernel's statistics forward carries no conv bias (HAS_BIAS)
    // (a statistics forward takes no bias / ReLU / addend in these kernels: PLAIN)
    if (!FLIP && STATS && (a.bias != nullptr || a.relu || a.addend != nullptr)) return false;
    if (FLIP && (STATS || (a.addend != nullptr && a.addend_sub)))
      return launch_halo<FLIP, STATS>(a, kHaloBase + 9, s) ||
             launch_halo<FLIP, STATS>(a, kHaloBase + 5, s);
    if (!halop_geom(cfg, a.B, a.GH, a.GW, a.CI, a.R, a.S, a.stride, a.pad, &pg, &bm, &ns, &nw,
                    &plds))
      return false;
    static const int xform_env = [] {
      const char* e = getenv("DMP_HALO64P_XFORM");
      return e && e[0] == '1' ? 1 : 0;
    }();
    pg.xform = xform_env;
    static const int stagger_env = [] {
      // on by default: ResNet-18 bs512 3.500 -> 3.486 ms/step, 3 interleaved
      // rounds (profiles/halo64p_stagger_ab_r5.txt); DMP_HALO64P_STAGGER=0 for A/B
      const char* e = getenv("DMP_HALO64P_STAGGER");
      return e && e[0] == '0' ? 0 : 1;
    }();
    pg.stagger = stagger_env;
    pg.xs = 1.f;
    pg.xh = 0.f;
    pg.xlo = -INFINITY;
    if constexpr (!(FLIP && STATS)) {
      if (nw == 8) launch_halop_t<256, 2, 8, FLIP, STATS>(a, pg, plds, s);
      else if (bm == 256) launch_halop_t<256, 2, 4, FLIP, STATS>(a, pg, plds, s);
      else launch_halop_t<128, 3, 4, FLIP, STATS>(a, pg, plds, s);
    }
    return true;
  }
  if (!halo_geom(cfg, a.GH, a.GW, a.CI, a.R, a.S, a.stride, a.pad, &g, &lds)) return false;
  // the statistics forward's epilogue has no bias / ReLU / addend (PLAIN in
  // halo_epilogue): such a conv takes the implicit GEMM instead
  if (!FLIP && STATS && (a.bias != nullptr || a.relu || a.addend != nullptr)) return false;
  switch (cfg - kHaloBase) {
#define X(i, BM, BN, BK, WM, WN, NS) \
  case i: launch_halo_t<BM, BN, BK, WM, WN, NS, FLIP, STATS>(a, g, lds, s); return true;
    DMP_HALO_CONFIGS(X)
#undef X
  }
  return false;
}

// stride-2 halo data-gradient tiles (conv_dgrad_s2_kernel): id, BM, BN, WM, WN
constexpr int kS2Base = 200;
// (wave tiles of 32 pixels x 64 channels or 64 x 32 per class: 4 classes x 8
// accumulator tiles = 128 registers)
#define DMP_S2_CONFIGS(X)      \
  X(0, 128, 64, 4, 1, 1)       \
  X(1, 256, 64, 8, 1, 1)       \
  X(2, 128, 128, 4, 2, 1)      \
  X(3, 256, 32, 4, 1, 1)       \
  X(4, 64, 64, 2, 1, 1)        \
  X(5, 112, 64, 7, 1, 1)       \
  X(6, 256, 64, 8, 1, 2)       \
  X(7, 128, 128, 4, 2, 2)      \
  X(8, 128, 64, 8, 1, 2)       \
  X(9, 112, 64, 7, 1, 2)
constexpr int kNumS2Configs = 10;
static bool s2_cfg(int cfg, int* bm, int* bn, int* nw, int* ns) {
  switch (cfg - kS2Base) {
#define X(i, BM, BN, WM, WN, NS) \
  case i: *bm = BM; *bn = BN; *nw = WM * WN; *ns = NS; return true;
    DMP_S2_CONFIGS(X)
#undef X
  }
  return false;
}
// geometry of a stride-2 halo dgrad config: dY (OH x OW, K channels) -> dX (H x W, N channels)
static bool s2_geom(int cfg, int H, int W, int OH, int OW, int K, int N, int R, int S, int stride,
                    int pad, HaloGeom* g, size_t* lds) {
  int bm, bn, nw, ns;
  if (!s2_cfg(cfg, &bm, &bn, &nw, &ns)) return false;
  if (R != 3 || S != 3 || stride != 2 || pad != 1 || H != 2 * OH || W != 2 * OW) return false;
  if (K % 32 != 0 || N % bn != 0) return false;
  const int img = OH * OW;
  HaloGeom h{};
  h.MV = bm;
  if (bm <= img) {
    if (bm % OW != 0 || img % bm != 0) return false;
    h.TH = bm / OW;
    h.TB = 1;
  } else {
    if (bm % img != 0) return false;
    h.TH = OH;
    h.TB = bm / img;
  }
  h.HROWS = h.TB * (h.TH + 1) * (OW + 1);
  h.A_INS = (h.HROWS + 15) / 16;
  if (h.A_INS > kHaloAPW * nw) return false;
  const size_t bytes = (size_t)ns * 2 * ((size_t)h.A_INS * 512 + (size_t)9 * bn * 32);
  if (bytes > 160 * 1024) return false;
  *g = h;
  *lds = bytes;
  return true;
}
bool conv_dgrad_s2_ok(int cfg, int H, int W, int OH, int OW, int K, int N, int R, int S, int stride,
                      int pad) {
  HaloGeom g;
  size_t lds;
  return s2_geom(cfg, H, W, OH, OW, K, N, R, S, stride, pad, &g, &lds);
}
int conv_dgrad_s2_base() { return kS2Base; }
int conv_dgrad_s2_num_configs() { return kNumS2Configs; }

template <int BM, int BN, int WM, int WN, int NS>
static void launch_s2_t(const ConvArgs& a, const HaloGeom& g, size_t lds, hipStream_t s) {
  auto kern = conv_dgrad_s2_kernel<BM, BN, WM, WN, NS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const long long M = (long long)a.B * a.GH * a.GW;   // class-grid pixels (= dY pixels)
  const dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)(a.CO / BN));
  hipLaunchKernelGGL(kern, grid, dim3(64 * WM * WN), lds, s, a, g);
}

int conv_fwd_num_mblocks(long long M, int CO, int cfg) {
  {
    int bm, bn, bk, nw, ns;
    if (halo_cfg(cfg, &bm, &bn, &bk, &nw, &ns)) return (int)((M + bm - 1) / bm);
  }
  if (cfg < 0 || cfg >= kNumConvConfigs) cfg = conv_default_config(M, CO);
  const int bm = config_bm(cfg);
  return (int)((M + bm - 1) / bm);
}

void launch_conv_fwd(const u16* x, const u16* w, u16* y, float* part, int B, int H, int W,
                     int CI, int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                     hipStream_t s, const float* bias, bool relu, const u16* addend) {
  // addend: a [B][OH][OW][CO] residual added before the ReLU (the inference-time
  // BatchNorm fold: BN(conv) + shortcut, ReLU = conv with folded weights + bias
  // + addend, ReLU -- ops/eval_fold.py)
  ConvArgs a{x, w, y, part, B, H, W, CI, OH, OW, CO, R, S, stride, pad,
             (long long)B * OH * OW, bias, addend, relu ? 1 : 0};
  if (cfg >= kHaloBase) {
    if (part ? launch_halo<false, true>(a, cfg, s) : launch_halo<false, false>(a, cfg, s)) return;
    cfg = -1;   // not applicable to this geometry: heuristic implicit-GEMM tile
  }
  if (cfg < 0 || cfg >= kNumConvConfigs) cfg = conv_default_config(a.M, CO);
  if (part) dispatch<0, true>(a, cfg, 1, s);
  else dispatch<0, false>(a, cfg, 1, s);
}

// dX (B,H,W,CI) from dY (B,OH,OW,CO) and Wt [CI][R][S][CO]; stride*stride parity classes.
void launch_conv_dgrad(const u16* dy, const u16* wt, u16* dx, int B, int H, int W, int CI,
                       int OH, int OW, int CO, int R, int S, int stride, int pad, int cfg,
                       hipStream_t s, const u16* addend, const BnBwdFuse* bnf,
                       bool addend_sub, const uint8_t* addend_mask) {
  const long long rows = (long long)B * ((H + stride - 1) / stride) * ((W + stride - 1) / stride);
  ConvArgs a{dy, wt, dx, nullptr, B, OH, OW, CO, H, W, CI, R, S, stride, pad, rows, nullptr,
             addend};
  a.addend_sub = addend_sub ? 1 : 0;
  a.addmask = addend ? addend_mask : nullptr;
  if (bnf) {
    a.part = bnf->part;
    a.bnx = bnf->x;
    a.bnmask = bnf->mask;
    a.bnstat = bnf->stats;
    a.bnrelu = bnf->relu;
  }
  if (cfg >= kS2Base && cfg < kS2Base + kNumS2Configs) {
    HaloGeom g;
    size_t lds;
    if (!bnf && s2_geom(cfg, H, W, OH, OW, CO, CI, R, S, stride, pad, &g, &lds)) {
      switch (cfg - kS2Base) {
#define X(i, BM, BN, WM, WN, NS) \
  case i: launch_s2_t<BM, BN, WM, WN, NS>(a, g, lds, s); return;
        DMP_S2_CONFIGS(X)
#undef X
      }
    }
    cfg = -1;   // not applicable: heuristic implicit-GEMM tile
  }
  if (cfg >= kHaloBase) {
    // stride 1, 3x3, pad 1: dX = the same conv over dY with Wt and mirrored taps
    if (bnf ? launch_halo<true, true>(a, cfg, s) : launch_halo<true, false>(a, cfg, s)) return;
    cfg = -1;
  }
  if (cfg < 0 || cfg >= kNumConvConfigs) cfg = conv_default_config(rows * stride * stride, CI);
  if (bnf) dispatch<1, true>(a, cfg, stride * stride, s);
  else dispatch<1, false>(a, cfg, stride * stride, s);
}

// x_sub[b][i][j][c] = x[b][2i][2j][c] (NHWC bf16, C % 8 == 0): the input of a
// 1x1 / stride-2 shortcut, gathered once so the shortcut runs as a stride-1 GEMM
__global__ void __launch_bounds__(256) subsample2_kernel(const u16* __restrict__ x,
                                                         u16* __restrict__ xs, int H, int W,
                                                         int C, int OH, int OW, long long nvec) {
  const int cv = C / 8;
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += step) {
    const int c8 = (int)(v % cv);
    const long long pix = v / cv;
    const int j = (int)(pix % OW);
    const long long t = pix / OW;
    const int i = (int)(t % OH);
    const long long b = t / OH;
    const long long src = ((b * H + 2 * i) * W + 2 * j) * C + c8 * 8;
    *reinterpret_cast<bf16x8*>(xs + v * 8) = *reinterpret_cast<const bf16x8*>(x + src);
  }
}

// dx[b][2i][2j][c] += xs[b][i][j][c] in place: the gradient of a subsampled alias
// added back onto a full-resolution data gradient (bf16, fp32 add, one rounding)
__global__ void __launch_bounds__(256) add_subsampled2_kernel(u16* __restrict__ dx,
                                                              const u16* __restrict__ xs, int H,
                                                              int W, int C, int OH, int OW,
                                                              long long nvec) {
  const int cv = C / 8;
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += step) {
    const int c8 = (int)(v % cv);
    const long long pix = v / cv;
    const int j = (int)(pix % OW);
    const long long t = pix / OW;
    const int i = (int)(t % OH);
    const long long b = t / OH;
    u16* d = dx + ((b * H + 2 * i) * W + 2 * j) * C + c8 * 8;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(d);
    const bf16x8 e = *reinterpret_cast<const bf16x8*>(xs + v * 8);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = f2bf(bf2f(a.v[k]) + bf2f(e.v[k]));
    *reinterpret_cast<bf16x8*>(d) = o;
  }
}

void launch_add_subsampled2(u16* dx, const u16* xs, int B, int H, int W, int C, hipStream_t s) {
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long long nvec = (long long)B * OH * OW * (C / 8);
  hipLaunchKernelGGL(add_subsampled2_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, dx,
                     xs, H, W, C, OH, OW, nvec);
}

void launch_subsample2(const u16* x, u16* xs, int B, int H, int W, int C, hipStream_t s) {
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long long nvec = (long long)B * OH * OW * (C / 8);
  hipLaunchKernelGGL(subsample2_kernel, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, x, xs, H,
                     W, C, OH, OW, nvec);
}

void launch_conv_weight_transpose(const u16* w, u16* wt, int CO, int RS, int CI, hipStream_t s) {
  const long long total = (long long)CO * RS * CI;
  hipLaunchKernelGGL(conv_weight_transpose_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s,
                     w, wt, CO, RS, CI);
}


}  // namespace dmp

namespace dmp {
// All conv weights of a model transposed in ONE launch: table[i] = {offset,
// CO, RS, CI} of weight i inside the flat bf16 shadow; W[co][rs][ci] at
// src+offset -> Wt[ci][rs][co] at dst+offset.  blockIdx.y = weight index.
// Every (rs) slice is a CO x CI matrix transposed through LDS in 64 x 64
// tiles: 128-B coalesced row reads and row writes (CO, CI multiples of 64 --
// the only weights the native dgrad consumes).
__global__ void __launch_bounds__(256) conv_weight_transpose_batched_kernel(
    const u16* __restrict__ src, u16* __restrict__ dst, const long long* __restrict__ table) {
  __shared__ u16 tile[64][66];
  const long long* t = table + 4 * blockIdx.y;
  const long long off = t[0];
  const int CO = (int)t[1], RS = (int)t[2], CI = (int)t[3];
  const int tco = CO / 64, tci = CI / 64;
  const int ntiles = RS * tco * tci;
  const u16* w = src + off;
  u16* wt = dst + off;
  const int tid = threadIdx.x, r = tid >> 2, c = (tid & 3) * 16;
  for (int tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int rs = tt / (tco * tci), rem = tt - rs * tco * tci;
    const int co0 = (rem / tci) * 64, ci0 = (rem % tci) * 64;
    // read row co0+r, columns ci0+c .. +15
    const uint4* g = reinterpret_cast<const uint4*>(w + ((long long)(co0 + r) * RS + rs) * CI + ci0 + c);
    const uint4 v0 = g[0], v1 = g[1];
    const u16* e0 = reinterpret_cast<const u16*>(&v0);
    const u16* e1 = reinterpret_cast<const u16*>(&v1);
#pragma unroll
    for (int k = 0; k < 8; ++k) { tile[r][c + k] = e0[k]; tile[r][c + 8 + k] = e1[k]; }
    __syncthreads();
    // write row ci0+r of Wt[.][rs][.], columns co0+c .. +15
    uint4 o0, o1;
    u16* f0 = reinterpret_cast<u16*>(&o0);
    u16* f1 = reinterpret_cast<u16*>(&o1);
#pragma unroll
    for (int k = 0; k < 8; ++k) { f0[k] = tile[c + k][r]; f1[k] = tile[c + 8 + k][r]; }
    uint4* d = reinterpret_cast<uint4*>(wt + ((long long)(ci0 + r) * RS + rs) * CO + co0 + c);
    d[0] = o0;
    d[1] = o1;
    __syncthreads();
  }
}

void launch_conv_weight_transpose_batched(const u16* src, u16* dst, const long long* table, int n,
                                          long long max_elems, hipStream_t s) {
  if (n <= 0) return;
  long long tiles = max_elems / 4096;
  int gx = (int)(tiles < 1 ? 1 : (tiles > 1024 ? 1024 : tiles));
  hipLaunchKernelGGL(conv_weight_transpose_batched_kernel, dim3(gx, n), dim3(256), 0, s, src, dst,
                     table);
}
}  // namespace dmp
