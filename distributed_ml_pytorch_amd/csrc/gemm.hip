// Dense bf16 GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_bf16) for the Linear
// layers (SURVEY §2.3 `addmm` / `mm` rows; the reference's nn.Linear heads,
// /root/reference/example/models.py:11-13,43, and the ViT-B/16 projections):
//
//   C[m][n] (+)= epilogue( sum_k A(m, k) * B(n, k) )
//
// A(m, k) = A[m*lda + k] (AT = false: k contiguous) or A[k*lda + m] (AT = true),
// B likewise.  The three passes of a linear layer Y = X W^T + b are:
//   fwd   Y  = X W^T        AT=0 BT=0   epilogue: + bias [, + addend] or GELU
//   dgrad dX = dY W          AT=0 BT=1   epilogue: plain, or * GELU'(h) (fused
//                                        GELU backward of the layer before)
//   wgrad dW += dY^T X       AT=1 BT=1   fp32 accumulate into the grad arena,
//                                        bias grad = row sums of dY^T (one extra
//                                        MFMA against an all-ones operand)
//
// Staging: every 64-deep k-tile of both operands is fetched by LDS DMA
// (buffer_load_dwordx4 ... lds: 16 B per lane, no VGPR round trip) into an
// NS-deep ring; one counted `s_waitcnt vmcnt` + one raw s_barrier per k-tile
// (NS-1 tiles in flight).  A k-contiguous operand lands as a [rows][64] image
// (128-B rows, 16-B chunk XOR swizzle applied on the SOURCE address) read with
// ds_read_b128; a k-strided operand lands as a [64][rows] image (32-B granule
// XOR swizzle) read with the gfx950 transposing ds_read_b64_tr_b16, which hands
// each lane 4 consecutive k of one column -- two such reads are exactly one
// MFMA operand fragment, in the same k order as the b128 fragment of the other
// operand, so mixed layouts multiply correctly.  Tails (M, N, K not multiples of
// the tile) read zeros through out-of-range buffer offsets and drop their
// stores the same way: no per-element branches.
//
// Workgroup -> tile map is XCD-aware: consecutive tiles along N of one M panel
// land on the same XCD (shared L2) under round-robin dispatch -- a speed
// choice only, any placement is correct.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace dmp {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr unsigned kOOBg = 0x80000000u;

// EPI_DRELU (data gradient): out = aux > 0 ? acc : 0 with aux = the layer's own
// forward INPUT -- the output of a ReLU (or of a dropout after one), so the
// data gradient leaves already multiplied by that ReLU's derivative and the
// producing layer skips its separate mask pass (ops/linear.py)
enum { EPI_STORE = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_ACC32 = 3, EPI_DRELU = 4 };

// epilogues that may read an aux [M][N] operand (register slots reserved)
constexpr bool has_aux_slots(int epi) {
  return epi == EPI_STORE || epi == EPI_DGELU || epi == EPI_DRELU;
}

struct GemmArgs {
  const u16* a;
  const u16* b;
  void* c;            // bf16 [M][ldc] (EPI 0-2) or fp32 [M][ldc] (EPI_ACC32)
  u16* c2;            // EPI_GELU: gelu(h) [M][ldc]  (h itself goes to c)
  const u16* bias;    // EPI_STORE / EPI_GELU: bf16 [N] (optional)
  const u16* aux;     // EPI_STORE: bf16 addend [M][ldc] (optional); EPI_DGELU: h [M][ldc]
  const uint8_t* auxmask;   // EPI_STORE: optional 1-bit mask of the addend (bit e of byte
                            // (m * ldc + n) / 8 keeps element (m, n + e); ldc == N): the
                            // residual gradient's deferred ReLU mask (ops/functional.py)
  float* dbias;       // EPI_ACC32: fp32 [M] += sum_k A(m, k) (optional)
  int M, N, K;
  int lda, ldb, ldc;
  int k_chunk;        // reduction rows per blockIdx.y (split-K), multiple of BK
  int tiles_n;
  int relu;           // EPI_STORE: max(0, .) after bias / addend (linear -> ReLU)
  float* part;        // EPI_STORE: optional BatchNorm slot sums [2][kBnSlots][N] of the
                      // stored bf16 outputs (a 1x1 conv feeding a BatchNorm)
  float* slab;        // EPI_ACC32 split-K: per-split fp32 partials [splits][M][N] written
                      // with plain stores, summed into C by gemm_slab_reduce_kernel
  // remainder split-K of the bf16-output passes (fwd / dgrad): blocks
  // [0, sk_full) own whole tiles; the T - sk_full tiles of the last, partial
  // round are cut into sk_split k-pieces of sk_kchunk reduction rows, one block
  // each (launched last, so the short pieces fill the final round).  Every piece
  // publishes its fp32 accumulators to sk_ws; the last to arrive (ticket in
  // sk_cnt[tile], zeroed per call) adds the others and runs the epilogue.
  int sk_full, sk_split, sk_kchunk;
  float* sk_ws;
  int* sk_cnt;
  // EPI_ACC32 split-K: deal (split, tile) pairs to the XCDs split-major, so one
  // XCD's blocks share a k-range (and so the operand panels its L2 holds)
  int xcd_k;
};

// Diagnostic build only (-DDMP_GEMM_STAMPS, scripts/gemm_stamps.cpp): per-block
// s_memrealtime stamps (100 MHz, one clock for every XCD) at kernel entry, after
// the prologue's first k-tile landed, after the k-loop and after the epilogue.  No
// stamp instruction exists in the extension build.
// cache policy of the bf16 output stores (buffer instruction aux bits): 2 = nt
// (streaming).  Measured with the stamped diagnostic build: -2 % on the QKV forward,
// -5.5 % on a 4096^2 K = 1024 forward, -1..2 % at K = 3072; sc1 (16) is slower
// (profiles/gemm_store_policy_r6.txt)
#ifndef DMP_GEMM_STORE_AUX
#define DMP_GEMM_STORE_AUX 2
#endif
#ifdef DMP_GEMM_STAMPS
__device__ unsigned long long g_gemm_stamps[1 << 16][4];
#define DMP_STAMP(i)                                                                  \
  do {                                                                                \
    if (threadIdx.x == 0) {                                                           \
      const unsigned b = blockIdx.x + blockIdx.y * gridDim.x;                         \
      if (b < (1u << 16)) g_gemm_stamps[b][i] = __builtin_amdgcn_s_memrealtime();     \
    }                                                                                 \
  } while (0)
#else
#define DMP_STAMP(i) do {} while (0)
#endif

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// LDS DMA from inline asm (the builtin makes hipcc wait vmcnt(0) before the
// next ds_read of ANY ring slot, serialising the pipeline); completion counted
// by hand with wait_vm.
__device__ __forceinline__ void gdma16(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                       u16* lds_wave_base) {
  const unsigned m0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave_base;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "{m0}"(m0));
}

template <int N>
__device__ __forceinline__ void gwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}

// [rows][BK] image, 16-B chunk c of row r holds logical chunk rswz(r, c) (an
// involution): each ds_read_b128 lane group (16 rows, one chunk) hits 16
// distinct slots.  BK = 64 (128-B rows, 2 per bank row): c ^= (r>>1)&7;
// BK = 32 (64-B rows, 4 per bank row): c ^= (-(r>>2))&3.  Rows 16 apart share
// the XOR.
template <int BK>
__device__ __forceinline__ int rswz(int row, int c) {
  if constexpr (BK == 64) return c ^ ((row >> 1) & 7);
  else return c ^ ((-(row >> 2)) & 3);
}

// [64][R] image (R >= 128 bf16 = whole bank rows): 32-B granule u of row r
// holds logical granule u ^ tf(r).  One half-wave tr read touches rows
// {8g + q : g = 0,1, q = 0..3} of one granule column; tf gives those 8 rows
// 8 distinct granules of the 256-B bank row -> conflict-free.
__device__ __forceinline__ int tf(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }
template <int R>
__device__ __forceinline__ int toff(int row, int col) {
  return row * R + (((col >> 4) ^ tf(row)) << 4) + (col & 15);
}

// One operand's per-lane DMA slots: PW 1-KiB wave-instructions per k-tile
// (waves wid < INS % NW issue one more when NW does not divide INS).  The
// per-lane byte offsets are computed once per block (recomputing them per
// stage cost ~12 VALU per DMA and measured 15-25 % slower on the wgrad tiles).
// 32-bit offsets; out-of-range pieces read zeros (kOOBg).
template <int R, bool T, int NW, int BK>
struct Stager {
  static constexpr int EL = R * BK;
  static constexpr int INS = EL / 512;
  static constexpr int PW = (INS + NW - 1) / NW;
  static constexpr int PW_MIN = INS / NW;
  static_assert(EL % 512 == 0, "whole 1-KiB DMA pieces");
  static_assert(!T || R % 128 == 0, "transposed image rows must be whole 256-B bank rows");
  unsigned off[PW];   // byte offset of the piece at k = kbase (kOOBg: row/col out of range)
  int kk[PW];         // k of the piece relative to the k-tile start

  // r0: tile origin along the operand's rows
  __device__ __forceinline__ void init(int wid, int lane, int r0, int rows, int ld, int kbase) {
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = ((wid + j * NW) % INS) * 512 + lane * 8;
      if constexpr (!T) {
        const int row = e / BK;
        const int kc = rswz<BK>(row, (e % BK) / 8) * 8;
        kk[j] = kc;
        off[j] = r0 + row < rows ? 2u * (unsigned)((r0 + row) * ld + kbase + kc) : kOOBg;
      } else {
        const int row = e / R, pch = (e % R) / 8;
        const int col = (((pch >> 1) ^ tf(row)) << 4) + (pch & 1) * 8;
        kk[j] = row;
        off[j] = r0 + col < rows ? 2u * (unsigned)((kbase + row) * ld + r0 + col) : kOOBg;
      }
    }
  }
  // k0: k-tile start relative to kbase; kend: valid k count relative to kbase
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, u16* img, int wid, int k0,
                                        int kend, int ld) {
    const unsigned delta = T ? 2u * (unsigned)(k0 * ld) : 2u * (unsigned)k0;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      if (j < PW_MIN || wid + j * NW < INS) {
        const bool ok = off[j] != kOOBg && k0 + kk[j] < kend;
        gdma16(rs, ok ? off[j] + delta : kOOBg, img + (wid + j * NW) * 512);
      }
    }
  }
};

// fragment of 16 rows/cols starting at `r` for k-step ks: row image via one
// ds_read_b128, transposed image via two ds_read_b64_tr_b16
template <int R, bool T, int BK>
__device__ __forceinline__ bf16x8 frag(const u16* img, int r, int ks, int lane) {
  if constexpr (!T) {
    const int row = r + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(img + row * BK + rswz<BK>(row, ks * 4 + (lane >> 4)) * 8);
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int row = ks * 32 + 8 * g + q;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + toff<R>(row, r + 4 * p)));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4_t*)(img + toff<R>(row + 4, r + 4 * p)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// One output tile per block (a persistent variant whose DMA ring ran across
// tile boundaries measured no faster on the ViT shapes and 15-70 % slower on
// the wgrad tiles: profiles/gemm_vs_hipblaslt_r2.txt).
//
// KG = 2 (weight gradients only): two groups of WM x WN waves share the block's
// output tile and split every staged 2*BK-deep k-tile between them (group g
// takes k-rows g*BK .. g*BK + BK - 1 of the [2*BK][rows] images); at the end
// group 1 parks its fp32 accumulators in the drained ring and group 0 adds them
// before the single flush.  One 8-wave block per CU then does the work of two
// 4-wave blocks with HALF the split-K partials through the fp32 atomics / slab
// (the ViT weight gradients spend ~25-30 % of their time there).
//
// PP = true: "ping-pong" k-loop for 8-wave tiles (WM = 2): the two wave rows run
// one barrier apart, so on every SIMD (waves w and w + 4) one wave issues its
// fragment reads and LDS DMA while the other runs its MFMA cluster.  Per k-tile
// (BK = 32, a 4-deep ring) and wave: [ds_read k-tile t | DMA k-tile t+3 | vmcnt:
// k-tile t+1 landed | lgkmcnt(0)] barrier [setprio 1, MFMAs, setprio 0] barrier.
// Row 0's read section of k-tile t lies between global barriers 2t-1 and 2t, row
// 1's between 2t and 2t+1 (it enters the loop one barrier late), so:
//   * k-tile t+1's DMAs were waited by every wave before barrier 2t+1, and its
//     first read (row 0) is after it;
//   * the DMA into ring slot (t+3) % 4 = (t-1) % 4 is issued after barrier 2t-1,
//     by which row 1's reads of k-tile t-1 completed (lgkmcnt(0) before it);
//   * past the last k-tile the DMAs read zeros into slots nobody reads again, so
//     every wave's vmcnt count stays uniform.
// OCC > 0: at least OCC waves per SIMD (the register budget that lets two 8-wave
// blocks share a CU, so one block's prologue / epilogue overlaps the other's MFMAs)
// (Round 6 also built a register-pipelined one-wave-per-SIMD 128x128 k-loop here; it measured
// slower than the ping-pong tiles and was removed: profiles/gemm_rp_tiles_r6.txt.)
template <int BM, int BN, int BK, int WM, int WN, int NS, bool AT, bool BT, int EPI, int KG = 1,
          bool PP = false, int OCC = 0>
__global__ void __launch_bounds__(64 * WM * WN * KG)
__attribute__((amdgpu_waves_per_eu(OCC > 0 ? OCC : 1))) gemm_kernel(GemmArgs g) {
  constexpr int NWG = WM * WN, NW = NWG * KG;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "wave tiles of 16x16 MFMAs");
  static_assert(KG == 1 || (KG == 2 && EPI == EPI_ACC32 && AT && BT),
                "k-groups only for the weight gradient (both operands k-strided)");
  constexpr int BKS = BK * KG;                      // k-rows per staged k-tile
  using SA = Stager<BM, AT, NW, BKS>;
  using SB = Stager<BN, BT, NW, BKS>;
  constexpr int STAGE = SA::EL + SB::EL;
  constexpr int INS_MIN = SA::PW_MIN + SB::PW_MIN;   // DMAs every wave issues per stage
  static_assert(NS >= 2 && (NS - 2) * INS_MIN < 64, "pipeline depth");
  constexpr bool TRANS_OUT = EPI != EPI_ACC32;   // lane owns 4 consecutive n of one m
  // the two-blocks-per-CU tiles (OCC > 0) have a ring smaller than the padded
  // epilogue tile: LDS sized for the larger of the two
  constexpr int EPI_EL = NW * (BM / WM) * (BN / WN + 8);
  constexpr int LDS_EL = (OCC > 0 && TRANS_OUT && EPI_EL > NS * STAGE) ? EPI_EL : NS * STAGE;
  __shared__ __attribute__((aligned(16))) u16 lds[LDS_EL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = KG == 1 ? 0 : wid / NWG, wq = KG == 1 ? wid : wid % NWG;
  const int wm = wq / WN, wn = wq % WN;

  // XCD-aware bijective remap of the tile id: blocks sharing an XCD take
  // consecutive tiles (neighbouring N tiles of one M panel)
  const int bid = blockIdx.x;
  // remainder split-K piece (see GemmArgs): tile sk_full + rt, k-piece `piece`
  const bool sk = TRANS_OUT && g.sk_split > 1 && bid >= g.sk_full;
  const int rt = sk ? (bid - g.sk_full) / g.sk_split : 0;
  const int piece = sk ? bid - g.sk_full - rt * g.sk_split : 0;
  const int G = TRANS_OUT && g.sk_split > 1 ? g.sk_full : gridDim.x;   // whole-tile blocks
  // weight gradient with split-K (g.xcd_k): the same deal over the linear block
  // id of the whole (tile, split) grid, split-major -- the blocks of one XCD take
  // consecutive tiles of ONE k-range instead of all k-ranges of fewer tiles, so
  // the operand panels one XCD's L2 must hold shrink (ViT-B/16 QKV dW: the 128x128
  // tiles over 4 k-ranges read 8 x the 19 MB input X from beyond L2 otherwise)
  const bool kdeal = EPI == EPI_ACC32 && g.xcd_k && gridDim.y > 1;
  const int L = kdeal ? bid + (int)blockIdx.y * G : bid;
  const int GL = kdeal ? G * (int)gridDim.y : G;
  const int xcd = L & 7, q8 = GL >> 3, r8 = GL & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ky = kdeal ? lin / G : (int)blockIdx.y;
  const int tile = sk ? g.sk_full + rt : (kdeal ? lin - ky * G : lin);
  const int tm = tile / g.tiles_n;
  const int m0 = tm * BM, n0 = (tile - tm * g.tiles_n) * BN;
  const int kbase = sk ? piece * g.sk_kchunk : ky * g.k_chunk;
  const int kend = min(g.K, kbase + (sk ? g.sk_kchunk : g.k_chunk)) - kbase;
  if (kend <= 0) return;   // (the host sizes pieces so that none is empty)
  const int KT = (kend + BKS - 1) / BKS;

  SA sa;
  SB sb;
  sa.init(wid, lane, m0, g.M, g.lda, kbase);
  sb.init(wid, lane, n0, g.N, g.ldb, kbase);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.a, 0, AT ? (int)(2LL * g.K * g.lda) : (int)(2LL * g.M * g.lda), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.b, 0, BT ? (int)(2LL * g.K * g.ldb) : (int)(2LL * g.N * g.ldb), 0x00020000);
  auto stage = [&](int buf, int kt) {
    u16* As = lds + buf * STAGE;
    sa.issue(rsA, As, wid, kt * BKS, kend, g.lda);
    sb.issue(rsB, As + SA::EL, wid, kt * BKS, kend, g.ldb);
  };

  f32x4 acc[TM][TN];
  f32x4 accb[TM];
  bf16x8 ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones.v[k] = 0x3f80;   // bf16 1.0
  const int ra = wm * (BM / WM), rb = wn * (BN / WN);
  bool do_bias = false;

  auto compute = [&](int buf) {
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + SA::EL;
#pragma unroll
    for (int ks0 = 0; ks0 < BK / 32; ++ks0) {
      const int ks = kg * (BK / 32) + ks0;          // this k-group's rows of the image
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<BM, AT, BKS>(As, ra + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag<BN, BT, BKS>(Bs, rb + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = TRANS_OUT ? mfma_bf16(bf[j], af[i], acc[i][j])
                                : mfma_bf16(af[i], bf[j], acc[i][j]);
      if (EPI == EPI_ACC32 && do_bias) {
#pragma unroll
        for (int i = 0; i < TM; ++i) accb[i] = mfma_bf16(af[i], ones, accb[i]);
      }
    }
  };

  // tile start: accumulators = bias (fwd) or 0
  auto tile_init = [&](int m0, int n0) {
    if constexpr (EPI == EPI_ACC32) {
      do_bias = g.dbias != nullptr && n0 == 0 && wn == 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + rb + j * 16 + 4 * (lane >> 4);
        f32x4 bv = {0.f, 0.f, 0.f, 0.f};
        if (EPI != EPI_DGELU && EPI != EPI_DRELU && g.bias != nullptr && n < g.N && piece == 0) {
          const uint2 raw = *reinterpret_cast<const uint2*>(g.bias + n);
          bv = f32x4{__uint_as_float(raw.x << 16), __uint_as_float(raw.x & 0xffff0000u),
                     __uint_as_float(raw.y << 16), __uint_as_float(raw.y & 0xffff0000u)};
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = bv;
      }
    }
  };

  auto epilogue = [&](int m0, int n0) {
    if constexpr (EPI == EPI_ACC32) {
      // D layout: lane holds rows m = 4*(lane>>4) + r of column n = lane & 15
      float* C = reinterpret_cast<float*>(g.c);
      const bool atomic = gridDim.y > 1;
      // split-K into a slab: plain stores (~6 TB/s chip-wide) instead of fp32
      // atomics (~1.3 TB/s of added bytes), reduced by a streaming pass after
      float* S = g.slab != nullptr ? g.slab + (long long)ky * g.M * g.N : nullptr;
      if (do_bias && (lane & 15) == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + ra + i * 16 + 4 * (lane >> 4) + r;
            if (m < g.M) atomicAdd(g.dbias + m, accb[i][r]);
          }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + rb + j * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + ra + i * 16 + 4 * (lane >> 4) + r;
            if (m < g.M && n < g.N) {
              if (S != nullptr) {
                S[(long long)m * g.N + n] = acc[i][j][r];
              } else {
                float* p = C + (long long)m * g.ldc + n;
                if (atomic) atomicAdd(p, acc[i][j][r]);
                else *p += acc[i][j][r];
              }
            }
          }
        }
    } else {
      // bf16 outputs: the D^T register layout (lane: 4 consecutive n of one m)
      // would make every store / aux load touch 16 rows x 32 B.  Each wave
      // stages its tile through LDS instead (free after the k-loop; row pitch
      // padded by 16 B) and re-reads it as rows of 16-B chunks: the epilogue
      // math, the aux load (GELU' pre-activation / addend) and the stores all
      // move whole row segments.
      constexpr int WROWS = BM / WM, WCOLS = BN / WN, CPR = WCOLS / 8, RPI = 64 / CPR;
      // 16-B row padding when it fits, else (256x256 ring) an XOR swizzle of the
      // 16-B chunks by row & 7 (needs a multiple of 8 chunks per row)
      constexpr bool SWZ = NW * WROWS * (WCOLS + 8) > LDS_EL;
      constexpr int PITCH = SWZ ? WCOLS : WCOLS + 8;
      static_assert(NW * WROWS * PITCH <= LDS_EL, "epilogue tile fits in the ring's LDS");
      static_assert(!SWZ || CPR % 8 == 0, "swizzled epilogue tile needs 8k chunks per row");
      auto pchunk = [](int row, int c) { return SWZ ? (c ^ (row & 7)) : c; };
      constexpr int NR = (WROWS + RPI - 1) / RPI;   // row segments per lane
      const int cbytes = (int)(2LL * g.M * g.ldc);
      const __amdgpu_buffer_rsrc_t rsC =
          __builtin_amdgcn_make_buffer_rsrc(g.c, 0, cbytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rsC2 = __builtin_amdgcn_make_buffer_rsrc(
          EPI == EPI_GELU ? (void*)g.c2 : g.c, 0, cbytes, 0x00020000);
      const bool has_aux = g.aux != nullptr;
      const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
          has_aux ? (void*)g.aux : g.c, 0, cbytes, 0x00020000);
      const int lrow = lane / CPR, ch = lane - lrow * CPR;
      const bool lane_on = lrow < RPI;
      const int n = n0 + rb + ch * 8;
      // BN partial sums of the stored values, per column (EPI_STORE, 16-B path)
      const bool stats = EPI == EPI_STORE && g.part != nullptr;
      float s_sum[8], s_sq[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s_sum[e] = 0.f; s_sq[e] = 0.f; }
      // an output width / row stride that is not whole 16-B pieces (10-class
      // heads, LeNet's 84 / 6 / 16 columns) is stored element by element
      const bool narrow = ((g.N | g.ldc) & 7) != 0;
      unsigned o[NR];
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        const int row = q * RPI + lrow, m = m0 + ra + row;
        o[q] = (lane_on && row < WROWS && m < g.M && n < g.N) ? 2u * (unsigned)(m * g.ldc + n)
                                                              : kOOBg;
      }
      // the aux row segments (GELU' pre-activation / addend) are fetched first,
      // so their latency overlaps the LDS staging below
      u32x4_t xa[has_aux_slots(EPI) ? NR : 1];
      if (!narrow && (EPI == EPI_DGELU || EPI == EPI_DRELU || (EPI == EPI_STORE && has_aux))) {
#pragma unroll
        for (int q = 0; q < (has_aux_slots(EPI) ? NR : 1); ++q)
          xa[q] = __builtin_amdgcn_raw_buffer_load_b128(rsX, o[q], 0, 0);
      }
      // deferred ReLU mask of the addend: one byte = this lane's 8 columns (the
      // host allows it only with ldc == N, 16-B row segments)
      const bool amask = EPI == EPI_STORE && has_aux && g.auxmask != nullptr && !narrow;
      unsigned mb[EPI == EPI_STORE ? NR : 1];
      if constexpr (EPI == EPI_STORE) {
        const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(
            amask ? (void*)g.auxmask : g.c, 0, cbytes / 16, 0x00020000);
#pragma unroll
        for (int q = 0; q < NR; ++q)
          mb[q] = amask ? __builtin_amdgcn_raw_buffer_load_b8(rsM, o[q] != kOOBg ? o[q] >> 4 : kOOBg,
                                                             0, 0)
                        : 0xffu;
      }
      __syncthreads();            // every wave is done reading the ring
      u16* wl = lds + wid * (WROWS * PITCH);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = i * 16 + (lane & 15), c16 = 2 * j + (lane >> 5);
          const int col = pchunk(row, c16) * 8 + 4 * ((lane >> 4) & 1);
          uint2 pk;
          pk.x = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
          pk.y = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
          *reinterpret_cast<uint2*>(wl + row * PITCH + col) = pk;
        }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        const int row = min(q * RPI + lrow, WROWS - 1);   // idle lanes re-read a valid row
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(wl + row * PITCH + pchunk(row, ch) * 8);
        bf16x8 xv;
        if (has_aux_slots(EPI)) {
          if (!narrow) {
            xv = __builtin_bit_cast(bf16x8, xa[has_aux_slots(EPI) ? q : 0]);
          } else if (has_aux) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              xv.v[e] = n + e < g.N ? (u16)__builtin_amdgcn_raw_buffer_load_b16(
                                          rsX, o[q] == kOOBg ? kOOBg : o[q] + 2u * e, 0, 0)
                                    : (u16)0;
          }
        }
        bf16x8 out, out2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = bf2f(v.v[e]);
          if constexpr (EPI == EPI_STORE) {
            float t = has_aux ? a + ((mb[q] >> e) & 1u ? bf2f(xv.v[e]) : 0.f) : a;
            if (g.relu) t = fmaxf(t, 0.f);
            out.v[e] = (has_aux || g.relu) ? f2bf(t) : v.v[e];
          } else if constexpr (EPI == EPI_GELU) {
            out.v[e] = v.v[e];                                 // h (pre-activation)
            out2.v[e] = f2bf(gelu_tanh(a, nullptr));           // gelu of the stored h
          } else if constexpr (EPI == EPI_DRELU) {   // xv = the layer's ReLU'd input
            out.v[e] = bf2f(xv.v[e]) > 0.f ? v.v[e] : (u16)0;
          } else {   // EPI_DGELU: xv = pre-activation h
            float d;
            gelu_tanh(bf2f(xv.v[e]), &d);
            out.v[e] = f2bf(a * d);
          }
        }
        if (stats && o[q] != kOOBg) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float yv = bf2f(out.v[e]);
            s_sum[e] += yv;
            s_sq[e] += yv * yv;
          }
        }
        if (!narrow) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, out), rsC, o[q], 0,
                                                 DMP_GEMM_STORE_AUX);
          if constexpr (EPI == EPI_GELU)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, out2), rsC2, o[q],
                                                   0, DMP_GEMM_STORE_AUX);
        } else if (o[q] != kOOBg) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (n + e < g.N) {
              __builtin_amdgcn_raw_buffer_store_b16(out.v[e], rsC, o[q] + 2u * e, 0, 0);
              if constexpr (EPI == EPI_GELU)
                __builtin_amdgcn_raw_buffer_store_b16(out2.v[e], rsC2, o[q] + 2u * e, 0, 0);
            }
          }
        }
      }
      if (stats) {
        // the RPI row lanes of each 8-column segment, then one atomic per
        // column per wave into slot (block % kBnSlots)
#pragma unroll
        for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s_sum[e] += __shfl_xor(s_sum[e], off, 64);
            s_sq[e] += __shfl_xor(s_sq[e], off, 64);
          }
        if (lrow == 0) {
          const int slot = (int)(blockIdx.x % kBnSlots);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (n + e < g.N) {
              atomicAdd(g.part + (long long)slot * g.N + n + e, s_sum[e]);
              atomicAdd(g.part + (long long)(kBnSlots + slot) * g.N + n + e, s_sq[e]);
            }
          }
        }
      }
    }
  };

  DMP_STAMP(0);
  // bias (fwd) into the accumulators before any DMA is in flight
  tile_init(m0, n0);
  if constexpr (PP) {
    static_assert(WM == 2 && KG == 1 && NS == 4 && BK == 32, "ping-pong tiles: 2 wave rows, BK 32, 4 slots");
    static_assert(SA::INS % NW == 0 && SB::INS % NW == 0, "uniform DMA count per wave");
    constexpr int PWK = SA::PW_MIN + SB::PW_MIN;   // DMAs per wave per k-tile
    const bool late = wm == 1;
#pragma unroll
    for (int s = 0; s < 3; ++s) stage(s, s);        // k-tiles past KT load zeros
    gwait_vm<2 * PWK>();                            // k-tile 0 landed (this wave)
    __builtin_amdgcn_s_barrier();
    DMP_STAMP(1);
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    for (int kt = 0; kt < KT; ++kt) {
      const u16* As = lds + (kt & 3) * STAGE;
      const u16* Bs = As + SA::EL;
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<BM, AT, BK>(As, ra + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag<BN, BT, BK>(Bs, rb + j * 16, 0, lane);
      stage((kt + 3) & 3, kt + 3);
      gwait_vm<2 * PWK>();                          // k-tile kt+1 landed; fragments read
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = TRANS_OUT ? mfma_bf16(bf[j], af[i], acc[i][j])
                                : mfma_bf16(af[i], bf[j], acc[i][j]);
      if (EPI == EPI_ACC32 && do_bias) {
#pragma unroll
        for (int i = 0; i < TM; ++i) accb[i] = mfma_bf16(af[i], ones, accb[i]);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!late) __builtin_amdgcn_s_barrier();
    gwait_vm<0>();
  } else {
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT) stage(s, s);
  for (int kt = 0; kt < KT; ++kt) {
    // k-tile kt landed for this wave (younger ones may still fly) ...
    if (kt + NS - 2 < KT) gwait_vm<(NS - 2) * INS_MIN>();
    else gwait_vm<0>();
    // ... and for every wave; everyone is done reading slot (kt-1) % NS
    __builtin_amdgcn_s_barrier();
    if (kt == 0) DMP_STAMP(1);
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < KT) stage((kt + NS - 1) % NS, kt + NS - 1);
    compute(kt % NS);
  }
  }
  DMP_STAMP(2);
  if constexpr (KG == 2) {
    // group 1 parks its partial sums in the drained ring, group 0 adds them
    gwait_vm<0>();
    __syncthreads();
    float* park = reinterpret_cast<float*>(lds);   // [NWG][TM*TN (+TM)][64 lanes] f32x4
    constexpr int PT = TM * TN + TM;
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(park + ((wq * PT + i * TN + j) * 64 + lane) * 4) = acc[i][j];
        *reinterpret_cast<f32x4*>(park + ((wq * PT + TM * TN + i) * 64 + lane) * 4) = accb[i];
      }
    }
    __syncthreads();
    if (kg == 1) return;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] += *reinterpret_cast<const f32x4*>(park + ((wq * PT + i * TN + j) * 64 + lane) * 4);
      accb[i] += *reinterpret_cast<const f32x4*>(park + ((wq * PT + TM * TN + i) * 64 + lane) * 4);
    }
  }
  if constexpr (TRANS_OUT) {
    if (sk) {
      // publish this piece's fp32 accumulators in the lane-native layout (16 B per
      // lane and fragment: whole lines), then take a ticket; the last piece to
      // arrive adds the others' (agent-scope release / acquire: the pieces of a
      // tile may run on any XCD, MI355X_MICROARCH.md "Workgroup dispatch")
      constexpr int FR = TM * TN * 256;   // floats per wave
      const int S = g.sk_split;
      float* mine = g.sk_ws + ((long long)(rt * S + piece) * NW + wid) * FR;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(mine + (i * TN + j) * 256 + lane * 4) = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // every wave's stores done; every wave past its last ring read
      int* flag = reinterpret_cast<int*>(lds);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(g.sk_cnt + rt, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == S - 1;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
      }
      __syncthreads();
      const bool last = *flag != 0;
      __syncthreads();   // the flag is read before the epilogue reuses the LDS
      if (!last) return;
      for (int p = 0; p < S; ++p) {
        if (p == piece) continue;
        const float* other = g.sk_ws + ((long long)(rt * S + p) * NW + wid) * FR;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] += *reinterpret_cast<const f32x4*>(other + (i * TN + j) * 256 + lane * 4);
      }
    }
  }
  epilogue(m0, n0);
  DMP_STAMP(3);
}

// ------------------------------------------------------- any-shape fallback
// Odd shapes the 16-B DMA tiles cannot take (a reduction length or output
// width that is not a multiple of 8: LeNet's 84-wide layer, 10-class heads)
// and tiny GEMMs: 64x64 output tile per 256-thread block, 4x4 outputs per
// thread, k staged through LDS 32 at a time as fp32 with the next stage
// prefetched into registers, same epilogues.
template <bool AT, bool BT, int EPI>
__global__ void __launch_bounds__(256) gemm_small_kernel(GemmArgs g) {
  constexpr int KS = 32;                       // k per LDS stage
  __shared__ float As[KS][65], Bs[KS][65];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int kbase = blockIdx.z * g.k_chunk;
  const int kend = min(g.K, kbase + g.k_chunk);
  const bool do_bias = EPI == EPI_ACC32 && g.dbias != nullptr && blockIdx.y == 0 && tx == 0;
  float acc[4][4] = {};
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
  // a lane's 8 staging elements of each operand: consecutive lanes walk the
  // operand's contiguous dimension (k for a row-major operand, rows for a
  // k-strided one); the next stage is fetched into registers while the
  // current one is multiplied (the loop is load-latency bound otherwise)
  auto coord = [&](int u, bool t, int& r, int& kk) {
    const int e = tid + 256 * u;
    if (t) { r = e & 63; kk = e >> 6; }
    else { r = e / KS; kk = e % KS; }
  };
  float pa[8], pb[8];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int r, kk;
      coord(u, AT, r, kk);
      const int k = k0 + kk, m = m0 + r;
      pa[u] = (k < kend && m < g.M)
                  ? bf2f(AT ? g.a[(long long)k * g.lda + m] : g.a[(long long)m * g.lda + k])
                  : 0.f;
      coord(u, BT, r, kk);
      const int kb = k0 + kk, n = n0 + r;
      pb[u] = (kb < kend && n < g.N)
                  ? bf2f(BT ? g.b[(long long)kb * g.ldb + n] : g.b[(long long)n * g.ldb + kb])
                  : 0.f;
    }
  };
  if (kbase < kend) fetch(kbase);
  for (int k0 = kbase; k0 < kend; k0 += KS) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int r, kk;
      coord(u, AT, r, kk);
      As[kk][r] = pa[u];
      coord(u, BT, r, kk);
      Bs[kk][r] = pb[u];
    }
    __syncthreads();
    if (k0 + KS < kend) fetch(k0 + KS);
#pragma unroll 8
    for (int kk = 0; kk < KS; ++kk) {
      float a4[4], b4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a4[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b4[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (do_bias) rsum[i] += a4[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a4[i], b4[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty + 16 * i;
    if (m >= g.M) continue;
    if (do_bias) atomicAdd(g.dbias + m, rsum[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx + 16 * j;
      if (n >= g.N) continue;
      const long long o = (long long)m * g.ldc + n;
      const float v = acc[i][j];
      if constexpr (EPI == EPI_ACC32) {
        float* C = reinterpret_cast<float*>(g.c);
        if (gridDim.z > 1) atomicAdd(C + o, v);
        else C[o] += v;
      } else {
        u16* C = reinterpret_cast<u16*>(g.c);
        const float b = (EPI != EPI_DGELU && EPI != EPI_DRELU && g.bias != nullptr)
                            ? bf2f(g.bias[n]) : 0.f;
        if constexpr (EPI == EPI_STORE) {
          const float t = v + b + (g.aux != nullptr ? bf2f(g.aux[o]) : 0.f);
          C[o] = f2bf(g.relu ? fmaxf(t, 0.f) : t);
        } else if constexpr (EPI == EPI_GELU) {
          const u16 h = f2bf(v + b);
          C[o] = h;
          g.c2[o] = f2bf(gelu_tanh(bf2f(h), nullptr));
        } else if constexpr (EPI == EPI_DRELU) {
          C[o] = bf2f(g.aux[o]) > 0.f ? f2bf(v) : (u16)0;
        } else {
          float d;
          gelu_tanh(bf2f(g.aux[o]), &d);
          C[o] = f2bf(v * d);
        }
      }
    }
  }
}

// C[m][n] (ldc) += sum over the splits of slab[s][m][n]; 4 columns per thread
// when rows are whole float4s
__global__ void __launch_bounds__(256) gemm_slab_reduce_kernel(const float* __restrict__ slab,
                                                               float* __restrict__ c, int M, int N,
                                                               int ldc, int splits) {
  const long long MN = (long long)M * N;
  const long long gs = (long long)gridDim.x * blockDim.x;
  if ((N & 3) == 0 && (ldc & 3) == 0) {
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < MN / 4; v += gs) {
      const long long e = v * 4;
      const long long m = e / N, n = e - m * N;
      float4 t = *reinterpret_cast<const float4*>(slab + e);
      for (int sp = 1; sp < splits; ++sp) {
        const float4 u = *reinterpret_cast<const float4*>(slab + sp * MN + e);
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      float4* o = reinterpret_cast<float4*>(c + m * ldc + n);
      float4 cv = *o;
      cv.x += t.x; cv.y += t.y; cv.z += t.z; cv.w += t.w;
      *o = cv;
    }
  } else {
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < MN; e += gs) {
      const long long m = e / N, n = e - m * N;
      float t = slab[e];
      for (int sp = 1; sp < splits; ++sp) t += slab[sp * MN + e];
      c[m * ldc + n] += t;
    }
  }
}

template <bool AT, bool BT, int EPI>
void launch_small(const GemmArgs& g, int splits, hipStream_t s) {
  hipLaunchKernelGGL((gemm_small_kernel<AT, BT, EPI>),
                     dim3((unsigned)((g.M + 63) / 64), (unsigned)((g.N + 63) / 64), (unsigned)splits),
                     dim3(256), 0, s, g);
}

// ------------------------------------------------------------------ configs
struct Cfg { int bm, bn, bk, wm, wn, ns, kg = 1, pp = 0, occ = 0; };
// LDS = ns * (bm + bn) * bk * 2 B.  Tile heights 160 / 192 exist for tile
// counts: M = 12608 tokens x N = 768 is 150 tiles of 256x256 (59 % of 256 CUs)
// but 237 of 160x256.  A k-strided (transposed) operand needs a tile side that
// is a multiple of 128 (whole 256-B LDS bank rows): gemm_config_ok().
constexpr Cfg kCfgs[] = {
    {256, 256, 64, 2, 4, 2},   // 0: 128 KiB, 8 waves (128x64 per wave), 1 block/CU
    {256, 128, 64, 4, 2, 3},   // 1: 144 KiB, 8 waves (64x64)
    {128, 256, 64, 2, 4, 3},   // 2: 144 KiB, 8 waves (64x64)
    {192, 256, 64, 2, 4, 2},   // 3: 112 KiB, 8 waves (96x64)
    {128, 128, 64, 2, 2, 2},   // 4:  64 KiB, 4 waves, 2 blocks/CU
    {160, 256, 64, 2, 4, 2},   // 5: 104 KiB, 8 waves (80x64)
    {256, 192, 64, 2, 4, 2},   // 6: 112 KiB, 8 waves (128x48)
    {128, 128, 32, 2, 2, 4},   // 7:  64 KiB, 4 waves, 2 blocks/CU, 3 k-tiles in flight
    {256, 128, 64, 2, 2, 3},   // 8: 144 KiB, 4 waves of 128x64 (1 wave / SIMD)
    {128, 128, 64, 2, 2, 2, 2},   // 9: wgrad only, 2 k-groups of 4 waves: 128 KiB, 1 block/CU
    {256, 256, 32, 2, 4, 4, 1, 1},   // 10: ping-pong k-loop (PP), 128 KiB, 8 waves of 128x64
    {128, 256, 32, 2, 4, 4, 1, 1},   // 11: PP, 96 KiB, 8 waves of 64x64
    {256, 128, 32, 2, 4, 4, 1, 1},   // 12: PP, 96 KiB, 8 waves of 128x32
    // two 8-wave blocks per CU (<= 128 VGPRs): 13-15
    {128, 256, 32, 2, 4, 2, 1, 0, 4},   // 13: 48 KiB, 8 waves of 64x64
    {128, 256, 32, 2, 4, 3, 1, 0, 4},   // 14: 72 KiB, 8 waves of 64x64
    {256, 128, 32, 4, 2, 2, 1, 0, 4},   // 15: 48 KiB, 8 waves of 64x64
};
// (4 waves of 128x128 per 256x256 / 192x256 tile, accumulators in AGPRs: 20-40 %
// slower than the 8-wave tiles on every ViT shape -- profiles/gemm_vs_hipblaslt_r2.txt)
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

constexpr bool cfg_ok(const Cfg& c, bool at, bool bt) {
  return (!at || c.bm % 128 == 0) && (!bt || c.bn % 128 == 0) && (c.kg == 1 || (at && bt));
}

// blocks of a config resident per CU (LDS, and the 256-VGPR 8-wave tiles)
constexpr int cfg_blocks_per_cu(const Cfg& c) {
  const int lds = c.ns * (c.bm + c.bn) * c.bk * 2;
  const int by_lds = (160 * 1024) / (lds > 0 ? lds : 1);
  const int by_regs = (c.occ > 0 || c.wm * c.wn * c.kg <= 4) ? 2 : 1;
  return by_lds < by_regs ? (by_lds < 1 ? 1 : by_lds) : by_regs;
}

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

// remainder split-K plan of a fwd / dgrad launch (GemmArgs sk_*): the whole
// rounds as usual, the last round's `rem` tiles in `sp` k-pieces (fewer than
// requested when the round has no room or K is short; sp = 1: no split)
struct SkPlan { int full = 0, rem = 0, sp = 1, kchunk = 0; };
SkPlan sk_plan(const Cfg& c, int M, int N, int K, int want) {
  SkPlan p;
  if (want <= 1) return p;
  const int tiles = ((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
  const int slots = num_cus() * cfg_blocks_per_cu(c);
  const int rem = tiles % slots;
  const int kt = (K + c.bk - 1) / c.bk;
  int sp = rem > 0 ? std::min(std::min(want, slots / rem), kt) : 1;
  if (sp <= 1) return p;
  const int kchunk = (kt + sp - 1) / sp * c.bk;
  sp = (K + kchunk - 1) / kchunk;   // no empty piece
  if (sp <= 1) return p;
  p.full = tiles - rem;
  p.rem = rem;
  p.sp = sp;
  p.kchunk = kchunk;
  return p;
}

template <int C, bool AT, bool BT, int EPI>
void launch_cfg(const GemmArgs& a, int splits, hipStream_t s) {
  constexpr Cfg c = kCfgs[C];
  if constexpr (!cfg_ok(c, AT, BT)) {
    throw std::runtime_error("gemm: tile config not valid for a k-strided operand");
  } else {
    GemmArgs g = a;
    g.tiles_n = (g.N + c.bn - 1) / c.bn;
    const int tiles = ((g.M + c.bm - 1) / c.bm) * g.tiles_n;
    int grid_x = tiles, grid_y = splits;
    if (EPI != EPI_ACC32 && g.sk_split > 1) {
      const SkPlan p = sk_plan(c, g.M, g.N, g.K, g.sk_split);
      g.sk_split = p.sp;
      if (p.sp > 1) {
        g.sk_full = p.full;
        g.sk_kchunk = p.kchunk;
        grid_x = p.full + p.rem * p.sp;
      }
      grid_y = 1;
    } else {
      g.sk_split = 1;
    }
    if constexpr (c.kg == 1 || EPI == EPI_ACC32)
      hipLaunchKernelGGL((gemm_kernel<c.bm, c.bn, c.bk, c.wm, c.wn, c.ns, AT, BT, EPI, c.kg,
                                      c.pp != 0, c.occ>),
                         dim3((unsigned)grid_x, (unsigned)grid_y), dim3(64 * c.wm * c.wn * c.kg), 0,
                         s, g);
    else
      throw std::runtime_error("gemm: k-group configs are weight-gradient only");
  }
}

template <bool AT, bool BT, int EPI>
void launch_mode(int cfg, const GemmArgs& a, int splits, hipStream_t s) {
  switch (cfg) {
    case -1: launch_small<AT, BT, EPI>(a, splits, s); break;
    case 0: launch_cfg<0, AT, BT, EPI>(a, splits, s); break;
    case 1: launch_cfg<1, AT, BT, EPI>(a, splits, s); break;
    case 2: launch_cfg<2, AT, BT, EPI>(a, splits, s); break;
    case 3: launch_cfg<3, AT, BT, EPI>(a, splits, s); break;
    case 4: launch_cfg<4, AT, BT, EPI>(a, splits, s); break;
    case 5: launch_cfg<5, AT, BT, EPI>(a, splits, s); break;
    case 6: launch_cfg<6, AT, BT, EPI>(a, splits, s); break;
    case 7: launch_cfg<7, AT, BT, EPI>(a, splits, s); break;
    case 8: launch_cfg<8, AT, BT, EPI>(a, splits, s); break;
    case 9: launch_cfg<9, AT, BT, EPI>(a, splits, s); break;
    case 10: launch_cfg<10, AT, BT, EPI>(a, splits, s); break;
    case 11: launch_cfg<11, AT, BT, EPI>(a, splits, s); break;
    case 12: launch_cfg<12, AT, BT, EPI>(a, splits, s); break;
    case 13: launch_cfg<13, AT, BT, EPI>(a, splits, s); break;
    case 14: launch_cfg<14, AT, BT, EPI>(a, splits, s); break;
    default: launch_cfg<15, AT, BT, EPI>(a, splits, s); break;
  }
}

}  // namespace

int gemm_num_configs() { return kNumCfgs; }

bool gemm_config_ok(int mode, int cfg) {
  if (cfg == -1) return true;
  if (cfg < 0 || cfg >= kNumCfgs) return false;
  return cfg_ok(kCfgs[cfg], mode == 2, mode >= 1);
}

void gemm_config_info(int cfg, int* info) {
  const Cfg& c = kCfgs[cfg];
  info[0] = c.bm;
  info[1] = c.bn;
  info[2] = 64 * c.wm * c.wn * c.kg;
  info[3] = c.ns;
  info[4] = c.bk;
}

namespace {
int g_xcd_k = -1;   // DMP_GEMM_XCD_K (default 1): split-major XCD deal of wgrad split-K
}
void gemm_set_xcd_k(int on) { g_xcd_k = on ? 1 : 0; }

// mode 0: fwd (C = A B^T, EPI 0 or 1), 1: dgrad (A [M][K], B [K][N]; EPI 0 or 2),
// 2: wgrad (A [K][M], B [K][N]; fp32 accumulate)
void launch_gemm(int mode, int epi, int cfg, const uint16_t* a, int lda, const uint16_t* b,
                 int ldb, void* c, int ldc, uint16_t* c2, const uint16_t* bias,
                 const uint16_t* aux, float* dbias, int M, int N, int K, int splits,
                 hipStream_t s, bool relu, float* part, float* slab, float* sk_ws, int* sk_cnt,
                 const uint8_t* auxmask) {
  GemmArgs g{};
  if (g_xcd_k < 0) {
    const char* e = std::getenv("DMP_GEMM_XCD_K");
    g_xcd_k = (e == nullptr || e[0] != '0') ? 1 : 0;
  }
  g.xcd_k = g_xcd_k;
  g.auxmask = aux != nullptr && epi == EPI_STORE ? auxmask : nullptr;
  g.relu = relu ? 1 : 0;
  g.part = part;
  g.a = a; g.b = b; g.c = c; g.c2 = c2; g.bias = bias; g.aux = aux; g.dbias = dbias;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  // fwd / dgrad: `splits` > 1 asks for the remainder split-K (needs sk_ws / sk_cnt)
  if (mode != 2 && splits > 1 && cfg >= 0 && sk_ws != nullptr && sk_cnt != nullptr) {
    g.sk_split = splits;
    g.sk_ws = sk_ws;
    g.sk_cnt = sk_cnt;
  }
  if (splits < 1 || mode != 2) splits = 1;   // split-K only for the fp32-accumulating pass
  g.k_chunk = ((K + splits - 1) / splits + 63) / 64 * 64;   // whole k-tiles of any BK
  splits = (K + g.k_chunk - 1) / g.k_chunk;
  if (mode == 0) {
    if (epi == EPI_GELU) launch_mode<false, false, EPI_GELU>(cfg, g, 1, s);
    else launch_mode<false, false, EPI_STORE>(cfg, g, 1, s);
  } else if (mode == 1) {
    if (epi == EPI_DGELU) launch_mode<false, true, EPI_DGELU>(cfg, g, 1, s);
    else if (epi == EPI_DRELU) launch_mode<false, true, EPI_DRELU>(cfg, g, 1, s);
    else launch_mode<false, true, EPI_STORE>(cfg, g, 1, s);
  } else {
    // slab split-K only for the MFMA tiles with more than one split
    if (slab != nullptr && splits > 1 && cfg >= 0) g.slab = slab;
    launch_mode<true, true, EPI_ACC32>(cfg, g, splits, s);
    if (g.slab != nullptr) {
      const long long work = ((N & 3) == 0 && (ldc & 3) == 0) ? (long long)M * N / 4
                                                               : (long long)M * N;
      hipLaunchKernelGGL(gemm_slab_reduce_kernel, dim3(stream_grid(work, 256)), dim3(256), 0, s,
                         slab, reinterpret_cast<float*>(c), M, N, ldc, splits);
    }
  }
}

void gemm_sk_sizes(int cfg, int M, int N, int K, int splits, long long* ws_floats, int* counters) {
  *ws_floats = 0;
  *counters = 0;
  if (cfg < 0 || cfg >= kNumCfgs || splits <= 1) return;
  const Cfg& c = kCfgs[cfg];
  if (c.kg != 1) return;
  const SkPlan p = sk_plan(c, M, N, K, splits);
  if (p.sp <= 1) return;
  *ws_floats = (long long)p.rem * p.sp * c.bm * c.bn;
  *counters = p.rem;
}

// effective split count launch_gemm uses for (K, requested splits) in mode 2
int gemm_effective_splits(int K, int splits) {
  if (splits < 1) splits = 1;
  const int k_chunk = ((K + splits - 1) / splits + 63) / 64 * 64;
  return (K + k_chunk - 1) / k_chunk;
}

}  // namespace dmp
