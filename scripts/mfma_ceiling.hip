// MFMA-loop ceiling microbenchmark ("ceiling first").
//
// The bare LDS -> register -> MFMA loop of the conv kernels, with nothing else:
// no global->LDS staging, no barriers in the loop, no epilogue.  A block fills
// a 64 KiB LDS image with random bf16 once, then every wave runs NSTEP
// (tap, k-step)-like steps: read its A and B fragments for the step from LDS at
// a row offset that moves every step (as the halo kernels' taps do), MFMA them
// into its accumulators, fragments double-buffered in registers (the reads of
// step s+1 issued among step s's MFMAs, like conv.hip).  Variants:
//   shape 16 : v_mfma_f32_16x16x32_bf16, wave tile (16*TM) x (16*TN)
//   shape 32 : v_mfma_f32_32x32x16_bf16, wave tile (32*TM) x (32*TN)
//   mode REG : register-fed (fragments read once, kept live) -- MFMA pipe + clock only
//   mode LDS : both operands' fragments re-read from LDS every step
//   mode AL  : A re-read from LDS every step, B register-resident across the loop
//              (round 6: "one operand held in registers")
// at NW waves per block and BPC blocks per CU.  Random operands throughout
// (zero data raises the clock: MI355X_MICROARCH.md, DVFS give-back).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o build/mfma_ceiling scripts/mfma_ceiling.hip
// Run:   build/mfma_ceiling   (one table; TF/s against the 2.5 PF dense bf16 peak)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr int kRows = 512;             // LDS image: 512 rows x 64 bf16 (128-B rows) = 64 KiB
constexpr int kRowBytes = 128;

// 16-B chunk swizzle of a 128-B row image: 16 distinct slots for every
// ds_read_b128 lane group, for 16-row (16x16x32) and 32-row (32x32x16) fragments
__device__ __forceinline__ int swz(int row, int c) { return c ^ ((row >> 1) & 7); }

__device__ __forceinline__ s16x8 rd(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const s16x8*>(lds + (row & (kRows - 1)) * kRowBytes + swz(row, chunk) * 16);
}

enum { REG = 0, LDS = 1, AL = 2 };

template <int SHAPE, int TM, int TN, int NW, int MODE>
__global__ void __launch_bounds__(64 * NW) mfma_loop(const short* __restrict__ src, float* out,
                                                      int nstep, int rowstep) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // fill the image with random bf16 (64 KiB per block)
  for (int i = tid; i < kRows * kRowBytes / 16; i += 64 * NW)
    reinterpret_cast<s16x8*>(lds)[i] = reinterpret_cast<const s16x8*>(src)[(blockIdx.x * 97 + i) & 8191];
  __syncthreads();
  constexpr int FR = SHAPE == 16 ? 16 : 32;            // fragment rows
  constexpr int KSUB = SHAPE == 16 ? 1 : 2;            // MFMAs along K per 32-deep step
  const int lr = lane % FR, kh = lane / FR;            // fragment row, k group
  const int abase = wid * 37 + lr, bbase = 256 + wid * 53 + lr;
  typedef typename std::conditional<SHAPE == 16, f32x4, f32x16>::type acc_t;
  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = acc_t{};
  s16x8 af[2][KSUB][TM], bf[2][KSUB][TN];
  auto load = [&](int st, int slot) {
    const int off = (st % 9) * rowstep;               // moves like a halo tap
#pragma unroll
    for (int k = 0; k < KSUB; ++k) {
      // 16x16x32: k group kh in 0..3 -> chunk kh (+4 for the second half of a
      // 128-B row); 32x32x16: k group kh in 0..1, sub-step k -> chunk 2k + kh
      const int ch = SHAPE == 16 ? kh + 4 * (st & 1) : 2 * k + kh + 4 * (st & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[slot][k][i] = rd(lds, abase + off + i * FR, ch);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[slot][k][j] = rd(lds, bbase + off + j * FR, ch);
    }
  };
  load(0, 0);
  for (int st = 0; st < nstep; st += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cur = h, nxt = h ^ 1;
      if (MODE == LDS) {
        load(st + h + 1, nxt);
      } else if (MODE == AL) {
        const int off = ((st + h + 1) % 9) * rowstep;
#pragma unroll
        for (int k = 0; k < KSUB; ++k) {
          const int ch = SHAPE == 16 ? kh + 4 * ((st + h + 1) & 1) : 2 * k + kh + 4 * ((st + h + 1) & 1);
#pragma unroll
          for (int i = 0; i < TM; ++i) af[nxt][k][i] = rd(lds, abase + off + i * FR, ch);
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bf[0][k][j]));
        }
      } else {
#pragma unroll
        for (int k = 0; k < KSUB; ++k) {
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[cur][k][i]));
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bf[cur][k][j]));
        }
      }
#pragma unroll
      for (int k = 0; k < KSUB; ++k)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const bf16x8_t a = __builtin_bit_cast(bf16x8_t, MODE != REG ? af[cur][k][i] : af[0][k][i]);
            const bf16x8_t b = __builtin_bit_cast(bf16x8_t, MODE == LDS ? bf[cur][k][j] : bf[0][k][j]);
            if constexpr (SHAPE == 16)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc[i][j], 0, 0, 0);
          }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < (SHAPE == 16 ? 4 : 16); ++r) s += acc[i][j][r];
  out[blockIdx.x * 64 * NW + tid] = s;
}

template <int SHAPE, int TM, int TN, int NW, int MODE>
void run(const char* name, const short* src, float* out, int bpc, int ncu, double clk_ghz) {
  const int nstep = 4096, rowstep = 35;
  auto k = mfma_loop<SHAPE, TM, TN, NW, MODE>;
  const size_t lds = kRows * kRowBytes;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int grid = ncu * bpc;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, 0, src, out, nstep, rowstep);
  CHECK(hipEventRecord(a));
  const int reps = 10;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, 0, src, out, nstep, rowstep);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double m = (SHAPE == 16 ? 16.0 : 32.0);
  const double flop = 2.0 * (m * TM) * (m * TN) * 32.0 * nstep * (double)grid * NW * reps;
  const double tf = flop / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD at the nominal clock: SIMD time / MFMAs it issued
  const double mf_per_simd = (double)nstep * TM * TN * (SHAPE == 16 ? 1 : 2) * NW * bpc / 4.0 * reps;
  const double cyc = (ms * 1e-3) * clk_ghz * 1e9 / mf_per_simd;
  std::printf("%-34s bpc %d  %8.1f TF/s  %5.1f %% of 2.5 PF  %6.2f cyc/MFMA@%.1fGHz (ideal %d)\n",
              name, bpc, tf, 100.0 * tf / 2500.0, cyc, clk_ghz, SHAPE == 16 ? 16 : 32);
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<short> h(8192 * 8);
  unsigned s = 12345u;
  for (auto& v : h) {   // uniform random bf16 in about [-1, 1)
    s = s * 1664525u + 1013904223u;
    const float f = ((s >> 8) & 0xffff) / 32768.0f - 1.0f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (short)(u >> 16);
  }
  short* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, (size_t)ncu * 2 * 512 * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const double clk = 2.4;
  std::printf("MFMA loop ceiling, %d CUs, random bf16, 4096 32-deep steps per wave\n", ncu);
  // the halo kernels' wave tiles, 16x16x32
  run<16, 4, 4, 4, LDS>("16x16x32 64x64 LDS  4 waves", src, out, 1, ncu, clk);
  run<16, 4, 4, 4, LDS>("16x16x32 64x64 LDS  4 waves", src, out, 2, ncu, clk);
  run<16, 2, 4, 8, LDS>("16x16x32 32x64 LDS  8 waves", src, out, 1, ncu, clk);
  run<16, 4, 4, 8, LDS>("16x16x32 64x64 LDS  8 waves", src, out, 1, ncu, clk);
  run<16, 8, 4, 4, LDS>("16x16x32 128x64 LDS 4 waves", src, out, 1, ncu, clk);
  run<16, 4, 4, 4, REG>("16x16x32 64x64 REG  4 waves", src, out, 1, ncu, clk);
  run<16, 4, 4, 8, REG>("16x16x32 64x64 REG  8 waves", src, out, 1, ncu, clk);
  // the same wave tiles on 32x32x16
  run<32, 2, 2, 4, LDS>("32x32x16 64x64 LDS  4 waves", src, out, 1, ncu, clk);
  run<32, 2, 2, 4, LDS>("32x32x16 64x64 LDS  4 waves", src, out, 2, ncu, clk);
  run<32, 1, 2, 8, LDS>("32x32x16 32x64 LDS  8 waves", src, out, 1, ncu, clk);
  run<32, 2, 2, 8, LDS>("32x32x16 64x64 LDS  8 waves", src, out, 1, ncu, clk);
  run<32, 4, 2, 4, LDS>("32x32x16 128x64 LDS 4 waves", src, out, 1, ncu, clk);
  run<32, 2, 2, 4, REG>("32x32x16 64x64 REG  4 waves", src, out, 1, ncu, clk);
  run<32, 2, 2, 8, REG>("32x32x16 64x64 REG  8 waves", src, out, 1, ncu, clk);
  // round 6: more reuse per LDS byte: 128x64 / 64x128
  // wave tiles at two waves per SIMD (8 waves, 128 fp32 accumulators per lane),
  // and one operand register-resident across the loop
  run<16, 8, 4, 8, LDS>("16x16x32 128x64 LDS 8 waves", src, out, 1, ncu, clk);
  run<32, 4, 2, 8, LDS>("32x32x16 128x64 LDS 8 waves", src, out, 1, ncu, clk);
  run<32, 2, 4, 8, LDS>("32x32x16 64x128 LDS 8 waves", src, out, 1, ncu, clk);
  run<16, 4, 4, 8, AL>("16x16x32 64x64 A-LDS B-REG 8 waves", src, out, 1, ncu, clk);
  run<16, 8, 4, 8, AL>("16x16x32 128x64 A-LDS B-REG 8 wv", src, out, 1, ncu, clk);
  run<32, 2, 2, 8, AL>("32x32x16 64x64 A-LDS B-REG 8 waves", src, out, 1, ncu, clk);
  run<32, 4, 2, 8, AL>("32x32x16 128x64 A-LDS B-REG 8 wv", src, out, 1, ncu, clk);
  run<32, 4, 2, 4, AL>("32x32x16 128x64 A-LDS B-REG 4 wv", src, out, 1, ncu, clk);
  // 128x128 wave tiles at ONE wave per SIMD (256 fp32 accumulators per lane in the
  // unified file): half the LDS bytes per FLOP of 128x64, no partner wave
  run<16, 8, 8, 4, LDS>("16x16x32 128x128 LDS 4 waves", src, out, 1, ncu, clk);
  run<32, 4, 4, 4, LDS>("32x32x16 128x128 LDS 4 waves", src, out, 1, ncu, clk);
  run<32, 4, 4, 4, REG>("32x32x16 128x128 REG 4 waves", src, out, 1, ncu, clk);
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
