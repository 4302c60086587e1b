// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this package.
//
// Conventions used by every kernel file:
//   * wave = 64 lanes (hard-coded, never warpSize tricks from 32-lane hardware);
//   * bf16 is carried as raw `uint16_t` bits; f32 <-> bf16 via bit arithmetic
//     (round-to-nearest-even) so memory-bound kernels stay vectorised (16 B/lane);
//   * every launcher takes an explicit hipStream_t (graph-capturable: no malloc,
//     no sync inside launch functions).
#pragma once

#include <hip/hip_runtime.h>

#include "bn_slots.h"
#include <stdint.h>

namespace dmp {

constexpr int kWave = 64;

using u16 = uint16_t;
using u32 = uint32_t;
using u8 = uint8_t;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

struct alignas(16) bf16x8 { u16 v[8]; };
struct alignas(8) bf16x4 { u16 v[4]; };

// 512-thread workgroups put two waves on each SIMD; the second-dispatched half
// (waves 4-7) loses VALU-issue arbitration (priority, then age) on every
// segment.  One static s_setprio 1 for that half before the main loop, no
// per-segment flips (MI355X_MICROARCH.md "Two waves per SIMD", item 4).
// DMP_PRIO_YOUNG=0 at compile time for A/B.
#ifndef DMP_PRIO_YOUNG
#define DMP_PRIO_YOUNG 1
#endif
__device__ __forceinline__ void prio_young_half(int wid) {
  if (DMP_PRIO_YOUNG && wid >= 4) __builtin_amdgcn_s_setprio(1);
}

__device__ __forceinline__ float bf2f(u16 h) {
  return __uint_as_float(((u32)h) << 16);
}

// Round-to-nearest-even f32 -> bf16: a plain cast lowers to gfx950's
// v_cvt_pk_bf16_f32 (one instruction per pair, NaN-preserving), instead of
// the 5-instruction integer RNE sequence.
__device__ __forceinline__ u16 f2bf(float f) {
  return __builtin_bit_cast(u16, static_cast<__bf16>(f));
}

// tanh(u) = 1 - 2 / (1 + e^{2u}): one v_exp_f32 + one v_rcp_f32 instead of
// the ~30-instruction libm tanhf (the GELU pass was VALU-bound with it).
__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __expf(2.f * u);
  return 1.f - 2.f * __frcp_rn(1.f + e);
}

// tanh-approximated GELU; *dgelu (optional) receives d gelu / dx
__device__ __forceinline__ float gelu_tanh(float x, float* dgelu) {
  constexpr float c0 = 0.7978845608028654f, c1 = 0.044715f;
  const float x2 = x * x;
  const float u = c0 * x * (1.f + c1 * x2);
  const float t = fast_tanh(u);
  if (dgelu) {
    const float du = c0 * (1.f + 3.f * c1 * x2);
    *dgelu = 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
  }
  return 0.5f * x * (1.f + t);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Grid size for a grid-stride memory-bound kernel: enough blocks to fill
// 256 CUs several times over, capped (Guideline 11).
inline int stream_grid(long long work_items, int block) {
  long long g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

}  // namespace dmp

#define DMP_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      throw std::runtime_error(std::string("HIP error: ") +                   \
                               hipGetErrorString(_e) + " at " __FILE__ ":" + \
                               std::to_string(__LINE__));                     \
    }                                                                         \
  } while (0)
