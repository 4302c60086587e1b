// Host-side shape arithmetic and 32-bit offset guards shared by the PyTorch
// bindings (bindings.cpp) and the sanitizer driver (host_check.cpp, `make asan`).
//
// Every HIP kernel here addresses its operands through buffer descriptors with
// 32-bit BYTE offsets (num_records is a 32-bit field), so a tensor the kernels
// touch must stay under 2 GiB; these checks are the only thing standing between
// an oversize batch and a wrapped offset.  Plain C++ (no torch, no HIP) so the
// sanitizer build can drive them over every model's shape set, including the
// rejection paths, with -fsanitize=address,undefined.
#pragma once

#include <cstdint>

namespace dmp {
namespace guard {

constexpr int64_t kTwoGiB = int64_t(1) << 31;

// output extent of a convolution / pooling window; <= 0 when empty or invalid
inline int64_t conv_out(int64_t in, int64_t pad, int64_t k, int64_t stride) {
  if (stride < 1 || pad < 0 || k < 1 || in < 1) return 0;
  const int64_t span = in + 2 * pad - k;
  return span < 0 ? 0 : span / stride + 1;
}

// a value that must fit the kernels' `int` arguments
inline bool fits_int(int64_t v) { return v >= 0 && v < kTwoGiB; }

// scale * a * b * c * d < limit, every factor >= 0, without overflowing int64
// on the way (checked factor by factor)
inline bool prod_lt(int64_t limit, int64_t scale, int64_t a, int64_t b, int64_t c, int64_t d) {
  int64_t e = scale;
  for (int64_t f : {a, b, c, d}) {
    if (f < 0) return false;
    if (f != 0 && e > INT64_MAX / f) return false;
    e *= f;
  }
  return e < limit;
}

// bf16 NHWC tensor of n*h*w*c elements addressable with 32-bit byte offsets
inline bool bf16_bytes_ok(int64_t n, int64_t h, int64_t w, int64_t c) {
  return prod_lt(kTwoGiB, 2, n, h, w, c);
}

// implicit-GEMM conv (conv.hip / conv_wgrad.hip): input, output and weight
// all under 2 GiB of bf16 (1 << 30 elements) and every extent an int
inline bool conv_offsets_ok(int64_t B, int64_t H, int64_t W, int64_t CI, int64_t OH, int64_t OW,
                            int64_t CO, int64_t R, int64_t S) {
  for (int64_t v : {B, H, W, CI, OH, OW, CO, R, S})
    if (!fits_int(v)) return false;
  return bf16_bytes_ok(B, H, W, CI) && bf16_bytes_ok(B, OH, OW, CO) &&
         bf16_bytes_ok(CO, CI, R, S);
}

// few-input-channel stem convs (conv_small.hip): 32-bit ELEMENT indexing of the
// output, 2 GiB of input
inline bool small_conv_ok(int64_t B, int64_t OH, int64_t OW, int64_t CO, int64_t x_numel) {
  for (int64_t v : {B, OH, OW, CO})
    if (!fits_int(v)) return false;
  return prod_lt(kTwoGiB, 1, B, OH, OW, CO) && x_numel >= 0 && x_numel < (int64_t(1) << 30);
}

// ImageNet stem (stem.hip): the [B, H/2, W/2, 64] output under 2 GiB
inline bool stem_batch_ok(int64_t B, int64_t H, int64_t W) {
  return fits_int(B) && bf16_bytes_ok(B, H / 2, W / 2, 64);
}

// a row-major [rows][ld] operand of `elem`-byte elements (gemm.hip)
inline bool rows_bytes_ok(int64_t elem, int64_t rows, int64_t ld) {
  if (elem <= 0 || rows < 0 || ld < 0) return false;
  if (rows != 0 && ld > INT64_MAX / rows / elem) return false;
  return elem * rows * ld < kTwoGiB;
}

}  // namespace guard
}  // namespace dmp
