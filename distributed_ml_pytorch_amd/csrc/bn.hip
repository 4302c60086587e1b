// Channels-last (NHWC) BatchNorm for training, with ReLU and residual-add fused.
//
// The reference models have no BatchNorm (/root/reference/example/models.py);
// it is needed by the BASELINE.json models (ResNet-18/50). Layout is [M, C]
// bf16 with M = N*H*W, every thread owning 8 consecutive channels (16 B).
//
// forward  : stats (per-block sums added into kBnSlots slot rows) -> finalize
//            (mean/invstd, running stats, folded scale/shift; re-zeroes the
//            slots) -> apply  y = relu(x*scale + shift [+ res])
// backward : reduce (sum dz, sum dz*xhat with dz = dy*[y>0]) -> finalize
//            (dgamma/dbeta accumulated straight into the fp32 grad arena, folded
//            dx coefficients) -> apply  dx = A*dz + Cc*x + Bc  [and dres = dz]
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace dmp {

__device__ __forceinline__ void load8(const u16* p, float v[8]) {
  const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = bf2f(r.v[k]);
}

__device__ __forceinline__ void store8(u16* p, const float v[8]) {
  bf16x8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = f2bf(v[k]);
  *reinterpret_cast<bf16x8*>(p) = r;
}

// Streaming loads / stores with an optional non-temporal hint (NT bit 1: loads,
// bit 2: stores; DMP_BN_NT, measured per shape in profiles/bn_nt_policy_r6.txt)
typedef unsigned bn_u32x4 __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ bf16x8 bn_ldv(const u16* p) {
  if constexpr ((NT & 1) != 0) {
    return __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(reinterpret_cast<const bn_u32x4*>(p)));
  } else {
    return *reinterpret_cast<const bf16x8*>(p);
  }
}
template <int NT>
__device__ __forceinline__ void bn_stv(u16* p, const bf16x8& r) {
  if constexpr ((NT & 2) != 0) {
    __builtin_nontemporal_store(__builtin_bit_cast(bn_u32x4, r), reinterpret_cast<bn_u32x4*>(p));
  } else {
    *reinterpret_cast<bf16x8*>(p) = r;
  }
}
template <int NT>
__device__ __forceinline__ void bn_st8(u16* p, const float v[8]) {
  bf16x8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = f2bf(v[k]);
  bn_stv<NT>(p, r);
}

// Pre-activation of the forward apply, shared by the forward and the backward's
// ReLU-mask recomputation so both round identically (explicit fma).
__device__ __forceinline__ float bn_pre(float x, float sc, float sh) { return __fmaf_rn(x, sc, sh); }

// ReLU mask source of the backward: 0 = no ReLU, 1 = from the saved output y
// (BN + residual + ReLU: the mask depends on the residual), 2 = recomputed from
// x and the folded scale/shift in stats (no residual): one tensor read fewer in
// both backward passes, 3 = a 1-bit-per-element mask the forward apply wrote
// beside y (BN + residual + ReLU): 1/16 of y's bytes in both backward passes.
// Mask layout: one byte per 8-channel vector (bit k = channel c0 + k), i.e.
// [M][C/8] bytes, the thread<->vector mapping of every kernel here.
__device__ __forceinline__ void relu_mask_bits(unsigned bits, float g[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) g[k] = (bits >> k) & 1u ? g[k] : 0.f;
}
__device__ __forceinline__ void relu_mask_from_x(const float xv[8], const float* __restrict__ stats,
                                                 int C, int c0, float g[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float y = fmaxf(bn_pre(xv[k], stats[2 * C + c0 + k], stats[3 * C + c0 + k]), 0.f);
    g[k] = bf2f(f2bf(y)) > 0.f ? g[k] : 0.f;   // exactly the y > 0 test on the stored y
  }
}

// -------- per-block channel partial sums --------------------------------
// MODE 0: s += x, q += x*x                       (forward statistics)
// MODE 1: s += dz, q += dz*(x-mean)*invstd        (backward reduction)
template <int MODE, int RELU, int NT = 0>
__global__ void __launch_bounds__(256) bn_partial_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const u16* __restrict__ y,
    const uint8_t* __restrict__ mask, const float* __restrict__ stats, float* __restrict__ part,
    long long M, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tpr = C >> 3;
  const int rpi = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const long long rows_per_blk = (M + gridDim.x - 1) / gridDim.x;
  const long long start = (long long)blockIdx.x * rows_per_blk;
  const long long end = min(M, start + rows_per_blk);
  float s[8], q[8], mean[8], inv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  if (MODE == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { mean[k] = stats[cg * 8 + k]; inv[k] = stats[C + cg * 8 + k]; }
  }
  auto accum = [&](const float xv[8], float g[8]) {
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += xv[k]; q[k] += xv[k] * xv[k]; }
    } else {
      if (RELU == 2) relu_mask_from_x(xv, stats, C, cg * 8, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += g[k]; q[k] += g[k] * (xv[k] - mean[k]) * inv[k]; }
    }
  };
  // 4 rows per trip with every load issued before any is consumed: the
  // one-row loop kept ~2 loads in flight per lane and ran at ~2.5 TB/s
  // (ResNet-50 bs128, gpurun_out/mprof/steady_resnet50.txt)
  constexpr int U = 4;
  if (r0 < rpi) {
    long long row = start + r0;
    for (; row + (U - 1) * rpi < end; row += U * rpi) {
      bf16x8 xr[U], dr[U], yr[U];
      unsigned mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long off = (row + u * rpi) * C + cg * 8;
        xr[u] = bn_ldv<NT>(x + off);
        if (MODE == 1) dr[u] = bn_ldv<NT>(dy + off);
        if (MODE == 1 && RELU == 1) yr[u] = bn_ldv<NT>(y + off);
        if (MODE == 1 && RELU == 3) mb[u] = mask[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float xv[8], g[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xv[k] = bf2f(xr[u].v[k]);
          g[k] = MODE == 1 ? bf2f(dr[u].v[k]) : 0.f;
          if (MODE == 1 && RELU == 1) g[k] = bf2f(yr[u].v[k]) > 0.f ? g[k] : 0.f;
        }
        if (MODE == 1 && RELU == 3) relu_mask_bits(mb[u], g);
        accum(xv, g);
      }
    }
    for (; row < end; row += rpi) {
      const long long off = row * C + cg * 8;
      float xv[8], g[8];
      load8(x + off, xv);
      if (MODE == 1) {
        load8(dy + off, g);
        if (RELU == 1) {
          float yv[8];
          load8(y + off, yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
        }
        if (RELU == 3) relu_mask_bits(mask[off >> 3], g);
      }
      accum(xv, g);
    }
  }
  // LDS reduce over the rpi row-lanes that share a channel group.
  float* ls = smem;            // [rpi][C]
  float* lq = smem + rpi * C;  // [rpi][C]
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { ls[r0 * C + cg * 8 + k] = s[k]; lq[r0 * C + cg * 8 + k] = q[k]; }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpi; ++r) { a += ls[r * C + c]; b += lq[r * C + c]; }
    const int slot = blockIdx.x % kBnSlots;
    atomicAdd(part + (long long)slot * C + c, a);
    atomicAdd(part + (long long)(kBnSlots + slot) * C + c, b);
  }
}

// -------- forward finalize: stats = [mean | invstd | scale | shift] -------
// Block = 64 channels x 16 partial-slices (1024 threads): coalesced loads of
// the [G][C] partial arrays, LDS tree over the slices.
// Reads the [2][G][C] slot sums of channel c and zeroes them (the slots are
// persistent and accumulated into by the next producer).
__device__ __forceinline__ void reduce_partials(float* __restrict__ part, int G, int C,
                                                int c, float& S, float& Q) {
  __shared__ float rs[16][64], rq[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // 4 independent accumulator pairs keep 8 loads in flight per thread (the
  // partial arrays come from conv epilogues with up to a few thousand blocks)
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  if (c < C) {
    float* ps = part + c;
    float* pq = part + (long long)G * C + c;
    int g = ty;
    for (; g + 48 < G; g += 64) {
      a0 += ps[(long long)g * C];        b0 += pq[(long long)g * C];
      a1 += ps[(long long)(g + 16) * C]; b1 += pq[(long long)(g + 16) * C];
      a2 += ps[(long long)(g + 32) * C]; b2 += pq[(long long)(g + 32) * C];
      a3 += ps[(long long)(g + 48) * C]; b3 += pq[(long long)(g + 48) * C];
    }
    for (; g < G; g += 16) { a0 += ps[(long long)g * C]; b0 += pq[(long long)g * C]; }
    for (g = ty; g < G; g += 16) { ps[(long long)g * C] = 0.f; pq[(long long)g * C] = 0.f; }
  }
  const float a = (a0 + a1) + (a2 + a3), b = (b0 + b1) + (b2 + b3);
  rs[ty][tx] = a;
  rq[ty][tx] = b;
  __syncthreads();
  if (ty == 0) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) { sa += rs[k][tx]; sb += rq[k][tx]; }
    S = sa;
    Q = sb;
  }
}

__global__ void __launch_bounds__(1024) bn_fwd_finalize_kernel(
    float* __restrict__ part, int G, long long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ running_mean,
    float* __restrict__ running_var, float momentum, float eps, float* __restrict__ stats,
    int use_running) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float S = 0.f, Q = 0.f;
  if (!use_running) reduce_partials(part, G, C, c, S, Q);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  float mean, var;
  if (use_running) {
    mean = running_mean[c];
    var = running_var[c];
  } else {
    mean = S / (float)M;
    var = fmaxf(Q / (float)M - mean * mean, 0.f);
    if (running_mean) {
      const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
    }
  }
  const float inv = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  const float sc = g * inv;
  stats[c] = mean;
  stats[C + c] = inv;
  stats[2 * C + c] = sc;
  stats[3 * C + c] = b - mean * sc;
}

// -------- forward apply --------------------------------------------------
template <bool RELU, bool RES, bool MASK = false>
__global__ void __launch_bounds__(256) bn_apply_kernel(
    const u16* __restrict__ x, const u16* __restrict__ res, const float* __restrict__ stats,
    u16* __restrict__ y, long long nvec, int C, uint8_t* __restrict__ mask = nullptr) {
  const int tpr = C >> 3;
  const float* scale = stats + 2 * C;
  const float* shift = stats + 3 * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % tpr) * 8;
    float xv[8];
    load8(x + v * 8, xv);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = bn_pre(xv[k], scale[c0 + k], shift[c0 + k]);
    if (RES) {
      float rv[8];
      load8(res + v * 8, rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] += rv[k];
    }
    if (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaxf(o[k], 0.f);
    }
    if (MASK) {
      bf16x8 r;
      unsigned bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        r.v[k] = f2bf(o[k]);
        bits |= (r.v[k] != 0 ? 1u : 0u) << k;   // the stored y > 0 (y >= 0 after the ReLU)
      }
      *reinterpret_cast<bf16x8*>(y + v * 8) = r;
      mask[v] = (uint8_t)bits;
    } else {
      store8(y + v * 8, o);
    }
  }
}

// -------- backward finalize: coef = [A | Bc | Cc] -----------------------------
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(
    float* __restrict__ part, int G, long long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ stats, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ coef) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float S = 0.f, Q = 0.f;
  reduce_partials(part, G, C, c, S, Q);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  const float db = S;   // sum dz
  const float dg = Q;   // sum dz * xhat
  if (dgamma) dgamma[c] += dg;
  if (dbeta) dbeta[c] += db;
  const float mean = stats[c], inv = stats[C + c];
  const float k1 = (gamma ? gamma[c] : 1.f) * inv;
  const float invM = 1.f / (float)M;
  // dx = k1*(dz - db/M - xhat*dg/M), xhat = (x-mean)*inv
  const float Cc = -k1 * inv * dg * invM;
  const float Bc = -k1 * db * invM - Cc * mean;
  coef[c] = k1;
  coef[C + c] = Bc;
  coef[2 * C + c] = Cc;
}

template <int RELU, bool WRITE_DRES>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const u16* __restrict__ y,
    const uint8_t* __restrict__ mask, const float* __restrict__ coef,
    const float* __restrict__ stats, u16* __restrict__ dx, u16* __restrict__ dres,
    long long nvec, int C) {
  const int tpr = C >> 3;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % tpr) * 8;
    float xv[8], g[8];
    load8(x + v * 8, xv);
    load8(dy + v * 8, g);
    if (RELU == 1) {
      float yv[8];
      load8(y + v * 8, yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
    } else if (RELU == 2) {
      relu_mask_from_x(xv, stats, C, c0, g);
    } else if (RELU == 3) {
      relu_mask_bits(mask[v], g);
    }
    if (WRITE_DRES) store8(dres + v * 8, g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = coef[c0 + k] * g[k] + coef[2 * C + c0 + k] * xv[k] + coef[C + c0 + k];
    store8(dx + v * 8, o);
  }
}

// ---------------------------------------------------------------- launchers
int bn_num_partials(long long M, int C) {
  // DMP_BN_PART_VPT / DMP_BN_PART_CAP: A/B knobs of the reduce grid
  static const long long vpt = [] {
    const char* e = std::getenv("DMP_BN_PART_VPT");
    return e ? std::max(1, std::atoi(e)) : 8;
  }();
  static const long long cap = [] {
    const char* e = std::getenv("DMP_BN_PART_CAP");
    return e ? std::max(1, std::atoi(e)) : 2048;
  }();
  long long vecs = M * (C / 8);
  long long g = vecs / (256 * vpt);   // >= 8 rows (two 4-row trips) per thread
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  if (g > M) g = M;
  return (int)g;
}

// forward apply; mask != nullptr (relu only) also writes the 1-bit ReLU mask
static void bn_apply(const u16* x, const u16* res, const float* stats, u16* y, uint8_t* mask,
                     long long M, int C, bool relu, hipStream_t s) {
  const long long nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, 256));
  if (relu && mask) {
    if (res) hipLaunchKernelGGL((bn_apply_kernel<true, true, true>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, mask);
    else hipLaunchKernelGGL((bn_apply_kernel<true, false, true>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, mask);
  } else if (relu) {
    if (res) hipLaunchKernelGGL((bn_apply_kernel<true, true>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, nullptr);
    else hipLaunchKernelGGL((bn_apply_kernel<true, false>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, nullptr);
  } else {
    if (res) hipLaunchKernelGGL((bn_apply_kernel<false, true>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, nullptr);
    else hipLaunchKernelGGL((bn_apply_kernel<false, false>), grid, dim3(256), 0, s, x, res, stats, y, nvec, C, nullptr);
  }
}

void launch_bn_fwd(const u16* x, const u16* res, u16* y, const float* gamma, const float* beta,
                   float* running_mean, float* running_var, float* stats, float* part,
                   long long M, int C, float momentum, float eps, bool training, bool relu,
                   hipStream_t s, uint8_t* mask) {
  const int G = bn_num_partials(M, C);
  const int rpi = 256 / (C / 8);
  const size_t lds = (size_t)rpi * C * 2 * sizeof(float);
  if (training) {
    hipLaunchKernelGGL((bn_partial_kernel<0, 0>), dim3(G), dim3(256), lds, s, x, nullptr,
                       nullptr, nullptr, nullptr, part, M, C);
  }
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, part,
                     kBnSlots, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                     stats, training ? 0 : 1);
  bn_apply(x, res, stats, y, mask, M, C, relu, s);
}

// ReLU mask of the backward: the 1-bit mask when given, else y, else (no
// residual in the forward) recomputed from x.
void launch_bn_bwd(const u16* x, const u16* dy, const u16* y, const float* gamma,
                   const float* stats, float* dgamma, float* dbeta, float* coef, float* part,
                   u16* dx, u16* dres, long long M, int C, bool relu, hipStream_t s,
                   const uint8_t* mask) {
  const int G = bn_num_partials(M, C);
  const int rpi = 256 / (C / 8);
  const size_t lds = (size_t)rpi * C * 2 * sizeof(float);
  const int mode = !relu ? 0 : (mask ? 3 : (y ? 1 : 2));
#define DMP_BN_PART(R)                                                                          \
  hipLaunchKernelGGL((bn_partial_kernel<1, R>), dim3(G), dim3(256), lds, s, x, dy, y, mask, stats, \
                     part, M, C)
  if (mode == 0) DMP_BN_PART(0);
  else if (mode == 1) DMP_BN_PART(1);
  else if (mode == 2) DMP_BN_PART(2);
  else DMP_BN_PART(3);
#undef DMP_BN_PART
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, part,
                     kBnSlots, M, C, gamma, stats, dgamma, dbeta, coef);
  const long long nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, 256));
#define DMP_BN_BAPPLY(R, D)                                                                   \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<R, D>), grid, dim3(256), 0, s, x, dy, y, mask, coef, \
                     stats, dx, dres, nvec, C)
  if (dres) {
    if (mode == 0) DMP_BN_BAPPLY(0, true);
    else if (mode == 1) DMP_BN_BAPPLY(1, true);
    else if (mode == 2) DMP_BN_BAPPLY(2, true);
    else DMP_BN_BAPPLY(3, true);
  } else {
    if (mode == 0) DMP_BN_BAPPLY(0, false);
    else if (mode == 1) DMP_BN_BAPPLY(1, false);
    else if (mode == 2) DMP_BN_BAPPLY(2, false);
    else DMP_BN_BAPPLY(3, false);
  }
#undef DMP_BN_BAPPLY
}


// -------- finalize folded into the apply passes --------------------------------
// The separate 1-block finalize launches (one forward + one backward per BN:
// 40 per ResNet-18 step, 106 per ResNet-50 step, each a dependent ~5 us dispatch
// on the critical path) disappear: every apply block reduces the kBnSlots slot
// sums of ITS channel slice itself (grid.y = C / CS slices of CS channels, so a
// block reads CS x 128 floats from L2, never all C) and derives the folded
// coefficients in LDS; all blocks of a slice run the same reduction in the same
// order, so they agree bit for bit.  Row-block 0 of each slice publishes
// stats / running stats (forward) or accumulates dgamma / dbeta (backward).
// The slots can no longer be re-zeroed by their reader (other blocks may still
// be reading), so each apply zeroes the OTHER direction's slots of the same
// layer, whose reader finished earlier: the forward apply zeroes the backward
// slots (read by the previous backward apply), the backward apply zeroes the
// forward slots (read by this step's forward apply).  The host tracks the
// leftovers of an unpaired pass (forward without backward) and zeroes them
// eagerly (ops/functional.py).
template <int CS>
__device__ __forceinline__ void slice_slot_sums(const float* __restrict__ part, int C, int cs0,
                                                float* __restrict__ lS, float* __restrict__ lQ) {
  constexpr int NG = 256 / CS;          // thread groups splitting the slots
  constexpr int PER = kBnSlots / NG;    // slots per thread (all loads independent)
  static_assert(kBnSlots % NG == 0, "slot split");
  __shared__ float rs[256], rq[256];
  const int t = threadIdx.x, ch = t % CS, grp = t / CS;
  const float* ps = part + cs0 + ch;
  const float* pq = part + (long long)kBnSlots * C + cs0 + ch;
  float a[PER], b[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    a[i] = ps[(long long)(grp + i * NG) * C];
    b[i] = pq[(long long)(grp + i * NG) * C];
  }
  float sa = 0.f, sb = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) { sa += a[i]; sb += b[i]; }
  rs[t] = sa;
  rq[t] = sb;
  __syncthreads();
  if (t < CS) {
    float ta = 0.f, tb = 0.f;
#pragma unroll
    for (int k = 0; k < NG; ++k) { ta += rs[k * CS + t]; tb += rq[k * CS + t]; }
    lS[t] = ta;
    lQ[t] = tb;
  }
}

// zero the [2][kBnSlots] rows of this block's channel slice in `zb` (rows spread
// over the slice's row blocks)
template <int CS>
__device__ __forceinline__ void slice_zero(float* __restrict__ zb, int C, int cs0) {
  if (zb == nullptr || threadIdx.x >= CS) return;
  for (int r = blockIdx.x; r < 2 * kBnSlots; r += gridDim.x)
    zb[(long long)r * C + cs0 + threadIdx.x] = 0.f;
}

// Forward prologue of a folded apply block: the slice's scale / shift into lS /
// lQ (M = the statistics' row count); block 0 publishes stats and the running
// statistics.  Ends with a barrier.
template <int CS>
__device__ __forceinline__ void fold_fwd_coefs(const float* __restrict__ part,
                                               float* __restrict__ zero_buf,
                                               const float* __restrict__ gamma,
                                               const float* __restrict__ beta,
                                               float* __restrict__ running_mean,
                                               float* __restrict__ running_var, float momentum,
                                               float eps, float* __restrict__ stats, long long M,
                                               int C, int cs0, float* lS, float* lQ) {
  const int t = threadIdx.x;
  slice_slot_sums<CS>(part, C, cs0, lS, lQ);
  if (t < CS) {   // same thread wrote lS[t] / lQ[t]: no barrier needed before the reuse
    const int c = cs0 + t;
    const float mean = lS[t] / (float)M;
    const float var = fmaxf(lQ[t] / (float)M - mean * mean, 0.f);
    const float inv = rsqrtf(var + eps);
    const float sc = (gamma ? gamma[c] : 1.f) * inv;
    const float sh = (beta ? beta[c] : 0.f) - mean * sc;
    if (blockIdx.x == 0) {
      stats[c] = mean;
      stats[C + c] = inv;
      stats[2 * C + c] = sc;
      stats[3 * C + c] = sh;
      if (running_mean) {
        const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
      }
    }
    lS[t] = sc;
    lQ[t] = sh;
  }
  slice_zero<CS>(zero_buf, C, cs0);
  __syncthreads();
}

template <int CS, bool RELU, bool RES, bool MASK, int NT = 0>
__global__ void __launch_bounds__(256) bn_apply_fold_kernel(
    const u16* __restrict__ x, const u16* __restrict__ res, const float* __restrict__ part,
    float* __restrict__ zero_buf, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps,
    float* __restrict__ stats, u16* __restrict__ y, uint8_t* __restrict__ mask, long long M,
    int C) {
  __shared__ float lS[CS], lQ[CS];
  const int t = threadIdx.x;
  const int cs0 = blockIdx.y * CS;
  fold_fwd_coefs<CS>(part, zero_buf, gamma, beta, running_mean, running_var, momentum, eps, stats,
                     M, C, cs0, lS, lQ);
  constexpr int TPR = CS / 8, RPI = 256 / TPR;
  const int cg = t % TPR, r0 = t / TPR;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = lS[cg * 8 + k]; sh[k] = lQ[cg * 8 + k]; }
  const long long rows_per_blk = (M + gridDim.x - 1) / gridDim.x;
  const long long start = (long long)blockIdx.x * rows_per_blk;
  const long long end = min(M, start + rows_per_blk);
  auto one = [&](const bf16x8& xr, const bf16x8& rr, long long off) {
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = bn_pre(bf2f(xr.v[k]), sc[k], sh[k]);
      if (RES) o[k] += bf2f(rr.v[k]);
      if (RELU) o[k] = fmaxf(o[k], 0.f);
    }
    if (MASK) {
      bf16x8 r;
      unsigned bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        r.v[k] = f2bf(o[k]);
        bits |= (r.v[k] != 0 ? 1u : 0u) << k;
      }
      bn_stv<NT>(y + off, r);
      mask[off >> 3] = (uint8_t)bits;
    } else {
      bn_st8<NT>(y + off, o);
    }
  };
  constexpr int U = 4;
  long long row = start + r0;
  const int cofs = cs0 + cg * 8;
  for (; row + (U - 1) * RPI < end; row += U * RPI) {
    bf16x8 xr[U], rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long off = (row + u * RPI) * C + cofs;
      xr[u] = bn_ldv<NT>(x + off);
      if (RES) rr[u] = bn_ldv<NT>(res + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(xr[u], rr[u], (row + u * RPI) * C + cofs);
  }
  for (; row < end; row += RPI) {
    const long long off = row * C + cofs;
    bf16x8 xr = *reinterpret_cast<const bf16x8*>(x + off), rr;
    if (RES) rr = *reinterpret_cast<const bf16x8*>(res + off);
    one(xr, rr, off);
  }
}

// Backward prologue of a folded apply block: dx = lS * dz + lC * x + lQ for the
// slice; block 0 accumulates dgamma / dbeta.  Ends with a barrier.
template <int CS>
__device__ __forceinline__ void fold_bwd_coefs(const float* __restrict__ part,
                                               float* __restrict__ zero_buf,
                                               const float* __restrict__ gamma,
                                               const float* __restrict__ stats,
                                               float* __restrict__ dgamma,
                                               float* __restrict__ dbeta, long long M, int C,
                                               int cs0, float* lS, float* lQ, float* lC) {
  const int t = threadIdx.x;
  slice_slot_sums<CS>(part, C, cs0, lS, lQ);
  if (t < CS) {
    const int c = cs0 + t;
    const float db = lS[t];   // sum dz
    const float dg = lQ[t];   // sum dz * xhat
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] += dg;
      if (dbeta) dbeta[c] += db;
    }
    const float mean = stats[c], inv = stats[C + c];
    const float k1 = (gamma ? gamma[c] : 1.f) * inv;
    const float invM = 1.f / (float)M;
    const float Cc = -k1 * inv * dg * invM;
    lS[t] = k1;
    lQ[t] = -k1 * db * invM - Cc * mean;
    lC[t] = Cc;
  }
  slice_zero<CS>(zero_buf, C, cs0);
  __syncthreads();
}

template <int CS, int RELU, bool WRITE_DRES, int NT = 0>
__global__ void __launch_bounds__(256) bn_bwd_apply_fold_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const u16* __restrict__ y,
    const uint8_t* __restrict__ mask, const float* __restrict__ part,
    float* __restrict__ zero_buf, const float* __restrict__ gamma,
    const float* __restrict__ stats, float* __restrict__ dgamma, float* __restrict__ dbeta,
    u16* __restrict__ dx, u16* __restrict__ dres, long long M, int C) {
  __shared__ float lS[CS], lQ[CS], lC[CS];
  const int t = threadIdx.x;
  const int cs0 = blockIdx.y * CS;
  fold_bwd_coefs<CS>(part, zero_buf, gamma, stats, dgamma, dbeta, M, C, cs0, lS, lQ, lC);
  constexpr int TPR = CS / 8, RPI = 256 / TPR;
  const int cg = t % TPR, r0 = t / TPR;
  const int cofs = cs0 + cg * 8;
  float ka[8], kb[8], kc[8], msc[8], msh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ka[k] = lS[cg * 8 + k];
    kb[k] = lQ[cg * 8 + k];
    kc[k] = lC[cg * 8 + k];
    if (RELU == 2) { msc[k] = stats[2 * C + cofs + k]; msh[k] = stats[3 * C + cofs + k]; }
  }
  const long long rows_per_blk = (M + gridDim.x - 1) / gridDim.x;
  const long long start = (long long)blockIdx.x * rows_per_blk;
  const long long end = min(M, start + rows_per_blk);
  auto one = [&](const bf16x8& xr, const bf16x8& dr, const bf16x8& yr, unsigned mb,
                 long long off) {
    float xv[8], g[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xv[k] = bf2f(xr.v[k]);
      g[k] = bf2f(dr.v[k]);
      if (RELU == 1) g[k] = bf2f(yr.v[k]) > 0.f ? g[k] : 0.f;
      if (RELU == 2) {
        const float yy = fmaxf(bn_pre(xv[k], msc[k], msh[k]), 0.f);
        g[k] = bf2f(f2bf(yy)) > 0.f ? g[k] : 0.f;
      }
    }
    if (RELU == 3) relu_mask_bits(mb, g);
    if (WRITE_DRES) bn_st8<NT>(dres + off, g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = ka[k] * g[k] + kc[k] * xv[k] + kb[k];
    bn_st8<NT>(dx + off, o);
  };
  constexpr int U = 4;
  long long row = start + r0;
  for (; row + (U - 1) * RPI < end; row += U * RPI) {
    bf16x8 xr[U], dr[U], yr[U];
    unsigned mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long off = (row + u * RPI) * C + cofs;
      xr[u] = bn_ldv<NT>(x + off);
      dr[u] = bn_ldv<NT>(dy + off);
      if (RELU == 1) yr[u] = bn_ldv<NT>(y + off);
      if (RELU == 3) mb[u] = mask[off >> 3];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(xr[u], dr[u], yr[u], mb[u], (row + u * RPI) * C + cofs);
  }
  for (; row < end; row += RPI) {
    const long long off = row * C + cofs;
    bf16x8 xr = *reinterpret_cast<const bf16x8*>(x + off);
    bf16x8 dr = *reinterpret_cast<const bf16x8*>(dy + off), yr;
    unsigned mb = 0;
    if (RELU == 1) yr = *reinterpret_cast<const bf16x8*>(y + off);
    if (RELU == 3) mb = mask[off >> 3];
    one(xr, dr, yr, mb, off);
  }
}

// -------- one-pass backward: reduce -> device-wide hand-off -> apply ----------
// The folded backward above is two launches per BatchNorm (bn_partial_kernel,
// then bn_bwd_apply_fold_kernel).  Here ONE launch of G blocks (G <= what the
// device holds at once: every block must be resident, see the host) does both:
//   1. each block reduces sum dz / sum dz*xhat over ITS rows [start, end) into
//      the kBnSlots slot sums (device-scope atomics, memory side);
//   2. arrival ticket (agent-scope release + atomic add on the slot buffer's
//      tail word 0); the LAST block to arrive (acquire) folds the slot sums into
//      the dx coefficients [3][C] (coef), accumulates dgamma / dbeta, then
//      publishes tail word 1 = 1 (release); the others poll it (acquire);
//   3. every block applies dx = k1*dz + Cc*x + kb to the SAME rows it reduced --
//      re-read from L2 / the Infinity Cache a moment after phase 1 streamed them.
// Tail words reset for the next call: word 0 by the last arriver before it
// releases, word 1 by the last block to depart (tail word 2 counts departures),
// so the slot buffer's tail is zero again when the kernel ends.  The poll is
// bounded (~0.1 s): a grid that could not be co-resident ends with wrong dx
// instead of hanging the GPU, and sets tail word 3 (a test reads it).
// Slot hygiene as in the fold kernels: the forward slots (zero_buf) are zeroed
// here, the backward slots by the next forward apply.
template <int RELU, bool WRITE_DRES>
__global__ void __launch_bounds__(256) bn_bwd_onepass_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, const u16* __restrict__ y,
    const uint8_t* __restrict__ mask, float* __restrict__ part, float* __restrict__ zero_buf,
    const float* __restrict__ gamma, const float* __restrict__ stats, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ coef, u16* __restrict__ dx,
    u16* __restrict__ dres, long long M, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int last_flag;
  const int tpr = C >> 3, rpi = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, r0 = t / tpr;
  const int G = gridDim.x;
  const long long rows_per_blk = (M + G - 1) / G;
  const long long start = (long long)blockIdx.x * rows_per_blk;
  const long long end = min(M, start + rows_per_blk);
  int* tail = reinterpret_cast<int*>(part + 2LL * kBnSlots * C);
  const int c0 = cg * 8;
  float msc[8], msh[8];
  if (RELU == 2) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      msc[k] = r0 < rpi ? stats[2 * C + c0 + k] : 0.f;
      msh[k] = r0 < rpi ? stats[3 * C + c0 + k] : 0.f;
    }
  }
  // dz of 8 channels from the loaded vectors (ReLU mask by mode)
  auto dz8 = [&](const bf16x8& xr, const bf16x8& dr, const bf16x8& yr, unsigned mb, float xv[8],
                 float g[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xv[k] = bf2f(xr.v[k]);
      g[k] = bf2f(dr.v[k]);
      if (RELU == 1) g[k] = bf2f(yr.v[k]) > 0.f ? g[k] : 0.f;
      if (RELU == 2) {
        const float yy = fmaxf(bn_pre(xv[k], msc[k], msh[k]), 0.f);
        g[k] = bf2f(f2bf(yy)) > 0.f ? g[k] : 0.f;
      }
    }
    if (RELU == 3) relu_mask_bits(mb, g);
  };
  constexpr int U = 4;
  auto load_rows = [&](long long row, bf16x8 (&xr)[U], bf16x8 (&dr)[U], bf16x8 (&yr)[U],
                       unsigned (&mb)[U], int nu) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < nu) {
        const long long off = (row + u * rpi) * C + c0;
        xr[u] = *reinterpret_cast<const bf16x8*>(x + off);
        dr[u] = *reinterpret_cast<const bf16x8*>(dy + off);
        if (RELU == 1) yr[u] = *reinterpret_cast<const bf16x8*>(y + off);
        if (RELU == 3) mb[u] = mask[off >> 3];
      }
    }
  };
  // ---- phase 1: this block's partial sums
  {
    float s[8], q[8], mean[8], inv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[k] = 0.f;
      q[k] = 0.f;
      mean[k] = r0 < rpi ? stats[c0 + k] : 0.f;
      inv[k] = r0 < rpi ? stats[C + c0 + k] : 0.f;
    }
    if (r0 < rpi) {
      for (long long row = start + r0; row < end; row += U * rpi) {
        const int nu = (int)min<long long>(U, (end - row + rpi - 1) / rpi);
        bf16x8 xr[U], dr[U], yr[U];
        unsigned mb[U];
        load_rows(row, xr, dr, yr, mb, nu);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < nu) {
            float xv[8], g[8];
            dz8(xr[u], dr[u], yr[u], mb[u], xv, g);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              s[k] += g[k];
              q[k] += g[k] * (xv[k] - mean[k]) * inv[k];
            }
          }
        }
      }
    }
    float* ls = smem;            // [rpi][C]
    float* lq = smem + rpi * C;  // [rpi][C]
    if (r0 < rpi) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { ls[r0 * C + c0 + k] = s[k]; lq[r0 * C + c0 + k] = q[k]; }
    }
    __syncthreads();
    const int slot = blockIdx.x % kBnSlots;
    for (int c = t; c < C; c += 256) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < rpi; ++r) { a += ls[r * C + c]; b += lq[r * C + c]; }
      atomicAdd(part + (long long)slot * C + c, a);
      atomicAdd(part + (long long)(kBnSlots + slot) * C + c, b);
    }
  }
  // the forward slots this layer's forward apply consumed: zero (rows spread)
  if (zero_buf != nullptr)
    for (long long e = (long long)blockIdx.x * 256 + t; e < 2LL * kBnSlots * C; e += 256LL * G)
      zero_buf[e] = 0.f;
  // ---- phase 2: arrival; the last block folds the sums into the coefficients
  __syncthreads();   // every thread's slot atomics are issued
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int ticket = __hip_atomic_fetch_add(tail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = ticket == G - 1;
  }
  __syncthreads();
  if (last_flag) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const float invM = 1.f / (float)M;
    for (int c = t; c < C; c += 256) {
      float db = 0.f, dg = 0.f;
      // plain loads after the acquire (independent, so they pipeline; atomic
      // loads here serialised into one round trip each)
      float a[kBnSlots], b[kBnSlots];
#pragma unroll
      for (int sl = 0; sl < kBnSlots; ++sl) {
        a[sl] = part[(long long)sl * C + c];
        b[sl] = part[(long long)(kBnSlots + sl) * C + c];
      }
#pragma unroll
      for (int sl = 0; sl < kBnSlots; ++sl) { db += a[sl]; dg += b[sl]; }
      if (dgamma) dgamma[c] += dg;
      if (dbeta) dbeta[c] += db;
      const float mean = stats[c], inv = stats[C + c];
      const float k1 = (gamma ? gamma[c] : 1.f) * inv;
      const float Cc = -k1 * inv * dg * invM;
      coef[c] = k1;
      coef[C + c] = -k1 * db * invM - Cc * mean;
      coef[2 * C + c] = Cc;
    }
    __syncthreads();
    if (t == 0) {
      __hip_atomic_store(tail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(tail + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (t == 0) {
    int it = 0;
    while (__hip_atomic_load(tail + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > (1 << 22)) {
        // never co-resident (CUs taken by another stream's kernel): give up rather
        // than hang, and make it LOUD -- this block's dx becomes NaN (the
        // divergence watchdog stops the run) instead of silently using stale
        // coefficients; tail + 3 records it for a host-side check
        __hip_atomic_store(tail + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag = -1;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const float poison = last_flag == -1 ? __builtin_nanf("") : 0.f;
  float ka[8], kb[8], kc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ka[k] = r0 < rpi ? coef[c0 + k] + poison : 0.f;
    kb[k] = r0 < rpi ? coef[C + c0 + k] + poison : 0.f;
    kc[k] = r0 < rpi ? coef[2 * C + c0 + k] + poison : 0.f;
  }
  __syncthreads();   // every thread has its coefficients before the departure below
  if (t == 0) {      // departure: the last block out re-arms the release flag
    const int d = __hip_atomic_fetch_add(tail + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == G - 1) {
      __hip_atomic_store(tail + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tail + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // ---- phase 3: apply to this block's rows
  if (r0 < rpi) {
    for (long long row = start + r0; row < end; row += U * rpi) {
      const int nu = (int)min<long long>(U, (end - row + rpi - 1) / rpi);
      bf16x8 xr[U], dr[U], yr[U];
      unsigned mb[U];
      load_rows(row, xr, dr, yr, mb, nu);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < nu) {
          const long long off = (row + u * rpi) * C + c0;
          float xv[8], g[8], o[8];
          dz8(xr[u], dr[u], yr[u], mb[u], xv, g);
          if (WRITE_DRES) store8(dres + off, g);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = ka[k] * g[k] + kc[k] * xv[k] + kb[k];
          store8(dx + off, o);
        }
      }
    }
  }
}

// blocks of the one-pass backward: 1 per CU (co-resident with room to spare: 256 threads,
// <= 16 KiB of LDS, 3-4 blocks fit a CU), fewer when the rows run out; 0 = two launches
static int onepass_blocks(long long M, int C) {
  static const int mode = [] {
    const char* e = std::getenv("DMP_BN_BWD_ONEPASS");
    return e ? std::atoi(e) : 0;   // opt-in until it measures faster in the step
  }();
  if (mode == 0 || C % 8 != 0 || C > 2048) return 0;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long long rpi = 256 / (C / 8);
  long long g = std::min<long long>(cus, (M + 4 * rpi - 1) / (4 * rpi));
  return (int)std::max<long long>(1, g);
}

// cache policy of the streaming BN passes (CS = 64 slices): bit 1 non-temporal
// loads, bit 2 non-temporal stores (DMP_BN_NT, default 0)
static int bn_nt_policy() {
  static const int v = [] {
    const char* e = std::getenv("DMP_BN_NT");
    return e ? (std::atoi(e) & 3) : 0;
  }();
  return v;
}

static int fold_cs(int C) { return C % 64 == 0 ? 64 : C % 32 == 0 ? 32 : C % 16 == 0 ? 16 : 8; }

// row blocks per slice: >= 4 vectors per thread (DMP_BN_FOLD_VPT), at most 1024
// blocks in all (DMP_BN_FOLD_CAP).  The per-block slot reduction is CS x 128
// floats from L2; the streaming pass needs the blocks: ResNet-18 bs512 3.77
// ms/step unfolded, 4.15 at 32 vectors per thread, 3.66 at 8, 3.65 at 4
// (profiles/bn_fold_stem3_r2.txt).  Cap 1024 vs 2048: ResNet-50 bs128 -0.14
// ms/step, ResNet-18 unchanged; 512 and 4096 slower (profiles/bn_grid_knobs_r4.txt).
// Small tensors (the reference batch): a grid of fewer than DMP_BN_FOLD_SMALL blocks
// at 4 vectors per thread goes to 1 vector per thread instead -- more blocks for a
// latency-bound pass (profiles/bn_grid_knobs_r6.txt)
static dim3 fold_grid(long long M, int C, int cs, long long cap_blocks = 0) {
  static const long long vpt = [] {
    const char* e = std::getenv("DMP_BN_FOLD_VPT");
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  static const long long total = [] {
    const char* e = std::getenv("DMP_BN_FOLD_CAP");
    return e ? std::max(1, std::atoi(e)) : 1024;
  }();
  static const long long small = [] {
    const char* e = std::getenv("DMP_BN_FOLD_SMALL");
    return e ? std::max(0, std::atoi(e)) : 512;
  }();
  const long long nsl = C / cs;
  const long long vecs = M * (cs / 8);   // per slice
  long long nrb = (vecs + 256 * vpt - 1) / (256 * vpt);
  if (nrb * nsl < small) nrb = (vecs + 255) / 256;
  const long long cap = std::max<long long>(1, (cap_blocks > 0 ? cap_blocks : total) / nsl);
  nrb = std::max<long long>(1, std::min(nrb, std::min(cap, M)));
  return dim3((unsigned)nrb, (unsigned)nsl);
}

void launch_bn_fwd_fold(const u16* x, const u16* res, u16* y, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, float* stats,
                        float* part, float* zero_buf, long long M, int C, float momentum,
                        float eps, bool relu, bool have_partials, hipStream_t s, uint8_t* mask) {
  if (!have_partials) {
    const int G = bn_num_partials(M, C);
    const int rpi = 256 / (C / 8);
    const size_t lds = (size_t)rpi * C * 2 * sizeof(float);
    hipLaunchKernelGGL((bn_partial_kernel<0, 0>), dim3(G), dim3(256), lds, s, x, nullptr,
                       nullptr, nullptr, nullptr, part, M, C);
  }
  const int cs = fold_cs(C);
  const dim3 grid = fold_grid(M, C, cs);
#define DMP_FOLD_F(CS, R, S, K, NT)                                                              \
  hipLaunchKernelGGL((bn_apply_fold_kernel<CS, R, S, K, NT>), grid, dim3(256), 0, s, x, res, part, \
                     zero_buf, gamma, beta, running_mean, running_var, momentum, eps, stats, y,     \
                     mask, M, C)
#define DMP_FOLD_FV(CS, NT)                                   \
  if (relu && mask) {                                          \
    if (res) DMP_FOLD_F(CS, true, true, true, NT);             \
    else DMP_FOLD_F(CS, true, false, true, NT);                \
  } else if (relu) {                                           \
    if (res) DMP_FOLD_F(CS, true, true, false, NT);            \
    else DMP_FOLD_F(CS, true, false, false, NT);               \
  } else {                                                     \
    if (res) DMP_FOLD_F(CS, false, true, false, NT);           \
    else DMP_FOLD_F(CS, false, false, false, NT);              \
  }
  const int nt = bn_nt_policy();
  if (cs == 64) {
    if (nt == 1) { DMP_FOLD_FV(64, 1) }
    else if (nt == 2) { DMP_FOLD_FV(64, 2) }
    else if (nt == 3) { DMP_FOLD_FV(64, 3) }
    else { DMP_FOLD_FV(64, 0) }
  }
  else if (cs == 32) { DMP_FOLD_FV(32, 0) }
  else if (cs == 16) { DMP_FOLD_FV(16, 0) }
  else { DMP_FOLD_FV(8, 0) }
#undef DMP_FOLD_FV
#undef DMP_FOLD_F
}

// backward reduce grid: bn_num_partials, or for a small tensor (fewer than
// DMP_BN_PART_SMALL blocks at 8 vectors per thread) 2 vectors per thread
static int bn_bwd_partials(long long M, int C) {
  static const int small = [] {
    const char* e = std::getenv("DMP_BN_PART_SMALL");
    return e ? std::max(0, std::atoi(e)) : 256;
  }();
  const int G = bn_num_partials(M, C);
  if (G >= small) return G;
  const long long g = M * (C / 8) / (256 * 2);
  return (int)std::max<long long>(G, std::min<long long>(g, std::min<long long>(2048, M)));
}

void launch_bn_bwd_fold(const u16* x, const u16* dy, const u16* y, const float* gamma,
                        const float* stats, float* dgamma, float* dbeta, float* part,
                        float* zero_buf, u16* dx, u16* dres, long long M, int C, bool relu,
                        hipStream_t s, const uint8_t* mask, float* coef) {
  const int G = bn_bwd_partials(M, C);
  const int rpi = 256 / (C / 8);
  const size_t lds = (size_t)rpi * C * 2 * sizeof(float);
  const int mode = !relu ? 0 : (mask ? 3 : (y ? 1 : 2));
  const int G1 = coef != nullptr ? onepass_blocks(M, C) : 0;
  if (G1 > 0) {
#define DMP_BN_ONE(R, D)                                                                       \
  hipLaunchKernelGGL((bn_bwd_onepass_kernel<R, D>), dim3(G1), dim3(256), lds, s, x, dy, y, mask, \
                     part, zero_buf, gamma, stats, dgamma, dbeta, coef, dx, dres, M, C)
    if (dres) {
      if (mode == 0) DMP_BN_ONE(0, true);
      else if (mode == 1) DMP_BN_ONE(1, true);
      else if (mode == 2) DMP_BN_ONE(2, true);
      else DMP_BN_ONE(3, true);
    } else {
      if (mode == 0) DMP_BN_ONE(0, false);
      else if (mode == 1) DMP_BN_ONE(1, false);
      else if (mode == 2) DMP_BN_ONE(2, false);
      else DMP_BN_ONE(3, false);
    }
#undef DMP_BN_ONE
    return;
  }
  const int nt = bn_nt_policy();
#define DMP_BN_PART(R, NT)                                                                          \
  hipLaunchKernelGGL((bn_partial_kernel<1, R, NT>), dim3(G), dim3(256), lds, s, x, dy, y, mask, stats, \
                     part, M, C)
#define DMP_BN_PARTV(R)                         \
  if ((nt & 1) != 0) DMP_BN_PART(R, 1);         \
  else DMP_BN_PART(R, 0);
  if (mode == 0) { DMP_BN_PARTV(0) }
  else if (mode == 1) { DMP_BN_PARTV(1) }
  else if (mode == 2) { DMP_BN_PARTV(2) }
  else { DMP_BN_PARTV(3) }
#undef DMP_BN_PARTV
#undef DMP_BN_PART
  const int cs = fold_cs(C);
  const dim3 grid = fold_grid(M, C, cs);
#define DMP_FOLD_B(CS, R, D, NT)                                                                   \
  hipLaunchKernelGGL((bn_bwd_apply_fold_kernel<CS, R, D, NT>), grid, dim3(256), 0, s, x, dy, y, mask, \
                     part, zero_buf, gamma, stats, dgamma, dbeta, dx, dres, M, C)
#define DMP_FOLD_BV(CS, NT)                                                \
  if (dres) {                                                              \
    if (mode == 0) DMP_FOLD_B(CS, 0, true, NT);                            \
    else if (mode == 1) DMP_FOLD_B(CS, 1, true, NT);                       \
    else if (mode == 2) DMP_FOLD_B(CS, 2, true, NT);                       \
    else DMP_FOLD_B(CS, 3, true, NT);                                      \
  } else {                                                                 \
    if (mode == 0) DMP_FOLD_B(CS, 0, false, NT);                           \
    else if (mode == 1) DMP_FOLD_B(CS, 1, false, NT);                      \
    else if (mode == 2) DMP_FOLD_B(CS, 2, false, NT);                      \
    else DMP_FOLD_B(CS, 3, false, NT);                                     \
  }
  if (cs == 64) {
    if (nt == 1) { DMP_FOLD_BV(64, 1) }
    else if (nt == 2) { DMP_FOLD_BV(64, 2) }
    else if (nt == 3) { DMP_FOLD_BV(64, 3) }
    else { DMP_FOLD_BV(64, 0) }
  }
  else if (cs == 32) { DMP_FOLD_BV(32, 0) }
  else if (cs == 16) { DMP_FOLD_BV(16, 0) }
  else { DMP_FOLD_BV(8, 0) }
#undef DMP_FOLD_BV
#undef DMP_FOLD_B
}

// -------- BatchNorm + ReLU + max pool, fused (the ImageNet ResNet stem) --------
// conv7x7/s2 -> BN -> ReLU -> maxpool 3x3/s2/p1 (ResNet-50 bs128: a 205 MB
// 112x112x64 activation).  Unfused, the BN apply wrote y (205 MB) for the pool
// to read back, and the backward materialised dy = maxpool_bwd(dp) (205 MB)
// for both BN backward passes to read: bn_apply 94 + maxpool 110 us forward,
// maxpool_bwd 137 + reduce 92 + apply 116 us backward
// (profiles/resnet50_step_dispatches_r4.txt).  Fused:
//   forward   each pooled output applies the folded scale / shift + ReLU to its
//             K x K taps of the raw conv output x and keeps the max and its tap;
//             y never exists.
//   backward  the reduce runs over the pooled windows (dp, taps, xm); the apply
//             gathers dz(h, w) = sum of dp over the windows whose saved argmax is
//             this tap -- dp and the uint8 taps are 1/4 and 1/8 of x's bytes --
//             so dy is never written or read.
// The forward is bit-identical to the unfused ops: the tap values are rounded to
// bf16 before the compare (the pool saw stored bf16 y), and a window whose max
// is 0 records tap 255 (the pool's relu_in rule: relu' = 0 everywhere in it);
// it also keeps the raw x of every window's winning tap (xm, pooled-sized) for
// the backward reduce.  The backward apply's gathered dz is rounded to bf16 (the
// unfused dy was stored).  The ReLU mask of the BN backward is implied: only a
// tap with y = max > 0 can receive gradient.
// 32-bit-offset buffer loads (one VGPR per address instead of a 64-bit pointer;
// an out-of-range offset returns zeros without a memory access): the fused pool
// kernels keep 10-20 loads per lane in flight
typedef unsigned int bnu32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int bnu32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kBnOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bn_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ bf16x8 bn_ld16(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
__device__ __forceinline__ uint2 bn_ld8(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  const bnu32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
  return make_uint2(v.x, v.y);
}

// One un-pooled row's gather, split into a load phase (every load of U rows is
// issued before any is consumed: one row per trip kept ~9 loads in flight per
// lane and ran the backward pair at 132 + 149 us) and a reduce phase.
template <int K, int S, int P>
struct PoolGather {
  static constexpr int KS = (K + S - 1) / S;   // pooled outputs per input row / column, at most
  bf16x8 gv[KS][KS];
  uint2 iv[KS][KS];
  bf16x8 xr;
  int h, w, hlo, hhi, wlo, whi;

  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rsx, __amdgpu_buffer_rsrc_t rsdp,
                                       __amdgpu_buffer_rsrc_t rsidx, int row, bool live, int H,
                                       int W, int C, int Ho, int Wo, int cofs) {
    w = row % W;
    const int r = row / W;
    h = r % H;
    const int n = r / H;
    hlo = max(0, (h + P - K + S) / S);
    hhi = live ? min(Ho - 1, (h + P) / S) : -1;     // a dead row gathers nothing
    wlo = max(0, (w + P - K + S) / S);
    whi = min(Wo - 1, (w + P) / S);
    xr = bn_ld16(rsx, live ? 2u * (unsigned)(row * C + cofs) : kBnOOB);
#pragma unroll
    for (int a = 0; a < KS; ++a)
#pragma unroll
      for (int b = 0; b < KS; ++b) {
        const bool ok = hlo + a <= hhi && wlo + b <= whi;
        const unsigned o = (unsigned)(((n * Ho + hlo + a) * Wo + wlo + b) * C + cofs);
        gv[a][b] = bn_ld16(rsdp, ok ? 2u * o : kBnOOB);
        iv[a][b] = bn_ld8(rsidx, ok ? o : kBnOOB);
      }
  }

  // dz of the 8 channels (rounded to bf16 as the unfused pool's stored dy) and x
  __device__ __forceinline__ void reduce(float g[8], float xv[8]) const {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < KS; ++a)
#pragma unroll
      for (int b = 0; b < KS; ++b) {
        const int ho = hlo + a, wo = wlo + b;
        if (ho <= hhi && wo <= whi) {
          const u32 me = (u32)((h - (ho * S - P)) * K + (w - (wo * S - P)));
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const u32 bi = ((k < 4 ? iv[a][b].x : iv[a][b].y) >> (8 * (k & 3))) & 0xffu;
            if (bi == me) acc[k] += bf2f(gv[a][b].v[k]);
          }
        }
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g[k] = bf2f(f2bf(acc[k]));
      xv[k] = bf2f(xr.v[k]);
    }
  }
};

constexpr int kPoolFwdU = 2, kPoolApplyU = 2;   // rows per trip

template <int CS, int K, int S, int P>
__global__ void __launch_bounds__(256) bn_relu_maxpool_fold_kernel(
    const u16* __restrict__ x, const float* __restrict__ part, float* __restrict__ zero_buf,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps,
    float* __restrict__ stats, u16* __restrict__ y, uint8_t* __restrict__ idx,
    u16* __restrict__ xm, int N, int H, int W, int C, int Ho, int Wo) {
  __shared__ float lS[CS], lQ[CS];
  const int t = threadIdx.x;
  const int cs0 = blockIdx.y * CS;
  fold_fwd_coefs<CS>(part, zero_buf, gamma, beta, running_mean, running_var, momentum, eps, stats,
                     (long long)N * H * W, C, cs0, lS, lQ);
  constexpr int TPR = CS / 8, RPI = 256 / TPR, U = kPoolFwdU;
  const int cg = t % TPR, r0 = t / TPR;
  const int cofs = cs0 + cg * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = lS[cg * 8 + k]; sh[k] = lQ[cg * 8 + k]; }
  const int Mo = N * Ho * Wo;
  const __amdgpu_buffer_rsrc_t rsx = bn_rsrc(x, 2LL * N * H * W * C);
  const int rows_per_blk = (Mo + gridDim.x - 1) / gridDim.x;
  const int start = blockIdx.x * rows_per_blk;
  const int end = min(Mo, start + rows_per_blk);
  for (int row0 = start + r0; row0 < end; row0 += U * RPI) {
    bf16x8 v[U][K][K];                // every tap of U pooled rows in flight together
    int h0[U], w0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * RPI;
      const int wo = row % Wo, r = row / Wo;
      const int ho = r % Ho, n = r / Ho;
      h0[u] = row < end ? ho * S - P : -K - 1;        // a dead row loads no tap
      w0[u] = wo * S - P;
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
          v[u][i][j] = bn_ld16(
              rsx, (unsigned)(h0[u] + i) < (unsigned)H && (unsigned)(w0[u] + j) < (unsigned)W
                       ? 2u * (unsigned)(((n * H + h0[u] + i) * W + w0[u] + j) * C + cofs)
                       : kBnOOB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * RPI;
      if (row >= end) break;
      float best[8];
      u32 bi[8];
      bf16x8 bx;                      // the raw x of the winning tap (backward reduce)
#pragma unroll
      for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; bx.v[k] = 0; }
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
          if ((unsigned)(h0[u] + i) < (unsigned)H && (unsigned)(w0[u] + j) < (unsigned)W) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float f = bf2f(f2bf(fmaxf(bn_pre(bf2f(v[u][i][j].v[k]), sc[k], sh[k]), 0.f)));
              if (f > best[k]) {
                best[k] = f;
                bi[k] = (u32)(i * K + j);
                bx.v[k] = v[u][i][j].v[k];
              }
            }
          }
        }
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o.v[k] = f2bf(best[k]);
        if (!(best[k] > 0.f)) {
          bi[k] = 255;
          bx.v[k] = 0;
        }
      }
      const long long off = (long long)row * C + cofs;
      *reinterpret_cast<bf16x8*>(y + off) = o;
      *reinterpret_cast<bf16x8*>(xm + off) = bx;
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      *reinterpret_cast<uint2*>(idx + off) = packed;
    }
  }
}

// backward reduce pass over the POOLED rows: dz is non-zero only at a window's
// winning tap, so sum dz = sum over windows of dp and sum dz * xhat = sum over
// windows of dp * xhat(x at the winning tap), the x the forward kept in xm
// (reads dp, the taps and xm: 1/4 + 1/8 + 1/4 of x's bytes; the gathering form
// over the un-pooled rows read x whole: ResNet-50 stem 94.0 -> 22.9 us, for
// 75.5 -> 91.8 us in the forward that writes xm).  Windows sharing a winning tap
// add their dp unrounded (the unfused path rounded the per-tap sum to bf16
// first: this reduce is the more exact one).
__global__ void __launch_bounds__(256) pooled_bn_partial_kernel(
    const u16* __restrict__ dp, const uint8_t* __restrict__ idx, const u16* __restrict__ xm,
    const float* __restrict__ stats, float* __restrict__ part, long long Mo, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int U = 4;
  const int tpr = C >> 3;
  const int rpi = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const long long rows_per_blk = (Mo + gridDim.x - 1) / gridDim.x;
  const long long start = (long long)blockIdx.x * rows_per_blk;
  const long long end = min(Mo, start + rows_per_blk);
  float s[8], q[8], mean[8], inv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s[k] = 0.f;
    q[k] = 0.f;
    mean[k] = stats[cg * 8 + k];
    inv[k] = stats[C + cg * 8 + k];
  }
  auto accum = [&](const bf16x8& g, const uint2& iv, const bf16x8& xr) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32 bi = ((k < 4 ? iv.x : iv.y) >> (8 * (k & 3))) & 0xffu;
      const float gv = bi != 255u ? bf2f(g.v[k]) : 0.f;
      s[k] += gv;
      q[k] += gv * (bf2f(xr.v[k]) - mean[k]) * inv[k];
    }
  };
  if (r0 < rpi) {
    long long row = start + r0;
    for (; row + (U - 1) * rpi < end; row += U * rpi) {
      bf16x8 gr[U], xr[U];
      uint2 iv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long off = (row + u * rpi) * C + cg * 8;
        gr[u] = *reinterpret_cast<const bf16x8*>(dp + off);
        iv[u] = *reinterpret_cast<const uint2*>(idx + off);
        xr[u] = *reinterpret_cast<const bf16x8*>(xm + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) accum(gr[u], iv[u], xr[u]);
    }
    for (; row < end; row += rpi) {
      const long long off = row * C + cg * 8;
      accum(*reinterpret_cast<const bf16x8*>(dp + off), *reinterpret_cast<const uint2*>(idx + off),
            *reinterpret_cast<const bf16x8*>(xm + off));
    }
  }
  float* ls = smem;            // [rpi][C]
  float* lq = smem + rpi * C;  // [rpi][C]
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { ls[r0 * C + cg * 8 + k] = s[k]; lq[r0 * C + cg * 8 + k] = q[k]; }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < rpi; ++rr) { a += ls[rr * C + c]; b += lq[rr * C + c]; }
    const int slot = blockIdx.x % kBnSlots;
    atomicAdd(part + (long long)slot * C + c, a);
    atomicAdd(part + (long long)(kBnSlots + slot) * C + c, b);
  }
}

template <int CS, int K, int S, int P>
__global__ void __launch_bounds__(256) maxpool_bn_bwd_apply_fold_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dp, const uint8_t* __restrict__ idx,
    const float* __restrict__ part, float* __restrict__ zero_buf, const float* __restrict__ gamma,
    const float* __restrict__ stats, float* __restrict__ dgamma, float* __restrict__ dbeta,
    u16* __restrict__ dx, int N, int H, int W, int C, int Ho, int Wo) {
  __shared__ float lS[CS], lQ[CS], lC[CS];
  const int t = threadIdx.x;
  const int cs0 = blockIdx.y * CS;
  const int M = N * H * W;
  fold_bwd_coefs<CS>(part, zero_buf, gamma, stats, dgamma, dbeta, M, C, cs0, lS, lQ, lC);
  constexpr int TPR = CS / 8, RPI = 256 / TPR, U = kPoolApplyU;
  const int cg = t % TPR, r0 = t / TPR;
  const int cofs = cs0 + cg * 8;
  float ka[8], kb[8], kc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ka[k] = lS[cg * 8 + k];
    kb[k] = lQ[cg * 8 + k];
    kc[k] = lC[cg * 8 + k];
  }
  const __amdgpu_buffer_rsrc_t rsx = bn_rsrc(x, 2LL * M * C);
  const __amdgpu_buffer_rsrc_t rsdp = bn_rsrc(dp, 2LL * N * Ho * Wo * C);
  const __amdgpu_buffer_rsrc_t rsidx = bn_rsrc(idx, (long long)N * Ho * Wo * C);
  const int rows_per_blk = (M + gridDim.x - 1) / gridDim.x;
  const int start = blockIdx.x * rows_per_blk;
  const int end = min(M, start + rows_per_blk);
  for (int row0 = start + r0; row0 < end; row0 += U * RPI) {
    PoolGather<K, S, P> pg[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * RPI;
      pg[u].load(rsx, rsdp, rsidx, row, row < end, H, W, C, Ho, Wo, cofs);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * RPI;
      if (row >= end) break;
      float xv[8], g[8], o[8];
      pg[u].reduce(g, xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = ka[k] * g[k] + kc[k] * xv[k] + kb[k];
      store8(dx + (long long)row * C + cofs, o);
    }
  }
}

int maxpool_out(int H, int K, int S, int P);   // pool.hip

bool bn_maxpool_supported(int C, int K, int S, int P) {
  return C % 64 == 0 && C <= 2048 && K == 3 && S == 2 && P == 1;
}

void launch_bn_relu_maxpool_fold(const u16* x, u16* y, uint8_t* idx, u16* xm, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var,
                                 float* stats, float* part, float* zero_buf, int N, int H, int W,
                                 int C, float momentum, float eps, bool have_partials,
                                 hipStream_t s) {
  const long long M = (long long)N * H * W;
  if (!have_partials) {
    const int G = bn_num_partials(M, C);
    const size_t lds = (size_t)(256 / (C / 8)) * C * 2 * sizeof(float);
    hipLaunchKernelGGL((bn_partial_kernel<0, 0>), dim3(G), dim3(256), lds, s, x, nullptr,
                       nullptr, nullptr, nullptr, part, M, C);
  }
  const int Ho = maxpool_out(H, 3, 2, 1), Wo = maxpool_out(W, 3, 2, 1);
  // the pool kernels keep 2048 blocks (1024: fwd 75 -> 94, bwd apply 109 -> 116 us)
  const dim3 grid = fold_grid((long long)N * Ho * Wo, C, 64, 2048);
  hipLaunchKernelGGL((bn_relu_maxpool_fold_kernel<64, 3, 2, 1>), grid, dim3(256), 0, s, x, part,
                     zero_buf, gamma, beta, running_mean, running_var, momentum, eps, stats, y, idx,
                     xm, N, H, W, C, Ho, Wo);
}

void launch_maxpool_bn_bwd_fold(const u16* x, const u16* dp, const uint8_t* idx,
                                const u16* xm, const float* gamma, const float* stats, float* dgamma,
                                float* dbeta, float* part, float* zero_buf, u16* dx, int N, int H,
                                int W, int C, hipStream_t s) {
  const long long M = (long long)N * H * W;
  const int Ho = maxpool_out(H, 3, 2, 1), Wo = maxpool_out(W, 3, 2, 1);
  const long long Mo = (long long)N * Ho * Wo;
  const int G = bn_num_partials(Mo, C);
  const size_t lds = (size_t)(256 / (C / 8)) * C * 2 * sizeof(float);
  hipLaunchKernelGGL(pooled_bn_partial_kernel, dim3(G), dim3(256), lds, s, dp, idx, xm, stats,
                     part, Mo, C);
  hipLaunchKernelGGL((maxpool_bn_bwd_apply_fold_kernel<64, 3, 2, 1>), fold_grid(M, C, 64, 2048),
                     dim3(256), 0, s, x, dp, idx, part, zero_buf, gamma, stats, dgamma, dbeta, dx,
                     N, H, W, C, Ho, Wo);
}

}  // namespace dmp

namespace dmp {
// BN backward whose reductions were already made per block by the consuming
// conv's data-gradient epilogue (conv.hip bnb_*, which also applied the ReLU
// mask: dz arrives masked): finalize + a mask-free apply, no reduce pass.
void launch_bn_bwd_from_partials(const u16* x, const u16* dz, const float* gamma,
                                 const float* stats, float* dgamma, float* dbeta, float* coef,
                                 float* part, u16* dx, long long M, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, part,
                     kBnSlots, M, C, gamma, stats, dgamma, dbeta, coef);
  const long long nvec = M * C / 8;
  hipLaunchKernelGGL((bn_bwd_apply_kernel<0, false>), dim3(stream_grid(nvec, 256)), dim3(256), 0,
                     s, x, dz, nullptr, nullptr, coef, stats, dx, nullptr, nvec, C);
}

// BN forward whose statistics were already reduced per block by the producing
// conv's epilogue (conv.hip STATS): finalize + apply only, no stats pass over x.
void launch_bn_fwd_partials(const u16* x, const u16* res, u16* y, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            float* stats, float* part, long long M, int C,
                            float momentum, float eps, bool relu, hipStream_t s, uint8_t* mask) {
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, part,
                     kBnSlots, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                     stats, 0);
  bn_apply(x, res, stats, y, mask, M, C, relu, s);
}
}  // namespace dmp

namespace dmp {
// ------------------------------------------------ inference-time BatchNorm folding
// Eval-mode BN is a per-channel affine map of its input, so BN(conv(x, W)) +
// residual, ReLU = conv(x, W * s) + t (+ residual), ReLU with
//   s[co] = gamma / sqrt(running_var + eps),  t[co] = beta + (conv_bias - running_mean) * s:
// the conv's own epilogue (bias, residual addend, ReLU) then IS the BN -- no
// statistics, finalize or apply pass (the reference's evaluation loop,
// /root/reference/example/main.py:110-125).  One launch per conv, once per
// evaluation pass (ops/eval_fold.py): every thread scales one weight of one
// output channel (fp32 master -> bf16 compute weight, ONE rounding as the
// arena's bf16 shadow has; any elements-per-channel count, e.g. the 27 of a
// 3x3x3 stem); threads co < CO also write t (fp32 for the conv epilogues, bf16
// for the GEMM route).
__global__ void __launch_bounds__(256) bn_fold_weights_kernel(
    const float* __restrict__ w, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ rmean, const float* __restrict__ rvar, const float* __restrict__ cbias,
    u16* __restrict__ w16, float* __restrict__ b32, u16* __restrict__ b16, long long n,
    int per_co, int CO, float eps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int co = (int)(i / per_co);
    const float s = (gamma ? gamma[co] : 1.f) * rsqrtf(rvar[co] + eps);
    w16[i] = f2bf(w[i] * s);
  }
  if (i < CO) {
    const int co = (int)i;
    const float s = (gamma ? gamma[co] : 1.f) * rsqrtf(rvar[co] + eps);
    const float t = (beta ? beta[co] : 0.f) + ((cbias ? cbias[co] : 0.f) - rmean[co]) * s;
    if (b32) b32[co] = t;
    if (b16) b16[co] = f2bf(t);
  }
}

void launch_bn_fold_weights(const float* w, const float* gamma, const float* beta,
                            const float* rmean, const float* rvar, const float* cbias,
                            uint16_t* w16, float* b32, uint16_t* b16, long long n, int CO,
                            float eps, hipStream_t s) {
  const long long threads = n > CO ? n : CO;
  hipLaunchKernelGGL(bn_fold_weights_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     s, w, gamma, beta, rmean, rvar, cbias, w16, b32, b16, n, (int)(n / CO), CO,
                     eps);
}
}  // namespace dmp
