// Flat-arena optimizer / parameter-server kernels (memory-bound, 16 B per lane).
//
// Reference behaviour being re-implemented (not translated):
//   * worker step  /root/reference/asgd/optim/Asynchronous.py:54-68
//       acc += -lr * g          (accumulated_gradients.add_(-lr, gradients))
//       p   += -lr * g          (per-tensor local SGD)
//     here: ONE pass over the flat fp32 arena that also refreshes the bf16
//     compute shadow, instead of a per-step torch.cat ravel + 2 axpys + N
//     per-tensor adds.
//   * PS apply  (missing asgd/server.py, contract in SURVEY.md C7)
//       shard += delta          (delta already carries -lr)
//
// All buffers are padded by the arena to a multiple of 64 elements and are
// 256-B aligned, so n % 4 == 0 always holds (asserted on the host side).
#include "common.h"

#include <algorithm>

namespace dmp {

// g      : fp32 gradient (flat)         [n]
// p      : fp32 worker parameters       [n]   (in/out)
// acc    : fp32 push accumulator        [n]   (in/out, may be null)
// mom    : fp32 momentum buffer         [n]   (in/out, may be null)
// w16    : bf16 compute shadow of p     [n]   (out, may be null)
__global__ void __launch_bounds__(256) asgd_fused_step_kernel(
    const float4* __restrict__ g, float4* __restrict__ p, float4* __restrict__ acc,
    float4* __restrict__ mom, bf16x4* __restrict__ w16, long long n4, float lr,
    float weight_decay, float momentum, float dampening, int nesterov) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 gv = g[i];
    float4 pv = p[i];
    if (weight_decay != 0.f) {
      gv.x += weight_decay * pv.x; gv.y += weight_decay * pv.y;
      gv.z += weight_decay * pv.z; gv.w += weight_decay * pv.w;
    }
    if (mom) {
      float4 m = mom[i];
      const float d = 1.f - dampening;
      m.x = momentum * m.x + d * gv.x; m.y = momentum * m.y + d * gv.y;
      m.z = momentum * m.z + d * gv.z; m.w = momentum * m.w + d * gv.w;
      mom[i] = m;
      if (nesterov) {
        gv.x += momentum * m.x; gv.y += momentum * m.y;
        gv.z += momentum * m.z; gv.w += momentum * m.w;
      } else {
        gv = m;
      }
    }
    const float4 d = make_float4(-lr * gv.x, -lr * gv.y, -lr * gv.z, -lr * gv.w);
    if (acc) {
      float4 a = acc[i];
      a.x += d.x; a.y += d.y; a.z += d.z; a.w += d.w;
      acc[i] = a;
    }
    pv.x += d.x; pv.y += d.y; pv.z += d.z; pv.w += d.w;
    p[i] = pv;
    if (w16) {
      bf16x4 o;
      o.v[0] = f2bf(pv.x); o.v[1] = f2bf(pv.y); o.v[2] = f2bf(pv.z); o.v[3] = f2bf(pv.w);
      w16[i] = o;
    }
  }
}

// shard += scale * delta (fp32 delta)      -- PS GradientUpdate apply
// optional: mirror the new shard into bf16 for low-precision pulls.
__global__ void __launch_bounds__(256) ps_apply_f32_kernel(
    float4* __restrict__ shard, const float4* __restrict__ delta, bf16x4* __restrict__ mirror,
    long long n4, float scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 s = shard[i];
    const float4 d = delta[i];
    s.x += scale * d.x; s.y += scale * d.y; s.z += scale * d.z; s.w += scale * d.w;
    shard[i] = s;
    if (mirror) {
      bf16x4 o;
      o.v[0] = f2bf(s.x); o.v[1] = f2bf(s.y); o.v[2] = f2bf(s.z); o.v[3] = f2bf(s.w);
      mirror[i] = o;
    }
  }
}

// shard += scale * delta (bf16 wire-format delta)
__global__ void __launch_bounds__(256) ps_apply_bf16_kernel(
    float4* __restrict__ shard, const bf16x4* __restrict__ delta, bf16x4* __restrict__ mirror,
    long long n4, float scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 s = shard[i];
    const bf16x4 d = delta[i];
    s.x += scale * bf2f(d.v[0]); s.y += scale * bf2f(d.v[1]);
    s.z += scale * bf2f(d.v[2]); s.w += scale * bf2f(d.v[3]);
    shard[i] = s;
    if (mirror) {
      bf16x4 o;
      o.v[0] = f2bf(s.x); o.v[1] = f2bf(s.y); o.v[2] = f2bf(s.z); o.v[3] = f2bf(s.w);
      mirror[i] = o;
    }
  }
}

// shard += scale * delta with fp32 global atomics (no-return
// global_atomic_add_f32): the completion-ordered PS applies each worker's delta
// on that worker's own link stream, so applies of different workers may run at
// the same time on one shard ("or use fp32 atomics").  Lane i
// of a wave adds element base + i: every wave-instruction covers 256 contiguous
// bytes, the full-rate shape of MI355X_MICROARCH.md §Global float atomics.
template <typename D>
__global__ void __launch_bounds__(256) ps_apply_atomic_kernel(float* __restrict__ shard,
                                                              const D* __restrict__ delta,
                                                              long long n, float scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float d;
    if constexpr (sizeof(D) == 4) d = delta[i];
    else d = bf2f(delta[i]);
    unsafeAtomicAdd(shard + i, scale * d);
  }
}

// Applied-count of a PS shard: the version a reply is stamped with
// (parallel/server.py, parallel/async_sharded.py; SURVEY §7.3(3) "a version
// counter is the basis for staleness-bounded pulls").  ps_count runs on the
// applying stream right after the apply kernel, so the count only moves once an
// apply has wholly landed; ps_stamp runs on the replying stream BEFORE the
// snapshot copy, so a stamp counts only applies the snapshot fully contains
// (applies still in flight on other link streams may show up in some elements,
// never in the count).  Both are agent-scope atomics: the counting and reading
// streams may run on any XCD (MI355X_MICROARCH.md "Workgroup dispatch").
__global__ void __launch_bounds__(64) ps_count_kernel(int* __restrict__ cnt, int add, int set) {
  if (threadIdx.x == 0) {
    if (set) __hip_atomic_exchange(cnt, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(cnt, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(64) ps_stamp_kernel(int* __restrict__ cnt,
                                                      float* __restrict__ dst) {
  if (threadIdx.x == 0) {
    const int v = __hip_atomic_fetch_add(cnt, 0, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    dst[0] = (float)v;
  }
}

// Pull landing: p = src (fp32 or bf16 wire), w16 = bf16(p). Optionally the
// delta the worker accumulated since the snapshot is re-applied on top
// (keep_local: p = src + acc), which keeps not-yet-pushed local progress
// instead of discarding it (the reference overwrote it).
__global__ void __launch_bounds__(256) pull_land_f32_kernel(
    float4* __restrict__ p, const float4* __restrict__ src, const float4* __restrict__ acc,
    bf16x4* __restrict__ w16, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = src[i];
    if (acc) {
      const float4 a = acc[i];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    p[i] = v;
    if (w16) {
      bf16x4 o;
      o.v[0] = f2bf(v.x); o.v[1] = f2bf(v.y); o.v[2] = f2bf(v.z); o.v[3] = f2bf(v.w);
      w16[i] = o;
    }
  }
}

__global__ void __launch_bounds__(256) pull_land_bf16_kernel(
    float4* __restrict__ p, const bf16x4* __restrict__ src, const float4* __restrict__ acc,
    bf16x4* __restrict__ w16, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const bf16x4 s = src[i];
    float4 v = make_float4(bf2f(s.v[0]), bf2f(s.v[1]), bf2f(s.v[2]), bf2f(s.v[3]));
    if (acc) {
      const float4 a = acc[i];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    p[i] = v;
    if (w16) {
      bf16x4 o;
      o.v[0] = f2bf(v.x); o.v[1] = f2bf(v.y); o.v[2] = f2bf(v.z); o.v[3] = f2bf(v.w);
      w16[i] = o;
    }
  }
}

// Push hand-off: out = acc (fp32 or bf16 wire), acc = 0. One pass replaces the
// reference's "send(acc); acc.zero_()" (Asynchronous.py:58-60) and makes the
// send buffer a private snapshot so the next step may keep accumulating.
__global__ void __launch_bounds__(256) push_handoff_kernel(
    float4* __restrict__ acc, float4* __restrict__ out32, bf16x4* __restrict__ out16,
    long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = acc[i];
    if (out32) out32[i] = a;
    if (out16) {
      bf16x4 o;
      o.v[0] = f2bf(a.x); o.v[1] = f2bf(a.y); o.v[2] = f2bf(a.z); o.v[3] = f2bf(a.w);
      out16[i] = o;
    }
    acc[i] = z;
  }
}

// fp32 -> bf16 cast (flat), used to initialise the compute shadow.
__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(
    const float4* __restrict__ src, bf16x4* __restrict__ dst, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = src[i];
    bf16x4 o;
    o.v[0] = f2bf(a.x); o.v[1] = f2bf(a.y); o.v[2] = f2bf(a.z); o.v[3] = f2bf(a.w);
    dst[i] = o;
  }
}

// Sum of squares of a flat fp32 buffer (grad-norm / divergence watchdog).
// Writes one partial per block; the host side sums <=2048 partials.
__global__ void __launch_bounds__(256) sumsq_partial_kernel(
    const float4* __restrict__ x, float* __restrict__ partial, long long n4) {
  __shared__ float red[4];
  float s = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = x[i];
    s += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Zero fill of a dense buffer, 16 B per lane (the grad arena at every step
// start).  A kernel, not hipMemsetAsync: a memset node captured into the step's
// hipGraph was NOT ordered behind the previous replay's kernels on this stack
// (ROCm 7.x): back-to-back replays without a host sync zeroed the arena while
// the previous step's weight-gradient atomics / fused update still used it, and
// training went non-finite within tens of steps (scripts/nan_hunt.py A/B:
// 3 of 3 memset runs diverged at least once, 0 of 6 with a kernel).
__global__ void __launch_bounds__(256) zero_fill_kernel(float4* __restrict__ x, long long n4,
                                                         float* __restrict__ tail, int ntail) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float4 z = {0.f, 0.f, 0.f, 0.f};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) x[i] = z;
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) tail[threadIdx.x] = 0.f;
}

// ---------------------------------------------------------------- launchers
void launch_zero_fill(void* p, long long bytes, hipStream_t s) {
  // bytes % 4 == 0 and 16-B aligned base (torch allocations); the < 16-B tail
  // is handled by block 0
  const long long n4 = bytes / 16;
  const int ntail = (int)((bytes - n4 * 16) / 4);
  hipLaunchKernelGGL(zero_fill_kernel, dim3(stream_grid(n4 > 0 ? n4 : 1, 256)), dim3(256), 0, s,
                     (float4*)p, n4, (float*)p + n4 * 4, ntail);
}

void launch_asgd_fused_step(const float* g, float* p, float* acc, float* mom, u16* w16,
                            long long n, float lr, float wd, float momentum, float dampening,
                            bool nesterov, hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(asgd_fused_step_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (const float4*)g, (float4*)p, (float4*)acc, (float4*)mom, (bf16x4*)w16, n4,
                     lr, wd, momentum, dampening, nesterov ? 1 : 0);
}

void launch_ps_apply_f32(float* shard, const float* delta, u16* mirror, long long n, float scale,
                         hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(ps_apply_f32_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (float4*)shard, (const float4*)delta, (bf16x4*)mirror, n4, scale);
}

void launch_ps_apply_bf16(float* shard, const u16* delta, u16* mirror, long long n, float scale,
                          hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(ps_apply_bf16_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (float4*)shard, (const bf16x4*)delta, (bf16x4*)mirror, n4, scale);
}

void launch_ps_apply_atomic(float* shard, const void* delta, bool bf16, long long n, float scale,
                            hipStream_t s) {
  if (n <= 0) return;   // an empty shard: nothing to add (a 0-block grid is invalid)
  const int grid = (int)std::min<long long>((n + 255) / 256, 256LL * 16);
  if (bf16)
    hipLaunchKernelGGL(ps_apply_atomic_kernel<u16>, dim3(grid), dim3(256), 0, s, shard,
                       (const u16*)delta, n, scale);
  else
    hipLaunchKernelGGL(ps_apply_atomic_kernel<float>, dim3(grid), dim3(256), 0, s, shard,
                       (const float*)delta, n, scale);
}

void launch_ps_count(int* cnt, int add, bool set, hipStream_t s) {
  hipLaunchKernelGGL(ps_count_kernel, dim3(1), dim3(64), 0, s, cnt, add, set ? 1 : 0);
}

void launch_ps_stamp(int* cnt, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(ps_stamp_kernel, dim3(1), dim3(64), 0, s, cnt, dst);
}

void launch_pull_land_f32(float* p, const float* src, const float* acc, u16* w16, long long n,
                          hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(pull_land_f32_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (float4*)p, (const float4*)src, (const float4*)acc, (bf16x4*)w16, n4);
}

void launch_pull_land_bf16(float* p, const u16* src, const float* acc, u16* w16, long long n,
                           hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(pull_land_bf16_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (float4*)p, (const bf16x4*)src, (const float4*)acc, (bf16x4*)w16, n4);
}

void launch_push_handoff(float* acc, float* out32, u16* out16, long long n, hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(push_handoff_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (float4*)acc, (float4*)out32, (bf16x4*)out16, n4);
}

void launch_cast_f32_bf16(const float* src, u16* dst, long long n, hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s,
                     (const float4*)src, (bf16x4*)dst, n4);
}

int launch_sumsq_partial(const float* x, float* partial, long long n, hipStream_t s) {
  const long long n4 = n / 4;
  int grid = stream_grid(n4, 256);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(grid), dim3(256), 0, s, (const float4*)x,
                     partial, n4);
  return grid;
}

}  // namespace dmp
