// Per-block phase timing of the native GEMM tiles (diagnostic build of csrc/gemm.hip with
// -DDMP_GEMM_STAMPS: s_memrealtime stamps at kernel entry, first k-tile landed, end of the
// k-loop, end of the epilogue).  Splits one launch's time into prologue / k-loop /
// epilogue per block and shows how the blocks' rounds line up.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I distributed_ml_pytorch_amd/csrc \
//     scripts/gemm_stamps.cpp -o /tmp/gemm_stamps && /tmp/gemm_stamps 12608 2304 768 10
#define DMP_GEMM_STAMPS 1
#include "gemm.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 12608;
  const int N = argc > 2 ? std::atoi(argv[2]) : 2304;
  const int K = argc > 3 ? std::atoi(argv[3]) : 768;
  const int cfg = argc > 4 ? std::atoi(argv[4]) : 10;
  if (!dmp::gemm_config_ok(0, cfg)) { std::fprintf(stderr, "cfg %d not valid in fwd\n", cfg); return 1; }
  std::vector<uint16_t> h((size_t)std::max(M, N) * K);
  unsigned s = 1234567u;
  for (auto& v : h) {   // uniform random bf16 in about [-1, 1)
    s = s * 1664525u + 1013904223u;
    const float f = ((s >> 8) & 0xffff) / 32768.0f - 1.0f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (uint16_t)(u >> 16);
  }
  uint16_t *a, *b, *c, *bias;
  CK(hipMalloc(&a, 2ull * M * K));
  CK(hipMalloc(&b, 2ull * N * K));
  CK(hipMalloc(&c, 2ull * M * N));
  CK(hipMalloc(&bias, 2ull * N));
  CK(hipMemcpy(a, h.data(), 2ull * M * K, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, h.data(), 2ull * N * K, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data(), 2ull * N, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto run = [&]() {
    dmp::launch_gemm(0, 0, cfg, a, K, b, K, c, N, nullptr, bias, nullptr, nullptr, M, N, K, 1, st,
                     false, nullptr, nullptr, nullptr, nullptr, nullptr);
  };
  for (int i = 0; i < 5; ++i) run();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < 20; ++i) run();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> z(4u << 16, 0ull);
  CK(hipMemcpyToSymbol(HIP_SYMBOL(dmp::g_gemm_stamps), z.data(), z.size() * 8));
  run();
  CK(hipStreamSynchronize(st));
  CK(hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(dmp::g_gemm_stamps), z.size() * 8));
  int nb = 0;
  while (nb < (1 << 16) && z[4 * nb + 3] != 0) ++nb;
  unsigned long long t0 = ~0ull, tend = 0;
  for (int i = 0; i < nb; ++i) { t0 = std::min(t0, z[4 * i]); tend = std::max(tend, z[4 * i + 3]); }
  auto us = [](unsigned long long d) { return d / 100.0; };   // 100 MHz counter
  double pro = 0, loop = 0, epi = 0;
  std::vector<double> starts;
  for (int i = 0; i < nb; ++i) {
    pro += us(z[4 * i + 1] - z[4 * i]);
    loop += us(z[4 * i + 2] - z[4 * i + 1]);
    epi += us(z[4 * i + 3] - z[4 * i + 2]);
    starts.push_back(us(z[4 * i] - t0));
  }
  std::sort(starts.begin(), starts.end());
  std::printf("M=%d N=%d K=%d cfg %d: %.1f us per launch (events, 20 back to back); %d blocks\n", M,
              N, K, cfg, 1e3 * ms / 20, nb);
  std::printf("  stamped launch: first entry -> last epilogue end %.1f us\n", us(tend - t0));
  std::printf("  per block mean: prologue (entry -> k-tile 0 landed) %.2f us, k-loop %.2f us, "
              "epilogue %.2f us\n", pro / nb, loop / nb, epi / nb);
  std::printf("  block start times (us after the first): ");
  for (int q = 0; q <= 10; ++q) std::printf("p%d0 %.1f  ", q, starts[std::min(nb - 1, q * (nb - 1) / 10)]);
  std::printf("\n");
  // the second round: blocks that start after the first quarter of the launch
  int late = 0;
  double lpro = 0, lloop = 0, lepi = 0;
  for (int i = 0; i < nb; ++i)
    if (us(z[4 * i] - t0) > 0.25 * us(tend - t0)) {
      ++late;
      lpro += us(z[4 * i + 1] - z[4 * i]);
      lloop += us(z[4 * i + 2] - z[4 * i + 1]);
      lepi += us(z[4 * i + 3] - z[4 * i + 2]);
    }
  if (late)
    std::printf("  later-round blocks: %d, mean prologue %.2f / k-loop %.2f / epilogue %.2f us\n", late,
                lpro / late, lloop / late, lepi / late);
  return 0;
}
