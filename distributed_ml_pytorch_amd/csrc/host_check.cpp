// Sanitizer driver for the host-side C++ of the extension (`make asan`, SURVEY
// §5.2; tests/test_asan_cpu.py).  Built host-only (hipcc --cuda-host-only: the
// kernels' device code is not compiled, nothing is launched, no GPU needed) with
// -fsanitize=address,undefined, it drives every piece of host logic that turns a
// tensor shape into kernel geometry -- tile / config selection, LDS sizing,
// split-K counts, slab sizes, the 32-bit offset guards -- over the shape sets of
// every model the framework ships (ResNet-18 CIFAR at the reference's batch 64
// and the bench's 512, ResNet-50 ImageNet bs128, ViT-B/16 bs64, AlexNet, LeNet)
// plus oversize batches that must be REJECTED, not wrapped.  Any signed overflow,
// out-of-range shift or bad access in that arithmetic aborts the run (UBSan /
// ASan, -fno-sanitize-recover).  Exit status 0 and a summary line on success.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "geom_guard.h"
#include "launchers.h"

namespace {

int g_fail = 0;
long long g_checks = 0;

#define EXPECT(cond, ...)                                           \
  do {                                                              \
    ++g_checks;                                                     \
    if (!(cond)) {                                                  \
      std::fprintf(stderr, "FAIL %s:%d: %s | ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                            \
      std::fprintf(stderr, "\n");                                   \
      ++g_fail;                                                     \
    }                                                               \
  } while (0)

struct Conv {
  const char* model;
  int B, CI, H, W, CO, R, S, stride, pad;
};

int out_dim(int in, int pad, int k, int st) { return (int)dmp::guard::conv_out(in, pad, k, st); }

// every conv of a ResNet (BasicBlock / Bottleneck) at batch B
void resnet_convs(std::vector<Conv>& v, const char* name, int B, bool bottleneck, bool cifar) {
  int H = cifar ? 32 : 56, cin = 64;
  if (cifar) v.push_back({name, B, 3, 32, 32, 64, 3, 3, 1, 1});
  else v.push_back({name, B, 3, 224, 224, 64, 7, 7, 2, 3});
  const int blocks[4] = {2, 2, 2, 2}, blocks50[4] = {3, 4, 6, 3};
  for (int st = 0; st < 4; ++st) {
    const int planes = 64 << st;
    const int n = bottleneck ? blocks50[st] : blocks[st];
    for (int j = 0; j < n; ++j) {
      const int stride = (st > 0 && j == 0) ? 2 : 1;
      const int OH = out_dim(H, 1, 3, stride);
      if (bottleneck) {
        const int out = planes * 4;
        v.push_back({name, B, cin, H, H, planes, 1, 1, 1, 0});
        v.push_back({name, B, planes, H, H, planes, 3, 3, stride, 1});
        v.push_back({name, B, planes, OH, OH, out, 1, 1, 1, 0});
        if (stride != 1 || cin != out) {
          v.push_back({name, B, cin, H, H, out, 1, 1, stride, 0});
          v.push_back({name, B, cin, OH, OH, out, 1, 1, 1, 0});   // subsampled-alias form
        }
        cin = out;
      } else {
        v.push_back({name, B, cin, H, H, planes, 3, 3, stride, 1});
        v.push_back({name, B, planes, OH, OH, planes, 3, 3, 1, 1});
        if (stride != 1 || cin != planes) {
          v.push_back({name, B, cin, H, H, planes, 1, 1, stride, 0});
          v.push_back({name, B, cin, OH, OH, planes, 1, 1, 1, 0});
        }
        cin = planes;
      }
      H = OH;
    }
  }
}

void check_conv(const Conv& c) {
  const int OH = out_dim(c.H, c.pad, c.R, c.stride), OW = out_dim(c.W, c.pad, c.S, c.stride);
  EXPECT(OH > 0 && OW > 0, "%s empty output", c.model);
  const bool fits = dmp::guard::conv_offsets_ok(c.B, c.H, c.W, c.CI, OH, OW, c.CO, c.R, c.S);
  const long long M = (long long)c.B * OH * OW;
  if (c.CI >= 64 && fits) {
    // implicit-GEMM configs: tile info and M-block counts
    const int ncfg = dmp::conv_num_configs();
    EXPECT(ncfg > 0, "no conv configs");
    for (int cfg = 0; cfg < ncfg; ++cfg) {
      int info[8] = {0};
      dmp::conv_config_info(cfg, info);
      EXPECT(info[0] > 0 && info[1] > 0 && info[2] > 0 && info[3] > 0 && info[3] <= 1024,
             "cfg %d info %d %d %d %d", cfg, info[0], info[1], info[2], info[3]);
      const int mb = dmp::conv_fwd_num_mblocks(M, c.CO, cfg);
      EXPECT(mb > 0 && (long long)mb * info[0] >= M, "cfg %d M %lld -> %d blocks of %d", cfg, M,
             mb, info[0]);
    }
    const int dflt = dmp::conv_default_config(M, c.CO);
    EXPECT(dflt >= 0 && dflt < ncfg, "default cfg %d", dflt);
    // 3x3 stride-1 halo tiles (incl. the persistent 64-channel ones)
    int nhalo = 0;
    for (int i = 0; i < dmp::conv_num_halo_configs(); ++i)
      nhalo += dmp::conv_halo_ok(dmp::conv_halo_base() + i, c.H, c.W, c.CI, c.R, c.S, c.stride,
                                 c.pad);
    if (c.R == 3 && c.stride == 1 && c.pad == 1 && c.H >= 4)
      EXPECT(nhalo > 0, "%s: no halo config for %dx%dx%d", c.model, c.H, c.W, c.CI);
    // stride-2 halo data gradient: dY (OH x OW, CO) -> dX (H x W, CI)
    for (int i = 0; i < dmp::conv_dgrad_s2_num_configs(); ++i)
      dmp::conv_dgrad_s2_ok(dmp::conv_dgrad_s2_base() + i, c.H, c.W, OH, OW, c.CO, c.CI, c.R,
                            c.S, c.stride, c.pad);
    // halo weight gradient, atomic and slab (split-K partials) forms
    for (int i = 0; i < dmp::conv_wgrad_num_halo_configs(); ++i) {
      const int cfg = dmp::conv_wgrad_halo_base() + i;
      dmp::conv_wgrad_halo_ok(cfg, c.B, c.H, c.W, c.CI, c.CO, c.R, c.S, c.stride, c.pad);
      const int scfg = dmp::conv_wgrad_halo_slab_base() + i;
      const long long se = dmp::conv_wgrad_halo_slab_elems(scfg, c.B, c.H, c.W, c.CI, c.CO, c.R,
                                                           c.S, c.stride, c.pad);
      const bool ok = dmp::conv_wgrad_halo_ok(scfg, c.B, c.H, c.W, c.CI, c.CO, c.R, c.S,
                                              c.stride, c.pad);
      EXPECT(ok == (se > 0), "slab cfg %d: ok %d elems %lld", scfg, ok, se);
      if (se > 0)
        EXPECT(se % ((long long)c.CO * c.R * c.S * c.CI) == 0, "slab elems %lld", se);
    }
  } else if (c.CI < 64) {
    // stems: 3x3 MFMA stem, VALU small conv, ImageNet s2d stem
    dmp::stem3_supported(c.CI, c.R, c.S, c.CO, c.stride, c.pad, c.W);
    if (c.R * c.S * c.CI <= dmp::conv_small_max_k() &&
        dmp::guard::small_conv_ok(c.B, OH, OW, c.CO, (long long)c.B * c.CI * c.H * c.W)) {
      const long long P = (long long)c.B * OH * OW;
      EXPECT(dmp::conv_small_fwd_blocks(P) > 0, "small fwd blocks");
      EXPECT(dmp::conv_small_wgrad_blocks(P, c.CO, c.R, c.S, c.CI) > 0, "small wgrad blocks");
    }
    if (c.R == 7) {
      EXPECT(dmp::stem_supported(c.H, c.W), "imagenet stem %dx%d", c.H, c.W);
      EXPECT(dmp::guard::stem_batch_ok(c.B, c.H, c.W), "stem batch %d", c.B);
    }
  }
}

void check_gemm(int M, int N, int K) {
  for (int cfg = 0; cfg < dmp::gemm_num_configs(); ++cfg) {
    int info[8] = {0};
    dmp::gemm_config_info(cfg, info);
    EXPECT(info[0] > 0 && info[1] > 0 && info[2] > 0 && info[2] <= 1024, "gemm cfg %d", cfg);
    for (int mode = 0; mode < 3; ++mode) dmp::gemm_config_ok(mode, cfg);
  }
  for (int sp : {1, 2, 4, 8, 16, 64}) {
    const int e = dmp::gemm_effective_splits(K, sp);
    EXPECT(e >= 1 && e <= sp && e <= K, "splits(%d, %d) = %d", K, sp, e);
  }
  EXPECT(dmp::guard::rows_bytes_ok(2, M, K) && dmp::guard::rows_bytes_ok(2, N, K) &&
             dmp::guard::rows_bytes_ok(2, M, N),
         "gemm %dx%dx%d rejected", M, N, K);
}

void check_guards() {
  using namespace dmp::guard;
  // conv outputs
  EXPECT(conv_out(32, 1, 3, 1) == 32 && conv_out(32, 1, 3, 2) == 16 && conv_out(224, 3, 7, 2) == 112,
         "conv_out");
  EXPECT(conv_out(2, 0, 3, 1) == 0 && conv_out(8, 0, 3, 0) == 0, "conv_out empty / bad stride");
  // the largest ResNet-18 CIFAR activation that fits: 2^30 elements of bf16 at 64 ch
  EXPECT(conv_offsets_ok(16383, 32, 32, 64, 32, 32, 64, 3, 3), "16383 x 64 x 32 x 32 fits");
  EXPECT(!conv_offsets_ok(16384, 32, 32, 64, 32, 32, 64, 3, 3), "exactly 2 GiB must be rejected");
  EXPECT(!conv_offsets_ok(int64_t(1) << 40, 32, 32, 64, 32, 32, 64, 3, 3), "2^40 batch");
  EXPECT(!conv_offsets_ok(int64_t(1) << 62, 1 << 20, 1 << 20, 64, 1 << 20, 1 << 20, 64, 3, 3),
         "product overflowing int64 must be rejected, not wrapped");
  EXPECT(!conv_offsets_ok(-1, 32, 32, 64, 32, 32, 64, 3, 3), "negative batch");
  EXPECT(!conv_offsets_ok(2, 32, 32, 64, 32, 32, 1 << 21, 3, 3), "weight over 2 GiB");
  EXPECT(bf16_bytes_ok(1, 1, 1, (int64_t(1) << 30) - 1) && !bf16_bytes_ok(1, 1, 1, int64_t(1) << 30),
         "bf16 2 GiB edge");
  EXPECT(small_conv_ok(512, 32, 32, 64, 512LL * 3 * 32 * 32), "small conv bs512");
  EXPECT(!small_conv_ok(int64_t(1) << 16, 32, 32, 1 << 10, 3), "small conv output over 2^31");
  EXPECT(!small_conv_ok(1, 32, 32, 64, int64_t(1) << 30), "small conv input over 2 GiB");
  EXPECT(stem_batch_ok(128, 224, 224) && !stem_batch_ok(int64_t(1) << 20, 224, 224), "stem");
  EXPECT(rows_bytes_ok(2, 12608, 3072) && !rows_bytes_ok(4, int64_t(1) << 20, 1 << 10),
         "rows 2 GiB");
  EXPECT(!rows_bytes_ok(2, int64_t(1) << 62, int64_t(1) << 62), "rows overflow");
  EXPECT(!rows_bytes_ok(0, 1, 1) && !rows_bytes_ok(2, -1, 4), "rows bad args");
  // the halo / wgrad geometry must REJECT (not overflow on) batches past 2 GiB
  const int hb = dmp::conv_halo_base();
  for (int i = 0; i < dmp::conv_num_halo_configs(); ++i)
    dmp::conv_halo_ok(hb + i, 32, 32, 64, 3, 3, 1, 1);
  for (int i = 0; i < dmp::conv_wgrad_num_halo_configs(); ++i) {
    const int cfg = dmp::conv_wgrad_halo_base() + i;
    EXPECT(!dmp::conv_wgrad_halo_ok(cfg, 1 << 20, 32, 32, 64, 64, 3, 3, 1, 1),
           "wgrad cfg %d accepted a 2^20 batch", cfg);
    EXPECT(dmp::conv_wgrad_halo_slab_elems(dmp::conv_wgrad_halo_slab_base() + i, 1 << 20, 32, 32,
                                           64, 64, 3, 3, 1, 1) == 0,
           "slab for a rejected shape");
  }
}

}  // namespace

// DMP_ASAN_SELFTEST=asan|ubsan: a deliberate heap overflow / signed overflow,
// so the test can see that the sanitizers are really in the build
int selftest(const char* kind) {
  volatile int n = 8;
  if (kind[0] == 'a') {
    int* p = new int[n];
    p[0] = 1;
    const int v = p[n];            // one past the end: ASan heap-buffer-overflow
    delete[] p;
    return v;
  }
  volatile int big = 0x7fffffff;
  return big + n;                  // UBSan: signed integer overflow
}

int main() {
  if (const char* st = std::getenv("DMP_ASAN_SELFTEST")) return selftest(st);
  std::vector<Conv> convs;
  for (int B : {1, 8, 64, 512, 1024}) resnet_convs(convs, "resnet18-cifar", B, false, true);
  for (int B : {1, 32, 128}) resnet_convs(convs, "resnet50-imagenet", B, true, false);
  // AlexNet-CIFAR (/root/reference/example/models.py:25-49) and LeNet
  for (int B : {64, 10000}) {
    convs.push_back({"alexnet", B, 3, 32, 32, 64, 11, 11, 4, 5});
    convs.push_back({"alexnet", B, 64, 4, 4, 192, 5, 5, 1, 2});
    convs.push_back({"alexnet", B, 192, 2, 2, 384, 3, 3, 1, 1});
    convs.push_back({"alexnet", B, 384, 2, 2, 256, 3, 3, 1, 1});
    convs.push_back({"alexnet", B, 256, 2, 2, 256, 3, 3, 1, 1});
    convs.push_back({"lenet", B, 3, 32, 32, 6, 5, 5, 1, 0});
  }
  for (const Conv& c : convs) check_conv(c);
  // ViT-B/16 bs64 (197 tokens, D 768, MLP 3072) and the CNN heads
  for (int M : {64 * 197, 8 * 197, 64 * 196})
    for (int NK : {768, 2304, 3072}) {
      check_gemm(M, NK, 768);
      check_gemm(M, 768, NK);
    }
  check_gemm(512, 10, 512);
  check_gemm(128, 1000, 2048);
  EXPECT(dmp::layernorm_supported(768), "layernorm 768");
  EXPECT(dmp::attention_max_tokens() >= 197 && dmp::attention_head_dim() == 64, "attention");
  EXPECT(dmp::gap_linear_supported(512, 10), "gap_linear 512 -> 10");
  EXPECT(dmp::bn_maxpool_supported(64, 3, 2, 1) && !dmp::bn_maxpool_supported(64, 2, 2, 0),
         "bn_maxpool window");
  check_guards();
  std::printf("host_check: %lld checks over %zu conv shapes, %d failed\n", g_checks, convs.size(),
              g_fail);
  return g_fail == 0 ? 0 : 1;
}
