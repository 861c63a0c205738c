// Host-side AddressSanitizer / UBSan check of the C ABI's host logic (no GPU):
// the U-Net plan builder (topology, state_dict contract, aliases, layouts,
// workspace and gradient-workspace sizing, backward segments, traces) for the
// configuration families the package supports, plus the error paths of
// cwdm_unet_create and the shape-only helpers.  Built host-only
// (hipcc --cuda-host-only -fsanitize=address,undefined) by
// tests/test_asan_cpu.py; exits non-zero on the first contract violation,
// and ASan/UBSan abort on any memory error.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cwdm.h"

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                      \
    }                                                               \
  } while (0)

static cwdm_unet_config cfg(int mc, int nrb, std::vector<int> mult, int dtype, int updown, int freq, int in = 32,
                            int out = 8, int groups = 32) {
  cwdm_unet_config c;
  std::memset(&c, 0, sizeof(c));
  c.in_channels = in; c.model_channels = mc; c.out_channels = out; c.num_res_blocks = nrb;
  c.num_levels = (int)mult.size();
  for (size_t i = 0; i < mult.size(); ++i) c.channel_mult[i] = mult[i];
  c.num_groups = groups; c.dtype = dtype; c.resblock_updown = updown; c.use_freq = freq;
  return c;
}

static void exercise(const cwdm_unet_config& c, int64_t n) {
  cwdm_unet* u = nullptr;
  const int rc = cwdm_unet_create(&c, &u);
  CHECK(rc == CWDM_OK && u);
  if (rc != CWDM_OK) { std::fprintf(stderr, "  %s\n", cwdm_last_error()); return; }
  const int np = cwdm_unet_num_params(u);
  CHECK(np > 0);
  char name[256];
  int64_t shape[5];
  int nd = 0;
  int64_t numel = 0;
  for (int i = 0; i < np; ++i) {
    CHECK(cwdm_unet_param_info(u, i, name, sizeof(name), shape, &nd) == CWDM_OK);
    CHECK(nd >= 1 && nd <= 5 && std::strlen(name) > 0);
    int64_t k = 1;
    for (int d = 0; d < nd; ++d) k *= shape[d];
    numel += k;
  }
  CHECK(cwdm_unet_param_info(u, np, name, sizeof(name), shape, &nd) != CWDM_OK);   // out of range
  char small[4];
  CHECK(cwdm_unet_param_info(u, 0, small, sizeof(small), shape, &nd) == CWDM_OK && std::strlen(small) == 3);
  const int na = cwdm_unet_num_aliases(u);
  CHECK(na >= 0 && (c.use_freq || na == 0));
  for (int i = 0; i < na; ++i) {
    int owner = -1, before = -1;
    CHECK(cwdm_unet_alias_info(u, i, name, sizeof(name), &owner, &before) == CWDM_OK);
    CHECK(owner >= 0 && owner < np && before >= 0 && before <= np);
  }
  CHECK(cwdm_unet_alias_info(u, na, name, sizeof(name), nullptr, nullptr) != CWDM_OK);
  CHECK(cwdm_unet_packed_bytes(u) > numel);   // fp32 copies + packed weights
  for (int64_t b : {1, 2}) {
    const int64_t ws = cwdm_unet_workspace_bytes(u, b, n, n, 2 * n);
    CHECK(ws > 0);
    CHECK(cwdm_unet_flops(u, b, n, n, 2 * n) > 0);
    const int tc = cwdm_unet_trace_count(u);
    CHECK(tc > 0);
    for (int i = 0; i < tc; ++i) {
      int64_t off = 0;
      int ch = 0, lv = 0;
      CHECK(cwdm_unet_trace_info(u, i, b, n, n, 2 * n, &off, &ch, &lv) == CWDM_OK);
      CHECK(off < ws && ch > 0 && lv >= 0 && lv <= c.num_levels);
    }
    const int64_t gws = cwdm_unet_grad_workspace_bytes(u, b, n, n, 2 * n);
    CHECK(gws > 0);   // WavUNetModel trains too (Haar adjoint backward)
    CHECK(cwdm_unet_backward_flops(u, b, n, n, 2 * n) > 0);
  }
  CHECK(cwdm_unet_workspace_bytes(u, 0, n, n, n) < 0);
  {
    const int ns = cwdm_unet_backward_segments(u);
    CHECK(ns > 2);
    int64_t total = 0;
    for (int s = 0; s < ns; ++s) {
      int64_t off = -1, cnt = -1;
      CHECK(cwdm_unet_segment_range(u, s, &off, &cnt) == CWDM_OK);
      CHECK(off >= 0 && cnt >= 0 && off + cnt <= numel);
      total += cnt;
    }
    CHECK(total == numel);
    CHECK(cwdm_unet_packed_bwd_bytes(u) > 0);
  }
  cwdm_unet_destroy(u);
}

int main() {
  CHECK(cwdm_version() >= 2000);
  CHECK(cwdm_build_id() && std::strlen(cwdm_build_id()) > 0);
  for (int dt : {CWDM_F32, CWDM_BF16}) {
    exercise(cfg(64, 2, {1, 2, 2, 4, 4}, dt, 1, 0), 32);    // run.sh production topology
    exercise(cfg(64, 2, {1, 2, 2, 4, 4}, dt, 0, 0), 32);    // resblock_updown=False (stride-2 convs)
    exercise(cfg(32, 1, {1, 2}, dt, 1, 0, 32, 8, 8), 16);    // config-1 tiny model
    exercise(cfg(64, 2, {1, 2, 2, 4, 4}, dt, 1, 1), 32);    // WavUNetModel production topology
    exercise(cfg(32, 2, {1, 2}, dt, 1, 1, 32, 8, 8), 16);    // WavUNetModel tiny
    exercise(cfg(32, 1, {1, 1}, dt, 1, 1, 32, 8, 8), 16);    // WavUNetModel, one res block per level
    exercise(cfg(64, 2, {1, 2, 2}, dt, 1, 0, 256, 64), 56 / 4 * 4);  // config 5's 3-level U-Net
  }
  // error paths: each must fail with a message, never crash
  cwdm_unet* u = nullptr;
  CHECK(cwdm_unet_create(nullptr, &u) != CWDM_OK);
  auto bad = cfg(64, 2, {1, 2}, CWDM_BF16, 1, 0);
  bad.num_levels = 0;
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK && std::strlen(cwdm_last_error()) > 0);
  bad = cfg(64, 2, {1, 2}, 7, 1, 0);
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK);
  bad = cfg(64, 2, {1, 2}, CWDM_BF16, 1, 0, 20);
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK);                     // in_channels not a chunk multiple
  bad = cfg(64, 2, {1, 2}, CWDM_BF16, 1, 0, 32, 8, 7);
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK);                     // groups do not divide channels
  bad = cfg(32, 1, {1, 2}, CWDM_BF16, 1, 1);
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK);                     // WavUNet reuse with a channel change
  bad = cfg(32, 2, {1, 2}, CWDM_BF16, 0, 1);
  CHECK(cwdm_unet_create(&bad, &u) != CWDM_OK);                     // WavUNet without resblock_updown
  cwdm_unet_destroy(nullptr);
  // shape-only helpers
  CHECK(cwdm_conv3d_packed_bytes(64, 64, 3, CWDM_BF16) > 0 && cwdm_conv3d_packed_bytes(64, 64, 2, CWDM_BF16) < 0);
  CHECK(cwdm_conv3d_parts(CWDM_BF16, 56, 56, 56, 64) > 0);
  CHECK(cwdm_haar_nd_parts(3, 5, 4) == 1 && cwdm_haar_nd_parts(8, 8, 6) == 6);
  if (fails) {
    std::fprintf(stderr, "%d contract checks failed\n", fails);
    return 1;
  }
  std::printf("plan_asan: ok\n");
  return 0;
}
