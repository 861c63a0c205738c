// U-Net executor: builds the UNetModel topology of the run.sh configuration
// family (guided_diffusion/unet.py:482-725), owns the parameter
// naming contract (state_dict keys/shapes), packs weights into the kernel
// layouts and replays UNetModel.forward (unet.py:754-800) as a fixed list of
// GroupNorm-finalize and fused conv launches on one stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <cstdlib>
#include <vector>

#include "common.hpp"

namespace cwdm {
int launch_time_embed(const float* t, int B, int mc, const float* w1, const float* b1, const float* w2,
                      const float* b2, float* temb, hipStream_t s);
int launch_emb_proj(const float* temb, int B, int E, const float* W, const float* bias, int R, float* out,
                    hipStream_t s);
int launch_vec_add(const float* a, const float* b, float* out, int64_t n, hipStream_t s);
int launch_emb_bwd(const float* dEb, int R, int n, int B, const float* temb, int E, const float* W, float* dw,
                   float* db, float* dcb, float* dsil, hipStream_t s, int acc);
int launch_temb_bwd(const float* t, int B, int mc, const float* w1, const float* b1, const float* w2,
                    const float* temb, const float* dsil, float* dw1, float* db1, float* dw2, float* db2,
                    hipStream_t s);
int gn_silu_bwd_impl(const void* x0, int c0, const void* x1, int c1, const void* du, int du_mode, const float* ss,
                     const float* mr, const float* gamma, int groups, int64_t B, int64_t d, int64_t h, int64_t w,
                     int dtype, void* dx0, int acc0, void* dx1, int acc1, float* dgamma, float* dbeta, void* ws,
                     int64_t ws_bytes, float* chs, int64_t chs_stride, cwdm_stream_t stream, int acc_affine,
                     const float* pre_part = nullptr, int pre_nblk = 0, const float** coef_out = nullptr);
int gb_part_reduce(const float* part, int nblk, int C, int64_t B, int slices, float* out, hipStream_t s);
bool pw_gapply_ok(const cwdm_conv3d_desc* d);
int haar_nd_synth_add(int dtype, int64_t B, int64_t d, int64_t h, int64_t w, int C, const void* L, int64_t l_vs,
                      float lll, const void* H, int64_t h_vs, float high, void* fine, int acc, hipStream_t s);
int haar_nd_anal_add(int dtype, int64_t B, int64_t d, int64_t h, int64_t w, int C, const void* fine, void* L,
                     int64_t l_vs, float lll, int accL, void* H, int64_t h_vs, float high, int accH, hipStream_t s);
}  // namespace cwdm

using namespace cwdm;

namespace {

constexpr int64_t kAlign = 256;
inline int64_t align_up(int64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

struct Param { std::string name; std::vector<int64_t> shape; int64_t numel() const { int64_t n = 1; for (auto s : shape) n *= s; return n; } };

struct Tensor {
  int level, channels;
  int stats_kind = 0;  // producer of its (sum, sum^2) parts: 0 conv epilogue, 1 / 2 cwdm_haar_nd over its own /
                       // the half grid (analysis / synthesis output), -1 none (never GroupNorm'd)
};

struct GnStep {
  int src0, src1;       // tensor ids (src1 = -1 if none)
  int gamma_p, beta_p;  // param indices
  int64_t gamma_off, beta_off;
  int channels;
  int level;
  int ss_id;            // scale/shift buffer index
};

struct ConvStep {
  int a0, a1, amode, gn;        // gn = scale/shift buffer index or -1
  int w_p, b_p;                 // param indices of conv weight / bias
  int64_t w_off;                // packed weight byte offset
  int cin_a;
  int sb0, sb1;                 // 1x1 segment sources (-1 none)
  int ws_p, wsb_p;              // skip weight / bias params
  int64_t wsk_off;
  int cin_b;
  int bias_kind;                // 0 static packed bias, 1 emb-folded rows
  int64_t bias_off;             // packed byte offset (kind 0) or row offset (kind 1)
  int emb_w_p, emb_b_p;         // for kind 1: emb_layers params (pack)
  int res, rmode;
  int out;                      // tensor id, -1 = final fp32 output
  int cout;
  int level;                    // output level
  bool stats;
  int skip_conv = -1;           // conv1 of a block with a 1x1 skip: index of the block's conv2
  int64_t wsplit_off = -1;      // accurate fast mode: split-bf16 packed weights (cwdm_conv3d_pack_split), -1 none
  int64_t hsplit_off = -1;      // accurate fast mode, output head: K-expanded bf16 weights [hi | hi | lo] (head_split3_pack)
  int64_t xsplit_off = -1;      // accurate fast mode, small grids (level >= 2): the same for the bf16 small-grid kernel
  int64_t xsplit_sk_off = -1;   //   and for its 1x1 skip (k = 1)
  int s2 = 0;                   // stride-2 conv (Downsample.op) over a space-to-depth input: cin_a = 8 x its channels
};

struct S2dStep {  // space-to-depth of a Downsample conv's input (stride2.hip)
  int src, out, level_out, channels;
};

struct PoolStep {  // down-ResBlock pre-pass (cwdm_gn_silu_pool)
  int src, ss_id, out_h, out_x, level_out, channels;
};

struct HaarStep {  // WavUNetModel resampling / input pyramid (cwdm_haar_nd, wavelet_nd.hip)
  int src, high_in, out, high_out;  // tensor ids (-1 none)
  int inverse, all8;
  float lll_scale, high_scale;
  int emb_row;                      // emb projection row offset added after the resampling, -1 none
  bool stats;
  int level;                        // the coarse grid's level
};

struct Step { int kind; int idx; };  // kind 0 = gn, 1 = conv, 2 = pool pre-pass, 3 = space-to-depth, 4 = haar

// one ResBlock, for the backward (reverse order) and the gradient segments
struct Block {
  int g1, pool, c1, g2, c2;   // step indices (pool = -1 unless down)
  int x0, x1;                 // input tensors (x1 = -1 unless decoder concat)
  int updown;                 // 0 none, 1 up, 2 down; layers without a ResBlock (resblock_updown=False):
                              // 3 Downsample stride-2 conv (c1, pool = its S2dStep), 4 Upsample nearest + conv (c1);
                              // WavUNetModel ResBlocks: 5 down (DWT), 6 up (IDWT); 7 WaveletDownsample of the input
                              // pyramid (pool = its HaarStep, c1 = its conv, x0 = the pyramid level it transforms)
  int p_begin, p_end;         // parameter index range
  int emb_k;                  // index into emb_rows_*
  int hh = -1, hx = -1;       // WavUNetModel down / up blocks: HaarSteps of h (+ emb) and of x (x_upd)
};

}  // namespace

struct CopyJob {  // dst[0:n] = a[0:n] (+ b[0:n]): the fp32 parameter copies of a pack, one launch
  float* dst;
  const float* a;
  const float* b;
  long long n, blk0;
};

struct cwdm_unet {
  cwdm_unet_config cfg;
  // device job tables of the batched packs (uploaded when the job list changes)
  cwdm::PackJob* pack_tab = nullptr;
  cwdm::PackJob* bwd_tab = nullptr;
  CopyJob* copy_tab = nullptr;
  size_t pack_cap = 0, bwd_cap = 0, copy_cap = 0;
  std::vector<cwdm::PackJob> pack_cache, bwd_cache;
  std::vector<CopyJob> copy_cache;
  int E = 0;                      // time embed dim
  std::vector<Param> params;
  std::vector<Tensor> tensors;
  std::vector<GnStep> gns;
  std::vector<ConvStep> convs;
  std::vector<PoolStep> pools;
  std::vector<S2dStep> s2ds;
  std::vector<HaarStep> haars;
  std::vector<Step> steps;
  struct Alias { std::string name; int owner, before; };
  std::vector<Alias> aliases;     // WavUNetModel: second state_dict name of a reused parameter; before = the
                                  // parameter index it precedes in state_dict order
  std::vector<int> trace;         // tensor id per topology block (-1 = final output)
  std::vector<int> trace_level;
  int input_tensor = -1;          // pseudo tensor for x
  int R = 0;                      // emb projection rows
  std::vector<int> emb_rows_w, emb_rows_b, emb_rows_cb;  // per res block: emb weight/bias param, conv1 bias param
                                                         // (-1: the conv bias is not folded, WavUNet up/down)
  std::vector<int> emb_rows_off, emb_rows_n;
  int te_w1, te_b1, te_w2, te_b2;
  std::vector<Block> blocks;
  int head_g = -1, head_c = -1, head_p_begin = 0;
  std::vector<int64_t> goff;      // flat gradient offset (elements) per parameter
  int64_t grad_numel = 0;
  std::vector<int64_t> dg_off, dgs_off;  // packed dgrad weights per conv (-1 none)
  int64_t packed_bwd_bytes = 0;
  std::vector<char> ginit;        // backward: gradient buffer of tensor written yet
  int64_t off_te_w1, off_te_b1, off_te_w2, off_te_b2, off_emb_w, off_emb_b;
  int64_t packed_bytes = 0;
  int64_t split3_tmp = -1;      // fp32 staging of head_split3_pack (one region, the packs run in stream order)
  // profiling
  bool profiling = false;
  std::vector<hipEvent_t> ev;
  std::vector<double> ev_flops;
  std::vector<cwdm::ProfHook> hooks;  // per conv: the MFMA kernel launches inside it
  int ev_used = 0;

  int add_param(const std::string& n, std::vector<int64_t> s) {
    params.push_back({n, std::move(s)});
    return (int)params.size() - 1;
  }
};

namespace {

int esize(int dtype) { return dtype_size(dtype); }

void build(cwdm_unet* u) {
  const auto& c = u->cfg;
  const int mc = c.model_channels, E = 4 * mc;
  u->E = E;
  u->te_w1 = u->add_param("time_embed.0.weight", {E, mc});
  u->te_b1 = u->add_param("time_embed.0.bias", {E});
  u->te_w2 = u->add_param("time_embed.2.weight", {E, E});
  u->te_b2 = u->add_param("time_embed.2.bias", {E});

  auto new_tensor = [&](int level, int ch) {
    u->tensors.push_back({level, ch});
    return (int)u->tensors.size() - 1;
  };
  u->input_tensor = new_tensor(0, c.in_channels);

  // WavUNetModel's decoder registers one ResBlock under two prefixes
  // (wunet.py:648-687): while alias_from is set, names under it resolve to the
  // parameter of the same suffix under alias_to instead of a new parameter
  std::string alias_from, alias_to;
  auto addp = [&](const std::string& n, std::vector<int64_t> shape) {
    if (alias_from.empty() || n.compare(0, alias_from.size(), alias_from) != 0) return u->add_param(n, std::move(shape));
    const std::string owner = alias_to + n.substr(alias_from.size());
    for (size_t i = 0; i < u->params.size(); ++i)
      if (u->params[i].name == owner) {
        u->aliases.push_back({n, (int)i, (int)u->params.size()});
        return (int)i;
      }
    return -1;  // unreachable: the owner block was built first
  };
  auto conv_params = [&](const std::string& p, int co, int ci, int k, int* wp, int* bp) {
    *wp = addp(p + ".weight", {co, ci, k, k, k});
    *bp = addp(p + ".bias", {co});
  };

  // conv_in
  int h;
  {
    ConvStep cs{};
    conv_params("input_blocks.0.0", mc, c.in_channels, 3, &cs.w_p, &cs.b_p);
    cs.a0 = u->input_tensor; cs.a1 = -1; cs.amode = 0; cs.gn = -1; cs.cin_a = c.in_channels;
    cs.sb0 = cs.sb1 = -1; cs.ws_p = cs.wsb_p = -1; cs.cin_b = 0;
    cs.bias_kind = 0; cs.res = -1; cs.rmode = -1;
    cs.cout = mc; cs.level = 0; cs.stats = true;
    h = cs.out = new_tensor(0, mc);
    u->convs.push_back(cs);
    u->steps.push_back({1, (int)u->convs.size() - 1});
    u->trace.push_back(h);
    u->trace_level.push_back(0);
  }
  std::vector<int> stack{h};
  int level = 0;

  auto gn_step = [&](const std::string& p, int s0, int s1, int lvl) {
    GnStep g{};
    g.src0 = s0; g.src1 = s1;
    g.channels = u->tensors[s0].channels + (s1 >= 0 ? u->tensors[s1].channels : 0);
    g.gamma_p = addp(p + ".weight", {g.channels});
    g.beta_p = addp(p + ".bias", {g.channels});
    g.level = lvl;
    g.ss_id = (int)u->gns.size();
    u->gns.push_back(g);
    u->steps.push_back({0, g.ss_id});
    return g.ss_id;
  };

  auto haar_step = [&](const HaarStep& hs) {
    u->haars.push_back(hs);
    u->steps.push_back({4, (int)u->haars.size() - 1});
  };
  auto add_emb_row = [&](Block& blk, int wp, int bp, int cbp, int n) {
    u->emb_rows_w.push_back(wp); u->emb_rows_b.push_back(bp); u->emb_rows_cb.push_back(cbp);
    blk.emb_k = (int)u->emb_rows_off.size();
    u->emb_rows_off.push_back(u->R); u->emb_rows_n.push_back(n);
    const int row = u->R;
    u->R += n;
    return row;
  };

  // ResBlock (unet.py:185-311): returns output tensor.  updown 5 / 6: the
  // WavUNetModel ResBlock (wunet.py:210-269) that down/upsamples by DWT / IDWT
  // AFTER its first conv; skip_bands = the 7 high bands an up block inverts
  // with, *skip_out = the 7 high bands a down block returns.
  auto resblock = [&](const std::string& p, int x0, int x1, int cout, int updown, int skip_bands = -1,
                      int* skip_out = nullptr) {
    Block blk{};
    blk.p_begin = (int)u->params.size();
    blk.x0 = x0; blk.x1 = x1; blk.updown = updown; blk.pool = -1;
    const int lin = u->tensors[x0].level;
    const int cin = u->tensors[x0].channels + (x1 >= 0 ? u->tensors[x1].channels : 0);
    const int lout = (updown == 2 || updown == 5) ? lin + 1 : ((updown == 1 || updown == 6) ? lin - 1 : lin);
    int g1 = gn_step(p + ".in_layers.0", x0, x1, lin);
    blk.g1 = g1;
    if (updown >= 5) {
      const bool down = updown == 5;
      ConvStep c1{};
      conv_params(p + ".in_layers.2", cout, cin, 3, &c1.w_p, &c1.b_p);
      c1.emb_w_p = addp(p + ".emb_layers.1.weight", {cout, E});
      c1.emb_b_p = addp(p + ".emb_layers.1.bias", {cout});
      c1.a0 = x0; c1.a1 = -1; c1.amode = 0; c1.gn = g1; c1.cin_a = cin;
      c1.sb0 = c1.sb1 = -1; c1.ws_p = c1.wsb_p = -1; c1.cin_b = 0;
      c1.bias_kind = 0; c1.res = -1; c1.rmode = -1; c1.cout = cout; c1.level = lin; c1.stats = false;
      const int h1 = c1.out = new_tensor(lin, cout);
      u->tensors[h1].stats_kind = -1;
      u->convs.push_back(c1);
      blk.c1 = (int)u->convs.size() - 1;
      u->steps.push_back({1, blk.c1});
      const int row = add_emb_row(blk, c1.emb_w_p, c1.emb_b_p, -1, cout);
      // h: DWT -> LLL / 3 (+ the 7 high bands as the skip) or IDWT(3 h, skip); then + emb
      HaarStep hh{};
      hh.src = h1; hh.high_in = down ? -1 : skip_bands; hh.inverse = down ? 0 : 1; hh.all8 = 0;
      hh.lll_scale = down ? 1.f / 3.f : 3.f; hh.high_scale = 1.f;
      hh.out = new_tensor(lout, cout);
      u->tensors[hh.out].stats_kind = down ? 1 : 2;
      hh.high_out = -1;
      if (down) {
        hh.high_out = new_tensor(lout, 7 * cout);
        u->tensors[hh.high_out].stats_kind = -1;
      }
      hh.emb_row = row; hh.stats = true; hh.level = down ? lout : lin;
      haar_step(hh);
      blk.hh = (int)u->haars.size() - 1;
      if (skip_out) *skip_out = hh.high_out;
      // x: the same resampling, LLL only / with the same skip bands (x_upd)
      HaarStep hx = hh;
      hx.src = x0; hx.out = new_tensor(lout, cin); hx.high_out = -1; hx.emb_row = -1; hx.stats = false;
      u->tensors[hx.out].stats_kind = -1;
      haar_step(hx);
      blk.hx = (int)u->haars.size() - 1;
      const int g2 = gn_step(p + ".out_layers.0", hh.out, -1, lout);
      blk.g2 = g2;
      ConvStep c2{};
      conv_params(p + ".out_layers.3", cout, cout, 3, &c2.w_p, &c2.b_p);
      c2.a0 = hh.out; c2.a1 = -1; c2.amode = 0; c2.gn = g2; c2.cin_a = cout;
      c2.sb0 = c2.sb1 = -1; c2.ws_p = c2.wsb_p = -1; c2.cin_b = 0;
      c2.res = hx.out; c2.rmode = 0;  // up/down blocks keep the channel count (checked at create)
      c2.bias_kind = 0; c2.cout = cout; c2.level = lout; c2.stats = true;
      const int o = c2.out = new_tensor(lout, cout);
      u->convs.push_back(c2);
      blk.c2 = (int)u->convs.size() - 1;
      u->steps.push_back({1, blk.c2});
      blk.p_end = (int)u->params.size();
      u->blocks.push_back(blk);
      return o;
    }
    int xres = x0, xrmode = updown == 2 ? 2 : (updown == 1 ? 1 : 0);
    int a_src = x0, a_mode = updown, a_gn = g1;
    if (updown == 2) {
      // AvgPool(SiLU(GN(x))) and AvgPool(x) once, at the low resolution
      PoolStep ps{};
      ps.src = x0; ps.ss_id = g1; ps.level_out = lout; ps.channels = cin;
      ps.out_h = new_tensor(lout, cin);
      ps.out_x = new_tensor(lout, cin);
      u->pools.push_back(ps);
      u->steps.push_back({2, (int)u->pools.size() - 1});
      blk.pool = (int)u->pools.size() - 1;
      a_src = ps.out_h; a_mode = 0; a_gn = -1;
      xres = ps.out_x; xrmode = 0;
    }
    ConvStep c1{};
    conv_params(p + ".in_layers.2", cout, cin, 3, &c1.w_p, &c1.b_p);
    c1.emb_w_p = addp(p + ".emb_layers.1.weight", {cout, E});
    c1.emb_b_p = addp(p + ".emb_layers.1.bias", {cout});
    c1.a0 = a_src; c1.a1 = x1; c1.amode = a_mode; c1.gn = a_gn; c1.cin_a = cin;
    c1.sb0 = c1.sb1 = -1; c1.ws_p = c1.wsb_p = -1; c1.cin_b = 0;
    c1.bias_kind = 1; c1.bias_off = add_emb_row(blk, c1.emb_w_p, c1.emb_b_p, c1.b_p, cout);
    c1.res = -1; c1.rmode = -1; c1.cout = cout; c1.level = lout; c1.stats = true;
    int h1 = c1.out = new_tensor(lout, cout);
    u->convs.push_back(c1);
    blk.c1 = (int)u->convs.size() - 1;
    u->steps.push_back({1, (int)u->convs.size() - 1});

    int g2 = gn_step(p + ".out_layers.0", h1, -1, lout);
    blk.g2 = g2;
    ConvStep c2{};
    conv_params(p + ".out_layers.3", cout, cout, 3, &c2.w_p, &c2.b_p);
    c2.a0 = h1; c2.a1 = -1; c2.amode = 0; c2.gn = g2; c2.cin_a = cout;
    c2.sb0 = c2.sb1 = -1; c2.ws_p = c2.wsb_p = -1; c2.cin_b = 0;
    c2.res = -1; c2.rmode = -1;
    if (cin != cout) {
      conv_params(p + ".skip_connection", cout, cin, 1, &c2.ws_p, &c2.wsb_p);
      c2.sb0 = x0; c2.sb1 = x1; c2.cin_b = cin;
      u->convs[blk.c1].skip_conv = (int)u->convs.size();  // c2's index once pushed below
    } else {
      c2.res = xres;
      c2.rmode = xrmode;
    }
    c2.bias_kind = 0; c2.cout = cout; c2.level = lout; c2.stats = true;
    int o = c2.out = new_tensor(lout, cout);
    u->convs.push_back(c2);
    u->steps.push_back({1, (int)u->convs.size() - 1});
    blk.c2 = (int)u->convs.size() - 1;
    blk.p_end = (int)u->params.size();
    u->blocks.push_back(blk);
    return o;
  };

  // resblock_updown=False: Downsample(use_conv=True) = a stride-2 conv, run as
  // a stride-1 conv over the space-to-depth input; Upsample(use_conv=True) =
  // nearest x2 folded into the conv's gather (a_mode 1).  unet.py:40-100, :606-612, :700-706.
  auto resample_layer = [&](const std::string& p, int x, int down) {
    Block blk{};
    blk.p_begin = (int)u->params.size();
    blk.x0 = x; blk.x1 = -1; blk.updown = down ? 3 : 4; blk.pool = -1; blk.g1 = blk.g2 = blk.c2 = -1; blk.emb_k = -1;
    const int lin = u->tensors[x].level, chn = u->tensors[x].channels;
    const int lout = down ? lin + 1 : lin - 1;
    ConvStep cs{};
    conv_params(p, chn, chn, 3, &cs.w_p, &cs.b_p);
    cs.a1 = -1; cs.gn = -1; cs.sb0 = cs.sb1 = -1; cs.ws_p = cs.wsb_p = -1; cs.cin_b = 0;
    cs.bias_kind = 0; cs.res = -1; cs.rmode = -1; cs.cout = chn; cs.level = lout; cs.stats = true;
    if (down) {
      S2dStep sd{x, new_tensor(lout, 8 * chn), lout, chn};
      u->s2ds.push_back(sd);
      u->steps.push_back({3, (int)u->s2ds.size() - 1});
      blk.pool = (int)u->s2ds.size() - 1;
      cs.a0 = sd.out; cs.amode = 0; cs.cin_a = 8 * chn; cs.s2 = 1;
    } else {
      cs.a0 = x; cs.amode = 1; cs.cin_a = chn;
    }
    const int o = cs.out = new_tensor(lout, chn);
    u->convs.push_back(cs);
    u->steps.push_back({1, (int)u->convs.size() - 1});
    blk.c1 = (int)u->convs.size() - 1;
    blk.p_end = (int)u->params.size();
    u->blocks.push_back(blk);
    return o;
  };

  int ch = mc, idx = 1;
  const int nl = c.num_levels;
  if (c.use_freq) {
    // WavUNetModel (wunet.py:470-700, forward :754-795): every level ends in a
    // DWT ResBlock and a WaveletDownsample of the input pyramid; the decoder
    // has no concatenation, only the high-band skips into its IDWT ResBlocks
    std::vector<int> skips;
    int pyr = u->input_tensor;
    for (int l = 0; l < nl; ++l) {
      const int mult = c.channel_mult[l];
      for (int r = 0; r < c.num_res_blocks; ++r) {
        h = resblock("input_blocks." + std::to_string(idx) + ".0", h, -1, mult * mc, 0);
        ch = mult * mc;
        u->trace.push_back(h); u->trace_level.push_back(level);
        ++idx;
      }
      int sk = -1;
      h = resblock("input_blocks." + std::to_string(idx) + ".0", h, -1, ch, 5, -1, &sk);
      skips.push_back(sk);
      ++level;
      u->trace.push_back(h); u->trace_level.push_back(level);
      // WaveletDownsample (:131-145): conv(cat(8 bands) / 3) + h
      const int cp = u->tensors[pyr].channels;
      HaarStep hp{};
      hp.src = pyr; hp.high_in = -1; hp.high_out = -1; hp.inverse = 0; hp.all8 = 1;
      hp.lll_scale = hp.high_scale = 1.f / 3.f; hp.emb_row = -1; hp.stats = false; hp.level = level;
      hp.out = new_tensor(level, 8 * cp);
      u->tensors[hp.out].stats_kind = -1;
      haar_step(hp);
      Block pb{};   // the WaveletDownsample as a backward segment of its own
      pb.updown = 7; pb.pool = (int)u->haars.size() - 1; pb.x0 = pyr; pb.x1 = -1;
      pb.g1 = pb.g2 = pb.c2 = -1; pb.emb_k = -1;
      pb.p_begin = (int)u->params.size();
      ConvStep cs{};
      conv_params("input_blocks." + std::to_string(idx + 1) + ".0.conv", ch, 8 * cp, 3, &cs.w_p, &cs.b_p);
      cs.a0 = hp.out; cs.a1 = -1; cs.amode = 0; cs.gn = -1; cs.cin_a = 8 * cp;
      cs.sb0 = cs.sb1 = -1; cs.ws_p = cs.wsb_p = -1; cs.cin_b = 0;
      cs.bias_kind = 0; cs.res = h; cs.rmode = 0; cs.cout = ch; cs.level = level; cs.stats = true;
      h = pyr = cs.out = new_tensor(level, ch);
      u->convs.push_back(cs);
      u->steps.push_back({1, (int)u->convs.size() - 1});
      pb.c1 = (int)u->convs.size() - 1;
      pb.p_end = (int)u->params.size();
      u->blocks.push_back(pb);
      u->trace.push_back(h); u->trace_level.push_back(level);
      idx += 2;
    }
    h = resblock("middle_block.0", h, -1, ch, 0);
    u->trace.push_back(h); u->trace_level.push_back(level);
    h = resblock("middle_block.1", h, -1, ch, 0);
    u->trace.push_back(h); u->trace_level.push_back(level);
    idx = 0;
    for (int l = nl - 1; l >= 0; --l) {
      const int mult = c.channel_mult[l];
      const int sk = skips.back();  // popped by the level's first output block (hs.pop() skips the Nones)
      skips.pop_back();
      std::string owner;
      for (int i = 0; i <= c.num_res_blocks; ++i) {
        const std::string p = "output_blocks." + std::to_string(idx);
        if (i != c.num_res_blocks) {
          h = resblock(p + ".0", h, -1, mc * mult, 0);
          ch = mc * mult;
          owner = p + ".0";
        } else {
          // Sequential(<the level's last ResBlock again>, IDWT ResBlock)
          alias_from = p + ".0.";
          alias_to = owner + ".";
          h = resblock(p + ".0", h, -1, ch, 0);
          alias_from.clear();
          h = resblock(p + ".1", h, -1, ch, 6, sk);
          --level;
        }
        u->trace.push_back(h); u->trace_level.push_back(level);
        ++idx;
      }
    }
    for (int i = 0; i < c.num_res_blocks; ++i) {
      h = resblock("out_res." + std::to_string(i) + ".0", h, -1, ch, 0);
      u->trace.push_back(h); u->trace_level.push_back(level);
    }
  }
  for (int l = 0; l < nl && !c.use_freq; ++l) {
    const int mult = c.channel_mult[l];
    for (int r = 0; r < c.num_res_blocks; ++r) {
      h = resblock("input_blocks." + std::to_string(idx) + ".0", h, -1, mult * mc, 0);
      ch = mult * mc;
      stack.push_back(h);
      u->trace.push_back(h); u->trace_level.push_back(level);
      ++idx;
    }
    if (l != nl - 1) {
      const std::string p = "input_blocks." + std::to_string(idx) + ".0";
      h = c.resblock_updown ? resblock(p, h, -1, ch, 2) : resample_layer(p + ".op", h, 1);
      ++level;
      stack.push_back(h);
      u->trace.push_back(h); u->trace_level.push_back(level);
      ++idx;
    }
  }
  if (!c.use_freq) {
    h = resblock("middle_block.0", h, -1, ch, 0);
    u->trace.push_back(h); u->trace_level.push_back(level);
    h = resblock("middle_block.1", h, -1, ch, 0);
    u->trace.push_back(h); u->trace_level.push_back(level);
    idx = 0;
  }
  for (int l = nl - 1; l >= 0 && !c.use_freq; --l) {
    const int mult = c.channel_mult[l];
    for (int i = 0; i <= c.num_res_blocks; ++i) {
      int skip = stack.back();
      stack.pop_back();
      h = resblock("output_blocks." + std::to_string(idx) + ".0", h, skip, mc * mult, 0);
      ch = mc * mult;
      u->trace.push_back(h); u->trace_level.push_back(level);
      if (l && i == c.num_res_blocks) {
        const std::string p = "output_blocks." + std::to_string(idx) + ".1";
        h = c.resblock_updown ? resblock(p, h, -1, ch, 1) : resample_layer(p + ".conv", h, 0);
        --level;
        u->trace.push_back(h); u->trace_level.push_back(level);
      }
      ++idx;
    }
  }
  // out head
  u->head_p_begin = (int)u->params.size();
  int g = gn_step("out.0", h, -1, 0);
  u->head_g = g;
  ConvStep co{};
  conv_params("out.2", c.out_channels, ch, 3, &co.w_p, &co.b_p);
  co.a0 = h; co.a1 = -1; co.amode = 0; co.gn = g; co.cin_a = ch;
  co.sb0 = co.sb1 = -1; co.ws_p = co.wsb_p = -1; co.cin_b = 0;
  co.bias_kind = 0; co.res = -1; co.rmode = -1; co.cout = c.out_channels; co.level = 0; co.stats = false;
  co.out = -1;
  u->convs.push_back(co);
  u->head_c = (int)u->convs.size() - 1;
  u->steps.push_back({1, (int)u->convs.size() - 1});
  u->trace.push_back(-1); u->trace_level.push_back(0);

  // packed layout
  int64_t off = 0;
  auto take = [&](int64_t bytes) { int64_t o = off; off = align_up(off + bytes); return o; };
  u->off_te_w1 = take(u->params[u->te_w1].numel() * 4);
  u->off_te_b1 = take(u->params[u->te_b1].numel() * 4);
  u->off_te_w2 = take(u->params[u->te_w2].numel() * 4);
  u->off_te_b2 = take(u->params[u->te_b2].numel() * 4);
  u->off_emb_w = take((int64_t)u->R * E * 4);
  u->off_emb_b = take((int64_t)u->R * 4);
  int64_t split3_max = 0;
  for (auto& cs : u->convs) {
    cs.w_off = take(cwdm_conv3d_packed_bytes(cs.cout, cs.cin_a, 3, c.dtype));
    if (c.mfma_split && c.dtype == CWDM_F32 && !cs.s2 && cs.cout % 64 == 0 && cs.cin_a % 16 == 0)
      cs.wsplit_off = take(cwdm_conv3d_packed_split_bytes(cs.cout, cs.cin_a));
    if (c.mfma_split && c.dtype == CWDM_F32 && &cs == &u->convs[u->head_c] && cs.a1 < 0 && cs.amode == 0 &&
        cs.gn >= 0 && cs.cout <= 16 && cs.cin_a % 32 == 0 && 3 * cs.cin_a <= 256) {
      cs.hsplit_off = take(cwdm_conv3d_packed_bytes(cs.cout, 3 * cs.cin_a, 3, CWDM_BF16));
      split3_max = std::max(split3_max, (int64_t)3 * cs.cout * cs.cin_a * 27 * 4);
    }
    // the small grids' K-expanded split convs (unet_forward_impl, xsg_plan): every 3x3x3 conv
    // that can land on a grid below the wide kernels' minimum width
    if (c.mfma_split && c.dtype == CWDM_F32 && !cs.s2 && cs.level >= 2 && cs.amode <= 1 &&
        cs.cout % 64 == 0 && cs.cin_a % 32 == 0) {
      cs.xsplit_off = take(cwdm_conv3d_packed_bytes(cs.cout, 3 * cs.cin_a, 3, CWDM_BF16));
      split3_max = std::max(split3_max, (int64_t)3 * cs.cout * cs.cin_a * 27 * 4);
      if (cs.ws_p >= 0 && cs.cin_b % 32 == 0) {
        cs.xsplit_sk_off = take(cwdm_conv3d_packed_bytes(cs.cout, 3 * cs.cin_b, 1, CWDM_BF16));
        split3_max = std::max(split3_max, (int64_t)3 * cs.cout * cs.cin_b * 4);
      }
    }
    if (cs.ws_p >= 0) cs.wsk_off = take(cwdm_conv3d_packed_bytes(cs.cout, cs.cin_b, 1, c.dtype));
    if (cs.bias_kind == 0) cs.bias_off = take((int64_t)cs.cout * 4);
  }
  for (auto& gs : u->gns) {
    gs.gamma_off = take((int64_t)gs.channels * 4);
    gs.beta_off = take((int64_t)gs.channels * 4);
  }
  if (split3_max > 0) u->split3_tmp = take(split3_max);
  u->packed_bytes = off;

  // flat gradient layout (state_dict order, contiguous)
  int64_t go = 0;
  for (const auto& pr : u->params) { u->goff.push_back(go); go += pr.numel(); }
  u->grad_numel = go;
  // packed dgrad weights (every conv but conv_in, whose input needs no gradient)
  const int ck = 32 / esize(c.dtype);
  int64_t bo = 0;
  auto takeb = [&](int64_t bytes) { int64_t o = bo; bo = align_up(bo + bytes); return o; };
  for (size_t i = 0; i < u->convs.size(); ++i) {
    const auto& cs = u->convs[i];
    const int cpad = (int)((cs.cout + ck - 1) / ck * ck);
    u->dg_off.push_back(i == 0 ? -1 : takeb(cwdm_conv3d_packed_bytes(cs.cin_a, cpad, 3, c.dtype)));
    u->dgs_off.push_back(cs.ws_p >= 0 ? takeb(cwdm_conv3d_packed_bytes(cs.cin_b, cpad, 1, c.dtype)) : -1);
  }
  u->packed_bwd_bytes = bo;
}

}  // namespace
namespace cwdm {
bool v4_eligible(const cwdm_conv3d_desc* d);
bool v5_eligible(const cwdm_conv3d_desc* d, bool gn);
int head_split3_prep(const float* x, const float* gn, int64_t B, int64_t V, int C, void* x3, hipStream_t s);
int head_split3_pack(const float* w, int cout, int cin, float* tmp, void* out, hipStream_t s, int k);
int split3_prep(const float* x0, int c0, const float* x1, int c1, const float* gn, int64_t B, int64_t V, int cm,
                void* x3, hipStream_t s);
bool sg_skip_eligible(const cwdm_conv3d_desc* d);
int sg_skip_ksplit(const cwdm_conv3d_desc* d);
int sg_skip_launch(const cwdm_conv3d_desc* d, void* out, void* partial, hipStream_t s);
bool sg_eligible(const cwdm_conv3d_desc* d);
int sg_ksplit(const cwdm_conv3d_desc* d);
int64_t ksplit_slice_voxels(const cwdm_conv3d_desc* d);
extern thread_local bool g_sg_fp32x;
bool pw_split_eligible(const cwdm_conv3d_desc* d);
int pw_split_forward(const cwdm_conv3d_desc* d, hipStream_t s);
bool apply_skip_ok(int dtype, int C, int cout, int64_t B, int64_t vpb);
int gn_apply_skip(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B, int64_t vpb, int dtype,
                  const void* wskip, int cout, void* act, void* skip, hipStream_t s);
int v4_launch(const cwdm_conv3d_desc* d, const void* a0, int c0, const void* a1, int c1, int a0_cm,
              const void* res, int rmode, void* partial, hipStream_t s);
extern thread_local unsigned* g_sg_sync;
extern thread_local int g_stats_wg;         // conv3d_v5.hip: per-workgroup GroupNorm partials wanted
extern thread_local int64_t g_stats_rows;   // ... and the rows the last launch wrote (0: per tile)
int64_t sg_sync_bytes(int ksplit);
int64_t plan_sync_bytes();
bool head_eligible(const cwdm_conv3d_desc* d);
extern thread_local std::vector<PackJob>* g_pack_batch;  // conv3d.hip
int pack_batch_run(std::vector<PackJob>& jobs, int dtype, PackJob* table, std::vector<PackJob>& cache, hipStream_t s);
// conv3d_v4.hip: where conv3d_v4_forward's GroupNorm pre-pass writes the
// activated input (null: its own workspace), and whether it did
extern thread_local void* g_act_keep;
extern thread_local int g_act_kept;
struct ActKeepScope {
  void* ptr;
  explicit ActKeepScope(void* p) : ptr(p) { g_act_keep = p; g_act_kept = 0; }
  ~ActKeepScope() { g_act_keep = nullptr; }
  bool used() const { return g_act_kept != 0; }
};
}  // namespace cwdm
namespace {
// the small-grid conv's K-split arrival counters for one launch list: one block
// in the plan's workspace, zeroed once (a memset node) before the list -- each
// K-split launch leaves its counters zero again -- and handed to the launches
// for the duration of the call (conv3d_sg.hip)
struct SgSyncScope {
  SgSyncScope(void* block) { cwdm::g_sg_sync = reinterpret_cast<unsigned*>(block); }
  ~SgSyncScope() { cwdm::g_sg_sync = nullptr; }
};
// the small-grid kernel's fp32 output / residual, for the K-expanded split convs only
struct SgFp32xScope {
  SgFp32xScope() { cwdm::g_sg_fp32x = true; }
  ~SgFp32xScope() { cwdm::g_sg_fp32x = false; }
};
}  // namespace
namespace {

struct Layout {
  int64_t temb, ebias, split, split_bytes, sync;
  int64_t skipbuf = 0;          // conv2 residual written by the fused GroupNorm + 1x1-skip pass
  std::vector<char> skip_fused; // per conv1 with a skip: that pass is used
  std::vector<int64_t> t_off, s_off, s_parts;
  std::vector<int64_t> ss_off, mr_off;
  int64_t total;
  // training: the activated input (GroupNorm+SiLU, chunk-major) of every conv
  // whose forward pre-pass writes one, kept past the inference total for the
  // DMA-staged wgrad (cwdm_unet_train_workspace_bytes); -1 = not kept
  std::vector<int64_t> keep_off;
  int64_t train_total;
};

// shape-only descriptor of one conv step (pointers filled in by the forward)
cwdm_conv3d_desc conv_shape(const cwdm_unet* u, const ConvStep& cs, int64_t B, int64_t D, int64_t H, int64_t W) {
  cwdm_conv3d_desc d{};
  d.dtype = u->cfg.dtype;
  d.B = B; d.D = D >> cs.level; d.H = H >> cs.level; d.W = W >> cs.level;
  d.cout = cs.cout;
  d.a_c0 = u->tensors[cs.a0].channels;
  d.a_c1 = cs.a1 >= 0 ? u->tensors[cs.a1].channels : 0;
  d.a_mode = cs.amode;
  // presence flags only: they select the kernel path and size its workspace
  // (the DMA-staged kernel needs room for the GroupNorm+SiLU'd input and the skip)
  d.a_w = reinterpret_cast<const void*>(1);
  if (cs.gn >= 0) d.a_gn = reinterpret_cast<const float*>(1);
  if (cs.ws_p >= 0) {
    d.b_c0 = u->tensors[cs.sb0].channels;
    d.b_c1 = cs.sb1 >= 0 ? u->tensors[cs.sb1].channels : 0;
    d.b_w = reinterpret_cast<const void*>(1);  // presence flag only
  }
  d.res_mode = cs.rmode;
  d.out_dtype = cs.out < 0 ? CWDM_F32 : u->cfg.dtype;
  if (cs.wsplit_off >= 0) d.a_w_split = reinterpret_cast<const void*>(1);   // presence flag only
  return d;
}

// the accurate fast mode on a small grid: the fp32 conv d (GroupNorm+SiLU'd or plain input, optional 1x1
// skip) as ONE bf16 small-grid conv over the K-expanded split input [hi | lo | hi] of SiLU(GN(x))
// (cwdm::split3_prep, chunk-major) against the weights [hi | hi | lo] (cs.xsplit_off): the three
// products hi.hi + lo.hi + hi.lo of the split kernels, fp32 output and residual.  The 1x1 skip,
// if any, runs first into an fp32 residual buffer: the same K expansion on the small-grid kernel's
// 1x1 form (channels-last split of the raw input, cs.xsplit_sk_off), else pw_split.
// Workspace: x3 (the conv's or the skip's split input) | skip | K-split slices.
struct XsgPlan {
  bool ok = false;
  bool sk_sg = false;     // the skip on the small-grid kernel
  cwdm_conv3d_desc e{};   // the bf16 desc (pointers filled in by the forward)
  cwdm_conv3d_desc ek{};  //   and the skip's
  int64_t x3_bytes = 0, skip_bytes = 0, total = 0;
};
XsgPlan xsg_plan(const cwdm_unet* u, const ConvStep& cs, const cwdm_conv3d_desc& d) {
  XsgPlan x;
  if (cs.xsplit_off < 0 || d.res_mode > 1 || (d.b_w && d.res_mode >= 0)) return x;
  const int64_t sv = cs.amode == 1 ? (d.D / 2) * (d.H / 2) * (d.W / 2) : d.D * d.H * d.W;
  const int C = d.a_c0 + d.a_c1;
  cwdm_conv3d_desc e = d;
  e.dtype = CWDM_BF16;
  e.a_c0 = 3 * C; e.a_c1 = 0; e.a_gn = nullptr; e.a_w_split = nullptr;
  e.b_c0 = e.b_c1 = 0; e.b_w = nullptr;
  if (d.b_w) e.res_mode = 0;
  e.out_dtype = CWDM_F32;
  SgFp32xScope fx;
  if (!cwdm::sg_eligible(&e)) return x;
  x.e = e;
  x.x3_bytes = align_up(d.B * sv * 3 * C * 2);
  x.skip_bytes = d.b_w ? align_up(d.B * d.D * d.H * d.W * d.cout * 4) : 0;
  const int S = cwdm::sg_ksplit(&e);
  int64_t part = S > 1 ? (int64_t)S * d.B * cwdm::ksplit_slice_voxels(&e) * d.cout * 4 : 0;
  if (d.b_w && cs.xsplit_sk_off >= 0) {
    cwdm_conv3d_desc k = d;
    k.dtype = CWDM_BF16;
    k.a0 = k.a1 = nullptr; k.a_c0 = k.a_c1 = 0; k.a_gn = nullptr; k.a_w = nullptr; k.a_w_split = nullptr; k.a_mode = 0;
    k.b_c0 = 3 * (d.b_c0 + d.b_c1); k.b_c1 = 0; k.b1 = nullptr;
    k.bias = nullptr; k.bias_bstride = 0; k.stats = nullptr; k.res = nullptr; k.res_mode = -1;
    k.out_dtype = CWDM_F32;
    if (cwdm::sg_skip_eligible(&k)) {
      x.sk_sg = true;
      x.ek = k;
      x.x3_bytes = std::max(x.x3_bytes, align_up(d.B * d.D * d.H * d.W * k.b_c0 * 2));
      const int Sk = cwdm::sg_skip_ksplit(&k);
      if (Sk > 1) part = std::max(part, (int64_t)Sk * d.B * cwdm::ksplit_slice_voxels(&k) * d.cout * 4);
    }
  }
  x.total = x.x3_bytes + x.skip_bytes + part;
  (void)u;
  x.ok = true;
  return x;
}

Layout layout(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  Layout L;
  int64_t off = 0;
  auto take = [&](int64_t bytes) { int64_t o = off; off = align_up(off + bytes); return o; };
  L.sync = take(cwdm::plan_sync_bytes());   // first: a memset block at a 256-byte boundary
  L.temb = take(B * u->E * 4);
  L.ebias = take(B * (int64_t)u->R * 4);
  const int es = esize(u->cfg.dtype);
  for (size_t i = 0; i < u->tensors.size(); ++i) {
    const auto& t = u->tensors[i];
    const int64_t d = D >> t.level, h = H >> t.level, w = W >> t.level;
    if ((int)i == u->input_tensor) {
      L.t_off.push_back(-1); L.s_off.push_back(-1); L.s_parts.push_back(0);
      continue;
    }
    L.t_off.push_back(take(B * d * h * w * t.channels * es));
    const int64_t parts = t.stats_kind < 0    ? 0
                          : t.stats_kind == 1 ? cwdm_haar_nd_parts(d, h, w)
                          : t.stats_kind == 2 ? cwdm_haar_nd_parts(d / 2, h / 2, w / 2)
                                              : cwdm_conv3d_parts(u->cfg.dtype, d, h, w, t.channels);
    L.s_parts.push_back(parts);
    L.s_off.push_back(take(B * parts * t.channels * 2 * 4));
  }
  for (const auto& g : u->gns) L.ss_off.push_back(take(B * (int64_t)g.channels * 2 * 4));
  for (size_t i = 0; i < u->gns.size(); ++i) L.mr_off.push_back(take(B * (int64_t)u->cfg.num_groups * 2 * 4));
  int64_t split = 0;
  for (const auto& cs : u->convs) {
    cwdm_conv3d_desc d = conv_shape(u, cs, B, D, H, W);
    const int64_t n = cwdm_conv3d_workspace_bytes(&d);
    if (n > split) split = n;
    const XsgPlan xp = xsg_plan(u, cs, d);
    if (xp.ok && xp.total > split) split = xp.total;
  }
  L.split_bytes = split;
  L.split = take(split);
  // ResBlocks with a 1x1 skip whose convs run on the DMA kernel: GN1 and the
  // skip read x in one pass (cwdm::gn_apply_skip)
  L.skip_fused.assign(u->convs.size(), 0);
  int64_t skipb = 0;
  const char* fe = std::getenv("CWDM_SKIP_FUSE");  // "0": A/B switch for the fused pass
  const bool fuse = !(fe && fe[0] == '0');
  for (size_t i = 0; fuse && i < u->convs.size(); ++i) {
    const auto& c1 = u->convs[i];
    if (c1.skip_conv < 0 || c1.gn < 0 || c1.amode != 0) continue;
    const auto& c2 = u->convs[c1.skip_conv];
    cwdm_conv3d_desc d1 = conv_shape(u, c1, B, D, H, W), d2 = conv_shape(u, c2, B, D, H, W);
    const int64_t vpb = d1.D * d1.H * d1.W;
    if (!cwdm::v4_eligible(&d1) || !cwdm::v4_eligible(&d2) ||
        !cwdm::apply_skip_ok(u->cfg.dtype, c1.cin_a, c2.cout, B, vpb))
      continue;
    L.skip_fused[i] = 1;
    skipb = std::max(skipb, B * vpb * c2.cout * es);
  }
  L.skipbuf = take(skipb);
  L.total = off;
  L.keep_off.assign(u->convs.size(), -1);
  for (size_t i = 0; i < u->convs.size(); ++i) {
    const auto& cs = u->convs[i];
    cwdm_conv3d_desc d = conv_shape(u, cs, B, D, H, W);
    if (!dtype_half(u->cfg.dtype) || cs.gn < 0 || cs.amode > 1 || cs.s2 || cwdm::head_eligible(&d) ||
        !cwdm::v4_eligible(&d))
      continue;
    const int64_t sv = cs.amode == 1 ? (d.D / 2) * (d.H / 2) * (d.W / 2) : d.D * d.H * d.W;
    const int64_t cin = d.a_c0 + d.a_c1;
    if (sv * cin * 2 >= (1LL << 31)) continue;  // the DMA wgrad's per-batch buffer range
    L.keep_off[i] = take(B * sv * cin * es);
  }
  L.train_total = off;
  return L;
}

}  // namespace

namespace cwdm {
namespace {
__global__ void __launch_bounds__(256) copy_batch_kernel(const CopyJob* __restrict__ jobs, int njobs) {
  const long long bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const CopyJob j = jobs[lo];
  const long long base = (bid - j.blk0) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // 4 independent gathers in flight per thread
    const long long i = base + k * 256 + threadIdx.x;
    if (i < j.n) j.dst[i] = j.b ? j.a[i] + j.b[i] : j.a[i];
  }
}

__global__ void vec_add_kernel(const float* a, const float* b, float* o, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] + b[i];
}
}  // namespace
int launch_vec_add(const float* a, const float* b, float* out, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(vec_add_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, a, b, out, n);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
}  // namespace cwdm

extern "C" int cwdm_unet_create(const cwdm_unet_config* cfg, cwdm_unet** plan) {
  CWDM_REQUIRE(cfg && plan, CWDM_E_INVALID, "cwdm_unet_create: null pointer");
  CWDM_REQUIRE(cfg->num_levels >= 1 && cfg->num_levels <= 8, CWDM_E_INVALID, "cwdm_unet_create: 1..8 levels");
  CWDM_REQUIRE(cfg->model_channels > 0 && cfg->in_channels > 0 && cfg->out_channels > 0 && cfg->num_res_blocks >= 1,
               CWDM_E_INVALID, "cwdm_unet_create: bad channel config");
  CWDM_REQUIRE(dtype_compute(cfg->dtype), CWDM_E_INVALID, "cwdm_unet_create: bad dtype");
  CWDM_REQUIRE(cfg->num_groups > 0, CWDM_E_INVALID, "cwdm_unet_create: bad num_groups");
  const int ck = 32 / dtype_size(cfg->dtype);
  CWDM_REQUIRE(cfg->in_channels % ck == 0, CWDM_E_UNSUPPORTED,
               "cwdm_unet_create: in_channels must be a multiple of " + std::to_string(ck));
  for (int l = 0; l < cfg->num_levels; ++l) {
    const int ch = cfg->channel_mult[l] * cfg->model_channels;
    CWDM_REQUIRE(ch > 0 && ch % ck == 0 && (ch % 64 == 0 || ch % 32 == 0), CWDM_E_UNSUPPORTED,
                 "cwdm_unet_create: level channels must be multiples of 32 (and of the chunk)");
    CWDM_REQUIRE(ch % cfg->num_groups == 0, CWDM_E_INVALID, "cwdm_unet_create: channels not divisible by groups");
  }
  if (cfg->use_freq) {
    // WavUNetModel as script_util.create_model builds it (:268-292)
    CWDM_REQUIRE(cfg->resblock_updown, CWDM_E_UNSUPPORTED,
                 "cwdm_unet_create: use_freq needs resblock_updown=1 (wunet.Downsample with use_freq ignores its conv)");
    CWDM_REQUIRE(cfg->channel_mult[0] == 1, CWDM_E_UNSUPPORTED,
                 "cwdm_unet_create: use_freq: the output head takes model_channels (wunet.py:713), channel_mult[0] = 1");
    CWDM_REQUIRE(cfg->in_channels % 8 == 0 && cfg->in_channels <= 2048, CWDM_E_UNSUPPORTED,
                 "cwdm_unet_create: use_freq: the wavelet pyramid needs in_channels a multiple of 8");
    // the decoder re-runs each level's last ResBlock on its own output (wunet.py:648-687): that block must keep
    // its channel count, i.e. num_res_blocks >= 2 or no channel change into the level
    for (int l = 0; l < cfg->num_levels && cfg->num_res_blocks == 1; ++l) {
      const int prev = l == cfg->num_levels - 1 ? cfg->channel_mult[l] : cfg->channel_mult[l + 1];
      CWDM_REQUIRE(prev == cfg->channel_mult[l], CWDM_E_UNSUPPORTED,
                   "cwdm_unet_create: use_freq with num_res_blocks=1 needs equal channel_mult across levels "
                   "(the reused decoder ResBlock would see the wrong channel count, as in the reference)");
    }
  }
  auto* u = new cwdm_unet();
  u->cfg = *cfg;
  build(u);
  *plan = u;
  return CWDM_OK;
}

extern "C" void cwdm_unet_destroy(cwdm_unet* u) {
  if (!u) return;
  for (auto e : u->ev) (void)hipEventDestroy(e);
  (void)hipFree(u->pack_tab);
  (void)hipFree(u->bwd_tab);
  (void)hipFree(u->copy_tab);
  delete u;
}

extern "C" int cwdm_unet_num_params(const cwdm_unet* u) { return u ? (int)u->params.size() : -1; }

extern "C" int cwdm_unet_param_info(const cwdm_unet* u, int i, char* name, int cap, int64_t* shape, int* ndim) {
  CWDM_REQUIRE(u && i >= 0 && i < (int)u->params.size(), CWDM_E_INVALID, "cwdm_unet_param_info: bad index");
  const auto& p = u->params[i];
  if (name && cap > 0) {
    std::strncpy(name, p.name.c_str(), cap - 1);
    name[cap - 1] = 0;
  }
  if (ndim) *ndim = (int)p.shape.size();
  if (shape)
    for (size_t k = 0; k < p.shape.size() && k < 5; ++k) shape[k] = p.shape[k];
  return CWDM_OK;
}

extern "C" int cwdm_unet_num_aliases(const cwdm_unet* u) { return u ? (int)u->aliases.size() : -1; }

extern "C" int cwdm_unet_alias_info(const cwdm_unet* u, int i, char* name, int cap, int* owner, int* before) {
  CWDM_REQUIRE(u && i >= 0 && i < (int)u->aliases.size(), CWDM_E_INVALID, "cwdm_unet_alias_info: bad index");
  if (name && cap > 0) {
    std::strncpy(name, u->aliases[i].name.c_str(), cap - 1);
    name[cap - 1] = 0;
  }
  if (owner) *owner = u->aliases[i].owner;
  if (before) *before = u->aliases[i].before;
  return CWDM_OK;
}

extern "C" int64_t cwdm_unet_packed_bytes(const cwdm_unet* u) { return u ? u->packed_bytes : -1; }

// device table of n jobs (grown when needed)
template <typename J>
static int ensure_table(J*& tab, size_t& cap, size_t n) {
  if (n <= cap) return CWDM_OK;
  if (tab) CWDM_HIP(hipFree(tab));
  tab = nullptr;
  CWDM_HIP(hipMalloc(reinterpret_cast<void**>(&tab), n * sizeof(J)));
  cap = n;
  return CWDM_OK;
}

static int copy_batch_run(cwdm_unet* u, std::vector<CopyJob>& jobs, hipStream_t s) {
  if (jobs.empty()) return CWDM_OK;
  long long blk = 0;
  for (auto& j : jobs) {
    j.blk0 = blk;
    blk += (j.n + 1023) / 1024;
  }
  int rc;
  if ((rc = ensure_table(u->copy_tab, u->copy_cap, jobs.size()))) return rc;
  if (u->copy_cache.size() != jobs.size() ||
      std::memcmp(u->copy_cache.data(), jobs.data(), jobs.size() * sizeof(CopyJob))) {
    CWDM_HIP(hipMemcpyAsync(u->copy_tab, jobs.data(), jobs.size() * sizeof(CopyJob), hipMemcpyHostToDevice, s));
    CWDM_HIP(hipStreamSynchronize(s));
    u->copy_cache = jobs;
  }
  hipLaunchKernelGGL(cwdm::copy_batch_kernel, dim3((unsigned)blk), dim3(256), 0, s, u->copy_tab, (int)jobs.size());
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// collects every cwdm_conv3d_pack* of its scope into jobs (one launch later)
struct PackBatchScope {
  explicit PackBatchScope(std::vector<cwdm::PackJob>* v) { cwdm::g_pack_batch = v; }
  ~PackBatchScope() { cwdm::g_pack_batch = nullptr; }
};

// (the packs and the fp32 parameter copies each go out as one batched launch;
// one launch per parameter / conv cost ~2.5 ms per training step in copies,
// vec-adds and pack kernels)
extern "C" int cwdm_unet_pack(const cwdm_unet* uc, const float* const* P, void* packed, cwdm_stream_t stream) {
  CWDM_REQUIRE(uc && P && packed, CWDM_E_INVALID, "cwdm_unet_pack: null pointer");
  cwdm_unet* u = const_cast<cwdm_unet*>(uc);  // only the job-table cache changes
  hipStream_t s = (hipStream_t)stream;
  auto* base = reinterpret_cast<unsigned char*>(packed);
  std::vector<CopyJob> cj;
  auto cp = [&](int pi, int64_t off) {
    cj.push_back(CopyJob{reinterpret_cast<float*>(base + off), P[pi], nullptr, u->params[pi].numel(), 0});
  };
  cp(u->te_w1, u->off_te_w1);
  cp(u->te_b1, u->off_te_b1);
  cp(u->te_w2, u->off_te_w2);
  cp(u->te_b2, u->off_te_b2);
  float* ew = reinterpret_cast<float*>(base + u->off_emb_w);
  float* eb = reinterpret_cast<float*>(base + u->off_emb_b);
  for (size_t k = 0; k < u->emb_rows_w.size(); ++k) {
    const int64_t o = u->emb_rows_off[k], n = u->emb_rows_n[k];
    cj.push_back(CopyJob{ew + o * u->E, P[u->emb_rows_w[k]], nullptr, n * u->E, 0});
    cj.push_back(CopyJob{eb + o, P[u->emb_rows_b[k]], u->emb_rows_cb[k] < 0 ? nullptr : P[u->emb_rows_cb[k]], n, 0});
  }
  std::vector<cwdm::PackJob> jobs;
  int rc;
  {
    PackBatchScope scope(&jobs);
    for (const auto& cs : u->convs) {
      if (cs.s2) {
        if ((rc = cwdm_conv3d_pack_s2(P[cs.w_p], cs.cout, cs.cin_a / 8, u->cfg.dtype, base + cs.w_off, 0, stream)))
          return rc;
      } else if ((rc = cwdm_conv3d_pack(P[cs.w_p], cs.cout, cs.cin_a, 3, u->cfg.dtype, base + cs.w_off, stream))) {
        return rc;
      }
      if (cs.wsplit_off >= 0 &&
          (rc = cwdm_conv3d_pack_split(P[cs.w_p], cs.cout, cs.cin_a, base + cs.wsplit_off, stream)))
        return rc;
      if (cs.ws_p >= 0 &&
          (rc = cwdm_conv3d_pack(P[cs.ws_p], cs.cout, cs.cin_b, 1, u->cfg.dtype, base + cs.wsk_off, stream)))
        return rc;
      if (cs.bias_kind == 0)
        cj.push_back(CopyJob{reinterpret_cast<float*>(base + cs.bias_off), P[cs.b_p],
                             cs.wsb_p >= 0 ? P[cs.wsb_p] : nullptr, cs.cout, 0});
    }
  }
  // the accurate fast mode's K-expanded weights (head, small grids): bf16, so packed now, outside the
  // batch (which packs in the model's dtype)
  for (const auto& cs : u->convs) {
    float* tmp = reinterpret_cast<float*>(base + u->split3_tmp);
    for (const int64_t o : {cs.hsplit_off, cs.xsplit_off})
      if (o >= 0 && (rc = cwdm::head_split3_pack(P[cs.w_p], cs.cout, cs.cin_a, tmp, base + o, s, 3))) return rc;
    if (cs.xsplit_sk_off >= 0 &&
        (rc = cwdm::head_split3_pack(P[cs.ws_p], cs.cout, cs.cin_b, tmp, base + cs.xsplit_sk_off, s, 1)))
      return rc;
  }
  for (const auto& g : u->gns) {
    cp(g.gamma_p, g.gamma_off);
    cp(g.beta_p, g.beta_off);
  }
  if ((rc = copy_batch_run(u, cj, s))) return rc;
  if ((rc = ensure_table(u->pack_tab, u->pack_cap, jobs.size()))) return rc;
  return cwdm::pack_batch_run(jobs, u->cfg.dtype, u->pack_tab, u->pack_cache, s);
}

extern "C" int64_t cwdm_unet_workspace_bytes(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u || B <= 0 || D <= 0 || H <= 0 || W <= 0) return -1;
  return layout(u, B, D, H, W).total;
}

extern "C" int64_t cwdm_unet_train_workspace_bytes(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  const int64_t n = cwdm_unet_workspace_bytes(u, B, D, H, W);
  if (n < 0) return n;
  return layout(u, B, D, H, W).train_total;
}

extern "C" double cwdm_unet_flops(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u) return -1;
  double f = 0;
  for (const auto& cs : u->convs) {
    const double v = (double)B * (D >> cs.level) * (H >> cs.level) * (W >> cs.level);
    f += 2.0 * v * cs.cout * (27.0 * (cs.s2 ? cs.cin_a / 8 : cs.cin_a) + cs.cin_b);  // algorithmic (stride-2: 27 C taps)
  }
  return f;
}

namespace cwdm {
bool head_sampler_eligible(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a);  // conv3d_head.hip
int head_sampler_forward(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a, hipStream_t s);
}

// samp: run the sampling step on the output (cwdm_unet_forward_step); fused
// into the output head when it qualifies (*fused = 1), else after the forward.
static int unet_forward_impl(cwdm_unet* u, const void* packed, const void* x, const float* t, float* out,
                             int64_t B, int64_t D, int64_t H, int64_t W, void* ws, int64_t ws_bytes,
                             cwdm_stream_t stream, const cwdm_sampler_args* samp, int* fused) {
  CWDM_REQUIRE(u && packed && x && t && out && ws, CWDM_E_INVALID, "cwdm_unet_forward: null pointer");
  CWDM_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, CWDM_E_SHAPE, "cwdm_unet_forward: empty grid");
  const int64_t div = int64_t(1) << (u->cfg.num_levels - (u->cfg.use_freq ? 0 : 1));
  CWDM_REQUIRE(D % div == 0 && H % div == 0 && W % div == 0, CWDM_E_SHAPE,
               "cwdm_unet_forward: every subband edge must be divisible by " + std::to_string(div));
  Layout L = layout(u, B, D, H, W);
  CWDM_REQUIRE(ws_bytes >= L.total, CWDM_E_WORKSPACE,
               "cwdm_unet_forward: workspace too small (need " + std::to_string(L.total) + " bytes)");
  // a training-sized workspace keeps the convs' activated inputs for the backward
  const bool keep = L.train_total > L.total && ws_bytes >= L.train_total;
  hipStream_t s = (hipStream_t)stream;
  auto* pk = reinterpret_cast<const unsigned char*>(packed);
  auto* wb = reinterpret_cast<unsigned char*>(ws);
  CWDM_HIP(hipMemsetAsync(wb + L.sync, 0, cwdm::plan_sync_bytes(), s));
  SgSyncScope sync_scope(wb + L.sync);
  float* temb = reinterpret_cast<float*>(wb + L.temb);
  float* ebias = reinterpret_cast<float*>(wb + L.ebias);
  int rc;
  const float* f = nullptr;
  auto P = [&](int64_t off) { return reinterpret_cast<const float*>(pk + off); };
  if ((rc = launch_time_embed(t, (int)B, u->cfg.model_channels, P(u->off_te_w1), P(u->off_te_b1), P(u->off_te_w2),
                              P(u->off_te_b2), temb, s)))
    return rc;
  if ((rc = launch_emb_proj(temb, (int)B, u->E, P(u->off_emb_w), P(u->off_emb_b), u->R, ebias, s))) return rc;
  (void)f;
  auto tptr = [&](int id) -> const void* {
    if (id < 0) return nullptr;
    if (id == u->input_tensor) return x;
    return wb + L.t_off[id];
  };
  int conv_i = 0;
  struct ProfReset {
    ~ProfReset() { cwdm::g_prof = nullptr; }  // also on an early error return
  } prof_reset;
  const int es = esize(u->cfg.dtype);
  (void)es;
  if (u->profiling) {
    const size_t need = u->convs.size() * 4;
    while (u->ev.size() < need) {
      hipEvent_t e;
      CWDM_HIP(hipEventCreate(&e));
      u->ev.push_back(e);
    }
    u->ev_flops.assign(u->convs.size(), 0.0);
    u->hooks.assign(u->convs.size(), cwdm::ProfHook{});
    for (size_t i = 0; i < u->convs.size(); ++i)
      for (int k = 0; k < 4; ++k) u->hooks[i].ev[k >> 1][k & 1] = u->ev[4 * i + k];
    u->ev_used = 0;
  }
  // GroupNorm finalize offered to its consumer conv (cwdm::GnFinFuse: at the
  // small grids the conv's pre-pass computes it; any other route runs it
  // first).  A pending one whose consumer is not the next step runs on its own.
  // Env CWDM_GNFIN=0: every finalize as its own launch (A/B switch).
  static const bool fin_on = [] { const char* e = std::getenv("CWDM_GNFIN"); return !(e && e[0] == '0'); }();
  // statistics partial rows per tensor: the per-tile layout, or the rows of a warp-specialised conv
  // that summed them per workgroup (cwdm::g_stats_rows; env CWDM_STATS_WG=0: per tile everywhere)
  static const int stats_wg = [] { const char* e = std::getenv("CWDM_STATS_WG"); return !(e && e[0] == '0'); }();
  std::vector<int64_t> srows(L.s_parts);
  struct StatsWgScope {
    StatsWgScope() { cwdm::g_stats_wg = stats_wg; cwdm::g_stats_rows = 0; }
    ~StatsWgScope() { cwdm::g_stats_wg = 0; cwdm::g_stats_rows = 0; }
  } stats_wg_scope;
  int fin_pend = -1;
  auto fin_args = [&](int gi, cwdm::GnFinFuse& f) {
    const auto& g = u->gns[gi];
    f.s0 = reinterpret_cast<const float*>(wb + L.s_off[g.src0]); f.p0 = srows[g.src0];
    f.c0 = u->tensors[g.src0].channels;
    f.s1 = g.src1 >= 0 ? reinterpret_cast<const float*>(wb + L.s_off[g.src1]) : nullptr;
    f.p1 = g.src1 >= 0 ? srows[g.src1] : 0; f.c1 = g.src1 >= 0 ? u->tensors[g.src1].channels : 0;
    f.gamma = P(g.gamma_off); f.beta = P(g.beta_off); f.groups = u->cfg.num_groups;
    f.voxels = (D >> g.level) * (H >> g.level) * (W >> g.level); f.eps = 1e-5f;
    f.ss = reinterpret_cast<float*>(wb + L.ss_off[g.ss_id]); f.mr = reinterpret_cast<float*>(wb + L.mr_off[g.ss_id]);
    f.B = B;
    f.used = false;
  };
  auto flush_fin = [&]() -> int {
    if (fin_pend < 0) return CWDM_OK;
    cwdm::GnFinFuse f{};
    fin_args(fin_pend, f);
    fin_pend = -1;
    return cwdm_gn_finalize(f.s0, f.p0, f.c0, f.s1, f.p1, f.c1, f.gamma, f.beta, f.groups, B, f.voxels, f.eps, f.ss,
                            f.mr, stream);
  };
  for (const auto& st : u->steps) {
    if (fin_pend >= 0 && !(st.kind == 1 && u->convs[st.idx].gn == u->gns[fin_pend].ss_id) && (rc = flush_fin()))
      return rc;
    if (st.kind == 2) {
      const auto& ps = u->pools[st.idx];
      const int lv = ps.level_out;
      if ((rc = cwdm_gn_silu_pool(tptr(ps.src), ps.channels, reinterpret_cast<const float*>(wb + L.ss_off[ps.ss_id]),
                                  B, D >> lv, H >> lv, W >> lv, u->cfg.dtype, wb + L.t_off[ps.out_h],
                                  wb + L.t_off[ps.out_x], stream)))
        return rc;
      continue;
    }
    if (st.kind == 3) {
      const auto& sd = u->s2ds[st.idx];
      const int lv = sd.level_out;
      if ((rc = cwdm_space_to_depth(tptr(sd.src), sd.channels, B, D >> lv, H >> lv, W >> lv, u->cfg.dtype,
                                    wb + L.t_off[sd.out], 1, 0, stream)))
        return rc;
      continue;
    }
    if (st.kind == 4) {
      const auto& hs = u->haars[st.idx];
      const int lv = hs.level;
      cwdm_haar_nd_desc a{};
      a.dtype = u->cfg.dtype;
      a.B = B; a.d = D >> lv; a.h = H >> lv; a.w = W >> lv;
      a.C = u->tensors[hs.src].channels;
      a.inverse = hs.inverse; a.all8 = hs.all8;
      a.src = tptr(hs.src); a.high_in = tptr(hs.high_in);
      a.lll_scale = hs.lll_scale; a.high_scale = hs.high_scale;
      a.out = wb + L.t_off[hs.out];
      a.high_out = hs.high_out >= 0 ? wb + L.t_off[hs.high_out] : nullptr;
      a.bias = hs.emb_row >= 0 ? ebias + hs.emb_row : nullptr;
      a.bias_bstride = u->R;
      a.stats = hs.stats ? reinterpret_cast<float*>(wb + L.s_off[hs.out]) : nullptr;
      if ((rc = cwdm_haar_nd(&a, stream))) return rc;
      continue;
    }
    if (st.kind == 0) {
      fin_pend = st.idx;
      if (!fin_on && (rc = flush_fin())) return rc;
      continue;
    }
    const auto& cs = u->convs[st.idx];
    cwdm_conv3d_desc d = conv_shape(u, cs, B, D, H, W);
    d.a0 = tptr(cs.a0);
    d.a1 = tptr(cs.a1);
    d.workspace = wb + L.split;
    d.ws_bytes = L.split_bytes;
    d.a_gn = cs.gn >= 0 ? reinterpret_cast<const float*>(wb + L.ss_off[cs.gn]) : nullptr;
    d.a_w = pk + cs.w_off;
    d.a_w_split = cs.wsplit_off >= 0 ? pk + cs.wsplit_off : nullptr;
    if (cs.ws_p >= 0) {
      d.b0 = tptr(cs.sb0); d.b_c0 = u->tensors[cs.sb0].channels;
      d.b1 = tptr(cs.sb1); d.b_c1 = cs.sb1 >= 0 ? u->tensors[cs.sb1].channels : 0;
      d.b_w = pk + cs.wsk_off;
    }
    if (cs.bias_kind == 0) { d.bias = P(cs.bias_off); d.bias_bstride = 0; }
    else { d.bias = ebias + cs.bias_off; d.bias_bstride = u->R; }
    d.res = tptr(cs.res); d.res_mode = cs.rmode;
    if (cs.out < 0) { d.out = out; d.out_dtype = CWDM_F32; }
    else { d.out = wb + L.t_off[cs.out]; d.out_dtype = u->cfg.dtype; }
    d.stats = (cs.stats && cs.out >= 0) ? reinterpret_cast<float*>(wb + L.s_off[cs.out]) : nullptr;
    if (u->profiling) cwdm::g_prof = &u->hooks[conv_i];
    // a skip block's conv1 that applies GroupNorm in its own LDS (conv3d_v5,
    // inference) reads x raw: the fused GroupNorm + 1x1-skip pass would only
    // write an activated copy nobody reads; conv2 then runs the 1x1 skip itself
    auto skip_pass_at = [&](int ci) {
      if (!L.skip_fused[ci]) return false;
      if (keep) return true;
      const cwdm_conv3d_desc dc = conv_shape(u, u->convs[ci], B, D, H, W);
      return !cwdm::v5_eligible(&dc, true);
    };
    if (skip_pass_at(st.idx)) {
      // conv1 of a skip block: SiLU(GN1(x)) for this conv and W_skip . x for conv2 in one pass
      const auto& c2 = u->convs[cs.skip_conv];
      const int64_t vpb = d.D * d.H * d.W;
      void* act = keep && L.keep_off[st.idx] >= 0 ? wb + L.keep_off[st.idx] : wb + L.split;
      if ((rc = flush_fin())) return rc;
      if ((rc = cwdm::gn_apply_skip(d.a0, d.a_c0, d.a1, d.a_c1, d.a_gn, B, vpb, u->cfg.dtype, pk + c2.wsk_off,
                                    c2.cout, act, wb + L.skipbuf, s)))
        return rc;
      void* part = wb + L.split + ((B * vpb * (d.a_c0 + d.a_c1) * es + 255) & ~(int64_t)255);
      if ((rc = cwdm::v4_launch(&d, act, d.a_c0 + d.a_c1, nullptr, 0, 1, d.res, d.res_mode, part, s))) return rc;
    } else {
      if (cs.ws_p >= 0 && st.idx > 0 && u->convs[st.idx - 1].skip_conv == st.idx && skip_pass_at(st.idx - 1)) {
        // the skip was computed in conv1's GroupNorm pass: a plain residual here
        d.b0 = d.b1 = nullptr; d.b_c0 = d.b_c1 = 0; d.b_w = nullptr;
        d.res = wb + L.skipbuf; d.res_mode = 0;
      }
      const int64_t x3_bytes = B * d.D * d.H * d.W * 3 * d.a_c0 * 2;
      if (samp && cs.out < 0 && cwdm::head_sampler_eligible(&d, samp)) {
        if ((rc = flush_fin())) return rc;
        if ((rc = cwdm::head_sampler_forward(&d, samp, s))) return rc;
        if (fused) *fused = 1;
      } else if (cs.hsplit_off >= 0 && !keep && d.a_gn && x3_bytes <= L.split_bytes) {
        // the accurate fast mode's head: a bf16 head over the K-expanded split input (head_split3_prep)
        if ((rc = flush_fin())) return rc;
        void* x3 = wb + L.split;
        if ((rc = cwdm::head_split3_prep(reinterpret_cast<const float*>(d.a0), d.a_gn, B, d.D * d.H * d.W, d.a_c0, x3,
                                          s)))
          return rc;
        cwdm_conv3d_desc e = d;
        e.dtype = CWDM_BF16;
        e.a0 = x3; e.a_c0 = 3 * d.a_c0; e.a1 = nullptr; e.a_c1 = 0;
        e.a_gn = nullptr; e.a_w = pk + cs.hsplit_off; e.a_w_split = nullptr;
        e.workspace = nullptr; e.ws_bytes = 0;
        if ((rc = cwdm_conv3d_forward(&e, stream))) return rc;
      } else if (XsgPlan xp = keep ? XsgPlan{} : xsg_plan(u, cs, d); xp.ok && xp.total <= L.split_bytes) {
        // the accurate fast mode on a small grid: one bf16 small-grid conv over the K-expanded split input
        if ((rc = flush_fin())) return rc;
        unsigned char* x3 = wb + L.split;
        const void* res = d.res;
        int rmode = d.res_mode;
        SgFp32xScope fx;
        void* part = x3 + xp.x3_bytes + xp.skip_bytes;
        if (d.b_w && xp.sk_sg) {
          // the 1x1 skip first, into an fp32 residual: K-expanded split of the raw input on the small-grid kernel
          if ((rc = cwdm::split3_prep(reinterpret_cast<const float*>(d.b0), d.b_c0, reinterpret_cast<const float*>(d.b1),
                                      d.b_c1, nullptr, B, d.D * d.H * d.W, 0, x3, s)))
            return rc;
          cwdm_conv3d_desc k = xp.ek;
          k.b0 = x3; k.b_w = pk + cs.xsplit_sk_off;
          if ((rc = cwdm::sg_skip_launch(&k, x3 + xp.x3_bytes, cwdm::sg_skip_ksplit(&k) > 1 ? part : nullptr, s)))
            return rc;
          res = x3 + xp.x3_bytes; rmode = 0;
        } else if (d.b_w) {
          // the 1x1 skip first, into an fp32 residual (pw_split: the split products of the 1x1 weights)
          cwdm_conv3d_desc k = d;
          k.a0 = k.a1 = nullptr; k.a_c0 = k.a_c1 = 0; k.a_gn = nullptr; k.a_w = nullptr; k.a_mode = 0;
          k.bias = nullptr; k.bias_bstride = 0; k.stats = nullptr; k.res = nullptr; k.res_mode = -1;
          k.out = x3 + xp.x3_bytes; k.out_dtype = CWDM_F32;
          k.workspace = nullptr; k.ws_bytes = 0;
          if ((rc = cwdm::pw_split_eligible(&k) ? cwdm::pw_split_forward(&k, s) : cwdm_conv3d_forward(&k, stream)))
            return rc;
          res = k.out; rmode = 0;
        }
        const int64_t sv = cs.amode == 1 ? (d.D / 2) * (d.H / 2) * (d.W / 2) : d.D * d.H * d.W;
        if ((rc = cwdm::split3_prep(reinterpret_cast<const float*>(d.a0), d.a_c0, reinterpret_cast<const float*>(d.a1),
                                    d.a_c1, d.a_gn, B, sv, 1, x3, s)))
          return rc;
        cwdm_conv3d_desc e = xp.e;
        e.a0 = x3; e.a1 = nullptr; e.a_w = pk + cs.xsplit_off;
        e.bias = d.bias; e.bias_bstride = d.bias_bstride;
        e.res = res; e.res_mode = rmode;
        e.out = d.out; e.stats = d.stats;
        e.workspace = nullptr; e.ws_bytes = 0;
        if ((rc = cwdm::v4_launch(&e, x3, e.a_c0, nullptr, 0, 1, res, rmode, cwdm::sg_ksplit(&e) > 1 ? part : nullptr, s)))
          return rc;
      } else {
        cwdm::ActKeepScope ks(keep && L.keep_off[st.idx] >= 0 ? wb + L.keep_off[st.idx] : nullptr);
        cwdm::GnFinFuse ff{};
        const bool offer = fin_pend >= 0 && d.a_gn == reinterpret_cast<const float*>(wb + L.ss_off[u->gns[fin_pend].ss_id]);
        if (offer) {
          fin_args(fin_pend, ff);
          fin_pend = -1;
          cwdm::g_gnfin = &ff;
        } else if ((rc = flush_fin())) {
          return rc;
        }
        rc = cwdm_conv3d_forward(&d, stream);
        cwdm::g_gnfin = nullptr;
        if (rc) return rc;
        CWDM_REQUIRE(!offer || ff.used, CWDM_E_INVALID,
                     "cwdm_unet_forward: conv " + std::to_string(st.idx) + " did not take its GroupNorm finalize");
        CWDM_REQUIRE(!ks.ptr || ks.used(), CWDM_E_INVALID,
                     "cwdm_unet_forward: conv " + std::to_string(st.idx) + " did not keep its activated input");
      }
    }
    if (cwdm::g_stats_rows > 0) {
      if (cs.out >= 0) srows[cs.out] = cwdm::g_stats_rows;
      cwdm::g_stats_rows = 0;
    }
    if (u->profiling) {
      cwdm::g_prof = nullptr;
      u->ev_used = conv_i + 1;
    }
    ++conv_i;
  }
  return flush_fin();
}

extern "C" int cwdm_unet_forward(cwdm_unet* u, const void* packed, const void* x, const float* t, float* out,
                                 int64_t B, int64_t D, int64_t H, int64_t W, void* ws, int64_t ws_bytes,
                                 cwdm_stream_t stream) {
  return unet_forward_impl(u, packed, x, t, out, B, D, H, W, ws, ws_bytes, stream, nullptr, nullptr);
}

extern "C" int cwdm_unet_forward_step(cwdm_unet* u, const void* packed, const void* x, const float* t_model,
                                      const cwdm_sampler_args* step, int64_t B, int64_t D, int64_t H, int64_t W,
                                      void* ws, int64_t ws_bytes, int* fused, cwdm_stream_t stream) {
  CWDM_REQUIRE(step && step->model_out, CWDM_E_INVALID, "cwdm_unet_forward_step: null step / model_out");
  CWDM_REQUIRE(u && step->d == D && step->h == H && step->w == W && step->B == B &&
                   (step->levels == 2 || u->cfg.out_channels == 8),
               CWDM_E_SHAPE, "cwdm_unet_forward_step: the step's grid must be the forward's");
  int did = 0;
  int rc = unet_forward_impl(u, packed, x, t_model, const_cast<float*>(step->model_out), B, D, H, W, ws, ws_bytes,
                             stream, step, &did);
  if (fused) *fused = did;
  if (rc || did) return rc;
  return cwdm_sampler_step(step, stream);
}

extern "C" int cwdm_unet_trace_count(const cwdm_unet* u) { return u ? (int)u->trace.size() : -1; }

extern "C" int cwdm_unet_trace_info(const cwdm_unet* u, int i, int64_t B, int64_t D, int64_t H, int64_t W,
                                    int64_t* off, int* ch, int* level) {
  CWDM_REQUIRE(u && i >= 0 && i < (int)u->trace.size(), CWDM_E_INVALID, "cwdm_unet_trace_info: bad index");
  const int id = u->trace[i];
  Layout L = layout(u, B, D, H, W);
  if (off) *off = id >= 0 ? L.t_off[id] : -1;
  if (ch) *ch = id >= 0 ? u->tensors[id].channels : u->cfg.out_channels;
  if (level) *level = u->trace_level[i];
  return CWDM_OK;
}

extern "C" int cwdm_unet_set_profiling(cwdm_unet* u, int on) {
  CWDM_REQUIRE(u, CWDM_E_INVALID, "cwdm_unet_set_profiling: null plan");
  u->profiling = on != 0;
  return CWDM_OK;
}

extern "C" int cwdm_unet_profile_read(cwdm_unet* u, double* ms, double* flops, int* n) {
  CWDM_REQUIRE(u, CWDM_E_INVALID, "cwdm_unet_profile_read: null plan");
  double tot = 0, fl = 0;
  int launches = 0;
  for (int i = 0; i < u->ev_used; ++i) {
    const cwdm::ProfHook& h = u->hooks[i];
    for (int k = 0; k < h.n; ++k) {
      float m = 0;
      CWDM_HIP(hipEventElapsedTime(&m, h.ev[k][0], h.ev[k][1]));
      tot += m;
      fl += h.flops[k];
      ++launches;
    }
  }
  if (ms) *ms = tot;
  if (flops) *flops = fl;
  if (n) *n = launches;
  return CWDM_OK;
}

// ============================================================================
// Backward (training): the reverse of the launch list above, as torch autograd
// differentiates UNetModel.forward inside TrainLoop.forward_backward
// (guided_diffusion/train_util.py:396-462).  Per ResBlock, in reverse:
//   conv2: bias grad (channel sums), wgrad (input = SiLU(GN2(h1)) recomputed
//          in the staging), skip 1x1 wgrad + dgrad or residual adjoint,
//          dgrad (flipped/transposed weights, same implicit-GEMM kernel)
//   GN2:   SiLU/GroupNorm backward -> dh1
//   conv1: emb-projection grads (per-batch channel sums), wgrad, dgrad
//   GN1:   SiLU/GroupNorm backward with the up/down resample adjoint -> dx
// Gradient buffers live in grad_ws (one per forward tensor, compute dtype);
// the first writer of a buffer stores, later writers accumulate.
// ============================================================================
namespace {

struct GLayout {
  std::vector<int64_t> g_off;
  int64_t sync, tmp, dout, deb, dsil, gnws, gnws_bytes, split, split_bytes, wgws, wgws_bytes, dwe, chs, chs_bytes;
  int64_t gbp, gbp_bytes;   // fused GroupNorm-backward partials ([B][tiles][C][2]) + their slice sums
  int64_t total;
};

constexpr int kGbSlices = 64;   // slice sums of the fused GroupNorm-backward partials (cwdm::gb_part_reduce)

int ckpad(const cwdm_unet* u, int c) {
  const int ck = 32 / esize(u->cfg.dtype);
  return (c + ck - 1) / ck * ck;
}

// dgrad conv of conv step i as a forward conv descriptor (shape only)
cwdm_conv3d_desc dgrad_shape(const cwdm_unet* u, int i, int64_t B, int64_t D, int64_t H, int64_t W) {
  const auto& cs = u->convs[i];
  cwdm_conv3d_desc d{};
  d.dtype = u->cfg.dtype;
  d.B = B; d.D = D >> cs.level; d.H = H >> cs.level; d.W = W >> cs.level;
  d.cout = cs.cin_a;
  d.a_c0 = ckpad(u, cs.cout);
  d.a_mode = 0;
  d.a_w = reinterpret_cast<const void*>(1);
  d.res_mode = -1;
  d.out_dtype = u->cfg.dtype;
  return d;
}

GLayout glayout(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  GLayout G;
  int64_t off = 0;
  auto take = [&](int64_t bytes) { int64_t o = off; off = align_up(off + bytes); return o; };
  const int es = esize(u->cfg.dtype);
  G.sync = take(cwdm::plan_sync_bytes());
  for (size_t i = 0; i < u->tensors.size(); ++i) {
    const auto& t = u->tensors[i];
    if ((int)i == u->input_tensor) { G.g_off.push_back(-1); continue; }
    G.g_off.push_back(take(B * (D >> t.level) * (H >> t.level) * (W >> t.level) * t.channels * es));
  }
  int64_t tmp = 0, split = 0, gnws = 0, wgws = 0;
  for (const auto& cs : u->convs) {
    wgws = std::max(wgws, cwdm_conv3d_wgrad_workspace_bytes(cs.cout, cs.cin_a, 3));
    if (cs.ws_p >= 0) wgws = std::max(wgws, cwdm_conv3d_wgrad_workspace_bytes(cs.cout, cs.cin_b, 1));
  }
  for (size_t i = 1; i < u->convs.size(); ++i) {
    const auto& cs = u->convs[i];
    const int64_t v = B * (D >> cs.level) * (H >> cs.level) * (W >> cs.level);
    tmp = std::max(tmp, v * cs.cin_a * es);
    cwdm_conv3d_desc d = dgrad_shape(u, (int)i, B, D, H, W);
    split = std::max(split, (int64_t)cwdm_conv3d_workspace_bytes(&d));
  }
  for (const auto& g : u->gns) {
    const int lv = g.level;
    gnws = std::max(gnws, cwdm_gn_silu_bwd_workspace_bytes(g.channels, B, D >> lv, H >> lv, W >> lv));
  }
  G.tmp = take(tmp);
  G.dout = take(B * D * H * W * ckpad(u, u->cfg.out_channels) * es);
  G.deb = take(B * (int64_t)u->R * 4);
  G.dsil = take(B * (int64_t)u->E * 4);
  G.gnws_bytes = gnws;
  G.gnws = take(gnws);
  G.split_bytes = split;
  G.split = take(split);
  G.wgws = take(wgws);
  G.wgws_bytes = wgws;
  int64_t dwe = 0;   // expanded weight gradient of a stride-2 conv before folding
  for (const auto& cs : u->convs)
    if (cs.s2) dwe = std::max(dwe, (int64_t)cs.cout * cs.cin_a * 27 * 4);
  G.dwe = take(dwe);
  int64_t chs = 0;   // per-workgroup partials of the bias-gradient channel sums (fixed-order finish)
  for (const auto& cs : u->convs)
    chs = std::max(chs, cwdm_channel_sum_workspace_bytes(B, (D >> cs.level) * (H >> cs.level) * (W >> cs.level),
                                                         std::max(cs.cout, 8)));
  G.chs_bytes = chs;
  G.chs = take(chs);
  // the dgrad epilogue's GroupNorm-backward partials: one row per 32x4x4 tile
  // of the DMA conv (cwdm::GbwdFuse), then kGbSlices slice sums of them
  int64_t gbp = 0;
  for (const auto& g : u->gns) {
    const int lv = g.level;
    const int64_t tiles = ceil_div(W >> lv, 32) * ceil_div(H >> lv, 4) * ceil_div(D >> lv, 4);
    gbp = std::max(gbp, B * tiles * g.channels * 8 + align_up(B * (int64_t)kGbSlices * g.channels * 8));
  }
  G.gbp_bytes = gbp;
  G.gbp = take(gbp);
  G.total = off;
  return G;
}

}  // namespace

extern "C" int64_t cwdm_unet_packed_bwd_bytes(const cwdm_unet* u) { return u ? u->packed_bwd_bytes : -1; }

extern "C" int cwdm_unet_pack_bwd(const cwdm_unet* uc, const float* const* P, void* packed_bwd, cwdm_stream_t stream) {
  CWDM_REQUIRE(uc && P && packed_bwd, CWDM_E_INVALID, "cwdm_unet_pack_bwd: null pointer");
  cwdm_unet* u = const_cast<cwdm_unet*>(uc);  // only the job-table cache changes
  auto* base = reinterpret_cast<unsigned char*>(packed_bwd);
  int rc;
  std::vector<cwdm::PackJob> jobs;
  {
  PackBatchScope scope(&jobs);
  for (size_t i = 0; i < u->convs.size(); ++i) {
    const auto& cs = u->convs[i];
    if (u->dg_off[i] >= 0 && cs.s2 &&
        (rc = cwdm_conv3d_pack_s2(P[cs.w_p], cs.cout, cs.cin_a / 8, u->cfg.dtype, base + u->dg_off[i], 1, stream)))
      return rc;
    if (u->dg_off[i] >= 0 && !cs.s2 &&
        (rc = cwdm_conv3d_pack_dgrad(P[cs.w_p], cs.cout, cs.cin_a, 3, u->cfg.dtype, base + u->dg_off[i], stream)))
      return rc;
    if (u->dgs_off[i] >= 0 &&
        (rc = cwdm_conv3d_pack_dgrad(P[cs.ws_p], cs.cout, cs.cin_b, 1, u->cfg.dtype, base + u->dgs_off[i], stream)))
      return rc;
  }
  }
  if ((rc = ensure_table(u->bwd_tab, u->bwd_cap, jobs.size()))) return rc;
  return cwdm::pack_batch_run(jobs, u->cfg.dtype, u->bwd_tab, u->bwd_cache, (hipStream_t)stream);
}

extern "C" int64_t cwdm_unet_grad_workspace_bytes(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u || B <= 0 || D <= 0 || H <= 0 || W <= 0) return -1;
  return glayout(u, B, D, H, W).total;
}

extern "C" int cwdm_unet_backward_segments(const cwdm_unet* u) { return u ? (int)u->blocks.size() + 2 : -1; }

extern "C" int cwdm_unet_segment_range(const cwdm_unet* u, int seg, int64_t* off, int64_t* n) {
  CWDM_REQUIRE(u && seg >= 0 && seg < (int)u->blocks.size() + 2, CWDM_E_INVALID, "cwdm_unet_segment_range: bad seg");
  const int nb = (int)u->blocks.size();
  int pb, pe;
  if (seg == 0) { pb = u->head_p_begin; pe = (int)u->params.size(); }
  else if (seg <= nb) { const auto& b = u->blocks[nb - seg]; pb = b.p_begin; pe = b.p_end; }
  else { pb = 0; pe = u->blocks[0].p_begin; }
  const int64_t o = u->goff[pb];
  const int64_t e = pe < (int)u->params.size() ? u->goff[pe] : u->grad_numel;
  if (off) *off = o;
  if (n) *n = e - o;
  return CWDM_OK;
}

extern "C" double cwdm_unet_backward_flops(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u) return -1;
  double f = 0;
  for (size_t i = 0; i < u->convs.size(); ++i) {
    const auto& cs = u->convs[i];
    const double v = (double)B * (D >> cs.level) * (H >> cs.level) * (W >> cs.level);
    const double fwd = 2.0 * v * cs.cout * (27.0 * (cs.s2 ? cs.cin_a / 8 : cs.cin_a) + cs.cin_b);
    f += i == 0 ? fwd : 2 * fwd;  // wgrad (+ dgrad)
  }
  return f;
}

extern "C" int cwdm_unet_backward(cwdm_unet* u, const void* packed, const void* packed_bwd, const void* x,
                                  const float* t, const float* dout, float* grads, int64_t B, int64_t D, int64_t H,
                                  int64_t W, const void* ws, int64_t ws_bytes, void* gws, int64_t gws_bytes,
                                  int seg_begin, int seg_end, cwdm_stream_t stream) {
  CWDM_REQUIRE(u && packed && packed_bwd && x && t && dout && grads && ws && gws, CWDM_E_INVALID,
               "cwdm_unet_backward: null pointer");
  const int nseg = (int)u->blocks.size() + 2;
  CWDM_REQUIRE(0 <= seg_begin && seg_begin <= seg_end && seg_end <= nseg, CWDM_E_INVALID,
               "cwdm_unet_backward: bad segment range");
  CWDM_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, CWDM_E_SHAPE, "cwdm_unet_backward: empty grid");
  const int64_t div = int64_t(1) << (u->cfg.num_levels - (u->cfg.use_freq ? 0 : 1));
  CWDM_REQUIRE(D % div == 0 && H % div == 0 && W % div == 0, CWDM_E_SHAPE,
               "cwdm_unet_backward: every subband edge must be divisible by " + std::to_string(div));
  Layout L = layout(u, B, D, H, W);
  GLayout G = glayout(u, B, D, H, W);
  CWDM_REQUIRE(ws_bytes >= L.total, CWDM_E_WORKSPACE, "cwdm_unet_backward: forward workspace too small");
  CWDM_REQUIRE(gws_bytes >= G.total, CWDM_E_WORKSPACE,
               "cwdm_unet_backward: grad workspace too small (need " + std::to_string(G.total) + " bytes)");
  CWDM_REQUIRE(seg_begin == 0 || (int)u->ginit.size() == (int)u->tensors.size(), CWDM_E_INVALID,
               "cwdm_unet_backward: segment 0 must run first");
  hipStream_t s = (hipStream_t)stream;
  const int dt = u->cfg.dtype;
  const int es = esize(dt);
  auto* pk = reinterpret_cast<const unsigned char*>(packed);
  auto* pb = reinterpret_cast<const unsigned char*>(packed_bwd);
  auto* wb = reinterpret_cast<const unsigned char*>(ws);
  auto* gb = reinterpret_cast<unsigned char*>(gws);
  // (every call: a caller may run segments on a fresh grad workspace)
  CWDM_HIP(hipMemsetAsync(gb + G.sync, 0, cwdm::plan_sync_bytes(), s));
  SgSyncScope sync_scope(gb + G.sync);
  auto P = [&](int64_t off) { return reinterpret_cast<const float*>(pk + off); };
  auto GR = [&](int pi) { return grads + u->goff[pi]; };
  auto act = [&](int id) -> const void* {
    if (id < 0) return nullptr;
    if (id == u->input_tensor) return x;
    return wb + L.t_off[id];
  };
  auto grd = [&](int id) -> void* { return id < 0 ? nullptr : gb + G.g_off[id]; };
  auto vox = [&](int lv) { return (D >> lv) * (H >> lv) * (W >> lv); };
  const float* temb = reinterpret_cast<const float*>(wb + L.temb);
  float* deb = reinterpret_cast<float*>(gb + G.deb);
  float* dsil = reinterpret_cast<float*>(gb + G.dsil);
  void* tmp = gb + G.tmp;
  int rc;

  // first writer stores, later writers accumulate
  auto take_acc = [&](int id) -> int {
    if (id < 0) return 0;
    const int a = u->ginit[id] ? 1 : 0;
    u->ginit[id] = 1;
    return a;
  };
  auto ss_of = [&](int g) { return reinterpret_cast<const float*>(wb + L.ss_off[g]); };
  auto mr_of = [&](int g) { return reinterpret_cast<const float*>(wb + L.mr_off[g]); };

  auto wgrad = [&](int level, int ksize, const void* u0, int uc0, const void* u1, int uc1, int umode,
                   const float* ugn, const void* dy, int dy_cs, int cout, float* dw) -> int {
    cwdm_wgrad_desc d{};
    d.dtype = dt; d.B = B; d.D = D >> level; d.H = H >> level; d.W = W >> level; d.ksize = ksize;
    d.u0 = u0; d.u_c0 = uc0; d.u1 = u1; d.u_c1 = uc1; d.u_mode = umode; d.u_gn = ugn;
    d.dy = dy; d.dy_cs = dy_cs; d.cout = cout; d.dw = dw;
    d.workspace = gb + G.wgws;
    d.ws_bytes = G.wgws_bytes;
    return cwdm_conv3d_wgrad(&d, stream);
  };
  // conv ci's wgrad from the activated input its forward kept (training
  // workspace), else recomputed from the sources by the staging code
  const bool kept = L.train_total > L.total && ws_bytes >= L.train_total;
  auto wgrad_c = [&](int ci, int level, const void* u0, int uc0, const void* u1, int uc1, int umode,
                     const float* ugn, const void* dy, int dy_cs, int cout, float* dw) -> int {
    if (!kept || L.keep_off[ci] < 0) return wgrad(level, 3, u0, uc0, u1, uc1, umode, ugn, dy, dy_cs, cout, dw);
    cwdm_wgrad_desc d{};
    d.dtype = dt; d.B = B; d.D = D >> level; d.H = H >> level; d.W = W >> level; d.ksize = 3;
    d.u0 = wb + L.keep_off[ci]; d.u_c0 = uc0 + uc1; d.u_mode = umode; d.u_cm = 1;
    d.dy = dy; d.dy_cs = dy_cs; d.cout = cout; d.dw = dw;
    d.workspace = gb + G.wgws;
    d.ws_bytes = G.wgws_bytes;
    return cwdm_conv3d_wgrad(&d, stream);
  };
  auto dgrad = [&](int ci, const void* dy) -> int {
    cwdm_conv3d_desc d = dgrad_shape(u, ci, B, D, H, W);
    d.a0 = dy;
    d.a_w = pb + u->dg_off[ci];
    d.out = tmp;
    d.workspace = gb + G.split;
    d.ws_bytes = G.split_bytes;
    return cwdm_conv3d_forward(&d, stream);
  };
  // dgrad conv ci whose output du (tmp) feeds the SiLU(GroupNorm gi) backward at
  // the same grid, input x = (xid0, xid1): the conv's epilogue takes the reduce
  // pass of that backward when its kernel can (cwdm::GbwdFuse: 16-bit DMA conv,
  // no K split); pre then names the partials for gn_silu_bwd_impl
  struct Pre { const float* part = nullptr; int nblk = 0; };
  static const bool gb_on = [] { const char* e = std::getenv("CWDM_GBWD_FUSE"); return !(e && e[0] == '0'); }();
  float* gbp = reinterpret_cast<float*>(gb + G.gbp);
  auto dgrad_gn = [&](int ci, const void* dy, int gi, int xid0, int xid1, Pre& pre) -> int {
    pre = Pre{};
    if (!gb_on || G.gbp_bytes <= 0) return dgrad(ci, dy);
    const auto& g = u->gns[gi];
    cwdm::GbwdFuse f{};
    f.x0 = act(xid0); f.x1 = act(xid1); f.c0 = u->tensors[xid0].channels;
    f.ss = ss_of(gi); f.mr = mr_of(gi); f.groups = u->cfg.num_groups;
    f.part = gbp;
    f.part_bytes = G.gbp_bytes - align_up(B * (int64_t)kGbSlices * g.channels * 8);
    cwdm::g_gbwd = &f;
    const int r = dgrad(ci, dy);
    cwdm::g_gbwd = nullptr;
    if (r || !f.used) return r;
    if (f.nblk <= 512) {   // few tiles: gn_bwd_finalize reads them directly
      pre.part = gbp; pre.nblk = f.nblk;
      return CWDM_OK;
    }
    float* sl = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(gbp) + f.part_bytes);
    if (int rc2 = gb_part_reduce(gbp, f.nblk, g.channels, B, kGbSlices, sl, s)) return rc2;
    pre.part = sl; pre.nblk = kGbSlices;
    return CWDM_OK;
  };
  auto gn_bwd = [&](int gi, int x0, int x1, int du_mode, const Pre* pre = nullptr) -> int {
    const auto& g = u->gns[gi];
    const int lv = g.level;
    const int c0 = u->tensors[x0].channels, c1 = x1 >= 0 ? u->tensors[x1].channels : 0;
    const int a0 = take_acc(x0), a1 = take_acc(x1);
    // affine gradients accumulate (zeroed at segment 0): a reused WavUNetModel block adds its second use
    return gn_silu_bwd_impl(act(x0), c0, act(x1), c1, tmp, du_mode, ss_of(gi), mr_of(gi), P(g.gamma_off),
                            u->cfg.num_groups, B, D >> lv, H >> lv, W >> lv, dt, grd(x0), a0, grd(x1), a1,
                            GR(g.gamma_p), GR(g.beta_p), gb + G.gnws, G.gnws_bytes, nullptr, 0, stream, 1,
                            pre ? pre->part : nullptr, pre ? pre->nblk : 0);
  };

  for (int seg = seg_begin; seg < seg_end; ++seg) {
    const int nb = (int)u->blocks.size();
    if (seg == 0) {
      u->ginit.assign(u->tensors.size(), 0);
      CWDM_HIP(hipMemsetAsync(grads, 0, u->grad_numel * 4, s));
      CWDM_HIP(hipMemsetAsync(deb, 0, B * (int64_t)u->R * 4, s));
      CWDM_HIP(hipMemsetAsync(dsil, 0, B * (int64_t)u->E * 4, s));
      // output head: dout -> padded compute-dtype buffer
      const int oc = u->cfg.out_channels, ocp = ckpad(u, oc);
      const int64_t V0 = D * H * W;
      void* d16 = gb + G.dout;
      CWDM_HIP(hipMemsetAsync(d16, 0, B * V0 * ocp * es, s));
      const int64_t ss_[3] = {V0 * oc, 1, oc}, ds_[3] = {V0 * ocp, 1, ocp};
      if ((rc = cwdm_copy3(dout, CWDM_F32, ss_, d16, dt, ds_, B, oc, V0, stream))) return rc;
      const auto& co = u->convs[u->head_c];
      const auto& hg = u->gns[u->head_g];
      if ((rc = cwdm_channel_sum(d16, dt, B, V0, oc, ocp, nullptr, 0, GR(co.b_p), nullptr, gb + G.chs, G.chs_bytes,
                                 stream)))
        return rc;
      if ((rc = wgrad(0, 3, act(co.a0), co.cin_a, nullptr, 0, 0, ss_of(u->head_g), d16, ocp, oc, GR(co.w_p))))
        return rc;
      Pre pre;
      if ((rc = dgrad_gn(u->head_c, d16, u->head_g, hg.src0, -1, pre))) return rc;
      if ((rc = gn_bwd(u->head_g, hg.src0, -1, 0, &pre))) return rc;
      continue;
    }
    if (seg <= nb && u->blocks[nb - seg].updown == 7) {
      // WavUNetModel WaveletDownsample (wunet.py:131-145): out = conv(cat(DWT(pyr)) / 3) + h
      const Block& bk = u->blocks[nb - seg];
      const auto& cs = u->convs[bk.c1];
      const auto& hp = u->haars[bk.pool];
      const int o = cs.out;
      if ((rc = cwdm_channel_sum(grd(o), dt, B, vox(cs.level), cs.cout, cs.cout, nullptr, 0, GR(cs.b_p), nullptr,
                                 gb + G.chs, G.chs_bytes, stream)))
        return rc;
      if ((rc = wgrad(cs.level, 3, act(hp.out), cs.cin_a, nullptr, 0, 0, nullptr, grd(o), cs.cout, cs.cout,
                      GR(cs.w_p))))
        return rc;
      const int lv = cs.level;
      if ((rc = cwdm_resample_add(grd(cs.res), grd(o), cs.cout, B, D >> lv, H >> lv, W >> lv, 0, take_acc(cs.res), dt,
                                  stream)))
        return rc;
      if (hp.src != u->input_tensor) {   // the level-0 pyramid is the model input: no gradient
        if ((rc = dgrad(bk.c1, grd(o)))) return rc;
        const int cp = u->tensors[hp.src].channels;
        if ((rc = haar_nd_synth_add(dt, B, D >> lv, H >> lv, W >> lv, cp, tmp, 8LL * cp, hp.lll_scale,
                                    reinterpret_cast<unsigned char*>(tmp) + (int64_t)cp * es, 8LL * cp, hp.high_scale,
                                    grd(hp.src), take_acc(hp.src), s)))
          return rc;
      }
      continue;
    }
    if (seg <= nb && (u->blocks[nb - seg].updown == 5 || u->blocks[nb - seg].updown == 6)) {
      // WavUNetModel ResBlock that resamples by DWT / IDWT after its first conv (wunet.py:210-269)
      const Block& bk = u->blocks[nb - seg];
      const bool down = bk.updown == 5;
      const auto& c1 = u->convs[bk.c1];
      const auto& c2 = u->convs[bk.c2];
      const auto& hh = u->haars[bk.hh];
      const auto& hx = u->haars[bk.hx];
      const int lout = c2.level, lin = c1.level;
      const int64_t Vo = vox(lout);
      const int o = c2.out, h1 = c1.out, cout = c2.cout, cin = u->tensors[bk.x0].channels;
      // ---- conv2 + the residual x_upd
      if ((rc = cwdm_channel_sum(grd(o), dt, B, Vo, cout, cout, nullptr, 0, GR(c2.b_p), nullptr, gb + G.chs,
                                 G.chs_bytes, stream)))
        return rc;
      if ((rc = wgrad_c(bk.c2, lout, act(hh.out), cout, nullptr, 0, 0, ss_of(bk.g2), grd(o), cout, cout,
                        GR(c2.w_p))))
        return rc;
      if ((rc = cwdm_resample_add(grd(hx.out), grd(o), cout, B, D >> lout, H >> lout, W >> lout, 0, take_acc(hx.out),
                                  dt, stream)))
        return rc;
      Pre pre2;
      if ((rc = dgrad_gn(bk.c2, grd(o), bk.g2, hh.out, -1, pre2))) return rc;
      // ---- GN2 -> d(h + emb), with its channel sums = the emb projection's gradient
      const int k = bk.emb_k;
      const int roff = u->emb_rows_off[k], rn = u->emb_rows_n[k];
      {
        const auto& g = u->gns[bk.g2];
        if ((rc = gn_silu_bwd_impl(act(hh.out), cout, nullptr, 0, tmp, 0, ss_of(bk.g2), mr_of(bk.g2), P(g.gamma_off),
                                   u->cfg.num_groups, B, D >> lout, H >> lout, W >> lout, dt, grd(hh.out),
                                   take_acc(hh.out), nullptr, 0, GR(g.gamma_p), GR(g.beta_p), gb + G.gnws,
                                   G.gnws_bytes, deb + roff, u->R, stream, 1, pre2.part, pre2.nblk)))
          return rc;
      }
      if ((rc = launch_emb_bwd(deb + roff, u->R, rn, (int)B, temb, u->E, P(u->off_emb_w) + (int64_t)roff * u->E,
                               GR(u->emb_rows_w[k]), GR(u->emb_rows_b[k]), nullptr, dsil, s, 1)))
        return rc;
      // ---- the resampling adjoints (orthonormal Haar: analysis <-> synthesis)
      const int lc = down ? lout : lin;   // the coarse grid of this block's DWT / IDWT
      const int64_t dc = D >> lc, hc = H >> lc, wc = W >> lc;
      if (down) {
        // h = DWT(h1): LLL / 3 (+ emb) continues, the 7 high bands are the skip
        const int sk = hh.high_out;
        const void* dsk = u->ginit[sk] ? grd(sk) : nullptr;   // (no later user: zero)
        if ((rc = haar_nd_synth_add(dt, B, dc, hc, wc, cout, grd(hh.out), cout, hh.lll_scale, dsk, 7LL * cout,
                                    hh.high_scale, grd(h1), take_acc(h1), s)))
          return rc;
        if ((rc = haar_nd_synth_add(dt, B, dc, hc, wc, cin, grd(hx.out), cin, hx.lll_scale, nullptr, 0, 0.f,
                                    grd(bk.x0), take_acc(bk.x0), s)))
          return rc;
      } else {
        // h = IDWT(3 h1, skip) (+ emb), x_upd = IDWT(3 x, skip): both feed the skip bands' gradient
        const int sk = hh.high_in;
        if ((rc = haar_nd_anal_add(dt, B, dc, hc, wc, cout, grd(hh.out), grd(h1), cout, hh.lll_scale, take_acc(h1),
                                   grd(sk), 7LL * cout, hh.high_scale, take_acc(sk), s)))
          return rc;
        if ((rc = haar_nd_anal_add(dt, B, dc, hc, wc, cin, grd(hx.out), grd(bk.x0), cin, hx.lll_scale,
                                   take_acc(bk.x0), grd(sk), 7LL * cin, hx.high_scale, take_acc(sk), s)))
          return rc;
      }
      // ---- conv1 (own bias; the emb is added after the resampling) and GN1
      if ((rc = cwdm_channel_sum(grd(h1), dt, B, vox(lin), cout, cout, nullptr, 0, GR(c1.b_p), nullptr, gb + G.chs,
                                 G.chs_bytes, stream)))
        return rc;
      if ((rc = wgrad_c(bk.c1, lin, act(bk.x0), cin, nullptr, 0, 0, ss_of(bk.g1), grd(h1), cout, cout, GR(c1.w_p))))
        return rc;
      Pre pre1;
      if ((rc = dgrad_gn(bk.c1, grd(h1), bk.g1, bk.x0, -1, pre1))) return rc;
      if ((rc = gn_bwd(bk.g1, bk.x0, -1, 0, &pre1))) return rc;
      continue;
    }
    if (seg <= nb && u->blocks[nb - seg].updown >= 3) {
      // Downsample stride-2 conv / Upsample nearest + conv (resblock_updown=False)
      const Block& bk = u->blocks[nb - seg];
      const auto& cs = u->convs[bk.c1];
      const int o = cs.out, xt = bk.x0;
      const int chn = u->tensors[xt].channels, lx = u->tensors[xt].level;
      if ((rc = cwdm_channel_sum(grd(o), dt, B, vox(cs.level), cs.cout, cs.cout, nullptr, 0, GR(cs.b_p), nullptr,
                                 gb + G.chs, G.chs_bytes, stream)))
        return rc;
      if (bk.updown == 4) {
        if ((rc = wgrad(cs.level, 3, act(xt), chn, nullptr, 0, 1, nullptr, grd(o), cs.cout, cs.cout, GR(cs.w_p))))
          return rc;
        if ((rc = dgrad(bk.c1, grd(o)))) return rc;
        if ((rc = cwdm_resample_add(grd(xt), tmp, chn, B, D >> lx, H >> lx, W >> lx, 1, take_acc(xt), dt, stream)))
          return rc;
      } else {
        const auto& sd = u->s2ds[bk.pool];
        float* dwe = reinterpret_cast<float*>(gb + G.dwe);
        CWDM_HIP(hipMemsetAsync(dwe, 0, (int64_t)cs.cout * cs.cin_a * 27 * 4, s));
        if ((rc = wgrad(cs.level, 3, act(sd.out), cs.cin_a, nullptr, 0, 0, nullptr, grd(o), cs.cout, cs.cout, dwe)))
          return rc;
        if ((rc = cwdm_conv3d_s2_fold_dw(dwe, cs.cout, chn, GR(cs.w_p), 1, stream))) return rc;
        if ((rc = dgrad(bk.c1, grd(o)))) return rc;
        if ((rc = cwdm_space_to_depth(tmp, chn, B, D >> cs.level, H >> cs.level, W >> cs.level, dt, grd(xt), 0,
                                      take_acc(xt), stream)))
          return rc;
      }
      continue;
    }
    if (seg <= nb) {
      const Block& bk = u->blocks[nb - seg];
      const auto& c1 = u->convs[bk.c1];
      const auto& c2 = u->convs[bk.c2];
      const int lout = c2.level;
      const int64_t Vo = vox(lout);
      const int o = c2.out, h1 = c1.out;
      const int cout = c2.cout;
      // ---- conv2 (+ skip / residual)
      if ((rc = cwdm_channel_sum(grd(o), dt, B, Vo, cout, cout, nullptr, 0, GR(c2.b_p),
                                 c2.wsb_p >= 0 ? GR(c2.wsb_p) : nullptr, gb + G.chs, G.chs_bytes, stream)))
        return rc;
      if ((rc = wgrad_c(bk.c2, lout, act(h1), cout, nullptr, 0, 0, ss_of(bk.g2), grd(o), cout, cout, GR(c2.w_p))))
        return rc;
      // 1x1 skip dgrad into dx0 / dx1 (dual output); with skip_gapply the
      // GroupNorm-1 backward's apply pass rides in its epilogue (GapplyFuse),
      // so it runs after GN1's reduce / finalize below
      auto skip_dgrad = [&](cwdm::GapplyFuse* gf, bool dry) -> int {
        const int c0 = u->tensors[c2.sb0].channels, cc1 = c2.sb1 >= 0 ? u->tensors[c2.sb1].channels : 0;
        cwdm_conv3d_desc d{};
        d.dtype = dt; d.B = B; d.D = D >> lout; d.H = H >> lout; d.W = W >> lout;
        d.cout = c0 + cc1;
        d.b0 = grd(o); d.b_c0 = cout; d.b_w = pb + u->dgs_off[bk.c2];
        d.res_mode = -1;
        d.out = grd(c2.sb0); d.out_dtype = dt;
        if (c2.sb1 >= 0) { d.out1 = grd(c2.sb1); d.out_c0 = c0; }
        if (dry) return pw_gapply_ok(&d) ? 1 : 0;
        // equalise the store/accumulate state of the two outputs
        int a0 = take_acc(c2.sb0), a1 = c2.sb1 >= 0 ? take_acc(c2.sb1) : a0;
        if (a0 != a1) {
          const int zid = a0 ? c2.sb1 : c2.sb0;
          const auto& zt = u->tensors[zid];
          CWDM_HIP(hipMemsetAsync(grd(zid), 0, B * vox(zt.level) * zt.channels * es, s));
          a0 = a1 = 1;
        }
        d.accumulate = a0;
        d.workspace = gb + G.split; d.ws_bytes = G.split_bytes;
        cwdm::g_gapply = gf;
        const int r = cwdm_conv3d_forward(&d, stream);
        cwdm::g_gapply = nullptr;
        if (r) return r;
        CWDM_REQUIRE(!gf || gf->used, CWDM_E_UNSUPPORTED, "train plan: skip dgrad did not take the fused apply");
        return CWDM_OK;
      };
      static const bool gapply_on = [] { const char* e = std::getenv("CWDM_GAPPLY_FUSE"); return !(e && e[0] == '0'); }();
      const bool skip_gapply = c2.ws_p >= 0 && gapply_on && bk.updown == 0 && c2.sb0 == bk.x0 &&
                               c2.sb1 == bk.x1 && skip_dgrad(nullptr, true) == 1;
      if (c2.ws_p >= 0) {
        const int c0 = u->tensors[c2.sb0].channels, cc1 = c2.sb1 >= 0 ? u->tensors[c2.sb1].channels : 0;
        if ((rc = wgrad(lout, 1, act(c2.sb0), c0, act(c2.sb1), cc1, 0, nullptr, grd(o), cout, cout, GR(c2.ws_p))))
          return rc;
        if (!skip_gapply && (rc = skip_dgrad(nullptr, false))) return rc;
      } else {
        // identity residual (possibly through the block's resampling)
        const int xt = bk.x0;
        const int lx = u->tensors[xt].level;
        const int mode = bk.updown == 2 ? 2 : (bk.updown == 1 ? 1 : 0);
        if ((rc = cwdm_resample_add(grd(xt), grd(o), cout, B, D >> lx, H >> lx, W >> lx, mode, take_acc(xt), dt,
                                    stream)))
          return rc;
      }
      Pre pre2;
      if ((rc = dgrad_gn(bk.c2, grd(o), bk.g2, h1, -1, pre2))) return rc;
      // ---- GN2 -> dh1, with the per-channel sums of dh1 (the emb projection's
      // gradient) taken in the same pass when dh1 is written, not accumulated
      const int k = bk.emb_k;
      const int roff = u->emb_rows_off[k], rn = u->emb_rows_n[k];
      const bool fuse_sum = !u->ginit[h1];
      if (fuse_sum) {
        const auto& g = u->gns[bk.g2];
        if ((rc = gn_silu_bwd_impl(act(h1), cout, nullptr, 0, tmp, 0, ss_of(bk.g2), mr_of(bk.g2), P(g.gamma_off),
                                   u->cfg.num_groups, B, D >> lout, H >> lout, W >> lout, dt, grd(h1), take_acc(h1),
                                   nullptr, 0, GR(g.gamma_p), GR(g.beta_p), gb + G.gnws, G.gnws_bytes, deb + roff, u->R,
                                   stream, 1, pre2.part, pre2.nblk)))
          return rc;
      } else {
        if ((rc = gn_bwd(bk.g2, h1, -1, 0, &pre2))) return rc;
        if ((rc = cwdm_channel_sum(grd(h1), dt, B, Vo, cout, cout, deb + roff, u->R, nullptr, nullptr, gb + G.chs,
                                   G.chs_bytes, stream)))
          return rc;
      }
      // ---- conv1: emb projection, wgrad, dgrad
      if ((rc = launch_emb_bwd(deb + roff, u->R, rn, (int)B, temb, u->E, P(u->off_emb_w) + (int64_t)roff * u->E,
                               GR(u->emb_rows_w[k]), GR(u->emb_rows_b[k]), GR(u->emb_rows_cb[k]), dsil, s, 1)))
        return rc;
      if (bk.updown == 2) {
        const auto& ps = u->pools[bk.pool];
        if ((rc = wgrad(lout, 3, act(ps.out_h), ps.channels, nullptr, 0, 0, nullptr, grd(h1), cout, cout,
                        GR(c1.w_p))))
          return rc;
      } else {
        const int c0 = u->tensors[bk.x0].channels, cc1 = bk.x1 >= 0 ? u->tensors[bk.x1].channels : 0;
        if ((rc = wgrad_c(bk.c1, lout, act(bk.x0), c0, act(bk.x1), cc1, bk.updown == 1 ? 1 : 0, ss_of(bk.g1),
                          grd(h1), cout, cout, GR(c1.w_p))))
          return rc;
      }
      // ---- GN1 (+ resample adjoint) -> dx0 / dx1 (the reduce in the dgrad's epilogue
      // when the GroupNorm's grid is the conv's: no resampling in between)
      Pre pre1;
      if (bk.updown == 0) {
        if ((rc = dgrad_gn(bk.c1, grd(h1), bk.g1, bk.x0, bk.x1, pre1))) return rc;
      } else if ((rc = dgrad(bk.c1, grd(h1)))) {
        return rc;
      }
      if (skip_gapply) {
        // GN1 reduce / finalize, then the skip dgrad applying it: dx = skip + GN1 backward
        const auto& g = u->gns[bk.g1];
        const int c0 = u->tensors[bk.x0].channels, cc1 = bk.x1 >= 0 ? u->tensors[bk.x1].channels : 0;
        const float* coef = nullptr;
        if ((rc = gn_silu_bwd_impl(act(bk.x0), c0, act(bk.x1), cc1, tmp, 0, ss_of(bk.g1), mr_of(bk.g1),
                                   P(g.gamma_off), u->cfg.num_groups, B, D >> lout, H >> lout, W >> lout, dt,
                                   grd(bk.x0), 0, grd(bk.x1), 0, GR(g.gamma_p), GR(g.beta_p), gb + G.gnws,
                                   G.gnws_bytes, nullptr, 0, stream, 1, pre1.part, pre1.nblk, &coef)))
          return rc;
        cwdm::GapplyFuse gf{};
        gf.x0 = act(bk.x0); gf.x1 = act(bk.x1); gf.du = tmp; gf.ss = ss_of(bk.g1); gf.coef = coef;
        if ((rc = skip_dgrad(&gf, false))) return rc;
        continue;
      }
      if ((rc = gn_bwd(bk.g1, bk.x0, bk.x1, bk.updown == 1 ? 1 : (bk.updown == 2 ? 2 : 0), &pre1))) return rc;
      continue;
    }
    // conv_in + time_embed
    const auto& c0 = u->convs[0];
    const int64_t V0 = D * H * W;
    if ((rc = cwdm_channel_sum(grd(c0.out), dt, B, V0, c0.cout, c0.cout, nullptr, 0, GR(c0.b_p), nullptr, gb + G.chs,
                               G.chs_bytes, stream)))
      return rc;
    if ((rc = wgrad(0, 3, x, c0.cin_a, nullptr, 0, 0, nullptr, grd(c0.out), c0.cout, c0.cout, GR(c0.w_p)))) return rc;
    if ((rc = launch_temb_bwd(t, (int)B, u->cfg.model_channels, P(u->off_te_w1), P(u->off_te_b1), P(u->off_te_w2),
                              temb, dsil, GR(u->te_w1), GR(u->te_b1), GR(u->te_w2), GR(u->te_b2), s)))
      return rc;
  }
  return CWDM_OK;
}
