// U-Net executor: builds the UNetModel topology of the run.sh configuration
// family (guided_diffusion/unet.py:482-725), owns the parameter
// naming contract (state_dict keys/shapes), packs weights into the kernel
// layouts and replays UNetModel.forward (unet.py:754-800) as a fixed list of
// GroupNorm-finalize and fused conv launches on one stream.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"

namespace cwdm {
int launch_time_embed(const float* t, int B, int mc, const float* w1, const float* b1, const float* w2,
                      const float* b2, float* temb, hipStream_t s);
int launch_emb_proj(const float* temb, int B, int E, const float* W, const float* bias, int R, float* out,
                    hipStream_t s);
int launch_vec_add(const float* a, const float* b, float* out, int64_t n, hipStream_t s);
}  // namespace cwdm

using namespace cwdm;

namespace {

constexpr int64_t kAlign = 256;
inline int64_t align_up(int64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

struct Param { std::string name; std::vector<int64_t> shape; int64_t numel() const { int64_t n = 1; for (auto s : shape) n *= s; return n; } };

struct Tensor { int level; int channels; };

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
};

struct PoolStep {  // down-ResBlock pre-pass (cwdm_gn_silu_pool)
  int src, ss_id, out_h, out_x, level_out, channels;
};

struct Step { int kind; int idx; };  // kind 0 = gn, 1 = conv, 2 = pool pre-pass

}  // namespace

struct cwdm_unet {
  cwdm_unet_config cfg;
  int E = 0;                      // time embed dim
  std::vector<Param> params;
  std::vector<Tensor> tensors;
  std::vector<GnStep> gns;
  std::vector<ConvStep> convs;
  std::vector<PoolStep> pools;
  std::vector<Step> steps;
  std::vector<int> trace;         // tensor id per topology block (-1 = final output)
  std::vector<int> trace_level;
  int input_tensor = -1;          // pseudo tensor for x
  int R = 0;                      // emb projection rows
  std::vector<int> emb_rows_w, emb_rows_b, emb_rows_cb;  // per res block: emb weight/bias param, conv1 bias param
  std::vector<int> emb_rows_off, emb_rows_n;
  int te_w1, te_b1, te_w2, te_b2;
  int64_t off_te_w1, off_te_b1, off_te_w2, off_te_b2, off_emb_w, off_emb_b;
  int64_t packed_bytes = 0;
  // profiling
  bool profiling = false;
  std::vector<hipEvent_t> ev;
  std::vector<double> ev_flops;
  int ev_used = 0;

  int add_param(const std::string& n, std::vector<int64_t> s) {
    params.push_back({n, std::move(s)});
    return (int)params.size() - 1;
  }
};

namespace {

int esize(int dtype) { return dtype == CWDM_BF16 ? 2 : 4; }

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

  auto conv_params = [&](const std::string& p, int co, int ci, int k, int* wp, int* bp) {
    *wp = u->add_param(p + ".weight", {co, ci, k, k, k});
    *bp = u->add_param(p + ".bias", {co});
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
    g.gamma_p = u->add_param(p + ".weight", {g.channels});
    g.beta_p = u->add_param(p + ".bias", {g.channels});
    g.level = lvl;
    g.ss_id = (int)u->gns.size();
    u->gns.push_back(g);
    u->steps.push_back({0, g.ss_id});
    return g.ss_id;
  };

  // ResBlock (unet.py:185-311): returns output tensor
  auto resblock = [&](const std::string& p, int x0, int x1, int cout, int updown /*0 none 1 up 2 down*/) {
    const int lin = u->tensors[x0].level;
    const int cin = u->tensors[x0].channels + (x1 >= 0 ? u->tensors[x1].channels : 0);
    const int lout = updown == 2 ? lin + 1 : (updown == 1 ? lin - 1 : lin);
    int g1 = gn_step(p + ".in_layers.0", x0, x1, lin);
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
      a_src = ps.out_h; a_mode = 0; a_gn = -1;
      xres = ps.out_x; xrmode = 0;
    }
    ConvStep c1{};
    conv_params(p + ".in_layers.2", cout, cin, 3, &c1.w_p, &c1.b_p);
    c1.emb_w_p = u->add_param(p + ".emb_layers.1.weight", {cout, E});
    c1.emb_b_p = u->add_param(p + ".emb_layers.1.bias", {cout});
    c1.a0 = a_src; c1.a1 = x1; c1.amode = a_mode; c1.gn = a_gn; c1.cin_a = cin;
    c1.sb0 = c1.sb1 = -1; c1.ws_p = c1.wsb_p = -1; c1.cin_b = 0;
    c1.bias_kind = 1; c1.bias_off = u->R;
    u->emb_rows_w.push_back(c1.emb_w_p); u->emb_rows_b.push_back(c1.emb_b_p); u->emb_rows_cb.push_back(c1.b_p);
    u->emb_rows_off.push_back(u->R); u->emb_rows_n.push_back(cout);
    u->R += cout;
    c1.res = -1; c1.rmode = -1; c1.cout = cout; c1.level = lout; c1.stats = true;
    int h1 = c1.out = new_tensor(lout, cout);
    u->convs.push_back(c1);
    u->steps.push_back({1, (int)u->convs.size() - 1});

    int g2 = gn_step(p + ".out_layers.0", h1, -1, lout);
    ConvStep c2{};
    conv_params(p + ".out_layers.3", cout, cout, 3, &c2.w_p, &c2.b_p);
    c2.a0 = h1; c2.a1 = -1; c2.amode = 0; c2.gn = g2; c2.cin_a = cout;
    c2.sb0 = c2.sb1 = -1; c2.ws_p = c2.wsb_p = -1; c2.cin_b = 0;
    c2.res = -1; c2.rmode = -1;
    if (cin != cout) {
      conv_params(p + ".skip_connection", cout, cin, 1, &c2.ws_p, &c2.wsb_p);
      c2.sb0 = x0; c2.sb1 = x1; c2.cin_b = cin;
    } else {
      c2.res = xres;
      c2.rmode = xrmode;
    }
    c2.bias_kind = 0; c2.cout = cout; c2.level = lout; c2.stats = true;
    int o = c2.out = new_tensor(lout, cout);
    u->convs.push_back(c2);
    u->steps.push_back({1, (int)u->convs.size() - 1});
    return o;
  };

  int ch = mc, idx = 1;
  const int nl = c.num_levels;
  for (int l = 0; l < nl; ++l) {
    const int mult = c.channel_mult[l];
    for (int r = 0; r < c.num_res_blocks; ++r) {
      h = resblock("input_blocks." + std::to_string(idx) + ".0", h, -1, mult * mc, 0);
      ch = mult * mc;
      stack.push_back(h);
      u->trace.push_back(h); u->trace_level.push_back(level);
      ++idx;
    }
    if (l != nl - 1) {
      h = resblock("input_blocks." + std::to_string(idx) + ".0", h, -1, ch, 2);
      ++level;
      stack.push_back(h);
      u->trace.push_back(h); u->trace_level.push_back(level);
      ++idx;
    }
  }
  h = resblock("middle_block.0", h, -1, ch, 0);
  u->trace.push_back(h); u->trace_level.push_back(level);
  h = resblock("middle_block.1", h, -1, ch, 0);
  u->trace.push_back(h); u->trace_level.push_back(level);
  idx = 0;
  for (int l = nl - 1; l >= 0; --l) {
    const int mult = c.channel_mult[l];
    for (int i = 0; i <= c.num_res_blocks; ++i) {
      int skip = stack.back();
      stack.pop_back();
      h = resblock("output_blocks." + std::to_string(idx) + ".0", h, skip, mc * mult, 0);
      ch = mc * mult;
      u->trace.push_back(h); u->trace_level.push_back(level);
      if (l && i == c.num_res_blocks) {
        h = resblock("output_blocks." + std::to_string(idx) + ".1", h, -1, ch, 1);
        --level;
        u->trace.push_back(h); u->trace_level.push_back(level);
      }
      ++idx;
    }
  }
  // out head
  int g = gn_step("out.0", h, -1, 0);
  ConvStep co{};
  conv_params("out.2", c.out_channels, ch, 3, &co.w_p, &co.b_p);
  co.a0 = h; co.a1 = -1; co.amode = 0; co.gn = g; co.cin_a = ch;
  co.sb0 = co.sb1 = -1; co.ws_p = co.wsb_p = -1; co.cin_b = 0;
  co.bias_kind = 0; co.res = -1; co.rmode = -1; co.cout = c.out_channels; co.level = 0; co.stats = false;
  co.out = -1;
  u->convs.push_back(co);
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
  for (auto& cs : u->convs) {
    cs.w_off = take(cwdm_conv3d_packed_bytes(cs.cout, cs.cin_a, 3, c.dtype));
    if (cs.ws_p >= 0) cs.wsk_off = take(cwdm_conv3d_packed_bytes(cs.cout, cs.cin_b, 1, c.dtype));
    if (cs.bias_kind == 0) cs.bias_off = take((int64_t)cs.cout * 4);
  }
  for (auto& gs : u->gns) {
    gs.gamma_off = take((int64_t)gs.channels * 4);
    gs.beta_off = take((int64_t)gs.channels * 4);
  }
  u->packed_bytes = off;
}

struct Layout {
  int64_t temb, ebias, split, split_bytes;
  std::vector<int64_t> t_off, s_off, s_parts;
  std::vector<int64_t> ss_off, mr_off;
  int64_t total;
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
  if (cs.ws_p >= 0) {
    d.b_c0 = u->tensors[cs.sb0].channels;
    d.b_c1 = cs.sb1 >= 0 ? u->tensors[cs.sb1].channels : 0;
    d.b_w = reinterpret_cast<const void*>(1);  // presence flag only
  }
  d.res_mode = cs.rmode;
  d.out_dtype = cs.out < 0 ? CWDM_F32 : u->cfg.dtype;
  return d;
}

Layout layout(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  Layout L;
  int64_t off = 0;
  auto take = [&](int64_t bytes) { int64_t o = off; off = align_up(off + bytes); return o; };
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
    const int64_t parts = cwdm_conv3d_parts(u->cfg.dtype, d, h, w, t.channels);
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
  }
  L.split_bytes = split;
  L.split = take(split);
  L.total = off;
  return L;
}

}  // namespace

namespace cwdm {
namespace {
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
  CWDM_REQUIRE(cfg->dtype == CWDM_F32 || cfg->dtype == CWDM_BF16, CWDM_E_INVALID, "cwdm_unet_create: bad dtype");
  CWDM_REQUIRE(cfg->num_groups > 0, CWDM_E_INVALID, "cwdm_unet_create: bad num_groups");
  const int ck = cfg->dtype == CWDM_BF16 ? 16 : 8;
  CWDM_REQUIRE(cfg->in_channels % ck == 0, CWDM_E_UNSUPPORTED,
               "cwdm_unet_create: in_channels must be a multiple of " + std::to_string(ck));
  for (int l = 0; l < cfg->num_levels; ++l) {
    const int ch = cfg->channel_mult[l] * cfg->model_channels;
    CWDM_REQUIRE(ch > 0 && ch % ck == 0 && (ch % 64 == 0 || ch % 32 == 0), CWDM_E_UNSUPPORTED,
                 "cwdm_unet_create: level channels must be multiples of 32 (and of the chunk)");
    CWDM_REQUIRE(ch % cfg->num_groups == 0, CWDM_E_INVALID, "cwdm_unet_create: channels not divisible by groups");
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

extern "C" int64_t cwdm_unet_packed_bytes(const cwdm_unet* u) { return u ? u->packed_bytes : -1; }

extern "C" int cwdm_unet_pack(const cwdm_unet* u, const float* const* P, void* packed, cwdm_stream_t stream) {
  CWDM_REQUIRE(u && P && packed, CWDM_E_INVALID, "cwdm_unet_pack: null pointer");
  hipStream_t s = (hipStream_t)stream;
  auto* base = reinterpret_cast<unsigned char*>(packed);
  auto cp = [&](int pi, int64_t off) -> int {
    CWDM_HIP(hipMemcpyAsync(base + off, P[pi], u->params[pi].numel() * 4, hipMemcpyDeviceToDevice, s));
    return CWDM_OK;
  };
  int rc;
  if ((rc = cp(u->te_w1, u->off_te_w1)) || (rc = cp(u->te_b1, u->off_te_b1)) || (rc = cp(u->te_w2, u->off_te_w2)) ||
      (rc = cp(u->te_b2, u->off_te_b2)))
    return rc;
  float* ew = reinterpret_cast<float*>(base + u->off_emb_w);
  float* eb = reinterpret_cast<float*>(base + u->off_emb_b);
  for (size_t k = 0; k < u->emb_rows_w.size(); ++k) {
    const int64_t o = u->emb_rows_off[k], n = u->emb_rows_n[k];
    CWDM_HIP(hipMemcpyAsync(ew + o * u->E, P[u->emb_rows_w[k]], n * u->E * 4, hipMemcpyDeviceToDevice, s));
    if ((rc = launch_vec_add(P[u->emb_rows_b[k]], P[u->emb_rows_cb[k]], eb + o, n, s))) return rc;
  }
  for (const auto& cs : u->convs) {
    if ((rc = cwdm_conv3d_pack(P[cs.w_p], cs.cout, cs.cin_a, 3, u->cfg.dtype, base + cs.w_off, stream))) return rc;
    if (cs.ws_p >= 0 &&
        (rc = cwdm_conv3d_pack(P[cs.ws_p], cs.cout, cs.cin_b, 1, u->cfg.dtype, base + cs.wsk_off, stream)))
      return rc;
    if (cs.bias_kind == 0) {
      float* bo = reinterpret_cast<float*>(base + cs.bias_off);
      if (cs.wsb_p >= 0) {
        if ((rc = launch_vec_add(P[cs.b_p], P[cs.wsb_p], bo, cs.cout, s))) return rc;
      } else if ((rc = cp(cs.b_p, cs.bias_off))) {
        return rc;
      }
    }
  }
  for (const auto& g : u->gns) {
    if ((rc = cp(g.gamma_p, g.gamma_off)) || (rc = cp(g.beta_p, g.beta_off))) return rc;
  }
  return CWDM_OK;
}

extern "C" int64_t cwdm_unet_workspace_bytes(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u || B <= 0 || D <= 0 || H <= 0 || W <= 0) return -1;
  return layout(u, B, D, H, W).total;
}

extern "C" double cwdm_unet_flops(const cwdm_unet* u, int64_t B, int64_t D, int64_t H, int64_t W) {
  if (!u) return -1;
  double f = 0;
  for (const auto& cs : u->convs) {
    const double v = (double)B * (D >> cs.level) * (H >> cs.level) * (W >> cs.level);
    f += 2.0 * v * cs.cout * (27.0 * cs.cin_a + cs.cin_b);
  }
  return f;
}

extern "C" int cwdm_unet_forward(cwdm_unet* u, const void* packed, const void* x, const float* t, float* out,
                                 int64_t B, int64_t D, int64_t H, int64_t W, void* ws, int64_t ws_bytes,
                                 cwdm_stream_t stream) {
  CWDM_REQUIRE(u && packed && x && t && out && ws, CWDM_E_INVALID, "cwdm_unet_forward: null pointer");
  CWDM_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0, CWDM_E_SHAPE, "cwdm_unet_forward: empty grid");
  const int64_t div = int64_t(1) << (u->cfg.num_levels - 1);
  CWDM_REQUIRE(D % div == 0 && H % div == 0 && W % div == 0, CWDM_E_SHAPE,
               "cwdm_unet_forward: every subband edge must be divisible by " + std::to_string(div));
  Layout L = layout(u, B, D, H, W);
  CWDM_REQUIRE(ws_bytes >= L.total, CWDM_E_WORKSPACE,
               "cwdm_unet_forward: workspace too small (need " + std::to_string(L.total) + " bytes)");
  hipStream_t s = (hipStream_t)stream;
  auto* pk = reinterpret_cast<const unsigned char*>(packed);
  auto* wb = reinterpret_cast<unsigned char*>(ws);
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
  const int es = esize(u->cfg.dtype);
  (void)es;
  if (u->profiling) {
    const size_t need = u->convs.size() * 2;
    while (u->ev.size() < need) {
      hipEvent_t e;
      CWDM_HIP(hipEventCreate(&e));
      u->ev.push_back(e);
    }
    u->ev_flops.assign(u->convs.size(), 0.0);
    u->ev_used = 0;
  }
  for (const auto& st : u->steps) {
    if (st.kind == 2) {
      const auto& ps = u->pools[st.idx];
      const int lv = ps.level_out;
      if ((rc = cwdm_gn_silu_pool(tptr(ps.src), ps.channels, reinterpret_cast<const float*>(wb + L.ss_off[ps.ss_id]),
                                  B, D >> lv, H >> lv, W >> lv, u->cfg.dtype, wb + L.t_off[ps.out_h],
                                  wb + L.t_off[ps.out_x], stream)))
        return rc;
      continue;
    }
    if (st.kind == 0) {
      const auto& g = u->gns[st.idx];
      const int lv = g.level;
      const int64_t vox = (D >> lv) * (H >> lv) * (W >> lv);
      const int c0 = u->tensors[g.src0].channels, c1 = g.src1 >= 0 ? u->tensors[g.src1].channels : 0;
      if ((rc = cwdm_gn_finalize(reinterpret_cast<const float*>(wb + L.s_off[g.src0]), L.s_parts[g.src0], c0,
                                 g.src1 >= 0 ? reinterpret_cast<const float*>(wb + L.s_off[g.src1]) : nullptr,
                                 g.src1 >= 0 ? L.s_parts[g.src1] : 0, c1, P(g.gamma_off), P(g.beta_off),
                                 u->cfg.num_groups, B, vox, 1e-5f, reinterpret_cast<float*>(wb + L.ss_off[g.ss_id]),
                                 reinterpret_cast<float*>(wb + L.mr_off[g.ss_id]), stream)))
        return rc;
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
    if (u->profiling) CWDM_HIP(hipEventRecord(u->ev[2 * conv_i], s));
    if ((rc = cwdm_conv3d_forward(&d, stream))) return rc;
    if (u->profiling) {
      CWDM_HIP(hipEventRecord(u->ev[2 * conv_i + 1], s));
      u->ev_flops[conv_i] = 2.0 * B * d.D * d.H * d.W * cs.cout * (27.0 * cs.cin_a + cs.cin_b);
      u->ev_used = conv_i + 1;
    }
    ++conv_i;
  }
  return CWDM_OK;
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
  for (int i = 0; i < u->ev_used; ++i) {
    float m = 0;
    CWDM_HIP(hipEventElapsedTime(&m, u->ev[2 * i], u->ev[2 * i + 1]));
    tot += m;
    fl += u->ev_flops[i];
  }
  if (ms) *ms = tot;
  if (flops) *flops = fl;
  if (n) *n = u->ev_used;
  return CWDM_OK;
}
