// Score-network runtime: parameter store, weight packing and the forward plan of
// NCSN_LiDAR_small (LiDARGen/models/ncsnv2.py:420-518) over the libsdp kernels.
//
// Activations live in HBM as NHWC float32 carved from the caller's workspace; every
// InstanceNorm++ is split into per-tile statistics written by the producing conv's
// epilogue + a tiny finalize kernel + an affine/ELU prologue in the consuming conv, so no
// activation is ever re-read just for normalisation.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>


#include "net_internal.h"

using namespace sdp;

namespace {

struct Buf {
  float* p;
  int H, W, C;
};

struct Fwd {
  sdp_net* net;
  int B;
  hipStream_t st;
  float* stats;
  float* ss;
  float* mv;     // inpp_finalize scratch

  struct Opt {
    int pro = PRO_NONE;        // prologue
    bool bias = true;
    const float* res = nullptr;
    const float* up = nullptr;
    float* out2 = nullptr;
    const float* res2 = nullptr;
    bool epi_elu = false;
    bool stats = false;
    int dil = 1;
    bool circular = true;
    bool pool = false;
  };

  void conv(const Buf& in, const std::string& wkey, const Buf& out, const Opt& o) {
    const auto& hp = net->host.at(wkey + ".weight");
    ConvArgs a{};
    a.in = in.p;
    // forward weights: "#frag16" in the bf16 modes (16x16 MFMAs), "#frag" for exact fp32 (32x32)
    a.wf = net->mode == MODE_F32 ? reinterpret_cast<const uint4*>(net->P(wkey + ".weight#frag")) : nullptr;
    a.wf16 = net->mode == MODE_F32 ? nullptr : reinterpret_cast<const uint4*>(net->P(wkey + ".weight#frag16"));
    a.bias = o.bias ? net->P(wkey + ".bias") : nullptr;
    a.out = out.p;
    a.res = o.res;
    a.out2 = o.out2;
    a.res2 = o.res2;
    a.up = o.up;
    a.pro_ss = o.pro == PRO_AFFINE_ELU ? ss : net->P("#ident_ss");
    a.ss_bstride = o.pro == PRO_AFFINE_ELU ? 2 * in.C : 0;
    a.stats = o.stats ? stats : nullptr;
    a.B = B;
    a.H = in.H;
    a.W = in.W;
    a.Cin = in.C;
    a.Cout = out.C;
    a.dil = o.dil;
    a.circular = o.circular ? 1 : 0;
    a.pro_mode = o.pro;
    a.epi_elu = o.epi_elu ? 1 : 0;
    if ((int)hp.shape[1] != in.C || (int)hp.shape[0] != out.C) throw std::runtime_error("conv shape mismatch " + wkey);
    const char* why = "conv launch";
    const int ks = (int)hp.shape[2];
    sdp_net::ProfRec rec;
    if (net->profile) {
      rec.cls = "conv" + std::to_string(ks) + "x" + std::to_string(ks) + " " + std::to_string(in.C) + "->" +
                std::to_string(out.C) + " @" + std::to_string(in.H) + "x" + std::to_string(in.W) + " d" +
                std::to_string(o.dil) + (o.pool ? " pool" : "");
      rec.flops = 2.0 * B * in.H * in.W * (double)in.C * out.C * ks * ks;
      rec.bytes = 4.0 * B * ((double)in.H * in.W * in.C + (double)out.H * out.W * out.C) + 4.0 * out.C * in.C * ks * ks;
      rec.a = net->event();
      rec.b = net->event();
      chk(hipEventRecord(rec.a, st), "hipEventRecord");
    }
    hipError_t e = conv_mfma(net->mode, a, ks, o.pool, st, &why);
    if (e != hipSuccess) throw std::runtime_error(std::string(why) + " (" + wkey + ")");
    if (net->profile) {
      chk(hipEventRecord(rec.b, st), "hipEventRecord");
      net->prof.push_back(rec);
    }
  }

  // a non-conv launch under the profiler: class name + algorithmic bytes (HBM roofline)
  template <class F>
  void prof_launch(const std::string& cls, double bytes, F&& launch) {
    sdp_net::ProfRec rec;
    if (net->profile) {
      rec.cls = cls;
      rec.flops = 0;
      rec.bytes = bytes;
      rec.a = net->event();
      rec.b = net->event();
      chk(hipEventRecord(rec.a, st), "hipEventRecord");
    }
    launch();
    if (net->profile) {
      chk(hipEventRecord(rec.b, st), "hipEventRecord");
      net->prof.push_back(rec);
    }
  }

  // stats (written by the previous conv) -> scale/shift of InstanceNorm2dPlus `nkey`
  void norm(const std::string& nkey, int T, float cnt, int C) {
    prof_launch("inpp_finalize C" + std::to_string(C), (double)B * T * C * 8 + (double)B * C * 8, [&] {
      chk(inpp_finalize(stats, B, T, cnt, C, net->P(nkey + ".alpha"), net->P(nkey + ".gamma"), net->P(nkey + ".beta"),
                        ss, st, nullptr, mv),
          "inpp_finalize");
    });
  }
  void pool(const Buf& X, const Buf& P) {
    const double bytes = 2.0 * B * X.H * X.W * X.C * 4;
    prof_launch("maxpool5 " + std::to_string(X.C) + " @" + std::to_string(X.H) + "x" + std::to_string(X.W), bytes,
                [&] { chk(maxpool5(X.p, P.p, B, X.H, X.W, X.C, st), "maxpool5"); });
  }
  static int tiles(const Buf& b) { return b.H * b.W / 128; }

  // ResidualBlock.forward (layers.py:443-456); returns output in `out`, stats of out written
  void resblock(const std::string& k, const Buf& x, const Buf& t1, const Buf& t2, const Buf& out, bool down, int dil,
                bool want_stats, int x_tiles, float x_cnt) {
    norm(k + ".normalize1", x_tiles, x_cnt, x.C);
    Opt o1;
    o1.pro = PRO_AFFINE_ELU;
    o1.stats = true;
    o1.dil = dil;
    conv(x, k + ".conv1", t1, o1);
    norm(k + ".normalize2", tiles(t1), 128.f, t1.C);
    Opt o2;
    o2.pro = PRO_AFFINE_ELU;
    o2.stats = want_stats;
    o2.dil = dil;
    if (down && dil == 1) {
      // ConvMeanPool shortcut (1x1) pool-first: the 2x2 mean of the raw input (into `out`, free until
      // conv2 writes it), then the 1x1 conv at half resolution (a quarter of the FLOPs of conv-then-pool;
      // the same linear map, float rounding aside); then conv2 = ConvMeanPool 3x3
      const Buf xp{out.p, x.H / 2, x.W / 2, x.C};
      prof_launch("avgpool2 " + std::to_string(x.C) + " @" + std::to_string(x.H) + "x" + std::to_string(x.W),
                  1.25 * B * x.H * x.W * x.C * 4, [&] { chk(avgpool2(x.p, xp.p, B, x.H, x.W, x.C, st), "avgpool2"); });
      Opt os;
      os.circular = false;
      conv(xp, k + ".shortcut.conv", t2, os);
      o2.circular = false;
      o2.pool = true;
      o2.res = t2.p;
      conv(t1, k + ".conv2.conv", out, o2);
    } else if (down) {
      Opt os;
      os.dil = dil;
      conv(x, k + ".shortcut", t2, os);
      o2.res = t2.p;
      conv(t1, k + ".conv2", out, o2);
    } else {
      o2.res = x.p;
      conv(t1, k + ".conv2", out, o2);
    }
  }

  // RCUBlock (layers.py:126-134): n blocks of [ELU->conv->ELU->conv] + residual.
  // Result in slots[last]; uses tmp.  epi_elu on the final conv when a CRP follows.
  Buf rcu(const std::string& k, Buf x, int nblocks, const Buf& tmp, const Buf& o0, const Buf& o1, bool final_elu,
          bool final_stats) {
    Buf outs[2] = {o0, o1};
    for (int i = 0; i < nblocks; ++i) {
      Opt a;
      a.pro = PRO_ELU;
      a.bias = false;
      conv(x, k + "." + std::to_string(i + 1) + "_1_conv", tmp, a);
      Opt b;
      b.pro = PRO_ELU;
      b.bias = false;
      b.res = x.p;
      b.epi_elu = final_elu && i == nblocks - 1;
      b.stats = final_stats && i == nblocks - 1;
      const Buf& y = outs[i & 1];
      conv(tmp, k + "." + std::to_string(i + 1) + "_2_conv", y, b);
      x = y;
    }
    return x;
  }

  // CRPBlock (layers.py:76-83) on X = ELU(h) (already applied by the producer)
  // -> returns x2 ; slots: P (pool), Q (path), R (x1), S (x2)
  Buf crp(const std::string& k, const Buf& X, const Buf& P, const Buf& Qp, const Buf& R, const Buf& S) {
    pool(X, P);
    Opt a;
    a.bias = false;
    a.out2 = R.p;
    a.res2 = X.p;
    conv(P, k + ".convs.0", Qp, a);                   // path1 -> Qp ; x1 = path1 + X -> R
    pool(Buf{Qp.p, X.H, X.W, X.C}, P);
    Opt b;
    b.bias = false;
    b.res = R.p;
    conv(P, k + ".convs.1", S, b);                    // x2 = path2 + x1
    return S;
  }
};

}  // namespace

// ------------------------------------------------------------------------------ forward
static void forward_impl(sdp_net* net, const float* x, const int64_t* labels, float* out, int B, void* ws,
                         size_t ws_bytes, hipStream_t st, const LangevinArgs* lg = nullptr) {
  const int H = net->d.H, W = net->d.W, C = net->d.ngf, C2 = 2 * C;
  const int h = H / 2, w = W / 2;
  const size_t F = (size_t)B * H * W * C, Q = (size_t)B * h * w * C2;
  char* p = reinterpret_cast<char*>(ws);
  char* end = p + ws_bytes;
  auto take = [&](size_t n) {
    float* q = reinterpret_cast<float*>(p);
    p += ((n * 4 + 255) / 256) * 256;
    if (p > end) throw std::runtime_error("workspace too small");
    return q;
  };
  Fwd f{net, B, st, nullptr, nullptr, nullptr};
  f.stats = take((size_t)B * (H * W / 64) * C2 * 2);
  f.ss = take((size_t)B * C2 * 2);
  f.mv = take((size_t)B * C2 * 4);
  auto full = [&]() { return Buf{take(F), H, W, C}; };
  auto half = [&]() { return Buf{take(Q), h, w, C2}; };
  Buf L1 = full(), FA = full(), FB = full(), FC = full(), FD = full(), FE = full();
  Buf L2 = half(), L3 = half(), L4 = half(), QA = half(), QB = half(), QC = half(), QD = half(), QE = half();
  auto half128 = [&](const Buf& b) { return Buf{b.p, h, w, C}; };

  using Opt = Fwd::Opt;
  // begin_conv + input prep  -> FA (stats over 64-px tiles)
  f.prof_launch("begin_conv 4->128 @" + std::to_string(H) + "x" + std::to_string(W),
                (double)B * H * W * (2 * 4 + C * 4) + (double)B * (H * W / 64) * C * 8, [&] {
                  chk(begin_conv(x, net->P("begin_conv.weight"), net->P("begin_conv.bias"), FA.p, f.stats, B, H, W, st, net->mode),
                      "begin_conv");
                });
  // res1
  f.resblock("res1.0", FA, FB, FD, FC, false, 1, true, H * W / 64, 64.f);
  f.resblock("res1.1", FC, FB, FD, L1, false, 1, true, Fwd::tiles(FC), 128.f);
  // res2 (down: ConvMeanPool)
  f.resblock("res2.0", L1, FB, QA, QB, true, 1, true, Fwd::tiles(L1), 128.f);
  f.resblock("res2.1", QB, QA, QC, L2, false, 1, true, Fwd::tiles(L1), 32.f);
  // res3 (dilation 2), res4 (dilation 4)
  f.resblock("res3.0", L2, QA, QB, QC, true, 2, true, Fwd::tiles(L2), 128.f);
  f.resblock("res3.1", QC, QA, QB, L3, false, 2, true, Fwd::tiles(QC), 128.f);
  f.resblock("res4.0", L3, QA, QB, QC, true, 4, true, Fwd::tiles(L3), 128.f);
  f.resblock("res4.1", QC, QA, QB, L4, false, 4, false, Fwd::tiles(QC), 128.f);

  // refine1([L4]) : adapt RCU -> ELU -> CRP -> output RCU
  Buf a1 = f.rcu("refine1.adapt_convs.0", L4, 2, QA, QB, QC, true, false);          // ELU(h) in QC
  Buf x2 = f.crp("refine1.crp", a1, QA, QB, QD, QE);
  Buf ref1 = f.rcu("refine1.output_convs", x2, 1, QA, QB, QC, false, false);       // QB
  // refine2([L3, ref1]) ; ref1 lives in QB
  Buf hA = f.rcu("refine2.adapt_convs.0", L3, 2, QA, QC, QD, false, false);        // QD
  Buf hB = f.rcu("refine2.adapt_convs.1", ref1, 2, QA, QC, QE, false, false);      // QE
  {
    Opt o;
    f.conv(hA, "refine2.msf.convs.0", QA, o);                                      // m0 -> QA
    Opt o1;
    o1.res = QA.p;
    o1.epi_elu = true;
    f.conv(hB, "refine2.msf.convs.1", QB, o1);                                     // ELU(m0 + m1) -> QB
  }
  x2 = f.crp("refine2.crp", QB, QA, QC, QD, QE);                                   // QE
  Buf ref2 = f.rcu("refine2.output_convs", x2, 1, QA, QB, QC, false, false);       // QB
  // refine3([L2, ref2]) -> 128 channels at half resolution
  hA = f.rcu("refine3.adapt_convs.0", L2, 2, QA, QC, QD, false, false);            // QD
  hB = f.rcu("refine3.adapt_convs.1", ref2, 2, QA, QC, QE, false, false);          // QE
  {
    Opt o;
    f.conv(hA, "refine3.msf.convs.0", half128(QA), o);
    Opt o1;
    o1.res = QA.p;
    o1.epi_elu = true;
    f.conv(hB, "refine3.msf.convs.1", half128(QB), o1);
  }
  x2 = f.crp("refine3.crp", half128(QB), half128(QA), half128(QC), half128(QD), half128(QE));
  Buf ref3 = f.rcu("refine3.output_convs", x2, 1, half128(QA), half128(QB), half128(QC), false, false);  // QB
  // refine4([L1, ref3]) at full resolution
  hA = f.rcu("refine4.adapt_convs.0", L1, 2, FA, FB, FC, false, false);            // FC
  hB = f.rcu("refine4.adapt_convs.1", ref3, 2, half128(QA), half128(QC), half128(QD), false, false);  // QD
  {
    Opt o;
    f.conv(hB, "refine4.msf.convs.1", half128(QA), o);                             // m1 (half res) -> QA
    Opt o1;
    o1.up = QA.p;
    o1.epi_elu = true;
    f.conv(hA, "refine4.msf.convs.0", FD, o1);                                     // ELU(m0 + up(m1)) -> FD
  }
  x2 = f.crp("refine4.crp", FD, FA, FB, FE, FC);                                   // FC
  Buf o = f.rcu("refine4.output_convs", x2, 3, FA, FB, FD, false, true);           // FB, stats
  // head: IN++ -> ELU -> end_conv -> / sigmas[y]
  f.norm("normalizer", Fwd::tiles(o), 128.f, C);
  // with lg: + the fused Langevin update (x read + written, ref, mask, lik: 20 B per element; the
  // scores only when out is given)
  const double lg_bytes = lg ? (double)B * 2 * H * W * (20 + (out ? 4 : 0) + (lg->noise ? 4 : 0)) : B * 2.0 * H * W * 4;
  f.prof_launch(std::string(lg ? "end_conv+langevin" : "end_conv") + " 128->2 @" + std::to_string(H) + "x" +
                    std::to_string(W),
                (double)B * H * W * C * 4 + lg_bytes, [&] {
                  chk(end_conv(o.p, f.ss, net->P("end_conv.weight"), net->P("end_conv.bias"), net->P("sigmas"), labels,
                               out, B, H, W, C, st, lg, net->mode),
                      "end_conv");
                });
}

static size_t workspace_bytes_one(const sdp_net* net, int B) {
  const int H = net->d.H, W = net->d.W, C = net->d.ngf, C2 = 2 * C;
  const size_t F = (size_t)B * H * W * C, Q = (size_t)B * (H / 2) * (W / 2) * C2;
  auto r = [](size_t n) { return ((n * 4 + 255) / 256) * 256; };
  return r((size_t)B * (H * W / 64) * C2 * 2) + r((size_t)B * C2 * 2) + r((size_t)B * C2 * 4) + 6 * r(F) + 8 * r(Q);
}

// default of sdp_net::split: two part-batch forwards on two streams (forward_split; the A/B that
// set it: profiles/experiments/r02_split_streams_ab.log)
constexpr int kSplitDefault = 2;
static int split_ways(const sdp_net* net) { return net->split > 0 ? net->split : kSplitDefault; }

// part p of B images split k ways: [first, first + count)
static void split_part(int B, int k, int p, int& first, int& count) {
  first = (int)((long)B * p / k);
  count = (int)((long)B * (p + 1) / k) - first;
}

// room for one B-image forward, or for the part-batch forwards side by side (forward_split)
static size_t workspace_bytes(const sdp_net* net, int B) {
  size_t need = workspace_bytes_one(net, B);
  const int k = std::min(B, split_ways(net));
  if (k > 1) {
    size_t sum = 0;
    for (int p = 0; p < k; ++p) {
      int f, c;
      split_part(B, k, p, f, c);
      sum += workspace_bytes_one(net, c);
    }
    need = std::max(need, sum);
  }
  return need;
}

// The forward as k part-batch forwards on k streams (the caller's and the handle's own), joined by
// events.  Every conv launch of one forward is a lock-step grid: each workgroup owns a CU (LDS),
// so all of them stage their first chunks together and store their outputs together, and those
// bursts leave the matrix cores idle chip-wide; a grid that is not a whole number of rounds also
// idles CUs in its last one.  Concurrent part-size launches de-phase the bursts of one against the
// main loops of another and fill each other's last rounds.  Per-image results are unchanged: no op
// couples images (batch invariance), and the Langevin update of a part uses its own Philox counters
// (offset + first image * per-image counters).
static void forward_split(sdp_net* net, const float* x, const int64_t* labels, float* out, int B, void* ws,
                          size_t ws_bytes, hipStream_t st, const LangevinArgs* lg) {
  const int k = std::min(B, split_ways(net));
  if (k < 2 || net->profile) {
    forward_impl(net, x, labels, out, B, ws, ws_bytes, st, lg);
    return;
  }
  for (int p = 0; p + 1 < k; ++p) {
    if (!net->aux_stream[p])
      chk(hipStreamCreateWithFlags(&net->aux_stream[p], hipStreamNonBlocking), "hipStreamCreate");
    if (!net->ev_join[p]) chk(hipEventCreateWithFlags(&net->ev_join[p], hipEventDisableTiming), "hipEventCreate");
  }
  if (!net->ev_fork) chk(hipEventCreateWithFlags(&net->ev_fork, hipEventDisableTiming), "hipEventCreate");
  const size_t per = (size_t)2 * net->d.H * net->d.W;        // floats of one image (2 channels)
  char* w = reinterpret_cast<char*>(ws);
  chk(hipEventRecord(net->ev_fork, st), "hipEventRecord");
  for (int p = k - 1; p >= 0; --p) {                        // the caller's stream takes part 0, last
    int f, c;
    split_part(B, k, p, f, c);
    const size_t wb = workspace_bytes_one(net, c);
    hipStream_t s = p ? net->aux_stream[p - 1] : st;
    if (p) chk(hipStreamWaitEvent(s, net->ev_fork, 0), "hipStreamWaitEvent");
    LangevinArgs l{};
    if (lg) {
      l = *lg;
      l.x = lg->x + f * per;
      l.ref = lg->ref + f * per;
      l.mask = lg->mask + f * per;
      if (lg->noise) l.noise = lg->noise + f * per;
      if (lg->lik) l.lik = lg->lik + f * per;
      l.offset = lg->offset + f * per / 4;
    }
    forward_impl(net, x + f * per, labels + f, out ? out + f * per : nullptr, c, w, wb, s, lg ? &l : nullptr);
    w += wb;
    if (p) chk(hipEventRecord(net->ev_join[p - 1], s), "hipEventRecord");
  }
  for (int p = 0; p + 1 < k; ++p) chk(hipStreamWaitEvent(st, net->ev_join[p], 0), "hipStreamWaitEvent");
}

// ------------------------------------------------------------------------------ C ABI
static thread_local std::string g_err;

int sdp_fail(const std::string& m) {
  g_err = m;
  return -1;
}
static int fail(const std::string& m) { return sdp_fail(m); }

extern "C" {

int sdp_version(void) { return SDP_VERSION; }
const char* sdp_last_error(void) { return g_err.c_str(); }

int sdp_net_create(const sdp_net_desc* desc, sdp_net** out) {
  if (!desc || !out) return fail("sdp_net_create: null argument");
  if (desc->ngf != 128 || desc->channels != 2) return fail("sdp_net_create: only ngf=128, channels=2 are built");
  if (desc->H % 8 || desc->W % 128) return fail("sdp_net_create: H must be a multiple of 8 and W of 128");
  if (desc->precision < 0 || desc->precision > 2) return fail("sdp_net_create: bad precision");
  sdp_net* n = new sdp_net();
  n->d = *desc;
  n->mode = desc->precision;
  *out = n;
  return 0;
}

int sdp_net_set_param(sdp_net* net, const char* key, const float* data, const int64_t* shape, int ndim) {
  if (!net || !key || !data || (ndim > 0 && !shape)) return fail("sdp_net_set_param: null argument");
  HostParam hp;
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    hp.shape.push_back(shape[i]);
    n *= (size_t)shape[i];
  }
  hp.data.assign(data, data + n);
  net->host[key] = std::move(hp);
  net->finalized = false;
  return 0;
}

int sdp_net_finalize(sdp_net* net) {
  if (!net) return fail("sdp_net_finalize: null net");
  try {
    net->release();
    if (!net->host.count("sigmas")) return fail("sdp_net_finalize: missing sigmas");
    auto upload = [&](const std::string& k, const void* src, size_t bytes) {
      void* d = nullptr;
      chk(hipMalloc(&d, bytes), "hipMalloc");
      chk(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice), "hipMemcpy");
      net->dev[k] = d;
    };
    // every learnable parameter in one arena, 64-float aligned (sdp_net_param_info), in the order
    // the backward finishes their gradients (train.hip grad_completion_order; the parameters it
    // does not name, in key order after them): gradient buckets are then contiguous arena ranges
    net->layout.clear();
    size_t off = 0;
    std::vector<std::string> order;
    try {
      order = grad_completion_order(net);
    } catch (const std::exception&) {   // an incomplete parameter set: key order (its forward fails anyway)
      order.clear();
    }
    std::map<std::string, bool> placed;
    for (auto& kv : net->host)
      if (kv.first != "sigmas") order.push_back(kv.first);   // (duplicates skipped below)
    for (const auto& k : order) {
      auto it = net->host.find(k);
      if (it == net->host.end() || k == "sigmas" || placed[k]) continue;
      placed[k] = true;
      net->layout.push_back({k, off, it->second.data.size()});
      off += (it->second.data.size() + 63) / 64 * 64;
    }
    net->arena_floats = off;
    chk(hipMalloc(&net->arena, off * 4), "hipMalloc");
    net->arena_owned = true;
    for (auto& e : net->layout) {
      chk(hipMemcpy(net->arena + e.offset, net->host[e.key].data.data(), e.numel * 4, hipMemcpyHostToDevice), "hipMemcpy");
      net->dev[e.key] = net->arena + e.offset;
    }
    upload("sigmas", net->host["sigmas"].data.data(), net->host["sigmas"].data.size() * 4);
    for (auto& kv : net->host) {
      const HostParam& hp = kv.second;
      if (net->is_conv_w(kv.first) && (hp.shape[0] % 32 || hp.shape[1] % 32))
        return fail("sdp_net_finalize: conv channels must be /32: " + kv.first);
    }
    // identity (scale, shift) = (1, 0) rows for convs without an InstanceNorm++ prologue
    std::vector<float> ident(2 * 1024);
    for (size_t i = 0; i < ident.size(); i += 2) ident[i] = 1.f;
    upload("#ident_ss", ident.data(), ident.size() * 4);
    hipStream_t st;
    chk(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    net->repack(st);
    chk(hipStreamSynchronize(st), "hipStreamSynchronize");
    chk(hipStreamDestroy(st), "hipStreamDestroy");
    net->finalized = true;
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_finalize: ") + e.what());
  }
  return 0;
}

int sdp_net_param_arena_floats(const sdp_net* net, size_t* n) {
  if (!net || !n || !net->finalized) return fail("sdp_net_param_arena_floats: finalize first");
  *n = net->arena_floats;
  return 0;
}

int sdp_net_param_count(const sdp_net* net, int* n) {
  if (!net || !n || !net->finalized) return fail("sdp_net_param_count: finalize first");
  *n = (int)net->layout.size();
  return 0;
}

int sdp_net_param_info(const sdp_net* net, int i, char* key, size_t cap, size_t* offset, size_t* numel) {
  if (!net || !net->finalized || i < 0 || i >= (int)net->layout.size() || !key || cap == 0)
    return fail("sdp_net_param_info: bad argument");
  const auto& e = net->layout[i];
  std::strncpy(key, e.key.c_str(), cap - 1);
  key[cap - 1] = 0;
  if (offset) *offset = e.offset;
  if (numel) *numel = e.numel;
  return 0;
}

int sdp_net_bind_params(sdp_net* net, float* arena, void* stream) {
  if (!net || !arena || !net->finalized) return fail("sdp_net_bind_params: bad argument");
  try {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (arena != net->arena)
      chk(hipMemcpyAsync(arena, net->arena, net->arena_floats * 4, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    chk(hipStreamSynchronize(st), "hipStreamSynchronize");
    if (net->arena_owned) chk(hipFree(net->arena), "hipFree");
    net->arena = arena;
    net->arena_owned = false;
    for (auto& e : net->layout) net->dev[e.key] = arena + e.offset;
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_bind_params: ") + e.what());
  }
  return 0;
}

int sdp_net_repack(sdp_net* net, void* stream) {
  if (!net || !net->finalized) return fail("sdp_net_repack: finalize first");
  try {
    net->repack(reinterpret_cast<hipStream_t>(stream));
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_repack: ") + e.what());
  }
  return 0;
}

int sdp_net_workspace_size(const sdp_net* net, int B, size_t* bytes) {
  if (!net || !bytes || B <= 0) return fail("sdp_net_workspace_size: bad argument");
  *bytes = workspace_bytes(net, B);
  return 0;
}

int sdp_net_forward(sdp_net* net, const float* x, const int64_t* labels, float* out, int B, void* ws, size_t ws_bytes,
                    void* stream) {
  if (!net || !x || !labels || !out || !ws || B <= 0) return fail("sdp_net_forward: bad argument");
  if (!net->finalized) return fail("sdp_net_forward: call sdp_net_finalize first");
  if (ws_bytes < workspace_bytes(net, B)) return fail("sdp_net_forward: workspace too small");
  const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  try {
    forward_split(net, x, labels, out, B, ws, ws_bytes, st, nullptr);
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_forward: ") + e.what());
  }
  return 0;
}

int sdp_net_forward_langevin(sdp_net* net, float* x, const int64_t* labels, int B, const sdp_langevin_params* lp,
                             void* ws, size_t ws_bytes, void* stream) {
  if (!net || !x || !labels || !lp || !lp->ref || !lp->mask || !ws || B <= 0)
    return fail("sdp_net_forward_langevin: bad argument");
  if (!net->finalized) return fail("sdp_net_forward_langevin: call sdp_net_finalize first");
  if (ws_bytes < workspace_bytes(net, B)) return fail("sdp_net_forward_langevin: workspace too small");
  const LangevinArgs lg{x,         lp->ref,          lp->mask,  lp->noise,    lp->seed,         lp->offset, lp->step_size,
                        lp->noise_scale, lp->grad_ref, lp->nan_to_num, lp->lik_out, lp->absmax_bits};
  try {
    forward_split(net, x, labels, lp->grad_out, B, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream), &lg);
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_forward_langevin: ") + e.what());
  }
  return 0;
}

int sdp_net_set_split(sdp_net* net, int ways) {
  if (!net || ways < 0 || ways > SDP_MAX_SPLIT) return fail("sdp_net_set_split: ways must be 0 (default) .. 4");
  net->split = ways;
  return 0;
}

int sdp_net_profile_enable(sdp_net* net, int enable) {
  if (!net) return fail("sdp_net_profile_enable: null net");
  net->profile = enable != 0;
  return 0;
}

// Synchronise on the recorded events and aggregate them per conv class.  Writes up to
// `cap` rows of "class\tlaunches\ttotal_ms\tflops_per_launch\tbytes_per_launch\n" into buf (NUL-terminated)
// and releases the events.  Returns 0; *n_launches receives the number of launches read.
int sdp_net_profile_read(sdp_net* net, char* buf, size_t cap, int* n_launches) {
  if (!net || !buf || cap == 0) return fail("sdp_net_profile_read: bad argument");
  struct Agg { int n = 0; double ms = 0, flops = 0, bytes = 0; };
  std::map<std::string, Agg> agg;
  try {
    for (auto& r : net->prof) {
      chk(hipEventSynchronize(r.b), "hipEventSynchronize");
      float ms = 0.f;
      chk(hipEventElapsedTime(&ms, r.a, r.b), "hipEventElapsedTime");
      Agg& g = agg[r.cls];
      g.n += 1;
      g.ms += ms;
      g.flops = r.flops;
      g.bytes = r.bytes;
      net->ev_pool.push_back(r.a);
      net->ev_pool.push_back(r.b);
    }
  } catch (const std::exception& e) {
    return fail(std::string("sdp_net_profile_read: ") + e.what());
  }
  if (n_launches) *n_launches = (int)net->prof.size();
  net->prof.clear();
  std::string out;
  for (auto& kv : agg)
    out += kv.first + "\t" + std::to_string(kv.second.n) + "\t" + std::to_string(kv.second.ms) + "\t" +
           std::to_string(kv.second.flops) + "\t" + std::to_string(kv.second.bytes) + "\n";
  std::strncpy(buf, out.c_str(), cap - 1);
  buf[cap - 1] = 0;
  return 0;
}

int sdp_net_destroy(sdp_net* net) {
  delete net;
  return 0;
}

int sdp_langevin_step(float* x, const float* grad, const float* ref, const int32_t* mask, const float* noise,
                      uint64_t seed, uint64_t offset, float step_size, float noise_scale, float grad_ref, int nan_to_num,
                      int B, int C, int HW, float* lik_out, uint32_t* absmax_bits, void* stream) {
  if (!x || !grad || !ref || !mask || B <= 0 || C <= 0 || HW <= 0) return fail("sdp_langevin_step: bad argument");
  if (HW % 4) return fail("sdp_langevin_step: H*W must be a multiple of 4");
  hipError_t e = langevin_step(x, grad, ref, mask, noise, seed, offset, step_size, noise_scale, grad_ref, nan_to_num, B,
                               C, HW, lik_out, absmax_bits, reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? 0 : fail(std::string("sdp_langevin_step: ") + hipGetErrorString(e));
}

int sdp_axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask, const float* ref, float b,
                  int n, void* stream) {
  if (!x || n <= 0 || (g && !lik) || (!g && (!mask || !ref))) return fail("sdp_axpy_step: bad argument");
  hipError_t e = axpy_step(x, g, a, lik, mask, ref, b, (size_t)n, reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? 0 : fail(std::string("sdp_axpy_step: ") + hipGetErrorString(e));
}

}  // extern "C"
