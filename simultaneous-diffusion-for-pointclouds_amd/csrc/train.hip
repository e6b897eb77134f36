// DSM training runtime of NCSN_LiDAR_small (BASELINE config 5):
//   sdp_net_forward_train : the score-net forward of ncsnv2.py:484-518 with every tensor the
//                           backward needs kept in the caller's workspace (the "tape")
//   sdp_net_backward      : d loss / d parameters for a given d loss / d score -- loss.backward()
//                           of runners/ncsn_runner_kitti_simultaneous.py:229-232 -- written into a
//                           caller-owned gradient arena laid out like the parameter arena
//   sdp_dsm_loss          : anneal_dsm_score_estimation_with_mask (losses/dsm.py:67-119)
//   sdp_adam_ema_step     : optimizer.step() of torch.optim.Adam + EMAHelper.update (ema.py:16-21)
//
// The forward mirrors net.hip's fused plan (InstanceNorm++ statistics in conv epilogues, its
// affine + ELU in the consumer's prologue, residual / upsample / CRP sums as epilogues) but
// keeps its tensors.  The backward walks the graph in reverse with
//   data gradients  : conv_mfma_kernel on dy with flipped/transposed weights (conv_bwd.hip),
//                     fusing elu' and residual gradients into its epilogue,
//   weight gradients: conv_wgrad_kernel (wgrad.hip, MFMA with LDS transpose reads),
//   the rest        : train_aux.hip (IN++ backward, pooling / upsampling adjoints, biases).
// Workspace = forward tape + backward buffers, bump-allocated in a fixed order; a dry run of
// the same code computes its size (sdp_net_train_workspace_size).
#include <cmath>
#include <set>
#include <string>

#include "net_internal.h"

namespace sdp {

// an NHWC activation / gradient tensor of the tape: float32, or bf16 elements when the plan's h16 is set
// (p is then reinterpreted by the kernels: every launch below passes h16 along)
struct T4 {
  float* p;
  int H, W, C;
};

struct TrainPlan {
  sdp_net* net = nullptr;
  int B = 0, H = 0, W = 0, C = 0;
  hipStream_t st = nullptr;
  bool dry = true;
  // the bf16 tape (bf16 mode, sdp_net_set_tape): every activation and output gradient is stored once in
  // bf16 -- half the bytes of every conv's patch DMA and epilogue, of the weight gradient's two operand
  // streams and of the memory-bound adjoints; parameters, the gradient arena, statistics and the head's
  // scores stay float32
  bool h16 = false;
  char* base = nullptr;
  size_t cap = 0, used = 0;
  std::map<std::string, T4> saved;
  std::map<std::string, float*> fl;   // saved per-norm tables: "<key>#ss", "<key>#nst"
  std::map<std::string, uint8_t*> idxs;  // saved maxpool argmax indices
  float* stats = nullptr;
  float* mvs = nullptr;               // inpp_finalize scratch
  float* xin = nullptr;               // copy of the forward input [B,2,H,W]
  int64_t* lab = nullptr;             // copy of the labels
  // backward scratch
  float *wpart = nullptr, *bpart = nullptr, *spart = nullptr, *coef = nullptr, *ppart = nullptr, *epart = nullptr;
  size_t wpart_n = 0;
  float* grads = nullptr;
  // gradient completion: the parameters whose gradient each producer finishes, in backward order
  // (grad_order, recorded by every run, dry or not); with bucket events, events[i] is recorded on
  // the stream once the finished parameters cover the arena prefix [0, bucket_end[i])
  std::vector<std::string> grad_order;
  int n_buckets = 0, next_bucket = 0;
  const size_t* bucket_end = nullptr;
  hipEvent_t const* bucket_ev = nullptr;
  size_t done_prefix = 0;             // floats of the arena prefix whose gradients are final
  std::set<std::string> done_keys;    // parameters whose gradients are final
  size_t layout_pos = 0;              // net->layout entries [0, layout_pos) are all in done_keys
  size_t fwd_bytes = 0;
  size_t ws_need = 0;                 // forward + backward bytes (dry run), 0 = unknown

  // ------------------------------------------------------------------ allocation
  float* takeb(size_t nbytes) {
    const size_t bytes = (nbytes + 255) / 256 * 256;
    float* p = dry ? nullptr : reinterpret_cast<float*>(base + used);
    used += bytes;
    if (!dry && used > cap) throw std::runtime_error("training workspace too small");
    return p;
  }
  float* take(size_t nfloats) { return takeb(nfloats * 4); }
  T4 mk(int h, int w, int c) { return T4{takeb((size_t)B * h * w * c * (h16 ? 2 : 4)), h, w, c}; }
  T4 like(const T4& t) { return mk(t.H, t.W, t.C); }
  size_t n(const T4& t) const { return (size_t)B * t.H * t.W * t.C; }
  void ok(hipError_t e, const std::string& what) {
    if (e != hipSuccess) throw std::runtime_error(what + ": " + hipGetErrorString(e));
  }
  const float* P(const std::string& k) const { return net->P(k); }
  float* G(const std::string& k) const { return dry ? nullptr : net->grad_of(grads, k); }
  const T4& S(const std::string& k) const {
    auto it = saved.find(k);
    if (it == saved.end()) throw std::runtime_error("tape: missing " + k);
    return it->second;
  }
  float* F(const std::string& k) const {
    auto it = fl.find(k);
    if (it == fl.end()) throw std::runtime_error("tape: missing " + k);
    return it->second;
  }
  int ks_of(const std::string& wkey) const { return (int)net->host.at(wkey + ".weight").shape[2]; }
  // the gradients of `keys` are final once the launches enqueued so far have run.  The final prefix
  // advances only over layout entries that are ALL finished, in arena order: a parameter finished
  // out of layout order (e.g. a key-ordered fallback layout) never lets a bucket event fire over a
  // gradient that is still being written.  Invariant the bucket reducer relies on
  // (sdp/gradreduce.py): no launch writes a parameter's gradient range after finished() named it.
  void finished(std::initializer_list<std::string> keys) {
    for (const auto& k : keys) {
      grad_order.push_back(k);
      done_keys.insert(k);
    }
    if (dry) return;
    const auto& lay = net->layout;
    while (layout_pos < lay.size() && done_keys.count(lay[layout_pos].key)) {
      done_prefix = std::max(done_prefix, lay[layout_pos].offset + (lay[layout_pos].numel + 63) / 64 * 64);
      ++layout_pos;
    }
    while (next_bucket < n_buckets && done_prefix >= bucket_end[next_bucket])
      ok(hipEventRecord(bucket_ev[next_bucket++], st), "hipEventRecord (gradient bucket)");
  }

  // ------------------------------------------------------------------ forward pieces
  struct Opt {
    int pro = PRO_NONE;
    const float* ss = nullptr;
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
  void conv(const T4& in, const std::string& wkey, const T4& out, const Opt& o) {
    const auto& hp = net->host.at(wkey + ".weight");
    if ((int)hp.shape[1] != in.C || (int)hp.shape[0] != out.C) throw std::runtime_error("conv shape mismatch " + wkey);
    if (dry) return;
    ConvArgs a{};
    a.in = in.p;
    a.wf = net->mode == MODE_F32 ? reinterpret_cast<const uint4*>(P(wkey + ".weight#frag")) : nullptr;
    a.wf16 = net->mode == MODE_F32 ? nullptr : reinterpret_cast<const uint4*>(P(wkey + ".weight#frag16"));
    a.bias = o.bias ? P(wkey + ".bias") : nullptr;
    a.out = out.p;
    a.res = o.res;
    a.out2 = o.out2;
    a.res2 = o.res2;
    a.up = o.up;
    a.pro_ss = o.pro == PRO_AFFINE_ELU ? o.ss : P("#ident_ss");
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
    a.io16 = h16 ? 1 : 0;
    const char* why = "conv launch";
    ok(conv_mfma(net->mode, a, (int)hp.shape[2], o.pool, st, &why), std::string(why) + " (" + wkey + ")");
  }
  // statistics of the last stats-writing conv -> (scale, shift) + backward statistics of `nkey`
  void norm(const std::string& nkey, int T, float cnt, int c) {
    float* ss = take((size_t)B * c * 2);
    float* nst = take((size_t)B * c * 4);
    fl[nkey + "#ss"] = ss;
    fl[nkey + "#nst"] = nst;
    if (dry) return;
    ok(inpp_finalize(stats, B, T, cnt, c, P(nkey + ".alpha"), P(nkey + ".gamma"), P(nkey + ".beta"), ss, st, nst, mvs),
       "inpp_finalize " + nkey);
  }
  static int tiles(const T4& t) { return t.H * t.W / 128; }

  // ResidualBlock.forward (layers.py:443-456)
  T4 resf(const std::string& k, const T4& x, bool down, int dil, int x_tiles, float x_cnt) {
    saved[k + ".x"] = x;
    norm(k + ".normalize1", x_tiles, x_cnt, x.C);
    T4 h1 = like(x);
    Opt o1;
    o1.pro = PRO_AFFINE_ELU;
    o1.ss = F(k + ".normalize1#ss");
    o1.stats = true;
    o1.dil = dil;
    conv(x, k + ".conv1", h1, o1);
    saved[k + ".h1"] = h1;
    norm(k + ".normalize2", tiles(h1), 128.f, h1.C);
    Opt o2;
    o2.pro = PRO_AFFINE_ELU;
    o2.ss = F(k + ".normalize2#ss");
    o2.stats = true;
    o2.dil = dil;
    T4 out;
    if (down && dil == 1) {   // ConvMeanPool conv2 + ConvMeanPool 1x1 shortcut (layers.py:417-420)
      T4 s = mk(x.H / 2, x.W / 2, 2 * x.C);
      Opt os;
      os.circular = false;
      os.pool = true;
      conv(x, k + ".shortcut.conv", s, os);
      out = like(s);
      o2.circular = false;
      o2.pool = true;
      o2.res = s.p;
      conv(h1, k + ".conv2.conv", out, o2);
    } else if (down) {         // dilated: no resampling, dilated shortcut (layers.py:411-415)
      T4 s = like(x);
      Opt os;
      os.dil = dil;
      conv(x, k + ".shortcut", s, os);
      out = like(x);
      o2.res = s.p;
      conv(h1, k + ".conv2", out, o2);
    } else {
      out = like(x);
      o2.res = x.p;
      conv(h1, k + ".conv2", out, o2);
    }
    return out;
  }
  // RCUBlock (layers.py:126-134)
  T4 rcuf(const std::string& k, T4 x, int nb, bool final_elu, bool final_stats) {
    for (int i = 0; i < nb; ++i) {
      const std::string c1 = k + "." + std::to_string(i + 1) + "_1_conv", c2 = k + "." + std::to_string(i + 1) + "_2_conv";
      saved[k + ".x" + std::to_string(i)] = x;
      T4 t = like(x);
      Opt a;
      a.pro = PRO_ELU;
      a.bias = false;
      conv(x, c1, t, a);
      saved[k + ".t" + std::to_string(i)] = t;
      T4 y = like(x);
      Opt b;
      b.pro = PRO_ELU;
      b.bias = false;
      b.res = x.p;
      b.epi_elu = final_elu && i == nb - 1;
      b.stats = final_stats && i == nb - 1;
      conv(t, c2, y, b);
      x = y;
    }
    saved[k + ".out"] = x;
    return x;
  }
  // CRPBlock (layers.py:76-83) on X = ELU(h)
  T4 crpf(const std::string& k, const T4& X) {
    saved[k + ".X"] = X;
    T4 p1 = like(X), path1 = like(X), x1 = like(X), p2 = like(X), x2 = like(X);
    const size_t nidx = (n(X) + 3) / 4;                // argmax bytes, in floats
    uint8_t* i1 = reinterpret_cast<uint8_t*>(take(nidx));
    uint8_t* i2 = reinterpret_cast<uint8_t*>(take(nidx));
    idxs[k + ".i1"] = i1;
    idxs[k + ".i2"] = i2;
    if (!dry) ok(maxpool5(X.p, p1.p, B, X.H, X.W, X.C, st, i1, h16), "maxpool5");
    Opt a;
    a.bias = false;
    a.out2 = x1.p;
    a.res2 = X.p;
    conv(p1, k + ".convs.0", path1, a);
    if (!dry) ok(maxpool5(path1.p, p2.p, B, X.H, X.W, X.C, st, i2, h16), "maxpool5");
    Opt b;
    b.bias = false;
    b.res = x1.p;
    conv(p2, k + ".convs.1", x2, b);
    saved[k + ".p1"] = p1;
    saved[k + ".path1"] = path1;
    saved[k + ".p2"] = p2;
    return x2;
  }
  // RefineBlock (layers.py:234-249); MSF (layers.py:179-184) fused with the CRP's input ELU
  T4 refinef(const std::string& k, const T4& a, const T4* b, int cout, int n_out, bool final_stats) {
    T4 X;
    if (!b) {
      X = rcuf(k + ".adapt_convs.0", a, 2, true, false);
    } else {
      T4 hA = rcuf(k + ".adapt_convs.0", a, 2, false, false);
      T4 hB = rcuf(k + ".adapt_convs.1", *b, 2, false, false);
      if (hA.H == hB.H) {
        T4 m0 = mk(hA.H, hA.W, cout);
        conv(hA, k + ".msf.convs.0", m0, Opt{});
        X = like(m0);
        Opt o;
        o.res = m0.p;
        o.epi_elu = true;
        conv(hB, k + ".msf.convs.1", X, o);
      } else {
        T4 m1 = mk(hB.H, hB.W, cout);
        conv(hB, k + ".msf.convs.1", m1, Opt{});
        X = mk(hA.H, hA.W, cout);
        Opt o;
        o.up = m1.p;
        o.epi_elu = true;
        conv(hA, k + ".msf.convs.0", X, o);
      }
      saved[k + ".msf.X"] = X;
    }
    T4 x2 = crpf(k + ".crp", X);
    return rcuf(k + ".output_convs", x2, n_out, false, final_stats);
  }

  void forward(const float* x, const int64_t* labels, float* out) {
    used = 0;
    saved.clear();
    fl.clear();
    idxs.clear();
    xin = take((size_t)B * 2 * H * W);
    lab = reinterpret_cast<int64_t*>(take((size_t)B * 2));
    if (!dry) {
      ok(hipMemcpyAsync(xin, x, (size_t)B * 2 * H * W * 4, hipMemcpyDeviceToDevice, st), "copy x");
      ok(hipMemcpyAsync(lab, labels, (size_t)B * 8, hipMemcpyDeviceToDevice, st), "copy labels");
    }
    stats = take((size_t)B * (H * W / 64) * 2 * C * 2);
    mvs = take((size_t)B * 2 * C * 4);
    T4 x0 = mk(H, W, C);
    if (!dry)
      ok(begin_conv(xin, P("begin_conv.weight"), P("begin_conv.bias"), x0.p, stats, B, H, W, st, net->mode, h16),
         "begin_conv");
    T4 l1 = resf("res1.0", x0, false, 1, H * W / 64, 64.f);
    l1 = resf("res1.1", l1, false, 1, tiles(l1), 128.f);
    T4 l2 = resf("res2.0", l1, true, 1, tiles(l1), 128.f);
    l2 = resf("res2.1", l2, false, 1, tiles(l1), 32.f);
    T4 l3 = resf("res3.0", l2, true, 2, tiles(l2), 128.f);
    l3 = resf("res3.1", l3, false, 2, tiles(l3), 128.f);
    T4 l4 = resf("res4.0", l3, true, 4, tiles(l3), 128.f);
    l4 = resf("res4.1", l4, false, 4, tiles(l4), 128.f);
    T4 r1 = refinef("refine1", l4, nullptr, 2 * C, 1, false);
    T4 r2 = refinef("refine2", l3, &r1, 2 * C, 1, false);
    T4 r3 = refinef("refine3", l2, &r2, C, 1, false);
    T4 o = refinef("refine4", l1, &r3, C, 3, true);
    norm("normalizer", tiles(o), 128.f, C);
    if (!dry)
      ok(end_conv(o.p, F("normalizer#ss"), P("end_conv.weight"), P("end_conv.bias"), P("sigmas"), lab, out, B, H, W, C,
                  st, nullptr, net->mode, h16),
         "end_conv");
    fwd_bytes = used;
  }

  // ------------------------------------------------------------------ backward pieces
  void wgrad(const std::string& k, const T4& in, int pro, const float* ss, const T4& dy, int dil, bool circular, int ks,
             bool with_bias) {
    if (!dry) wgrad_launch(k, in, pro, ss, dy, dil, circular, ks, with_bias);
    if (with_bias) finished({k + ".weight", k + ".bias"});
    else finished({k + ".weight"});
  }
  void wgrad_launch(const std::string& k, const T4& in, int pro, const float* ss, const T4& dy, int dil, bool circular,
                    int ks, bool with_bias) {
    WgradArgs a{};
    a.in = in.p;
    a.pro_ss = pro == PRO_AFFINE_ELU ? ss : P("#ident_ss");
    a.ss_bstride = pro == PRO_AFFINE_ELU ? 2 * in.C : 0;
    a.pro_mode = pro;
    a.dy = dy.p;
    a.part = wpart;
    a.part_floats = wpart_n;
    a.bpart = bpart;
    a.B = B;
    a.H = in.H;
    a.W = in.W;
    a.Cin = in.C;
    a.Cout = dy.C;
    a.dil = dil;
    a.circular = circular ? 1 : 0;
    const char* why = "wgrad launch";
    ok(conv_wgrad(net->mode, a, ks, G(k + ".weight"), with_bias ? G(k + ".bias") : nullptr, 0, st, &why, h16),
       std::string(why) + " (" + k + ")");
  }
  void dgrad(const std::string& k, const T4& dy, const T4& dx, int dil, bool circular, int ks, int dact,
             const float* aux, const float* epi_ss, const float* res) {
    if (dry) return;
    ConvArgs a{};
    a.in = dy.p;
    a.wf16 = reinterpret_cast<const uint4*>(P(k + ".weight#dfrag16"));   // coalesced 16x16 order (train_aux.hip pack_slot16)
    a.out = dx.p;
    a.res = res;
    a.pro_ss = P("#ident_ss");
    a.B = B;
    a.H = dy.H;
    a.W = dy.W;
    a.Cin = dy.C;
    a.Cout = dx.C;
    a.dil = dil;
    a.circular = circular ? 1 : 0;
    a.pro_mode = PRO_NONE;
    a.aux = aux;
    a.epi_ss = epi_ss;
    a.dact = dact;
    a.io16 = h16 ? 1 : 0;
    const char* why = "dgrad launch";
    ok(conv_dgrad(net->mode, a, ks, st, &why), std::string(why) + " (" + k + ")");
  }
  void inpp_back(const std::string& nkey, const T4& g, const T4& h, const float* r1, const float* r2, const T4& out) {
    if (!dry)
      ok(inpp_backward(g.p, h.p, F(nkey + "#nst"), P(nkey + ".alpha"), P(nkey + ".gamma"), B, h.H * h.W, h.C, spart,
                       coef, ppart, G(nkey + ".alpha"), G(nkey + ".gamma"), G(nkey + ".beta"), r1, r2, out.p, st, h16),
         "inpp_backward " + nkey);
    finished({nkey + ".alpha", nkey + ".gamma", nkey + ".beta"});
  }

  T4 resb(const std::string& k, const T4& dout, bool down, int dil, const float* extra) {
    const T4 &x = S(k + ".x"), &h1 = S(k + ".h1");
    float *ss1 = F(k + ".normalize1#ss"), *ss2 = F(k + ".normalize2#ss");
    T4 g2 = like(h1);
    const float* sg;
    if (down && dil == 1) {
      T4 dyf = mk(x.H, x.W, dout.C);
      if (!dry) ok(unpool(dout.p, dyf.p, B, x.H, x.W, dout.C, st, h16), "unpool");
      wgrad(k + ".conv2.conv", h1, PRO_AFFINE_ELU, ss2, dyf, 1, false, 3, true);
      dgrad(k + ".conv2.conv", dyf, g2, 1, false, 3, 3, h1.p, ss2, nullptr);
      wgrad(k + ".shortcut.conv", x, PRO_NONE, nullptr, dyf, 1, false, 1, true);
      T4 sgb = like(x);
      dgrad(k + ".shortcut.conv", dyf, sgb, 1, false, 1, 0, nullptr, nullptr, nullptr);
      sg = sgb.p;
    } else {
      wgrad(k + ".conv2", h1, PRO_AFFINE_ELU, ss2, dout, dil, true, 3, true);
      dgrad(k + ".conv2", dout, g2, dil, true, 3, 3, h1.p, ss2, nullptr);
      if (down) {
        wgrad(k + ".shortcut", x, PRO_NONE, nullptr, dout, dil, true, 3, true);
        T4 sgb = like(x);
        dgrad(k + ".shortcut", dout, sgb, dil, true, 3, 0, nullptr, nullptr, nullptr);
        sg = sgb.p;
      } else {
        sg = dout.p;
      }
    }
    T4 dh1 = like(h1);
    inpp_back(k + ".normalize2", g2, h1, nullptr, nullptr, dh1);
    wgrad(k + ".conv1", x, PRO_AFFINE_ELU, ss1, dh1, dil, true, 3, true);
    T4 g1 = like(x);
    dgrad(k + ".conv1", dh1, g1, dil, true, 3, 3, x.p, ss1, nullptr);
    T4 dx = like(x);
    inpp_back(k + ".normalize1", g1, x, sg, extra, dx);
    return dx;
  }
  T4 rcub(const std::string& k, const T4& dxn, int nb, bool final_elu) {
    T4 d = dxn;
    if (final_elu) {
      T4 d2 = like(dxn);
      if (!dry) ok(elu_backward_post(dxn.p, S(k + ".out").p, nullptr, d2.p, n(d2), st, h16), "elu_backward");
      d = d2;
    }
    for (int i = nb - 1; i >= 0; --i) {
      const std::string c1 = k + "." + std::to_string(i + 1) + "_1_conv", c2 = k + "." + std::to_string(i + 1) + "_2_conv";
      const T4 &xi = S(k + ".x" + std::to_string(i)), &ti = S(k + ".t" + std::to_string(i));
      wgrad(c2, ti, PRO_ELU, nullptr, d, 1, true, 3, false);
      T4 dt = like(ti);
      dgrad(c2, d, dt, 1, true, 3, 1, ti.p, nullptr, nullptr);
      wgrad(c1, xi, PRO_ELU, nullptr, dt, 1, true, 3, false);
      T4 dn = like(xi);
      dgrad(c1, dt, dn, 1, true, 3, 1, xi.p, nullptr, d.p);
      d = dn;
    }
    return d;
  }
  T4 crpb(const std::string& k, const T4& dx2) {
    const T4 &X = S(k + ".X"), &p1 = S(k + ".p1"), &p2 = S(k + ".p2");
    wgrad(k + ".convs.1", p2, PRO_NONE, nullptr, dx2, 1, true, 3, false);
    T4 dp2 = like(X);
    dgrad(k + ".convs.1", dx2, dp2, 1, true, 3, 0, nullptr, nullptr, nullptr);
    T4 dpath1 = like(X);
    if (!dry)
      ok(maxpool5_backward(idxs.at(k + ".i2"), dp2.p, dx2.p, dpath1.p, B, X.H, X.W, X.C, st, h16), "maxpool5_backward");
    wgrad(k + ".convs.0", p1, PRO_NONE, nullptr, dpath1, 1, true, 3, false);
    T4 dp1 = like(X);
    dgrad(k + ".convs.0", dpath1, dp1, 1, true, 3, 0, nullptr, nullptr, nullptr);
    T4 dX = like(X);
    if (!dry) ok(maxpool5_backward(idxs.at(k + ".i1"), dp1.p, dx2.p, dX.p, B, X.H, X.W, X.C, st, h16), "maxpool5_backward");
    return dX;
  }
  // returns the gradients of the refine block's inputs (second one empty for refine1)
  std::pair<T4, T4> refineb(const std::string& k, const T4& dout, bool two, int n_out) {
    T4 dx2 = rcub(k + ".output_convs", dout, n_out, false);
    T4 dX = crpb(k + ".crp", dx2);
    if (!two) return {rcub(k + ".adapt_convs.0", dX, 2, true), T4{}};
    const T4 &X = S(k + ".msf.X"), &hA = S(k + ".adapt_convs.0.out"), &hB = S(k + ".adapt_convs.1.out");
    T4 dm = like(X);
    if (!dry) ok(elu_backward_post(dX.p, X.p, nullptr, dm.p, n(dm), st, h16), "elu_backward");
    T4 dm1 = dm;
    if (hB.H != hA.H) {
      dm1 = mk(hB.H, hB.W, X.C);
      if (!dry) ok(upsample_backward(dm.p, dm1.p, B, X.H, X.W, X.C, 0, st, h16), "upsample_backward");
    }
    wgrad(k + ".msf.convs.0", hA, PRO_NONE, nullptr, dm, 1, true, 3, true);
    T4 dhA = like(hA);
    dgrad(k + ".msf.convs.0", dm, dhA, 1, true, 3, 0, nullptr, nullptr, nullptr);
    wgrad(k + ".msf.convs.1", hB, PRO_NONE, nullptr, dm1, 1, true, 3, true);
    T4 dhB = like(hB);
    dgrad(k + ".msf.convs.1", dm1, dhB, 1, true, 3, 0, nullptr, nullptr, nullptr);
    return {rcub(k + ".adapt_convs.0", dhA, 2, false), rcub(k + ".adapt_convs.1", dhB, 2, false)};
  }

  void backward(const float* dscore, float* grad_arena) {
    used = fwd_bytes;
    grads = grad_arena;
    grad_order.clear();
    next_bucket = 0;
    done_prefix = 0;
    done_keys.clear();
    layout_pos = 0;
    // scratch (upper bounds over every layer of the network)
    wpart_n = (size_t)(WGRAD_TARGET_BLOCKS + 64) * 9 * 128 * 32;   // >= splits x 9 x Cin x Cout for every conv
    wpart = take(wpart_n);
    spart = take((size_t)B * (H * W / 512) * 256 * 2);   // inpp_backward: 512-pixel groups (train_aux.hip INPP_GRP)
    coef = take((size_t)B * 256 * 4);
    bpart = take(1024 * 256);
    ppart = take((size_t)B * 256 * 3);
    epart = take(head_wgrad_part_floats(B, H, W));
    if (!dry) ok(hipMemsetAsync(grads, 0, net->arena_floats * 4, st), "zero grads");

    // head: IN++ -> ELU -> end_conv -> / sigma
    const T4& o = S("refine4.output_convs.out");
    T4 g = like(o);
    if (!dry)
      ok(end_conv_backward(dscore, P("sigmas"), lab, P("end_conv.weight"), o.p, F("normalizer#ss"), g.p, epart,
                           G("end_conv.weight"), G("end_conv.bias"), B, H, W, st, h16),
         "end_conv_backward");
    finished({"end_conv.weight", "end_conv.bias"});
    T4 d_o = like(o);
    inpp_back("normalizer", g, o, nullptr, nullptr, d_o);
    auto r4 = refineb("refine4", d_o, true, 3);      // -> d L1 (part), d ref3
    auto r3 = refineb("refine3", r4.second, true, 1);  // -> d L2 (part), d ref2
    auto r2 = refineb("refine2", r3.second, true, 1);  // -> d L3 (part), d ref1
    auto r1 = refineb("refine1", r2.second, false, 1); // -> d L4
    T4 d = resb("res4.1", r1.first, false, 4, nullptr);
    d = resb("res4.0", d, true, 4, r2.first.p);        // + d L3 from refine2
    d = resb("res3.1", d, false, 2, nullptr);
    d = resb("res3.0", d, true, 2, r3.first.p);        // + d L2 from refine3
    d = resb("res2.1", d, false, 1, nullptr);
    d = resb("res2.0", d, true, 1, r4.first.p);        // + d L1 from refine4
    d = resb("res1.1", d, false, 1, nullptr);
    d = resb("res1.0", d, false, 1, nullptr);
    if (!dry)
      ok(begin_conv_wgrad(xin, d.p, epart, G("begin_conv.weight"), G("begin_conv.bias"), B, H, W, st, h16),
         "begin_conv_wgrad");
    finished({"begin_conv.weight", "begin_conv.bias"});
    done_prefix = net->arena_floats;   // every gradient is final: the remaining buckets complete here
    finished({});
  }
};

void destroy_plan(TrainPlan* p) { delete p; }

// The parameters in the order the backward finishes their gradients (a dry run of the plan: host
// bookkeeping only).  sdp_net_finalize lays the parameter arena out in this order, so the arena
// prefix whose gradients are final grows monotonically during sdp_net_backward -- the gradient
// buckets of sdp_net_backward_buckets are contiguous ranges that complete one after another.
std::vector<std::string> grad_completion_order(sdp_net* net) {
  TrainPlan p;
  p.net = net;
  p.B = 1;
  p.H = net->d.H;
  p.W = net->d.W;
  p.C = net->d.ngf;
  p.dry = true;
  p.forward(nullptr, nullptr, nullptr);
  p.backward(nullptr, nullptr);
  return p.grad_order;
}

static TrainPlan* plan_for(sdp_net* net, int B) {
  const bool h16 = net->mode == MODE_BF16 && net->tape16;
  if (net->plan && net->plan->B == B && net->plan->h16 == h16) return net->plan;
  if (net->plan) destroy_plan(net->plan);
  TrainPlan* p = new TrainPlan();
  p->net = net;
  p->B = B;
  p->h16 = h16;
  p->H = net->d.H;
  p->W = net->d.W;
  p->C = net->d.ngf;
  net->plan = p;
  return p;
}

static size_t train_ws_bytes(sdp_net* net, int B) {
  TrainPlan* p = plan_for(net, B);
  if (p->ws_need) return p->ws_need;
  p->dry = true;
  p->forward(nullptr, nullptr, nullptr);
  p->backward(nullptr, nullptr);
  p->ws_need = p->used;
  p->saved.clear();
  p->fl.clear();
  return p->ws_need;
}

}  // namespace sdp

using namespace sdp;

static int tfail(const std::string& m) { return sdp_fail(m); }

static void enable_training(sdp_net* net, hipStream_t st) {
  if (net->mode != MODE_F32X3 && net->mode != MODE_BF16) throw std::runtime_error("training needs fp32x3 or bf16");
  if (!net->train_packs) {
    net->train_packs = true;
    net->repack(st);
  }
}

extern "C" {

int sdp_net_set_tape(sdp_net* net, int bf16) {
  if (!net || bf16 < 0 || bf16 > 1) return tfail("sdp_net_set_tape: bad argument");
  net->tape16 = bf16 != 0;
  return 0;
}

int sdp_net_train_workspace_size(sdp_net* net, int B, size_t* bytes) {
  if (!net || !bytes || B <= 0 || !net->finalized) return tfail("sdp_net_train_workspace_size: bad argument");
  try {
    *bytes = train_ws_bytes(net, B);
  } catch (const std::exception& e) {
    return tfail(std::string("sdp_net_train_workspace_size: ") + e.what());
  }
  return 0;
}

int sdp_net_forward_train(sdp_net* net, const float* x, const int64_t* labels, float* out, int B, void* ws,
                          size_t ws_bytes, void* stream) {
  if (!net || !x || !labels || !out || !ws || B <= 0) return tfail("sdp_net_forward_train: bad argument");
  if (!net->finalized) return tfail("sdp_net_forward_train: call sdp_net_finalize first");
  try {
    const size_t need = train_ws_bytes(net, B);
    if (ws_bytes < need) return tfail("sdp_net_forward_train: workspace too small");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    enable_training(net, st);
    TrainPlan* p = plan_for(net, B);
    p->dry = false;
    p->st = st;
    p->base = reinterpret_cast<char*>(ws);
    p->cap = ws_bytes;
    p->forward(x, labels, out);
  } catch (const std::exception& e) {
    return tfail(std::string("sdp_net_forward_train: ") + e.what());
  }
  return 0;
}

int sdp_net_backward(sdp_net* net, const float* dscore, int B, void* ws, size_t ws_bytes, float* grads, void* stream) {
  if (!net || !dscore || !ws || !grads || B <= 0) return tfail("sdp_net_backward: bad argument");
  TrainPlan* p = net->plan;
  if (!p || p->dry || p->B != B || p->base != ws || p->saved.empty())
    return tfail("sdp_net_backward: no tape -- call sdp_net_forward_train with this workspace and batch first");
  try {
    p->st = reinterpret_cast<hipStream_t>(stream);
    p->cap = ws_bytes;
    p->backward(dscore, grads);
  } catch (const std::exception& e) {
    return tfail(std::string("sdp_net_backward: ") + e.what());
  }
  return 0;
}

int sdp_net_backward_buckets(sdp_net* net, const float* dscore, int B, void* ws, size_t ws_bytes, float* grads,
                             int n_buckets, const size_t* bucket_end, void* const* events, void* stream) {
  if (!net || !dscore || !ws || !grads || B <= 0 || n_buckets < 0 || (n_buckets && (!bucket_end || !events)))
    return tfail("sdp_net_backward_buckets: bad argument");
  for (int i = 0; i < n_buckets; ++i)
    if (!events[i] || (i && bucket_end[i] <= bucket_end[i - 1]) || bucket_end[i] > net->arena_floats)
      return tfail("sdp_net_backward_buckets: bucket ends must increase within the arena, events non-null");
  TrainPlan* p = net->plan;
  if (!p || p->dry || p->B != B || p->base != ws || p->saved.empty())
    return tfail("sdp_net_backward_buckets: no tape -- call sdp_net_forward_train with this workspace and batch first");
  try {
    p->st = reinterpret_cast<hipStream_t>(stream);
    p->cap = ws_bytes;
    p->n_buckets = n_buckets;
    p->bucket_end = bucket_end;
    p->bucket_ev = reinterpret_cast<hipEvent_t const*>(events);
    p->backward(dscore, grads);
    p->n_buckets = 0;
  } catch (const std::exception& e) {
    p->n_buckets = 0;
    return tfail(std::string("sdp_net_backward_buckets: ") + e.what());
  }
  return 0;
}

int sdp_dsm_loss(const float* score, const float* noise, const float* mask, const float* used_sigma, int B, int n_img,
                 float anneal_power, float* dscore, float* loss, float* loss_per, float* part, void* stream) {
  if (!score || !noise || !mask || !used_sigma || !dscore || !loss || !part || B <= 0 || n_img <= 0)
    return tfail("sdp_dsm_loss: bad argument");
  hipError_t e = dsm_loss(score, noise, mask, used_sigma, B, n_img, anneal_power, dscore, loss, loss_per, part,
                          reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? 0 : tfail(std::string("sdp_dsm_loss: ") + hipGetErrorString(e));
}

int sdp_adam_ema_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* ema_shadow, size_t n,
                      double lr, double beta1, double beta2, double eps, int step, double ema_mu, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || n == 0 || step < 1) return tfail("sdp_adam_ema_step: bad argument");
  return sdp_optim_ema_step(SDP_OPTIM_ADAM, params, grads, exp_avg, exp_avg_sq, nullptr, ema_shadow, n, lr, beta1, beta2,
                            eps, 0.0, step, ema_mu, stream);
}

int sdp_optim_ema_step(int kind, float* params, const float* grads, float* state0, float* state1, float* state2,
                       float* ema_shadow, size_t n, double lr, double beta1, double beta2, double eps,
                       double weight_decay, int step, double ema_mu, void* stream) {
  if (!params || !grads || !state0 || n == 0 || step < 1 || kind < SDP_OPTIM_ADAM || kind > SDP_OPTIM_SGD ||
      (kind == SDP_OPTIM_ADAM && !state1))
    return tfail("sdp_optim_ema_step: bad argument");
  OptimHyper h{};
  h.b1 = (float)beta1;
  h.b2 = (float)beta2;
  h.eps = (float)eps;
  h.weight_decay = (float)weight_decay;
  h.mu = (float)ema_mu;
  h.omb1 = (float)(1.0 - beta1);
  h.omb2 = (float)(1.0 - beta2);
  h.ommu = (float)(1.0 - ema_mu);
  h.first = step == 1;
  h.step_size = (float)lr;
  h.bc2_sqrt = 1.f;
  if (kind == SDP_OPTIM_ADAM) {   // torch: bias corrections in Python float (double), then lr / bc1, bc2 ** 0.5
    const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
    h.step_size = (float)(lr / bc1);
    h.bc2_sqrt = (float)std::sqrt(bc2);
  }
  hipError_t e = optim_ema(kind, params, grads, state0, kind == SDP_OPTIM_ADAM ? state1 : nullptr,
                           kind == SDP_OPTIM_ADAM ? state2 : nullptr, ema_shadow, n, h,
                           reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? 0 : tfail(std::string("sdp_optim_ema_step: ") + hipGetErrorString(e));
}

}  // extern "C"
