// sdp_net handle internals, shared by the forward runtime (net.hip) and the training
// runtime (train.hip).
#pragma once
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sdp.h"
#include "kernels.h"

namespace sdp {

struct HostParam {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

struct ParamEntry {
  std::string key;
  size_t offset, numel;   // floats within the parameter arena
};

inline void chk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int SDP_MAX_SPLIT = 4;   // part-batch streams of one forward (net.hip forward_split)

struct TrainPlan;   // train.hip
void destroy_plan(TrainPlan* p);

}  // namespace sdp

struct sdp_net {
  struct ProfRec {
    std::string cls;
    double flops;
    double bytes = 0;               // algorithmic HBM bytes of the launch (memory-bound kernels)
    hipEvent_t a, b;
  };
  sdp_net_desc d;
  bool profile = false;
  std::vector<ProfRec> prof;        // events of the forwards since the last read
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, sdp::HostParam> host;
  // device tensors: parameters (pointers into `arena`), "sigmas", "#ident_ss" and the packed
  // conv weights "<key>#frag16" (forward, bf16 modes) or "<key>#frag" (forward, exact fp32) and
  // "<key>#dfrag16" (data gradient in 16x16 fragment order, training only)
  std::map<std::string, void*> dev;
  std::vector<sdp::ParamEntry> layout;
  float* arena = nullptr;           // every learnable parameter, fp32, `layout` order
  size_t arena_floats = 0;
  bool arena_owned = false;         // false once the caller bound its own arena
  bool finalized = false;
  bool train_packs = false;         // keep the dgrad packings current in repack()
  bool tape16 = true;               // bf16 mode: the training tape in bf16 (sdp_net_set_tape)
  int mode = sdp::MODE_F32X3;
  sdp::TrainPlan* plan = nullptr;   // tape of the last sdp_net_forward_train
  int split = 0;                     // part-batch forwards (0: the default, 2)
  hipStream_t aux_stream[sdp::SDP_MAX_SPLIT - 1] = {};   // part-batch forwards 1.. (net.hip forward_split)
  hipEvent_t ev_fork = nullptr, ev_join[sdp::SDP_MAX_SPLIT - 1] = {};

  ~sdp_net() {
    release();
    for (auto& s : aux_stream)
      if (s) (void)hipStreamDestroy(s);
    for (auto& e : ev_join)
      if (e) (void)hipEventDestroy(e);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    for (auto& r : prof) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    for (auto e : ev_pool) (void)hipEventDestroy(e);
  }
  void release() {
    for (auto& kv : dev) {
      const bool in_arena = arena && kv.second >= (void*)arena && kv.second < (void*)(arena + arena_floats);
      if (!in_arena) (void)hipFree(kv.second);
    }
    dev.clear();
    if (pack_dev) (void)hipFree(pack_dev);
    pack_dev = nullptr;
    pack_dev_n = 0;
    pack_host.clear();
    if (arena_owned && arena) (void)hipFree(arena);
    arena = nullptr;
    arena_owned = false;
    if (plan) sdp::destroy_plan(plan);
    plan = nullptr;
  }
  hipEvent_t event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("hipEventCreate");
    return e;
  }
  const float* P(const std::string& k) const {
    auto it = dev.find(k);
    if (it == dev.end()) throw std::runtime_error("missing parameter " + k);
    return reinterpret_cast<const float*>(it->second);
  }
  float* grad_of(float* grads, const std::string& k) const {
    for (auto& e : layout)
      if (e.key == k) return grads + e.offset;
    throw std::runtime_error("no parameter " + k);
  }
  bool is_conv_w(const std::string& k) const {
    auto it = host.find(k);
    return it != host.end() && it->second.shape.size() == 4 && k != "begin_conv.weight" && k != "end_conv.weight";
  }
  // (re)build the fragment-ordered weights from the fp32 parameters on the device: one
  // launch over every conv (a descriptor table, re-uploaded when a parameter moves)
  std::vector<sdp::PackDesc> pack_host;
  sdp::PackDesc* pack_dev = nullptr;
  size_t pack_dev_n = 0, pack_total = 0;
  void repack(hipStream_t st) {
    std::vector<sdp::PackDesc> d;
    size_t total = 0;
    for (auto& kv : host) {
      if (!is_conv_w(kv.first)) continue;
      const auto& s = kv.second.shape;
      // packings: 0 = forward "#frag" (32x32 fragment order: the exact-fp32 forward), 3 = the forward in
      // 16x16 fragment order "#frag16" (bf16 modes), 4 = the data gradient in 16x16 fragment order
      // "#dfrag16" (training: bf16 modes); (1 was the data gradient in 32x32 order -- read in 16-B pieces
      // at a 64-B lane stride, and in bf16 mode only the hi half of each 32 B: replaced in round 6 --
      // 2 the Winograd packing, removed with its kernel)
      for (int dg = 0; dg < 5; ++dg) {
        if (dg == 0 && mode != sdp::MODE_F32) continue;
        if (dg == 1 || dg == 2) continue;
        if (dg == 3 && mode == sdp::MODE_F32) continue;
        if (dg == 4 && (!train_packs || mode == sdp::MODE_F32)) continue;
        const std::string fk = kv.first + (dg == 0 ? "#frag" : dg == 3 ? "#frag16" : "#dfrag16");
        const int nt = (int)(s[2] * s[3]);
        const size_t n = (size_t)s[0] * s[1] * nt;
        if (!dev.count(fk)) {
          void* p = nullptr;
          sdp::chk(hipMalloc(&p, n * 4), "hipMalloc");
          dev[fk] = p;
        }
        d.push_back(sdp::PackDesc{P(kv.first), reinterpret_cast<uint32_t*>(dev[fk]), (int)s[0], (int)s[1], nt, dg,
                                  total});
        total += n;
      }
    }
    const bool same = d.size() == pack_host.size() &&
                      std::equal(d.begin(), d.end(), pack_host.begin(), [](const sdp::PackDesc& x, const sdp::PackDesc& y) {
                        return x.w == y.w && x.out == y.out && x.begin == y.begin && x.dgrad == y.dgrad;
                      });
    if (!same) {
      if (pack_dev_n < d.size()) {
        if (pack_dev) sdp::chk(hipFree(pack_dev), "hipFree");
        sdp::chk(hipMalloc(&pack_dev, d.size() * sizeof(sdp::PackDesc)), "hipMalloc");
        pack_dev_n = d.size();
      }
      pack_host = d;
      sdp::chk(hipMemcpyAsync(pack_dev, pack_host.data(), d.size() * sizeof(sdp::PackDesc), hipMemcpyHostToDevice, st),
               "hipMemcpyAsync");
      pack_total = total;
    }
    sdp::chk(sdp::pack_weights_multi(pack_dev, (int)pack_host.size(), pack_total, mode, st), "pack_weights_multi");
  }
};

int sdp_fail(const std::string& m);

namespace sdp {
std::vector<std::string> grad_completion_order(sdp_net* net);   // train.hip
}
