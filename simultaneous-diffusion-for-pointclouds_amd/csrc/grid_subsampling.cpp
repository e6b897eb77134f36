// Voxel-grid subsampling of a point cloud on the HOST (the reference's only native code,
// LiDARGen/datasets/cpp_wrappers/cpp_subsampling): SURVEY §8(f)-3, used by the scene-completion
// dataset (datasets/kitti360_im_SceneCompletion.py:18-36, grid_size 0.05).  It is a CPU data-prep
// step ahead of the GPU range-image projection, so it stays host C++.
//
//   method 0 "barycenters"  grid_subsampling.cpp:46-102      per voxel: mean point, mean features,
//                                                           majority label per label column
//   method 1 "lidar"        grid_subsampling_lidar.cpp:46-120 per voxel: the point whose grid
//                                                           coordinates are best power-of-2 aligned
//
// Exactness.  The result order is the iteration order of a std::unordered_map keyed by the voxel
// index, filled in point order: the reference returns its cells in that order, so this file keeps
// the same container, the same key arithmetic (float corner / float divisions / size_t index)
// and the same first-touch insertion sequence, which makes the output bit-identical to the
// reference built with the same C++ library (oracle/_ref, tests/test_grid_subsampling_cpu.py).
// Majority labels break ties by the iteration order of the per-voxel label histogram
// (std::max_element keeps the first maximum), as the reference does.
//
// The lidar variant reads the alignment coordinates of point i from the two floats BEFORE its
// feature row (`(begin + i*fdim)[-2]`, `[-1]`: the last two features of point i-1).  For i = 0
// the reference reads two floats in front of the feature buffer (the allocator's size word: for
// any buffer below 16 GiB both floats truncate to int 0); here that read is defined as (0, 0).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/sdp.h"

int sdp_fail(const std::string& m);

namespace {

struct P3 {
  float x, y, z;
};

struct Voxel {
  int count = 0;
  int best = -1;                                   // lidar: alignment level of the kept point
  P3 sum{0.f, 0.f, 0.f};                           // barycenter: running sum; lidar: the kept point
  std::vector<float> feat;                         // [fdim]
  std::vector<std::unordered_map<int, int>> hist;  // [ldim] label -> votes
};

// alignment level of the (truncated) grid coordinates: the largest m in 1..16 such that both are
// non-multiples of every 2^k, k <= m (stops at the first k where either is a multiple)
int alignment(float gx, float gy) {
  const int ix = (int)gx, iy = (int)gy;
  int best = 0;
  for (int m = 1; m < 17; ++m) {
    const int p = (int)std::pow(2, m);
    if ((ix % p) && (iy % p)) best = m;
    else break;
  }
  return best;
}

}  // namespace

extern "C" int sdp_grid_subsample(const float* points, int64_t n, const float* features, int fdim,
                                  const int32_t* classes, int ldim, float sample_dl, int method, float* out_points,
                                  float* out_features, int32_t* out_classes, int64_t* out_n) {
  if (!points || n < 1 || !out_points || !out_n || (method != 0 && method != 1) || !(sample_dl > 0.f) ||
      (features && (fdim < 1 || !out_features)) || (classes && (ldim < 1 || !out_classes)))
    return sdp_fail("sdp_grid_subsample: bad argument");
  const bool use_f = features != nullptr, use_c = classes != nullptr;
  const size_t fd = use_f ? (size_t)fdim : 0, ld = use_c ? (size_t)ldim : 0;
  const P3* pts = reinterpret_cast<const P3*>(points);

  // grid corner and extent, in the reference's float arithmetic
  P3 lo = pts[0], hi = pts[0];
  for (int64_t i = 0; i < n; ++i) {
    const P3 p = pts[i];
    lo.x = p.x < lo.x ? p.x : lo.x; lo.y = p.y < lo.y ? p.y : lo.y; lo.z = p.z < lo.z ? p.z : lo.z;
    hi.x = p.x > hi.x ? p.x : hi.x; hi.y = p.y > hi.y ? p.y : hi.y; hi.z = p.z > hi.z ? p.z : hi.z;
  }
  const float inv = 1 / sample_dl;
  const P3 org{std::floor(lo.x * inv) * sample_dl, std::floor(lo.y * inv) * sample_dl, std::floor(lo.z * inv) * sample_dl};
  const size_t nx = (size_t)std::floor((hi.x - org.x) / sample_dl) + 1;
  const size_t ny = (size_t)std::floor((hi.y - org.y) / sample_dl) + 1;

  std::unordered_map<size_t, Voxel> cells;
  for (int64_t i = 0; i < n; ++i) {
    const P3 p = pts[i];
    const size_t key = (size_t)std::floor((p.x - org.x) / sample_dl) + nx * (size_t)std::floor((p.y - org.y) / sample_dl) +
                       nx * ny * (size_t)std::floor((p.z - org.z) / sample_dl);
    auto it = cells.find(key);
    if (it == cells.end()) {
      Voxel v;
      v.feat.assign(fd, 0.f);
      v.hist.resize(ld);
      it = cells.emplace(key, std::move(v)).first;
    }
    Voxel& v = it->second;
    const float* f = use_f ? features + (size_t)i * fd : nullptr;
    const int32_t* c = use_c ? classes + (size_t)i * ld : nullptr;
    if (method == 0) {
      ++v.count;
      v.sum.x += p.x; v.sum.y += p.y; v.sum.z += p.z;
      for (size_t k = 0; k < fd; ++k) v.feat[k] += f[k];
      for (size_t k = 0; k < ld; ++k) v.hist[k][c[k]] += 1;
      continue;
    }
    if (use_f) {      // keep the best-aligned point (strictly better replaces; the first always enters)
      const int b = i == 0 ? alignment(0.f, 0.f) : alignment(f[-2], f[-1]);
      if (v.best < b) {
        v.best = b;
        ++v.count;
        v.sum = p;
        for (size_t k = 0; k < fd; ++k) v.feat[k] = f[k];
        if (use_c) {
          v.hist.assign(ld, std::unordered_map<int, int>());
          for (size_t k = 0; k < ld; ++k) v.hist[k][c[k]] += 1;
        }
      }
    } else {          // no features: the last point of the voxel, labels voted over all of them
      ++v.count;
      v.sum = p;
      for (size_t k = 0; k < ld; ++k) v.hist[k][c[k]] += 1;
    }
  }

  int64_t m = 0;
  for (auto& kv : cells) {
    const Voxel& v = kv.second;
    P3 q = v.sum;
    if (method == 0) {
      const float s = (float)(1.0 / v.count);
      q = P3{q.x * s, q.y * s, q.z * s};
    }
    std::memcpy(out_points + 3 * m, &q, sizeof(P3));
    if (use_f) {
      const float cnt = (float)v.count;
      for (size_t k = 0; k < fd; ++k) out_features[m * fd + k] = method == 0 ? v.feat[k] / cnt : v.feat[k];
    }
    if (use_c) {
      for (size_t k = 0; k < ld; ++k) {
        auto top = v.hist[k].begin();
        for (auto h = v.hist[k].begin(); h != v.hist[k].end(); ++h)
          if (top->second < h->second) top = h;
        out_classes[m * ld + k] = top->first;
      }
    }
    ++m;
  }
  *out_n = m;
  return 0;
}
