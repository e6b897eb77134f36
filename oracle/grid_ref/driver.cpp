// TEST INFRASTRUCTURE ONLY: a ctypes entry point over the REFERENCE's own grid subsampling, compiled
// from its sources where they lie (oracle/build_ref.sh -> oracle/_ref/).  Built twice: with
// -DREF_LIDAR against grid_subsampling_lidar.cpp, without it against grid_subsampling.cpp (the two
// define different SampledData classes, so they cannot share one library).  Mirrors what
// wrapper.cpp:200-285 does around the call: vectors in, vectors out.
#include <cstdint>
#include <cstring>
#include <vector>

#ifdef REF_LIDAR
#include "grid_subsampling/grid_subsampling_lidar.h"
#define REF_FN grid_subsampling_lidar
#else
#include "grid_subsampling/grid_subsampling.h"
#define REF_FN grid_subsampling
#endif

extern "C" int64_t ref_grid_subsample(const float* points, int64_t n, const float* features, int fdim,
                                      const int32_t* classes, int ldim, float dl, float* out_points,
                                      float* out_features, int32_t* out_classes) {
  std::vector<PointXYZ> op((const PointXYZ*)points, (const PointXYZ*)points + n), sp;
  std::vector<float> of, sf;
  std::vector<int> oc, sc;
  if (features) of.assign(features, features + n * fdim);
  if (classes) oc.assign(classes, classes + n * ldim);
  REF_FN(op, sp, of, sf, oc, sc, dl, 0);
  std::memcpy(out_points, sp.data(), sp.size() * sizeof(PointXYZ));
  if (features) std::memcpy(out_features, sf.data(), sf.size() * sizeof(float));
  if (classes) std::memcpy(out_classes, sc.data(), sc.size() * sizeof(int));
  return (int64_t)sp.size();
}
