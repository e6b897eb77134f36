// KITTI-360 view rendering on the GPU: the per-view work of the three
// datasets' __getitem__ around point_cloud_to_range_image, so a scan goes from its .bin
// float32 [N][4] to the returned range images without the CPU DataLoader:
//   view_transform_kernel : pointVals = fromWorld @ (toWorld @ [x y z 1]^T) in float64 and
//                           the scan re-assembled as [x y z intensity] (kitti360_im_8Batch.py:
//                           146-190, kitti360_im_AllForOne.py:144-190); with no matrices it is
//                           the float32 -> float64 widening the projection sees for the goal
//                           scan and the densification input (numpy promotes them on the
//                           origin subtraction, lidar_utils.py:159);
//   view_gather_kernel    : scanPoints[index[index >= 0]] after index[:, :W/4] = -2, the
//                           row-major compaction of kitti360_im_simultenous_densification.py:
//                           186-203 (order kept: it decides the projection's tie rule);
//   view_finalize_kernel  : the post-processing of kitti360_im_8Batch.py:221-291 (and the
//                           AllForOne / densification variants): sky -> mask, log2 depth code,
//                           clip, optional roll, intensity cut at 1, the 3-row sky shift, the
//                           densification column mask, and the logical_not of the returned masks.
// float64 throughout, no contraction (-ffp-contract=off), as the reference's numpy.
#include <string>

#include "../../include/sdp.h"
#include "common.h"
#include "kernels.h"

int sdp_fail(const std::string& m);

namespace sdp {

constexpr double VIEW_MAX_RANGE = 2057.701;   // kitti360_im_8Batch.py:196

struct Mat4 {
  double m[16];   // row-major
};

// r = M v (numpy matmul of a 4x4 with a column; products summed left to right)
SDP_DEV void mat4_apply(const Mat4& M, const double v[4], double r[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r[i] = ((M.m[4 * i] * v[0] + M.m[4 * i + 1] * v[1]) + M.m[4 * i + 2] * v[2]) + M.m[4 * i + 3] * v[3];
}

__global__ __launch_bounds__(256) void view_transform_kernel(const float4* __restrict__ pts, long long n, Mat4 m1,
                                                             Mat4 m2, int nmat, double4* __restrict__ out) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 p = pts[i];
    double v[4] = {(double)p.x, (double)p.y, (double)p.z, 1.0}, t[4];
    if (nmat >= 1) {
      mat4_apply(m1, v, t);
      if (nmat >= 2) mat4_apply(m2, t, v);
      else for (int k = 0; k < 4; ++k) v[k] = t[k];
    }
    out[i] = make_double4(v[0], v[1], v[2], (double)p.w);
  }
}

// one workgroup of 1024 threads; thread t owns the contiguous pixel run [t*per, (t+1)*per)
__global__ __launch_bounds__(1024) void view_gather_kernel(const int64_t* __restrict__ index, int H, int W,
                                                           int blank_cols, const float4* __restrict__ pts,
                                                           double4* __restrict__ out, int* __restrict__ count) {
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int HW = H * W, per = (HW + 1023) / 1024;
  const int p0 = min(tid * per, HW), p1 = min(p0 + per, HW);
  auto valid = [&](int p) { return (p % W) >= blank_cols && index[p] >= 0; };
  int c = 0;
  for (int p = p0; p < p1; ++p) c += valid(p) ? 1 : 0;
  // exclusive scan: wave prefix by shuffles, then the 16 wave totals
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int base = 0, total = 0;
  for (int k = 0; k < 16; ++k) {
    base += k < wv ? wsum[k] : 0;
    total += wsum[k];
  }
  int o = base + inc - c;
  for (int p = p0; p < p1; ++p)
    if (valid(p)) {
      const float4 q = pts[index[p]];
      out[o++] = make_double4((double)q.x, (double)q.y, (double)q.z, (double)q.w);
    }
  if (tid == 0) *count = total;
}

struct FinalizeArgs {
  const double *depth, *inten, *goal_depth, *goal_inten;   // [H][W] projection outputs
  const uint8_t *obf, *sky;
  double *real, *goal;                                      // [C][H][W]
  uint8_t *notmask, *notsky;                                // [C][H][W], [H][W]
  int H, W, C, roll, variant, first_view;
};

SDP_DEV double depth_code(double d) {   // where(d >= maxRange, 0, d) + 0.0001 -> log2(. + 1) / 6 -> clip
  const double t = (d >= VIEW_MAX_RANGE ? 0.0 : d) + 0.0001;
  const double v = log2(t + 1.0) / 6.0;
  return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
}

SDP_DEV double inten_code(double x) {   // where(x >= 1, 0, x) + 0.0001 -> clip(0, 1)
  const double v = (x >= 1.0 ? 0.0 : x) + 0.0001;
  return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
}

__global__ __launch_bounds__(256) void view_finalize_kernel(FinalizeArgs a) {
  const int HW = a.H * a.W;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= HW) return;
  const int r = i / a.W, c = i % a.W;
  // np.roll(x, k, axis=1): out[:, c] = x[:, (c - k) mod W]; roll < 0 = no roll
  const int sc = a.roll >= 0 ? ((c - a.roll) % a.W + a.W) % a.W : c;
  const int s = r * a.W + sc;
  const double d = a.depth[s];
  bool m = a.obf[s] != 0 || d >= VIEW_MAX_RANGE;
  // the intensity test runs on the UNROLLED intensity against the rolled mask (8Batch:272,
  // AllForOne:276-279, densification:257-258)
  if (a.C == 2 && a.inten[i] >= 1.0) m = true;
  if (a.variant == SDP_VIEW_DENSIFICATION && a.first_view) m = c < a.W / 4;   // densification:274-282
  // sky[1:] = sky[:-1] three times: row r takes row max(r - 3, 0)
  const int sr = r >= 3 ? r - 3 : 0;
  a.notsky[i] = a.sky[sr * a.W + sc] ? 0 : 1;
  a.real[i] = depth_code(d);
  if (a.goal) a.goal[i] = depth_code(a.goal_depth[i]);
  a.notmask[i] = m ? 0 : 1;
  if (a.C == 2) {
    if (a.variant == SDP_VIEW_COMPLETION) {   // SceneCompletion: (real, real) and (mask, ones)
      a.real[HW + i] = a.real[i];
      a.notmask[HW + i] = 0;
    } else {
      a.real[HW + i] = inten_code(a.inten[s]);
      a.notmask[HW + i] = m ? 0 : 1;
    }
    if (a.goal) a.goal[HW + i] = inten_code(a.goal_inten[i]);
  }
}

}  // namespace sdp

extern "C" {

int sdp_view_transform(const float* points, int64_t n, const double* m1, const double* m2, double* out, void* stream) {
  if (n < 0 || (n > 0 && (!points || !out)) || (!m1 && m2)) return sdp_fail("sdp_view_transform: bad argument");
  if (n == 0) return 0;
  sdp::Mat4 A{}, B{};
  for (int k = 0; k < 16; ++k) {
    A.m[k] = m1 ? m1[k] : 0.0;
    B.m[k] = m2 ? m2[k] : 0.0;
  }
  const int nmat = m1 ? (m2 ? 2 : 1) : 0;
  const long long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(sdp::view_transform_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float4*>(points), (long long)n, A,
                     B, nmat, reinterpret_cast<double4*>(out));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : sdp_fail(std::string("sdp_view_transform: ") + hipGetErrorString(e));
}

int sdp_view_gather(const int64_t* index, int H, int W, int blank_cols, const float* points, double* out, int* count,
                    void* stream) {
  if (!index || !points || !out || !count || H < 1 || W < 1 || blank_cols < 0)
    return sdp_fail("sdp_view_gather: bad argument");
  hipLaunchKernelGGL(sdp::view_gather_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), index, H,
                     W, blank_cols, reinterpret_cast<const float4*>(points), reinterpret_cast<double4*>(out), count);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : sdp_fail(std::string("sdp_view_gather: ") + hipGetErrorString(e));
}

int sdp_view_finalize(const double* depth, const double* intensity, const uint8_t* obfuscation, const uint8_t* sky,
                      const double* goal_depth, const double* goal_intensity, int H, int W, int channels, int roll,
                      int variant, int first_view, double* real, uint8_t* notmask, uint8_t* notsky, double* goal,
                      void* stream) {
  const bool has_goal = goal != nullptr;
  if (!depth || !obfuscation || !sky || !real || !notmask || !notsky || H < 1 || W < 1 ||
      (has_goal && !goal_depth) || (variant != SDP_VIEW_COMPLETION && !has_goal) ||
      (channels != 1 && channels != 2) || (channels == 2 && (!intensity || (has_goal && !goal_intensity))) ||
      roll >= W || variant < SDP_VIEW_8BATCH || variant > SDP_VIEW_COMPLETION)
    return sdp_fail("sdp_view_finalize: bad argument");
  sdp::FinalizeArgs a{depth, intensity, goal_depth, goal_intensity, obfuscation, sky, real, goal, notmask, notsky,
                      H, W, channels, roll, variant, first_view};
  hipLaunchKernelGGL(sdp::view_finalize_kernel, dim3((H * W + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : sdp_fail(std::string("sdp_view_finalize: ") + hipGetErrorString(e));
}

}  // extern "C"
