// C ABI of the consistency merge: host-side geometry (KITTISampling.py:29-102) and launch.
#include <cmath>
#include <string>

#include "../../include/sdp.h"
#include "merge.h"

int sdp_fail(const std::string& m);

// reference evaluation order: no FMA contraction in this file (HIP __fmul_rn is a plain `*`)
#pragma clang fp contract(off)

namespace sdp {

static long floordiv(long a, long b) {  // Python // on ints
  long q = a / b, r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? q - 1 : q;
}

}  // namespace sdp

using namespace sdp;

extern "C" {

int sdp_merge_workspace_size(int n_src, int n_out, int H, int W, size_t* bytes) {
  if (!bytes || n_src <= 0 || n_out <= 0 || H <= 0 || W <= 0) return sdp_fail("sdp_merge_workspace_size: bad argument");
  *bytes = merge_ws_bytes(n_src, n_src, n_out, H, W);   // any megabatch size
  return 0;
}

int sdp_merge_workspace_bytes(int n_src, int aB, int n_out, int H, int W, size_t* bytes) {
  if (!bytes || n_src <= 0 || aB <= 0 || aB > n_src || n_out <= 0 || H <= 0 || W <= 0)
    return sdp_fail("sdp_merge_workspace_bytes: bad argument");
  *bytes = merge_ws_bytes(n_src, aB, n_out, H, W);
  return 0;
}

int sdp_consistency_merge_ev(float* x_all, int n_src, int aB, int o_begin, int n_out, int H, int W, const double* toWorld,
                             const double* fromWorld, const float* origins, const uint8_t* exist, const uint8_t* sky,
                             const int32_t* refmask, const sdp_merge_params* prm, const uint32_t* absmax_bits,
                             float* new_images, void* ws, size_t ws_bytes, void* stream, void* absmax_event) {
  if (!x_all || !prm || !exist || !sky || !refmask || !absmax_bits || !ws || aB <= 0 || n_out <= 0 || H <= 0 || W <= 0)
    return sdp_fail("sdp_consistency_merge: bad argument");
  if (prm->variant == SDP_MERGE_POSES && (!toWorld || !fromWorld))
    return sdp_fail("sdp_consistency_merge: POSES variant needs toWorld/fromWorld");
  if (prm->variant == SDP_MERGE_ORIGINS && !origins) return sdp_fail("sdp_consistency_merge: ORIGINS needs origins");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  MergeArgs a{};
  MergeGeom& g = a.g;
  g.H = H;
  g.W = W;
  const double deg = M_PI / 180.0;
  g.hA = (360.0 * deg) / W;
  g.vA = (28.0 * deg) / H;
  g.hMin = (double)floordiv((long)W * -180, 360) * g.hA + g.hA / 2;
  g.big = (int)((50L * H) / 28);
  g.bigMin = (double)floordiv(g.big, -2) * g.vA + g.vA / 2;
  g.vMin = (double)floordiv((long)H * -25, 28) * g.vA + g.vA / 2;
  a.x = x_all;
  a.xout = x_all;
  a.toWorld = toWorld;
  a.fromWorld = fromWorld;
  a.origins = origins;
  a.exist = exist;
  a.sky = sky;
  a.refmask = refmask;
  a.absmax = absmax_bits;
  a.n_src = n_src;
  a.aB = aB;
  a.o_begin = o_begin;
  a.n_out = n_out;
  a.variant = prm->variant;
  a.setting = prm->setting;
  a.smod = prm->sigma > 1.0f ? prm->sigma : 1.0f;
  a.allowance = prm->allowance;
  a.cc = prm->cc;
  // log2(tensor(0.2)+1)/6*sigmaMod in float32 (KITTISampling.py:272-274)
  const float l2 = (float)std::log2((double)(0.2f + 1.0f));
  a.min_code = (l2 / 6.0f) * a.smod;
  const char* why = "merge";
  hipError_t e = consistency_merge(a, ws, ws_bytes, new_images, st, &why, reinterpret_cast<hipEvent_t>(absmax_event));
  if (e != hipSuccess) return sdp_fail(std::string("sdp_consistency_merge: ") + why + " " + hipGetErrorString(e));
  return 0;
}

int sdp_consistency_merge(float* x_all, int n_src, int aB, int o_begin, int n_out, int H, int W, const double* toWorld,
                          const double* fromWorld, const float* origins, const uint8_t* exist, const uint8_t* sky,
                          const int32_t* refmask, const sdp_merge_params* prm, const uint32_t* absmax_bits,
                          float* new_images, void* ws, size_t ws_bytes, void* stream) {
  return sdp_consistency_merge_ev(x_all, n_src, aB, o_begin, n_out, H, W, toWorld, fromWorld, origins, exist, sky, refmask,
                                  prm, absmax_bits, new_images, ws, ws_bytes, stream, nullptr);
}

}  // extern "C"
