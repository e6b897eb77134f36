// Point cloud -> range image (the data front end): point_cloud_to_range_image
// of LiDARGen/datasets/lidar_utils.py:54-347, which the KITTI-360 datasets call for every
// view (datasets/kitti360_im_8Batch.py:199-212).  The reference sorts all points by depth on
// the CPU (argsort + np.unique) to keep the nearest point per pixel; here:
//   proj_depth_kernel : per point, float64 spherical bin (np.round = half-even = rint,
//                       clamped, row/col 0 excluded as inGrid does) and a 64-bit atomicMin of
//                       the depth's bit pattern (monotonic for depth >= 0) per pixel;
//   proj_index_kernel : per point again, atomicMin of the point index among the points whose
//                       depth equals the pixel minimum (the reference's quicksort leaves such
//                       ties unspecified; the lowest index is kept);
//   proj_pixel_kernel : per pixel, the winner's depth / xy / intensity / index into the
//                       flipped (both axes) output, empty pixels = maxRange / 0 / -1, and a
//                       nearest depth of exactly 0 left empty (tempDepth != 0, L254-261);
//   proj_sky_kernel   : the row-sequential sky / obfuscation scan (L283-306), one block per
//                       image, one thread per column, the 3-column sum through LDS.
// All geometry in float64, as the reference's numpy.
#include <string>

#include "../../include/sdp.h"
#include "common.h"
#include "kernels.h"

int sdp_fail(const std::string& m);

namespace sdp {

constexpr double PROJ_MAX_RANGE = 2057.701;

struct ProjGeom {
  int H, W;
  double hA, vA, hMin, vMin;
  double ox, oy, oz;
};

SDP_DEV bool proj_point(const double* __restrict__ pts, int stride, int i, const ProjGeom& g, int* pix, double* depth,
                        double* xy) {
  const double* p = pts + (size_t)i * stride;
  const double rx = p[0] - g.ox, ry = p[1] - g.oy, rz = p[2] - g.oz;
  const double xy2 = rx * rx + ry * ry;
  *depth = sqrt(xy2 + rz * rz);
  const double h = atan2(ry, rx);
  *xy = sqrt(xy2);
  const double v = atan2(rz, *xy);
  double cf = rint((h - g.hMin) / g.hA), rf = rint((v - g.vMin) / g.vA);
  cf = fmin(fmax(cf, 0.0), (double)(g.W - 1));
  rf = fmin(fmax(rf, 0.0), (double)(g.H - 1));
  const int col = (int)cf, row = (int)rf;
  *pix = row * g.W + col;
  return col > 0 && row > 0;   // inGrid (L196): after the clamp only row/col 0 can fail
}

__global__ void proj_depth_kernel(const double* __restrict__ pts, int stride, int N, ProjGeom g,
                                  unsigned long long* __restrict__ dbest) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    int pix;
    double d, xy;
    if (proj_point(pts, stride, i, g, &pix, &d, &xy)) atomicMin(&dbest[pix], (unsigned long long)__double_as_longlong(d));
  }
}

__global__ void proj_index_kernel(const double* __restrict__ pts, int stride, int N, ProjGeom g,
                                  const unsigned long long* __restrict__ dbest, unsigned int* __restrict__ ibest) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    int pix;
    double d, xy;
    if (proj_point(pts, stride, i, g, &pix, &d, &xy) && (unsigned long long)__double_as_longlong(d) == dbest[pix])
      atomicMin(&ibest[pix], (unsigned int)i);
  }
}

__global__ void proj_pixel_kernel(const double* __restrict__ pts, int stride, int has_int, ProjGeom g,
                                  const unsigned int* __restrict__ ibest, double* __restrict__ depth,
                                  double* __restrict__ inten, double* __restrict__ xy_out, int64_t* __restrict__ index) {
  const int n = g.H * g.W;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int o = n - 1 - q;   // np.flip of both axes
    double d = PROJ_MAX_RANGE, xy = PROJ_MAX_RANGE, it = 0.0;
    int64_t id = -1;
    const unsigned int w = ibest[q];
    if (w != 0xffffffffu) {
      int pix;
      double dd, xx;
      proj_point(pts, stride, (int)w, g, &pix, &dd, &xx);
      if (dd != 0.0) {
        d = dd;
        xy = xx;
        id = w;
        if (has_int) it = pts[(size_t)w * stride + 3];
      }
    }
    depth[o] = d;
    xy_out[o] = xy;
    if (inten) inten[o] = it;
    if (index) index[o] = id;
  }
}

// one block of W threads (W <= 1024): rows are sequential, columns parallel.  Each thread
// slides a (row-1, row, row+1) window down its column; the rows are fetched RC at a time into
// registers (one memory latency per RC rows instead of per row), and the 3-column sum goes
// through a double-buffered LDS row, so one barrier per row suffices.
constexpr int SKY_RC = 16;
__global__ __launch_bounds__(1024) void proj_sky_kernel(const double* __restrict__ xy, int H, int W,
                                                        uint8_t* __restrict__ obf, uint8_t* __restrict__ sky) {
  __shared__ int e[2][1024 + 2];
  const int c = threadIdx.x;
  const bool act = c < W;
  double md = PROJ_MAX_RANGE;
  bool prev_sky = true;                 // rows 0 and 1 are sky (L285-287)
  if (act) {
    obf[c] = 0;
    obf[W + c] = 0;
  }
  if (c < 2) {
    e[c][0] = 0;
    e[c][W + 1] = 0;
  }
  double xm1 = act ? xy[(size_t)W + c] : 0.0, x0 = act ? xy[(size_t)2 * W + c] : 0.0;   // rows 1, 2
  for (int r0 = 2; r0 < H - 1; r0 += SKY_RC) {
    double nx[SKY_RC];                  // rows r0+1 .. r0+RC
#pragma unroll
    for (int k = 0; k < SKY_RC; ++k) {
      const int rr = r0 + 1 + k;
      nx[k] = (act && rr < H) ? xy[(size_t)rr * W + c] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < SKY_RC; ++k) {
      const int row = r0 + k;
      if (row < H - 1) {                // uniform; no break, so the loop unrolls and nx stays in VGPRs
        const double xp1 = nx[k];
        int* eb = e[row & 1];
        if (act) {
          obf[(size_t)row * W + c] = x0 > md + 5 ? 1 : 0;
          eb[c + 1] = (x0 != md) + (xm1 != md) + (xp1 != md);
        }
        __syncthreads();
        if (act) {
          const int s3 = eb[c] + eb[c + 1] + eb[c + 2];
          const bool cur = s3 <= 1 && prev_sky;
          prev_sky = cur;
          if (!cur) md = fmin(x0, md);
        }
        xm1 = x0;
        x0 = xp1;
      }
    }
  }
  if (act) {
    obf[(size_t)(H - 1) * W + c] = x0 > md + 5 ? 1 : 0;   // x0 = row H-1 here
    for (int row = 0; row < H; ++row) sky[(size_t)row * W + c] = 0;   // skyMask[:] = False (L304)
  }
}

// the z-buffer words: nearest-depth bits and winner index start at all-ones
__global__ __launch_bounds__(256) void proj_init_kernel(unsigned long long* __restrict__ dbest,
                                                        unsigned int* __restrict__ ibest, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    dbest[i] = ~0ull;
    ibest[i] = ~0u;
  }
}

size_t range_project_ws_bytes(int H, int W) { return (size_t)H * W * (8 + 4 + 8); }

hipError_t range_project(const double* pts, int N, int stride, int has_int, double ox, double oy, double oz, int H,
                         int W, double* depth, double* inten, uint8_t* obf, uint8_t* sky, int64_t* index, void* ws,
                         hipStream_t st) {
  if (W > 1024 || H < 3 || stride < 3 || (has_int && stride < 4)) return hipErrorInvalidValue;
  ProjGeom g;
  g.H = H;
  g.W = W;
  const double deg = 3.14159265358979323846 / 180.0;   // math.radians(x) = x * (pi / 180)
  g.hA = (360.0 * deg) / W;
  g.vA = (28.0 * deg) / H;
  g.hMin = (double)(W / 2 * -1 - (W % 2 ? 1 : 0)) * g.hA + g.hA / 2;   // colCount // (-2)
  g.vMin = (3.0 - 28.0) * deg;           // math.radians(verticalPositive - verticalScope)
  g.ox = ox;
  g.oy = oy;
  g.oz = oz;
  const size_t n = (size_t)H * W;
  unsigned long long* dbest = reinterpret_cast<unsigned long long*>(ws);
  unsigned int* ibest = reinterpret_cast<unsigned int*>(dbest + n);
  double* xy = reinterpret_cast<double*>(reinterpret_cast<char*>(ibest) + ((n * 4 + 7) / 8) * 8);
  hipLaunchKernelGGL(proj_init_kernel, dim3((int)std::min<size_t>((n + 255) / 256, 1024)), dim3(256), 0, st, dbest,
                     ibest, n);
  const int grid = (int)std::min<size_t>(((size_t)N + 255) / 256, 4096);
  if (N > 0) {
    hipLaunchKernelGGL(proj_depth_kernel, dim3(grid), dim3(256), 0, st, pts, stride, N, g, dbest);
    hipLaunchKernelGGL(proj_index_kernel, dim3(grid), dim3(256), 0, st, pts, stride, N, g, dbest, ibest);
  }
  hipLaunchKernelGGL(proj_pixel_kernel, dim3((int)((n + 255) / 256)), dim3(256), 0, st, pts, stride, has_int, g, ibest,
                     depth, inten, xy, index);
  if (obf)   // callers that only need the depth / intensity (a goal scan) skip the sequential scan
    hipLaunchKernelGGL(proj_sky_kernel, dim3(1), dim3(((W + 63) / 64) * 64), 0, st, xy, H, W, obf, sky);
  return hipGetLastError();
}

}  // namespace sdp

extern "C" {

int sdp_range_project_workspace_size(int H, int W, size_t* bytes) {
  if (H < 3 || W < 1 || W > 1024 || !bytes) return sdp_fail("sdp_range_project_workspace_size: bad argument");
  *bytes = sdp::range_project_ws_bytes(H, W);
  return 0;
}

int sdp_range_project(const double* points, int N, int stride, int has_intensity, const double* origin, int H, int W,
                      double* depth, double* intensity, uint8_t* obfuscation, uint8_t* sky, int64_t* index, void* ws,
                      size_t ws_bytes, void* stream) {
  if ((!points && N > 0) || N < 0 || !origin || !depth || (!obfuscation) != (!sky) || !ws)
    return sdp_fail("sdp_range_project: bad argument");
  if (ws_bytes < sdp::range_project_ws_bytes(H, W)) return sdp_fail("sdp_range_project: workspace too small");
  hipError_t e = sdp::range_project(points, N, stride, has_intensity, origin[0], origin[1], origin[2], H, W, depth,
                                    intensity, obfuscation, sky, index, ws, reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? 0 : sdp_fail(std::string("sdp_range_project: ") + hipGetErrorString(e));
}

}  // extern "C"
