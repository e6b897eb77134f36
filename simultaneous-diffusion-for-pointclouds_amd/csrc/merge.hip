// Cross-view reprojection / consistency merge (gfx950).
//
// Restates KITTISampling.py:160-490 (pose matrices) and models/__init__.py:263-579 (origin
// offsets) without the reference's per-view argsort / stable sorts / unique_consecutive /
// sparse->dense: every (output view, source point) pair of a megabatch is projected once
// (float64, as the reference's numpy-derived angles promote) and scattered with atomics
// into a [114 x W] "big" grid per output view:
//     cnt (u32), sum of log-depth codes (f64), sum of intensities (f64),
//     nearest code (u64 atomicMin on the f64 bits; codes are >= 0 so the order is the
//     unsigned order), then the lowest source index among the nearest (second pass).
// Large megabatches scatter into several replicas of the grids (by source view) that a
// reduce pass folds, so no cell serialises one atomic per source view.
// A resolve pass turns a cell into the reference's controlled average (mean depth unless
// it exceeds the nearest depth + allowance), applies the negative-depth flip/roll and crop
// to the output view, and an apply pass adds cc * (-mask*(x - new)) on unknown pixels
// unless tooHigh.  Tie rule: equal nearest codes keep the lowest source index (the
// reference's unstable argsort leaves it unspecified).
#include "merge.h"

// reference evaluation order: no FMA contraction in this file (HIP __fmul_rn is a plain `*`)
#pragma clang fp contract(off)

namespace sdp {

// ---------------------------------------------------------------- K0: source points -> world
__global__ __launch_bounds__(256) void merge_world_kernel(MergeArgs a) {
  const int HW = a.g.H * a.g.W;
  const size_t n = (size_t)a.n_src * HW;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int v = i / HW, p = i % HW;
    const int r = p / a.g.W, c = p % a.g.W;
    const float x0 = a.x[(size_t)v * 2 * HW + p];
    // realDistance = (2^(|x|*6/smod) - 1) * (+-1), float32 (KITTISampling.py:164-166)
    const float e = __fdiv_rn(__fmul_rn(fabsf(x0), 6.0f), a.smod);
    float rd = __fsub_rn(exp2f(e), 1.0f);
    if (x0 < 0.f) rd = -rd;
    const double cz = a.trig[c], sz = a.trig[a.g.W + c];
    const double ce = a.trig[2 * a.g.W + r], se = a.trig[2 * a.g.W + a.g.H + r];
    const double rdd = (double)rd;
    double px = __dmul_rn(__dmul_rn(rdd, cz), ce);
    double py = __dmul_rn(__dmul_rn(rdd, sz), ce);
    double pz = __dmul_rn(rdd, se);
    const int vl = v % a.aB;
    double flag = a.exist[(size_t)vl * HW + p] ? 1.0 : 0.0;
    double4 w;
    if (a.variant == 0) {
      const double* T = a.toWorld + (size_t)v * 16;
      w.x = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[0], px), __dmul_rn(T[1], py)), __dmul_rn(T[2], pz)), T[3]);
      w.y = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[4], px), __dmul_rn(T[5], py)), __dmul_rn(T[6], pz)), T[7]);
      w.z = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[8], px), __dmul_rn(T[9], py)), __dmul_rn(T[10], pz)), T[11]);
    } else {
      w.x = __dadd_rn(px, (double)a.origins[vl * 3 + 0]);
      w.y = __dadd_rn(py, (double)a.origins[vl * 3 + 1]);
      w.z = __dadd_rn(pz, (double)a.origins[vl * 3 + 2]);
      if (!a.sky[(size_t)v * HW + p]) flag = 0.0;   // source sky gate (models/__init__.py:356-359)
    }
    w.w = flag;
    a.world[i] = w;
  }
}

struct Proj {
  int cell;     // -1 if not valid
  double code;  // log2(d+1)/6*smod
};

// project world point w into output view o (global index); noinline so K1 and K2 agree bitwise
__device__ __noinline__ Proj project(const MergeArgs& a, double4 w, int o) {
  Proj pr;
  pr.cell = -1;
  pr.code = 0.0;
  double qx, qy, qz;
  if (a.variant == 0) {
    const double* F = a.fromWorld + (size_t)o * 16;
    qx = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[0], w.x), __dmul_rn(F[1], w.y)), __dmul_rn(F[2], w.z)), F[3]);
    qy = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[4], w.x), __dmul_rn(F[5], w.y)), __dmul_rn(F[6], w.z)), F[7]);
    qz = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[8], w.x), __dmul_rn(F[9], w.y)), __dmul_rn(F[10], w.z)), F[11]);
  } else {
    const int ol = o % a.aB;
    qx = __dsub_rn(w.x, (double)a.origins[ol * 3 + 0]);
    qy = __dsub_rn(w.y, (double)a.origins[ol * 3 + 1]);
    qz = __dsub_rn(w.z, (double)a.origins[ol * 3 + 2]);
  }
  const double xy = __dadd_rn(__dmul_rn(qx, qx), __dmul_rn(qy, qy));
  const double dist = sqrt(__dadd_rn(xy, __dmul_rn(qz, qz)));
  const double code = __dmul_rn(__ddiv_rn(log2(__dadd_rn(dist, 1.0)), 6.0), (double)a.smod);
  const double h = atan2(qy, qx);
  const double e = atan2(qz, sqrt(xy));
  const double fc = rint(__ddiv_rn(__dsub_rn(h, a.g.hMin), a.g.hA));
  const double fr = rint(__ddiv_rn(__dsub_rn(e, a.g.bigMin), a.g.vA));
  const int col = a.g.W - 1 - (int)fc;
  const int row = a.g.big - 1 - (int)fr;
  bool ok = w.w != 0.0 && col > -1 && col < a.g.W && row > -1 && row < a.g.big;
  // setting 5 (kitti) / always (AllForOne): min-depth filter code > log2(1.2)/6*smod
  if (a.variant == 1 || a.setting == 5) ok = ok && code > (double)a.min_code;
  if (ok) pr.cell = row * a.g.W + col;
  pr.code = code;
  return pr;
}

// ---------------------------------------------------------------- K1: accumulate
__global__ __launch_bounds__(256) void merge_accum_kernel(MergeArgs a) {
  const int HW = a.g.H * a.g.W;
  const size_t per_out = (size_t)a.aB * HW;
  const size_t n = (size_t)a.n_out * per_out;
  const int cells = a.g.big * a.g.W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int ol = i / per_out;
    const int s = i % per_out;
    const int o = a.o_begin + ol;
    const int m0 = (o / a.aB) * a.aB;
    const int vl = s / HW, p = s % HW;
    const double4 w = a.world[(size_t)(m0 + vl) * HW + p];
    const Proj pr = project(a, w, o);
    if (pr.cell < 0) continue;
    const size_t ci = ((size_t)(vl % a.nrep) * a.n_out + ol) * cells + pr.cell;
    atomicAdd(&a.cnt[ci], 1u);
    atomicAdd(&a.sumL[ci], pr.code);
    atomicAdd(&a.sumI[ci], (double)a.x[((size_t)(m0 + vl) * 2 + 1) * HW + p]);
    atomicMin(&a.minkey[ci], (unsigned long long)__double_as_longlong(pr.code));
  }
}

// ---------------------------------------------------------------- K1b: fold the replicas
__global__ __launch_bounds__(256) void merge_reduce_kernel(MergeArgs a) {
  const size_t n = (size_t)a.n_out * a.g.big * a.g.W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t c = a.cnt[i];
    double l = a.sumL[i], in = a.sumI[i];
    unsigned long long mk = a.minkey[i];
    for (int r = 1; r < a.nrep; ++r) {
      const size_t j = (size_t)r * n + i;
      c += a.cnt[j];
      l = __dadd_rn(l, a.sumL[j]);
      in = __dadd_rn(in, a.sumI[j]);
      mk = a.minkey[j] < mk ? a.minkey[j] : mk;
    }
    a.cnt[i] = c;
    a.sumL[i] = l;
    a.sumI[i] = in;
    a.minkey[i] = mk;
  }
}

// ---------------------------------------------------------------- K2: lowest index among nearest
__global__ __launch_bounds__(256) void merge_minidx_kernel(MergeArgs a) {
  const int HW = a.g.H * a.g.W;
  const size_t per_out = (size_t)a.aB * HW;
  const size_t n = (size_t)a.n_out * per_out;
  const int cells = a.g.big * a.g.W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int ol = i / per_out;
    const int s = i % per_out;
    const int o = a.o_begin + ol;
    const int m0 = (o / a.aB) * a.aB;
    const int vl = s / HW, p = s % HW;
    const double4 w = a.world[(size_t)(m0 + vl) * HW + p];
    const Proj pr = project(a, w, o);
    if (pr.cell < 0) continue;
    const size_t ci = (size_t)ol * cells + pr.cell;
    if ((unsigned long long)__double_as_longlong(pr.code) == a.minkey[ci]) atomicMin(&a.minidx[ci], (uint32_t)s);
  }
}

// ---------------------------------------------------------------- K3: resolve cells -> new image
__global__ __launch_bounds__(256) void merge_resolve_kernel(MergeArgs a) {
  const int H = a.g.H, W = a.g.W, HW = H * W;
  const int cells = a.g.big * W;
  const size_t n = (size_t)a.n_out * HW;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int ol = i / HW, p = i % HW;
    const int r = p / W, c = p % W;
    const int o = a.o_begin + ol;
    const int m0 = (o / a.aB) * a.aB;
    const bool neg = a.x[(size_t)o * 2 * HW + p] < 0.f;
    const int brow = neg ? (H - 1 - r) : (r + a.g.big - H);
    const int bcol = neg ? ((c - W / 2) % W + W) % W : c;
    const size_t ci = (size_t)ol * cells + brow * W + bcol;
    const uint32_t nn = a.cnt[ci];
    double code = 0.0;
    float inten = 0.f;
    if (nn > 0) {
      const float scaling = (float)nn;   // float32(n + 1e-9) == n for n >= 1
      const double Abar = __ddiv_rn(a.sumL[ci], (double)scaling);
      const float Ibar = __fdiv_rn((float)a.sumI[ci], scaling);
      const bool controlled = a.variant == 0 || a.setting >= 7;
      if (controlled) {
        const double lmin = __longlong_as_double((long long)a.minkey[ci]);
        const uint32_t s = a.minidx[ci];
        const int vl = s / HW, ps = s % HW;
        const float Imin = a.x[((size_t)(m0 + vl) * 2 + 1) * HW + ps];
        const double sm = (double)a.smod;
        const double A = exp2(__dmul_rn(fabs(Abar), 6.0) / sm) - 1.0;
        const double M = exp2(__dmul_rn(fabs(lmin), 6.0) / sm) - 1.0;
        const double allow = (double)a.allowance;
        const bool cond = A > M + allow;
        inten = cond ? Imin : Ibar;
        const double D = cond ? M + allow / 5.0 : A;
        code = __dmul_rn(log2(D + 1.0) / 6.0, sm);
      } else {
        code = Abar;
        inten = Ibar;
      }
    }
    const float depth = (float)(neg ? -code : code);
    const bool m = nn > 0 && a.exist[p] && a.sky[(size_t)o * HW + p];
    if (a.newimg) {
      a.newimg[((size_t)ol * 2 + 0) * HW + p] = depth;
      a.newimg[((size_t)ol * 2 + 1) * HW + p] = inten;
    }
    a.maskimg[i] = m ? 1 : 0;
  }
}

// ---------------------------------------------------------------- K4: apply correction
__global__ __launch_bounds__(256) void merge_apply_kernel(MergeArgs a) {
  const int HW = a.g.H * a.g.W;
  const size_t n = (size_t)a.n_out * 2 * HW;
  const float mx = __uint_as_float(*a.absmax);
  const bool too_high = __fdiv_rn(__fmul_rn(mx, 6.0f), a.smod) > 50.0f;   // KITTISampling.py:162
  if (too_high) return;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int ol = i / (2 * HW);
    const int rem = i % (2 * HW);
    const int p = rem % HW;
    const int o = a.o_begin + ol;
    const size_t xi = (size_t)o * 2 * HW + rem;
    if (!a.maskimg[(size_t)ol * HW + p] || a.refmask[xi] != 0) continue;
    const float xv = a.xout[xi];
    const float nv = a.newimg[((size_t)ol * 2) * HW + rem];
    const float corr = -__fsub_rn(xv, nv);
    a.xout[xi] = __fadd_rn(xv, __fmul_rn(a.cc, corr));
  }
}

static int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 256 * 16); }

// replicas of the accumulator grids: 1 up to a 7-view megabatch, then one per 2 views, at most 8
// (measured on one MI355X, 4 output views: a 32-view megabatch costs 25.4 ms/step with one
// grid, 18.6 ms with 8 replicas, 19.1 ms with 16)
int merge_replicas(int aB) { return aB < 8 ? 1 : (aB / 2 > 8 ? 8 : aB / 2); }

size_t merge_ws_bytes(int n_src, int n_out, int H, int W) {
  const int big = (int)((25 * 2) * (long)H / 28);
  const size_t cells = (size_t)big * W;
  const int R = merge_replicas(n_src);                // aB <= n_src
  size_t b = 0;
  b += (size_t)n_src * H * W * sizeof(double4);      // world
  b += (size_t)R * n_out * cells * (4 + 8 + 8 + 8) + 4 * 256;  // cnt, sumL, sumI, minkey (replicated)
  b += (size_t)n_out * cells * 4;                    // minidx
  b += (size_t)n_out * 2 * H * W * 4;                // newimg (internal)
  b += (size_t)n_out * H * W;                        // maskimg
  return b + 1024;
}

hipError_t consistency_merge(MergeArgs a, void* ws, size_t ws_bytes, float* new_out, hipStream_t st, const char** why) {
  const int H = a.g.H, W = a.g.W;
  const size_t cells = (size_t)a.g.big * W;
  if (ws_bytes < merge_ws_bytes(a.n_src, a.n_out, H, W)) { *why = "merge: workspace too small"; return hipErrorInvalidValue; }
  if (a.n_src % a.aB || a.o_begin < 0 || a.o_begin + a.n_out > a.n_src) { *why = "merge: bad view ranges"; return hipErrorInvalidValue; }
  if (W % 2) { *why = "merge: W must be even"; return hipErrorInvalidValue; }
  char* p = reinterpret_cast<char*>(ws);
  auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) & ~size_t(255); return q; };
  a.world = reinterpret_cast<double4*>(take((size_t)a.n_src * H * W * sizeof(double4)));
  a.nrep = merge_replicas(a.aB);
  const size_t rc = (size_t)a.nrep * a.n_out * cells;
  char* acc0 = p;
  a.cnt = reinterpret_cast<uint32_t*>(take(rc * 4));
  a.sumL = reinterpret_cast<double*>(take(rc * 8));
  a.sumI = reinterpret_cast<double*>(take(rc * 8));
  char* ff0 = p;
  a.minkey = reinterpret_cast<unsigned long long*>(take(rc * 8));
  a.minidx = reinterpret_cast<uint32_t*>(take((size_t)a.n_out * cells * 4));
  char* ff1 = p;
  a.newimg = new_out ? new_out : reinterpret_cast<float*>(take((size_t)a.n_out * 2 * H * W * 4));
  a.maskimg = reinterpret_cast<uint8_t*>(take((size_t)a.n_out * H * W));
  hipError_t e;
  if ((e = hipMemsetAsync(acc0, 0, ff0 - acc0, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(ff0, 0xFF, ff1 - ff0, st)) != hipSuccess) return e;
  const size_t nw = (size_t)a.n_src * H * W, npair = (size_t)a.n_out * a.aB * H * W, nout = (size_t)a.n_out * H * W;
  hipLaunchKernelGGL(merge_world_kernel, dim3(grid_for(nw)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(merge_accum_kernel, dim3(grid_for(npair)), dim3(256), 0, st, a);
  if (a.nrep > 1) hipLaunchKernelGGL(merge_reduce_kernel, dim3(grid_for((size_t)a.n_out * cells)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(merge_minidx_kernel, dim3(grid_for(npair)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(merge_resolve_kernel, dim3(grid_for(nout)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(merge_apply_kernel, dim3(grid_for(2 * nout)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace sdp
