// Fused annealed-Langevin update (gfx950), HBM-bound elementwise pass (langevin.h holds the
// per-element arithmetic, shared with the end_conv epilogue of sdp_net_forward_langevin).
// The same pass emits max|x_new[:,0]| (float bits, atomicMax) for the merge's tooHigh test
// (KITTISampling.py:162) and, when asked, lik for the denoise step (KITTISampling.py:505 uses
// the last loop step's grad_likelihood).
#include "langevin.h"

// reference evaluation order: no FMA contraction in this file (HIP __fmul_rn is a plain `*`)
#pragma clang fp contract(off)

namespace sdp {

// x, g, ref, mask, noise: [B][C][HW]; one thread = 4 consecutive elements (HW % 4 == 0)
__global__ __launch_bounds__(256) void langevin_kernel(LangevinArgs a, const float* __restrict__ g, int C, int HW,
                                                       size_t n4) {
  uint32_t local_max = 0u;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 l;
    const float4 o = langevin_group(a, i, reinterpret_cast<const float4*>(g)[i], l);
    reinterpret_cast<float4*>(a.x)[i] = o;
    if (a.lik) reinterpret_cast<float4*>(a.lik)[i] = l;
    if (a.absmax && ((i * 4) / HW) % C == 0) local_max = max(local_max, absmax4(o));
  }
  // wave max, then block max in LDS: ONE atomic per block (same-address atomics serialise at
  // the L2 -- one per wave cost ~10 us of a 16 us launch at 4 views)
  if (a.absmax) block_absmax<4>(local_max, a.absmax);
}

// x <- (x + a*g) + b*lik ; or, with g == null: x <- x + b*(-mask*(x - ref))
__global__ __launch_bounds__(256) void axpy_kernel(float* __restrict__ x, const float* __restrict__ g, float a,
                                                   const float* __restrict__ lik, const int32_t* __restrict__ mask,
                                                   const float* __restrict__ ref, float b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float xv = x[i];
    if (g) {
      x[i] = __fadd_rn(__fadd_rn(xv, __fmul_rn(a, g[i])), __fmul_rn(b, lik[i]));
    } else {
      const float l = __fmul_rn((float)(-mask[i]), __fsub_rn(xv, ref[i]));
      x[i] = __fadd_rn(xv, __fmul_rn(b, l));
    }
  }
}

static int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 256 * 8); }

hipError_t langevin_step(float* x, const float* g, const float* ref, const int32_t* mask, const float* noise,
                         uint64_t seed, uint64_t offset, float step, float nscale, float gref, int n2n, int B, int C,
                         int HW, float* lik_out, uint32_t* absmax, hipStream_t st) {
  const size_t n4 = (size_t)B * C * HW / 4;
  // with the absmax reduction: at most 256 blocks (one atomic each), each thread a few float4s
  const int grid = absmax ? (int)std::min<size_t>((n4 + 255) / 256, 256) : grid_for(n4);
  const LangevinArgs a{x, ref, mask, noise, seed, offset, step, nscale, gref, n2n, lik_out, absmax};
  hipLaunchKernelGGL(langevin_kernel, dim3(grid), dim3(256), 0, st, a, g, C, HW, n4);
  return hipGetLastError();
}

hipError_t axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask, const float* ref, float b,
                     size_t n, hipStream_t st) {
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, g, a, lik, mask, ref, b, n);
  return hipGetLastError();
}

}  // namespace sdp
