// Fused annealed-Langevin update (gfx950), HBM-bound elementwise pass.
//
//   grad = nan_to_num(scorenet(x, labels))                   KITTISampling.py:137-138
//   lik  = -mask * (x - ref)                                  KITTISampling.py:144
//   x    = x + step*grad + grad_ref*lik + noise*sqrt(2*step)  KITTISampling.py:156
//
// Evaluated in float32 with the reference's association and no FMA contraction, so with an
// injected noise buffer it is bit-identical to the PyTorch CPU path.  Without one, noise is
// N(0,1) from Philox4x32-10 + Box-Muller (the reference's torch.randn_like stream cannot be
// reproduced on a different device anyway).  The same pass emits max|x_new[:,0]| (float bits,
// atomicMax) for the merge's tooHigh test (KITTISampling.py:162) and, when asked, lik for the
// denoise step (KITTISampling.py:505 uses the last loop step's grad_likelihood).
#include "common.h"

// reference evaluation order: no FMA contraction in this file (HIP __fmul_rn is a plain `*`)
#pragma clang fp contract(off)

namespace sdp {

struct Philox {
  static SDP_DEV uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  static SDP_DEV uint4 run(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

SDP_DEV float u01(uint32_t v) { return ((float)v + 0.5f) * 2.3283064365386963e-10f; }  // (0,1)

SDP_DEV float4 normal4(uint64_t seed, uint64_t ctr) {
  const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u),
                              make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float r1 = sqrtf(-2.f * __logf(u01(r.x))), r2 = sqrtf(-2.f * __logf(u01(r.z)));
  float s1, c1, s2, c2;
  __sincosf(6.283185307179586f * u01(r.y), &s1, &c1);
  __sincosf(6.283185307179586f * u01(r.w), &s2, &c2);
  return make_float4(r1 * c1, r1 * s1, r2 * c2, r2 * s2);
}

SDP_DEV float nan2num(float g) {
  if (g != g) return 0.f;
  if (g == INFINITY) return 3.4028234663852886e38f;
  if (g == -INFINITY) return -3.4028234663852886e38f;
  return g;
}

// x, g, ref, mask, noise: [B][C][HW]; one thread = 4 consecutive elements (HW % 4 == 0)
__global__ __launch_bounds__(256) void langevin_kernel(float* __restrict__ x, const float* __restrict__ g,
                                                       const float* __restrict__ ref, const int32_t* __restrict__ mask,
                                                       const float* __restrict__ noise, uint64_t seed, uint64_t offset,
                                                       float step, float nscale, float gref, int n2n, int C, int HW,
                                                       size_t n4, float* __restrict__ lik_out,
                                                       uint32_t* __restrict__ absmax) {
  uint32_t local_max = 0u;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 xv = reinterpret_cast<const float4*>(x)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    const float4 rv = reinterpret_cast<const float4*>(ref)[i];
    const int4 mv = reinterpret_cast<const int4*>(mask)[i];
    const float4 nv = noise ? reinterpret_cast<const float4*>(noise)[i] : normal4(seed, offset + i);
    const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ga[4] = {gv.x, gv.y, gv.z, gv.w};
    const float ra[4] = {rv.x, rv.y, rv.z, rv.w}, na[4] = {nv.x, nv.y, nv.z, nv.w};
    const int ma[4] = {mv.x, mv.y, mv.z, mv.w};
    float o[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gg = n2n ? nan2num(ga[k]) : ga[k];
      l[k] = __fmul_rn((float)(-ma[k]), __fsub_rn(xa[k], ra[k]));
      float v = __fadd_rn(xa[k], __fmul_rn(step, gg));
      v = __fadd_rn(v, __fmul_rn(gref, l[k]));
      o[k] = __fadd_rn(v, __fmul_rn(na[k], nscale));
    }
    reinterpret_cast<float4*>(x)[i] = make_float4(o[0], o[1], o[2], o[3]);
    if (lik_out) reinterpret_cast<float4*>(lik_out)[i] = make_float4(l[0], l[1], l[2], l[3]);
    if (absmax) {
      const size_t e = i * 4;
      if ((e / HW) % C == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) local_max = max(local_max, __float_as_uint(fabsf(o[k])));
      }
    }
  }
  if (absmax) {
    // wave max, then block max in LDS: ONE atomic per block (same-address atomics serialise
    // at the L2 -- one per wave cost ~10 us of a 16 us launch at 4 views)
    __shared__ uint32_t wmax[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) local_max = max(local_max, (uint32_t)__shfl_xor((int)local_max, off));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = local_max;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
      if (m) atomicMax(absmax, m);
    }
  }
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
  hipLaunchKernelGGL(langevin_kernel, dim3(grid), dim3(256), 0, st, x, g, ref, mask, noise, seed, offset, step,
                     nscale, gref, n2n, C, HW, n4, lik_out, absmax);
  return hipGetLastError();
}

hipError_t axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask, const float* ref, float b,
                     size_t n, hipStream_t st) {
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, g, a, lik, mask, ref, b, n);
  return hipGetLastError();
}

}  // namespace sdp
