// The annealed-Langevin update of one float4 group, shared by the stand-alone Langevin kernel
// (langevin.hip) and the end_conv epilogue that fuses it into the score-net forward (aux.hip).
//
//   grad = nan_to_num(scorenet(x, labels))                   KITTISampling.py:137-138
//   lik  = -mask * (x - ref)                                  KITTISampling.py:144
//   x    = x + step*grad + grad_ref*lik + noise*sqrt(2*step)  KITTISampling.py:156
//
// Evaluated in float32 with the reference's association and no FMA contraction (the pragma in
// each function body holds whatever the including file's -ffp-contract is), so with an injected
// noise buffer it is bit-identical to the PyTorch CPU path, and the fused and stand-alone forms
// agree bit for bit.  Without a noise buffer, noise is N(0,1) from Philox4x32-10 + Box-Muller,
// one counter per 4 consecutive elements of [B][C][HW].
#pragma once
#include "common.h"

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

SDP_DEV float u01(uint32_t v) {
#pragma clang fp contract(off)
  return ((float)v + 0.5f) * 2.3283064365386963e-10f;   // (0,1)
}

SDP_DEV float4 normal4(uint64_t seed, uint64_t ctr) {
#pragma clang fp contract(off)
  const uint4 r = Philox::run(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u),
                              make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  // builtins, not the header functions sqrtf/__logf: those carry the including file's `contract`
  // flag into llvm.sqrt/llvm.log, whose expansions then differ by an ulp between files
  const float r1 = __builtin_sqrtf(-2.f * __builtin_logf(u01(r.x)));
  const float r2 = __builtin_sqrtf(-2.f * __builtin_logf(u01(r.z)));
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

// one Langevin step's operands; x is updated in place
struct LangevinArgs {
  float* x;
  const float* ref;
  const int32_t* mask;
  const float* noise;      // nullable: Philox
  uint64_t seed, offset;   // Philox key, counter of float4 group 0
  float step, nscale, gref;
  int n2n;                 // nan_to_num(grad)
  float* lik;              // nullable: grad_likelihood out
  uint32_t* absmax;        // nullable: atomicMax of |x_new[:,0]| float bits
};

// float4 group i of [B][C][HW] (group index = element index / 4): new x and lik
SDP_DEV float4 langevin_group(const LangevinArgs& a, size_t i, float4 gv, float4& lik) {
#pragma clang fp contract(off)
  const float4 xv = reinterpret_cast<const float4*>(a.x)[i];
  const float4 rv = reinterpret_cast<const float4*>(a.ref)[i];
  const int4 mv = reinterpret_cast<const int4*>(a.mask)[i];
  const float4 nv = a.noise ? reinterpret_cast<const float4*>(a.noise)[i] : normal4(a.seed, a.offset + i);
  const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ga[4] = {gv.x, gv.y, gv.z, gv.w};
  const float ra[4] = {rv.x, rv.y, rv.z, rv.w}, na[4] = {nv.x, nv.y, nv.z, nv.w};
  const int ma[4] = {mv.x, mv.y, mv.z, mv.w};
  float o[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gg = a.n2n ? nan2num(ga[k]) : ga[k];
    // plain operators under this body's pragma (HIP's __fmul_rn / __fadd_rn are header functions
    // compiled under the including file's contraction setting)
    l[k] = (float)(-ma[k]) * (xa[k] - ra[k]);
    float v = xa[k] + a.step * gg;
    v = v + a.gref * l[k];
    o[k] = v + na[k] * a.nscale;
  }
  lik = make_float4(l[0], l[1], l[2], l[3]);
  return make_float4(o[0], o[1], o[2], o[3]);
}

SDP_DEV uint32_t absmax4(float4 o) {
  return max(max(__float_as_uint(fabsf(o.x)), __float_as_uint(fabsf(o.y))),
             max(__float_as_uint(fabsf(o.z)), __float_as_uint(fabsf(o.w))));
}

// block max of v (every thread of the block calls it) -> one atomicMax, skipped when the running
// maximum is already larger (same-address atomics serialise at the L2)
template <int NWAVES>
SDP_DEV void block_absmax(uint32_t v, uint32_t* absmax) {
  __shared__ uint32_t wmax[NWAVES];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t m = 0;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) m = max(m, wmax[w]);
    if (m > *reinterpret_cast<volatile uint32_t*>(absmax)) atomicMax(absmax, m);
  }
}

}  // namespace sdp
