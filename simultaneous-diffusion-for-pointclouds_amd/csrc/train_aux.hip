// Memory-bound / small kernels of the DSM training step (BASELINE config 5):
//   pack_weights   : fp32 [Cout][Cin][k][k] -> MFMA fragment order (forward, or the flipped +
//                    transposed "dgrad" packing) on the device, so weights updated by the
//                    optimizer are re-packed without a host round trip
//   InstanceNorm++ backward (normalization.py:163-176): per-tile (sum g, sum g*xhat) ->
//                    per-(b,c) coefficients dh = k1*g + k2*h + k3 and the alpha/gamma/beta
//                    gradients -> the apply pass
//   unpool         : adjoint of ConvMeanPool's 2x2 mean (layers.py:309-313)
//   maxpool5 bwd   : adjoint of MaxPool2d(5, 1, 2) (layers.py:70) from the forward's argmax indices
//   upsample bwd   : adjoint of F.interpolate(bilinear, align_corners=True) (layers.py:182)
//   elu bwd        : dy * elu'(from the ELU output)
//   begin/end conv : weight gradients of the 4->128 / 128->2 convs, data gradient of end_conv
//   dsm loss       : anneal_dsm_score_estimation_with_mask (losses/dsm.py:67-119) + d loss/d score
//   adam_ema       : torch.optim.Adam step (losses/__init__.py:10-20) + EMAHelper.update (ema.py:16-21)
#include "common.h"
#include "kernels.h"

namespace sdp {

SDP_DEV float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- weight packing
// Fragment order consumed by conv_mfma_kernel: [chunk = Cin'/32][tap][nb = Cout'/32][lane 64][16 slots of 4 B]
// F32  : slot q of lane l = W'[nb*32 + (l&31)][chunk*32 + 16*(l>>5) + q]
// BF16 : 16-bit element (s, hl, j) of lane l, s in {0,1}, hl in {hi, lo}, j < 8:
//        ci' = chunk*32 + 16*s + 8*(l>>5) + j ; hi = bf16(w), lo = bf16(w - hi)
// dgrad: W'[o][i][tap] = W[i][o][k*k-1-tap]   (Cout' = Cin, Cin' = Cout)
SDP_DEV uint32_t pack_slot(const float* __restrict__ w, int Cout, int Cin, int NT, int mode, int dgrad, size_t i) {
  const int Co = dgrad ? Cin : Cout;
  const int NB = Co / 32;
  const int slot = i & 15;
  size_t r = i >> 4;
  const int lane = r & 63;
  r >>= 6;
  const int nb = r % NB;
  r /= NB;
  const int tap = r % NT;
  const int ch = r / NT;
  const int co = nb * 32 + (lane & 31), h = lane >> 5;
  auto wv = [&](int ci) -> float {
    return dgrad ? w[((size_t)ci * Cin + co) * NT + (NT - 1 - tap)] : w[((size_t)co * Cin + ci) * NT + tap];
  };
  if (mode == MODE_F32) return __float_as_uint(wv(ch * 32 + 16 * h + slot));
  const int s = slot >> 3, hl = (slot >> 2) & 1, j0 = (slot & 3) * 2;
  uint32_t pk = 0;
  for (int e = 0; e < 2; ++e) {
    const float f = wv(ch * 32 + 16 * s + 8 * h + j0 + e);
    const __bf16 hi = (__bf16)f;
    const __bf16 q = hl ? (__bf16)(f - (float)hi) : hi;
    pk |= (uint32_t)__builtin_bit_cast(uint16_t, q) << (16 * e);
  }
  return pk;
}

// 16x16 fragment order of the bf16 modes (conv_mfma_kernel SH = 16): [chunk][tap][nf = Cout'/16][hl][lane 64]
// [4 words = 8 bf16]; lane l: Cout' nf*16 + l%16, channels chunk*32 + 8 (l/16) + 0..7 (hl: hi / lo part),
// so every fragment load of a wave reads 1 KiB contiguous (bf16 mode reads the hi blocks only).  dgrad:
// the data gradient's flipped + transposed weights W'[o][i][tap] = W[i][o][k*k-1-tap] (Cout' = Cin) --
// the same lane layout serves as the MFMA's A operand (the transposed D = W x X data gradient)
SDP_DEV uint32_t pack_slot16(const float* __restrict__ w, int Cout, int Cin, int NT, int mode, int dgrad, size_t i) {
  const int NF = (dgrad ? Cin : Cout) / 16;
  const int word = i & 3;
  const int lane = (i >> 2) & 63;
  const int hl = (i >> 8) & 1;
  size_t r = i >> 9;
  const int nf = r % NF;
  r /= NF;
  const int tap = r % NT;
  const int ch = r / NT;
  const int co = nf * 16 + (lane & 15);
  uint32_t pk = 0;
  for (int e = 0; e < 2; ++e) {
    const int ci = ch * 32 + 8 * (lane >> 4) + word * 2 + e;
    const float f = dgrad ? w[((size_t)ci * Cin + co) * NT + (NT - 1 - tap)] : w[((size_t)co * Cin + ci) * NT + tap];
    const __bf16 hi = (__bf16)f;
    const __bf16 q = (hl && mode == MODE_F32X3) ? (__bf16)(f - (float)hi) : hi;
    pk |= (uint32_t)__builtin_bit_cast(uint16_t, q) << (16 * e);
  }
  return pk;
}

__global__ void pack_weights_kernel(const float* __restrict__ w, uint32_t* __restrict__ out, int Cout, int Cin, int NT,
                                    int mode, int dgrad) {
  const size_t n = (size_t)Cout * Cin * NT;    // output 32-bit slots
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = pack_slot(w, Cout, Cin, NT, mode, dgrad, i);
}

// every conv of the network in one launch (the re-pack after each optimizer step):
// blockIdx.y picks the conv, the x blocks stride over its slots
__global__ void pack_weights_multi_kernel(const PackDesc* __restrict__ d, int mode) {
  const PackDesc e = d[blockIdx.y];
  const size_t n = (size_t)e.Cout * e.Cin * e.NT;
  for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < n; j += (size_t)gridDim.x * blockDim.x)
    e.out[j] = e.dgrad >= 3 ? pack_slot16(e.w, e.Cout, e.Cin, e.NT, mode, e.dgrad == 4, j)
                            : pack_slot(e.w, e.Cout, e.Cin, e.NT, mode, e.dgrad, j);
}

hipError_t pack_weights_multi(const PackDesc* d, int nd, size_t total, int mode, hipStream_t st) {
  if (nd <= 0) return hipSuccess;
  (void)total;
  // 512 blocks per conv: each thread re-packs a few slots (its loads wait behind its previous
  // slot's store -- loads and stores retire in order -- so the chain per thread is kept short)
  hipLaunchKernelGGL(pack_weights_multi_kernel, dim3(512, nd), dim3(256), 0, st, d, mode);
  return hipGetLastError();
}

hipError_t pack_weights(const float* w, uint32_t* out, int Cout, int Cin, int k, int mode, int dgrad, hipStream_t st) {
  const size_t n = (size_t)Cout * Cin * k * k;
  const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(grid), dim3(256), 0, st, w, out, Cout, Cin, k * k, mode, dgrad);
  return hipGetLastError();
}

// ---------------------------------------------------------------- InstanceNorm++ backward
// part[b][grp][c] = (sum g, sum g * (h - mean) * rstd) over the INPP_GRP pixels of group grp.
// 1024-thread blocks (4x the waves of 256-thread ones) with four independent loads in flight per
// thread, so the reduce streams g and h at HBM rate while the finalize still sums only HW / 512
// groups per image.
constexpr int INPP_GRP = 512, INPP_NT = 1024;
template <typename TA>
__global__ __launch_bounds__(INPP_NT) void inpp_bwd_reduce_kernel(const TA* __restrict__ g, const TA* __restrict__ h,
                                                                  const float4* __restrict__ nst, float2* __restrict__ part,
                                                                  int HW, int C) {
  __shared__ float2 red[INPP_NT * 4];
  const int b = blockIdx.y, grp = blockIdx.x, ngrp = gridDim.x;
  const int C4 = C / 4, PL = INPP_NT / C4, tid = threadIdx.x;
  const int c4 = tid % C4, pl = tid / C4;
  const size_t base = ((size_t)b * HW + (size_t)grp * INPP_GRP) * C;
  float4 mu, rs;
  {
    const float4 n0 = nst[(size_t)b * C + c4 * 4], n1 = nst[(size_t)b * C + c4 * 4 + 1];
    const float4 n2 = nst[(size_t)b * C + c4 * 4 + 2], n3 = nst[(size_t)b * C + c4 * 4 + 3];
    mu = make_float4(n0.x, n1.x, n2.x, n3.x);
    rs = make_float4(n0.y, n1.y, n2.y, n3.y);
  }
  float sg[4] = {0.f, 0.f, 0.f, 0.f}, sx[4] = {0.f, 0.f, 0.f, 0.f};
  const int npp = INPP_GRP / PL;   // pixels per thread: 8 (C = 64) .. 64 (C = 512), a multiple of 4
  for (int j = 0; j < npp; j += 4) {
    float4 gv[4], hv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t o = base + (size_t)(pl + (j + u) * PL) * C + c4 * 4;
      gv[u] = ldg4(g, o);
      hv[u] = ldg4(h, o);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sg[0] += gv[u].x; sg[1] += gv[u].y; sg[2] += gv[u].z; sg[3] += gv[u].w;
      sx[0] = fmaf(gv[u].x, (hv[u].x - mu.x) * rs.x, sx[0]);
      sx[1] = fmaf(gv[u].y, (hv[u].y - mu.y) * rs.y, sx[1]);
      sx[2] = fmaf(gv[u].z, (hv[u].z - mu.z) * rs.z, sx[2]);
      sx[3] = fmaf(gv[u].w, (hv[u].w - mu.w) * rs.w, sx[3]);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[(pl * C4 + c4) * 4 + k] = make_float2(sg[k], sx[k]);
  __syncthreads();
  for (int i = tid; i < C; i += INPP_NT) {
    float a0 = 0.f, a1 = 0.f;
    for (int k = 0; k < PL; ++k) {
      const float2 v = red[(k * C4 + i / 4) * 4 + (i & 3)];
      a0 += v.x;
      a1 += v.y;
    }
    part[((size_t)b * ngrp + grp) * C + i] = make_float2(a0, a1);
  }
}

// One 1024-thread block.  Per image: G_c, Gx_c (f64 over the groups), then the channel-mean
// path of IN++: mhat = (mu - m)/sqrt(v + eps) with the unbiased v over C channels.
//   dh = gamma*rstd*(g - G/N - xhat*Gx/N) + dmu/N = k1*g + k2*(h - mean) + k3
//   d mhat_c = alpha_c*gamma_c*G_c ; du_c = tinv*(dmhat_c - mhat_c*sum(dmhat*mhat)/(C-1)) ;
//   dmu_c = du_c - mean_c(du)
//   dgamma += Gx + alpha*mhat*G ; dbeta += G ; dalpha += gamma*mhat*G
__global__ __launch_bounds__(1024) void inpp_bwd_finalize_kernel(const float2* __restrict__ part, int ngrp, float N,
                                                                 const float4* __restrict__ nst,
                                                                 const float* __restrict__ alpha,
                                                                 const float* __restrict__ gamma, int C,
                                                                 float4* __restrict__ coef, float* __restrict__ ppart) {
  __shared__ double r0[1024], r1[1024];
  const int b = blockIdx.x, tid = threadIdx.x, Gt = 1024 / C, gi = tid / C, c = tid % C;
  double s0 = 0.0, s1 = 0.0;
  for (int k = gi; k < ngrp; k += Gt) {
    const float2 v = part[((size_t)b * ngrp + k) * C + c];
    s0 += v.x;
    s1 += v.y;
  }
  r0[tid] = s0;
  r1[tid] = s1;
  __syncthreads();
  if (gi == 0)
    for (int k = 1; k < Gt; ++k) {
      s0 += r0[k * C + c];
      s1 += r1[k * C + c];
    }
  __syncthreads();
  const float4 ns = nst[(size_t)b * C + c];   // mean, rstd, mhat, tinv
  const double Gc = s0, Gx = s1;
  const double al = alpha[c], gm = gamma[c];
  const double dmh = al * gm * Gc;
  if (gi == 0) r0[c] = dmh * ns.z;
  __syncthreads();
  for (int s = C / 2; s > 0; s >>= 1) {
    if (gi == 0 && c < s) r0[c] += r0[c + s];
    __syncthreads();
  }
  const double A = r0[0];
  const double du = (double)ns.w * (dmh - (double)ns.z * A / (C - 1));
  if (gi == 0) r1[c] = du;
  __syncthreads();
  for (int s = C / 2; s > 0; s >>= 1) {
    if (gi == 0 && c < s) r1[c] += r1[c + s];
    __syncthreads();
  }
  if (gi != 0) return;
  const double dmu = du - r1[0] / C;
  // dh = k1*g + k2*(h - mean) + k3: centring h before the product keeps the cancellation
  // between the xhat and mean terms out of float32
  const double rs = ns.y;
  const double k1 = gm * rs;
  const double k2 = -gm * rs * rs * Gx / N;
  const double k3 = -gm * rs * Gc / N + dmu / N;
  coef[(size_t)b * C + c] = make_float4((float)k1, (float)k2, (float)k3, ns.x);
  float* pp = ppart + ((size_t)b * C + c) * 3;
  pp[0] = (float)(gm * (double)ns.z * Gc);          // d alpha
  pp[1] = (float)(Gx + al * (double)ns.z * Gc);     // d gamma
  pp[2] = (float)Gc;                                // d beta
}

// parameter gradients = sum over the images of the per-image partials (fixed order)
__global__ void inpp_bwd_params_kernel(const float* __restrict__ ppart, int B, int C, float* __restrict__ dalpha,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, g = 0.0, be = 0.0;
  for (int b = 0; b < B; ++b) {
    const float* pp = ppart + ((size_t)b * C + c) * 3;
    a += pp[0];
    g += pp[1];
    be += pp[2];
  }
  dalpha[c] = (float)a;
  dgamma[c] = (float)g;
  dbeta[c] = (float)be;
}

// out = k1*g + k2*(h - mean) + k3 (+ r1) (+ r2).  Grid (blocks, B): a thread's channel group is
// fixed (the block stride is a multiple of C/4), so its 4 coefficient rows are loaded once per image
template <typename TA>
__global__ __launch_bounds__(256) void inpp_bwd_apply_kernel(const TA* __restrict__ g, const TA* __restrict__ h,
                                                             const float4* __restrict__ coef, const TA* __restrict__ r1,
                                                             const TA* __restrict__ r2, TA* __restrict__ out, int HW,
                                                             int C) {
  // (__restrict__ on every operand -- the calls are elementwise, so even an in-place one is safe --
  // lets the next iteration's loads issue before this one's store: loads and stores retire in order)
  const int C4 = C / 4;
  const int b = blockIdx.y;
  const size_t n4 = (size_t)HW * C4, off = (size_t)b * n4;
  const size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  const int c = (int)(i0 % C4) * 4;
  const float4* cf = coef + (size_t)b * C + c;
  const float4 k0 = cf[0], kk1 = cf[1], kk2 = cf[2], kk3 = cf[3];
#pragma unroll 2
  for (size_t i = i0; i < n4; i += stride) {
    const size_t e = (off + i) * 4;
    const float4 gv = ldg4(g, e), hv = ldg4(h, e);
    float4 v = make_float4(fmaf(k0.x, gv.x, fmaf(k0.y, hv.x - k0.w, k0.z)), fmaf(kk1.x, gv.y, fmaf(kk1.y, hv.y - kk1.w, kk1.z)),
                           fmaf(kk2.x, gv.z, fmaf(kk2.y, hv.z - kk2.w, kk2.z)), fmaf(kk3.x, gv.w, fmaf(kk3.y, hv.w - kk3.w, kk3.z)));
    if (r1) {
      const float4 t = ldg4(r1, e);
      v = make_float4(v.x + t.x, v.y + t.y, v.z + t.z, v.w + t.w);
    }
    if (r2) {
      const float4 t = ldg4(r2, e);
      v = make_float4(v.x + t.x, v.y + t.y, v.z + t.z, v.w + t.w);
    }
    stg4(out, e, v);
  }
}

static int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 256 * 32); }

// Channel range: C a power of two in [32, 512] (the network's norms are 128 and 256 wide): the reduce
// block's 1024 threads hold C/4 channel groups x 4096/C pixel lanes, C/4 must divide 256 (the apply
// kernel's channel-fixed stride) and each lane's share of a 512-pixel group a multiple of 4
// (C % 32 == 0); anything else returns hipErrorInvalidValue (kernels.h).
template <typename TA>
static hipError_t inpp_backward_t(const TA* g, const TA* h, const float* nst, const float* alpha, const float* gamma,
                                  int B, int HW, int C, float* part, float* coef, float* ppart, float* dalpha,
                                  float* dgamma, float* dbeta, const TA* r1, const TA* r2, TA* out, hipStream_t st) {
  if (HW % INPP_GRP || C % 4 || C > 512 || (256 % (C / 4)) || (INPP_GRP / (INPP_NT / (C / 4))) % 4) return hipErrorInvalidValue;
  const int ngrp = HW / INPP_GRP;
  hipLaunchKernelGGL(inpp_bwd_reduce_kernel<TA>, dim3(ngrp, B), dim3(INPP_NT), 0, st, g, h,
                     reinterpret_cast<const float4*>(nst), reinterpret_cast<float2*>(part), HW, C);
  hipLaunchKernelGGL(inpp_bwd_finalize_kernel, dim3(B), dim3(1024), 0, st, reinterpret_cast<const float2*>(part), ngrp,
                     (float)HW, reinterpret_cast<const float4*>(nst), alpha, gamma, C, reinterpret_cast<float4*>(coef),
                     ppart);
  hipLaunchKernelGGL(inpp_bwd_params_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ppart, B, C, dalpha, dgamma, dbeta);
  // per image: 2048 blocks at most, the stride a multiple of C/4 (256 threads, C/4 divides 256)
  const size_t n4 = (size_t)HW * C / 4;
  const int nb = (int)std::min<size_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(inpp_bwd_apply_kernel<TA>, dim3(nb, B), dim3(256), 0, st, g, h,
                     reinterpret_cast<const float4*>(coef), r1, r2, out, HW, C);
  return hipGetLastError();
}

hipError_t inpp_backward(const float* g, const float* h, const float* nst, const float* alpha, const float* gamma, int B,
                         int HW, int C, float* part, float* coef, float* ppart, float* dalpha, float* dgamma,
                         float* dbeta, const float* r1, const float* r2, float* out, hipStream_t st, bool h16) {
  if (!h16) return inpp_backward_t(g, h, nst, alpha, gamma, B, HW, C, part, coef, ppart, dalpha, dgamma, dbeta, r1, r2, out, st);
  auto H = [](const float* p) { return reinterpret_cast<const __bf16*>(p); };
  return inpp_backward_t(H(g), H(h), nst, alpha, gamma, B, HW, C, part, coef, ppart, dalpha, dgamma, dbeta, H(r1), H(r2),
                         reinterpret_cast<__bf16*>(out), st);
}

// ---------------------------------------------------------------- pooling / upsampling adjoints
// ConvMeanPool: out = (o00 + o10 + o01 + o11)/4 -> d o_yx = dout[y/2][x/2] / 4   (dst full-res)
template <typename TA>
__global__ void unpool_kernel(const TA* __restrict__ dout, TA* __restrict__ dst, int H, int W, int C, size_t n4) {
  const int C4 = C / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    size_t p = i / C4;
    const int x = p % W;
    p /= W;
    const int y = p % H;
    const size_t b = p / H;
    const float4 v = ldg4(dout, (((b * (H / 2) + y / 2) * (W / 2) + x / 2) * C4 + c4) * 4);
    stg4(dst, i * 4, make_float4(v.x * 0.25f, v.y * 0.25f, v.z * 0.25f, v.w * 0.25f));
  }
}

// dst[q] = (res ? res[q] : 0) + sum over the windows p containing q whose argmax (idx, written
// by the forward maxpool5) is q of dp[p].  A block owns a 32-column x 32-channel strip of a
// run of rows and walks down it with a 5-row ring of window centres (idx + dp, 2-column halo)
// in LDS; the next row is fetched into registers while the current one is summed, so every
// input byte is read from HBM ~1.1 times and each of the 25 checks per output reads LDS.
// Positions outside the image get an index no window offset matches.
constexpr int MPB_W = 32, MPB_CB = 32;
template <typename TA>
__global__ __launch_bounds__(256) void maxpool5_bwd_kernel(const TA* __restrict__ dp, const uchar4* __restrict__ idx,
                                                           const TA* __restrict__ res, TA* __restrict__ dst, int H,
                                                           int W, int C, int rpb) {
  constexpr int C4B = MPB_CB / 4, PC = MPB_W + 4, RU = PC * C4B;   // 288 16-B units per ring row
  __shared__ float4 sd[5 * RU];
  __shared__ uchar4 si[5 * RU];
  const int tid = threadIdx.x;
  const int tw = W / MPB_W, tc = C / MPB_CB, nch = (H + rpb - 1) / rpb;
  int t = blockIdx.x;
  const int cb = t % tc;
  t /= tc;
  const int tx = t % tw;
  t /= tw;
  const int chunk = t % nch;
  const size_t b = t / nch;
  const int y0 = chunk * rpb, y1 = min(H, y0 + rpb), x0 = tx * MPB_W, c40 = cb * C4B, C4 = C / 4;
  float4 d[2];
  uchar4 k[2];
  auto fetch = [&](int row) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = tid + h * 256, xx = x0 - 2 + u / C4B;
      if (u < RU && row >= 0 && row < H && xx >= 0 && xx < W) {
        const size_t j = ((b * H + row) * W + xx) * C4 + c40 + u % C4B;
        d[h] = ldg4(dp, j * 4);
        k[h] = idx[j];
      } else {
        d[h] = make_float4(0.f, 0.f, 0.f, 0.f);
        k[h] = make_uchar4(255, 255, 255, 255);
      }
    }
  };
  auto put = [&](int slot) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = tid + h * 256;
      if (u < RU) {
        sd[slot * RU + u] = d[h];
        si[slot * RU + u] = k[h];
      }
    }
  };
  for (int r = 0; r < 4; ++r) {      // rows y0-2 .. y0+1 -> slots 0..3
    fetch(y0 - 2 + r);
    put(r);
  }
  fetch(y0 + 2);
  const int c4 = tid % C4B, col = tid / C4B;   // 32 columns x 8 channel groups
  int base = 0;                                 // slot of row y-2
  for (int y = y0; y < y1; ++y) {
    put(base == 0 ? 4 : base - 1);              // row y+2
    __syncthreads();
    fetch(y + 3);
    const size_t o = ((b * H + y) * W + x0 + col) * C4 + c40 + c4;
    float4 s = res ? ldg4(res, o * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int dy = -2; dy <= 2; ++dy) {
      int sl = base + dy + 2;
      sl = sl >= 5 ? sl - 5 : sl;
#pragma unroll
      for (int dx = -2; dx <= 2; ++dx) {      // window centre (y+dy, x+dx); q sits at its offset (-dy, -dx)
        const int u = sl * RU + (col + 2 + dx) * C4B + c4;
        const uchar4 kk = si[u];
        const unsigned char want = (unsigned char)((2 - dy) * 5 + (2 - dx));
        if (kk.x == want || kk.y == want || kk.z == want || kk.w == want) {
          const float4 dd = sd[u];
          if (kk.x == want) s.x += dd.x;
          if (kk.y == want) s.y += dd.y;
          if (kk.z == want) s.z += dd.z;
          if (kk.w == want) s.w += dd.w;
        }
      }
    }
    stg4(dst, o * 4, s);
    base = base == 4 ? 0 : base + 1;
    __syncthreads();
  }
}

// The bf16-tape form of maxpool5_bwd_kernel: 8-channel units (16 B of dp, 8 B of indices) -- each of the 25
// window checks reads one 8-byte index word from LDS for 8 channels (a SWAR byte compare) instead of one
// 4-byte word per 4 channels -- over 32-column x 64-channel strips, otherwise the same ring walk, the same
// fixed summation order (dy, dx), so the result is deterministic.
constexpr int MPH_W = 32, MPH_C = 64;
__global__ __launch_bounds__(256) void maxpool5_bwd_h16_kernel(const __bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                                                               const __bf16* __restrict__ res, __bf16* __restrict__ dst,
                                                               int H, int W, int C, int rpb) {
  constexpr int C8B = MPH_C / 8, PC = MPH_W + 4, RU = PC * C8B;   // 288 units per ring row
  __shared__ uint4 sd[5 * RU];
  __shared__ uint2 si[5 * RU];
  const int tid = threadIdx.x;
  const int tw = W / MPH_W, tc = C / MPH_C, nch = (H + rpb - 1) / rpb;
  int t = blockIdx.x;
  const int cb = t % tc;
  t /= tc;
  const int tx = t % tw;
  t /= tw;
  const int chunk = t % nch;
  const size_t b = t / nch;
  const int y0 = chunk * rpb, y1 = min(H, y0 + rpb), x0 = tx * MPH_W;
  uint4 d[2];
  uint2 k[2];
  auto fetch = [&](int row) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = tid + h * 256, xx = x0 - 2 + u / C8B;
      if (u < RU && row >= 0 && row < H && xx >= 0 && xx < W) {
        const size_t e = ((b * H + row) * W + xx) * C + cb * MPH_C + (u % C8B) * 8;
        d[h] = *reinterpret_cast<const uint4*>(dp + e);
        k[h] = *reinterpret_cast<const uint2*>(idx + e);
      } else {
        d[h] = make_uint4(0u, 0u, 0u, 0u);
        k[h] = make_uint2(0xffffffffu, 0xffffffffu);   // no window offset matches
      }
    }
  };
  auto put = [&](int slot) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = tid + h * 256;
      if (u < RU) {
        sd[slot * RU + u] = d[h];
        si[slot * RU + u] = k[h];
      }
    }
  };
  for (int r = 0; r < 4; ++r) {
    fetch(y0 - 2 + r);
    put(r);
  }
  fetch(y0 + 2);
  const int c8 = tid % C8B, col = tid / C8B;   // 32 columns x 8 channel units
  int base = 0;
  for (int y = y0; y < y1; ++y) {
    put(base == 0 ? 4 : base - 1);
    __syncthreads();
    fetch(y + 3);
    const size_t o = ((b * H + y) * W + x0 + col) * C + cb * MPH_C + c8 * 8;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (res) {
      const uint4 rv = *reinterpret_cast<const uint4*>(res + o);
      const float4 lo = bf4_to_f4(make_uint2(rv.x, rv.y)), hi = bf4_to_f4(make_uint2(rv.z, rv.w));
      s[0] = lo.x; s[1] = lo.y; s[2] = lo.z; s[3] = lo.w; s[4] = hi.x; s[5] = hi.y; s[6] = hi.z; s[7] = hi.w;
    }
#pragma unroll
    for (int dy = -2; dy <= 2; ++dy) {
      int sl = base + dy + 2;
      sl = sl >= 5 ? sl - 5 : sl;
#pragma unroll
      for (int dx = -2; dx <= 2; ++dx) {
        const int u = sl * RU + (col + 2 + dx) * C8B + c8;
        const uint2 kk = si[u];
        const uint32_t want = (uint32_t)((2 - dy) * 5 + (2 - dx)) * 0x01010101u;
        const uint32_t e0 = kk.x ^ want, e1 = kk.y ^ want;   // zero bytes where the index matches
        const uint32_t z0 = (e0 - 0x01010101u) & ~e0 & 0x80808080u, z1 = (e1 - 0x01010101u) & ~e1 & 0x80808080u;
        if (z0 | z1) {
          const uint4 dd = sd[u];
          const uint32_t w[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t byte = ((e < 4 ? kk.x : kk.y) >> (8 * (e & 3))) & 0xffu;
            const float v = (e & 1) ? __uint_as_float(w[e >> 1] & 0xffff0000u) : __uint_as_float(w[e >> 1] << 16);
            if (byte == ((2 - dy) * 5 + (2 - dx))) s[e] += v;
          }
        }
      }
    }
    *reinterpret_cast<uint4*>(dst + o) = make_uint4(pack_bf2(s[0], s[1]), pack_bf2(s[2], s[3]), pack_bf2(s[4], s[5]),
                                                     pack_bf2(s[6], s[7]));
    base = base == 4 ? 0 : base + 1;
    __syncthreads();
  }
}

// adjoint of the bilinear align_corners upsample [h][w] -> [H][W] (forward: conv epilogue `up`):
// dlow[i][j] += sum_{y,x} wy(y,i) wx(x,j) g[y][x]  (gather over the few y, x that reach (i, j))
SDP_DEV void up_weights(int o, int n_lo, float scale, int* i0, int* i1, float* w0, float* w1) {
  const float f = scale * (float)o;
  const int a = (int)f;
  const int ap = a < n_lo - 1 ? 1 : 0;
  *i0 = a;
  *i1 = a + ap;
  *w1 = f - (float)a;
  *w0 = 1.f - *w1;
}

template <typename TA>
__global__ void upsample_bwd_kernel(const TA* __restrict__ g, TA* __restrict__ dlow, int H, int W, int C,
                                    int accumulate, size_t n4) {
  const int h = H / 2, w = W / 2, C4 = C / 4;
  const float sh = (float)(h - 1) / (float)(H - 1), sw = (float)(w - 1) / (float)(W - 1);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    size_t p = i / C4;
    const int j = p % w;
    p /= w;
    const int ii = p % h;
    const size_t b = p / h;
    // high-res rows whose source rows include ii: scale*y in (ii-1, ii+1]
    const int ylo = max(0, (int)floorf((float)(ii - 1) / sh) - 1), yhi = min(H - 1, (int)ceilf((float)(ii + 1) / sh) + 1);
    const int xlo = max(0, (int)floorf((float)(j - 1) / sw) - 1), xhi = min(W - 1, (int)ceilf((float)(j + 1) / sw) + 1);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int y = ylo; y <= yhi; ++y) {
      int a0, a1;
      float u0, u1;
      up_weights(y, h, sh, &a0, &a1, &u0, &u1);
      const float wy = (a0 == ii ? u0 : 0.f) + (a1 == ii ? u1 : 0.f);
      if (wy == 0.f) continue;
      for (int x = xlo; x <= xhi; ++x) {
        int b0, b1;
        float v0, v1;
        up_weights(x, w, sw, &b0, &b1, &v0, &v1);
        const float wx = (b0 == j ? v0 : 0.f) + (b1 == j ? v1 : 0.f);
        if (wx == 0.f) continue;
        const float4 gv = ldg4(g, (((b * H + y) * W + x) * C4 + c4) * 4);
        const float ww = wy * wx;
        s = make_float4(fmaf(ww, gv.x, s.x), fmaf(ww, gv.y, s.y), fmaf(ww, gv.z, s.z), fmaf(ww, gv.w, s.w));
      }
    }
    if (accumulate) {
      const float4 t = ldg4(dlow, i * 4);
      s = make_float4(s.x + t.x, s.y + t.y, s.z + t.z, s.w + t.w);
    }
    stg4(dlow, i * 4, s);
  }
}

// dst = dy * elu'(from the ELU output y) (+ res)
template <typename TA>
__global__ void elu_bwd_post_kernel(const TA* __restrict__ dy, const TA* __restrict__ y,
                                    const TA* __restrict__ res, TA* __restrict__ dst, size_t n4) {
#pragma unroll 2
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 d = ldg4(dy, i * 4), yv = ldg4(y, i * 4);
    float4 v = make_float4(d.x * elu_grad(yv.x, 2), d.y * elu_grad(yv.y, 2), d.z * elu_grad(yv.z, 2),
                           d.w * elu_grad(yv.w, 2));
    if (res) {
      const float4 t = ldg4(res, i * 4);
      v = make_float4(v.x + t.x, v.y + t.y, v.z + t.z, v.w + t.w);
    }
    stg4(dst, i * 4, v);
  }
}

// dst = a + b (float4 lanes)
template <typename TA>
__global__ void add_kernel(const TA* __restrict__ a, const TA* __restrict__ b, TA* __restrict__ dst, size_t n4) {
#pragma unroll 2
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 x = ldg4(a, i * 4), y = ldg4(b, i * 4);
    stg4(dst, i * 4, make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w));
  }
}

// out[i] = sum_k part[k*stride + i] (fixed order); block = 32 outputs x 8 K-groups
__global__ __launch_bounds__(256) void sum_rows_kernel(const float* __restrict__ part, int K, int n, int stride,
                                                       float* __restrict__ out) {
  __shared__ double red[8][32];
  const int il = threadIdx.x & 31, kg = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + il;
  double s = 0.0;
  if (i < n)
    for (int k = kg; k < K; k += 8) s += part[(size_t)k * stride + i];
  red[kg][il] = s;
  __syncthreads();
  if (kg == 0 && i < n) {
    for (int g = 1; g < 8; ++g) s += red[g][il];
    out[i] = (float)s;
  }
}

static hipError_t sum_rows(const float* part, int K, int n, int stride, float* out, hipStream_t st) {
  hipLaunchKernelGGL(sum_rows_kernel, dim3((n + 31) / 32), dim3(256), 0, st, part, K, n, stride, out);
  return hipGetLastError();
}

#define SDP_H16(p) reinterpret_cast<const __bf16*>(p)
#define SDP_H16W(p) reinterpret_cast<__bf16*>(p)
hipError_t unpool(const float* dout, float* dst, int B, int H, int W, int C, hipStream_t st, bool h16) {
  const size_t n4 = (size_t)B * H * W * C / 4;
  if (h16) hipLaunchKernelGGL(unpool_kernel<__bf16>, dim3(grid_for(n4)), dim3(256), 0, st, SDP_H16(dout), SDP_H16W(dst), H, W, C, n4);
  else hipLaunchKernelGGL(unpool_kernel<float>, dim3(grid_for(n4)), dim3(256), 0, st, dout, dst, H, W, C, n4);
  return hipGetLastError();
}

hipError_t maxpool5_backward(const uint8_t* idx, const float* dp, const float* res, float* dst, int B, int H, int W, int C,
                             hipStream_t st, bool h16) {
  if (W % MPB_W || C % MPB_CB) return hipErrorInvalidValue;
  const int strips = B * (W / MPB_W) * (C / MPB_CB);
  int rpb = H;                                  // split the rows only as far as needed to fill the chip
  while (rpb > 8 && (long)strips * ((H + rpb - 1) / rpb) < 2048) rpb = (rpb + 1) / 2;
  const int nb = strips * ((H + rpb - 1) / rpb);
  if (h16) {
    if (C % MPH_C) return hipErrorInvalidValue;
    const int strips16 = B * (W / MPH_W) * (C / MPH_C);
    int rpb16 = H;
    while (rpb16 > 8 && (long)strips16 * ((H + rpb16 - 1) / rpb16) < 2048) rpb16 = (rpb16 + 1) / 2;
    hipLaunchKernelGGL(maxpool5_bwd_h16_kernel, dim3(strips16 * ((H + rpb16 - 1) / rpb16)), dim3(256), 0, st, SDP_H16(dp), idx,
                       SDP_H16(res), SDP_H16W(dst), H, W, C, rpb16);
  } else
    hipLaunchKernelGGL(maxpool5_bwd_kernel<float>, dim3(nb), dim3(256), 0, st, dp, reinterpret_cast<const uchar4*>(idx), res,
                       dst, H, W, C, rpb);
  return hipGetLastError();
}

hipError_t upsample_backward(const float* g, float* dlow, int B, int H, int W, int C, int accumulate, hipStream_t st, bool h16) {
  const size_t n4 = (size_t)B * (H / 2) * (W / 2) * C / 4;
  if (h16)
    hipLaunchKernelGGL(upsample_bwd_kernel<__bf16>, dim3(grid_for(n4)), dim3(256), 0, st, SDP_H16(g), SDP_H16W(dlow), H, W, C,
                       accumulate, n4);
  else
    hipLaunchKernelGGL(upsample_bwd_kernel<float>, dim3(grid_for(n4)), dim3(256), 0, st, g, dlow, H, W, C, accumulate, n4);
  return hipGetLastError();
}

hipError_t elu_backward_post(const float* dy, const float* y, const float* res, float* dst, size_t n, hipStream_t st, bool h16) {
  if (h16)
    hipLaunchKernelGGL(elu_bwd_post_kernel<__bf16>, dim3(grid_for(n / 4)), dim3(256), 0, st, SDP_H16(dy), SDP_H16(y), SDP_H16(res),
                       SDP_H16W(dst), n / 4);
  else
    hipLaunchKernelGGL(elu_bwd_post_kernel<float>, dim3(grid_for(n / 4)), dim3(256), 0, st, dy, y, res, dst, n / 4);
  return hipGetLastError();
}

hipError_t add_tensors(const float* a, const float* b, float* dst, size_t n, hipStream_t st, bool h16) {
  if (h16)
    hipLaunchKernelGGL(add_kernel<__bf16>, dim3(grid_for(n / 4)), dim3(256), 0, st, SDP_H16(a), SDP_H16(b), SDP_H16W(dst), n / 4);
  else
    hipLaunchKernelGGL(add_kernel<float>, dim3(grid_for(n / 4)), dim3(256), 0, st, a, b, dst, n / 4);
  return hipGetLastError();
}

// ---------------------------------------------------------------- begin_conv weight gradient
// dW[co][ci][tap] = sum_p dx0[p][co] * in4[p + tap - (1,1)][ci] (zero pad), db[co] = sum_p dx0[p][co]
// in4 = (2x-1, 2x-1, linspace W, linspace H) (ncsnv2.py:485-496).  Block: ROWS rows x 64 px.
SDP_DEV float linspace01_t(int i, int n) {
  if (n == 1) return 0.f;
  const float step = 1.0f / (float)(n - 1);
  return i < n / 2 ? step * (float)i : 1.0f - step * (float)(n - 1 - i);
}

// 8 rows per block: B * H/8 * W/64 blocks (1024 at B=8, 64x1024) keep four waves per SIMD in flight; 32 rows gave
// 256 blocks, one wave per SIMD, and every LDS read of the FMA loop stood exposed (387 us per call at B=8)
constexpr int BW_ROWS = 8;
template <typename TA>
__global__ __launch_bounds__(256) void begin_wgrad_kernel(const float* __restrict__ x, const TA* __restrict__ dy,
                                                          float* __restrict__ part, int H, int W) {
  __shared__ float sp[4][3][66];
  __shared__ float sd[64][129];
  const int tid = threadIdx.x, co = tid & 127, half = tid >> 7;
  const int tiles_row = W / 64, rows_blk = H / BW_ROWS;
  const int per_img = rows_blk * tiles_row;
  const int b = blockIdx.x / per_img, t = blockIdx.x % per_img;
  const int y0 = (t / tiles_row) * BW_ROWS, x0 = (t % tiles_row) * 64;
  float acc[18];
#pragma unroll
  for (int k = 0; k < 18; ++k) acc[k] = 0.f;
  float db = 0.f;
  for (int r = 0; r < BW_ROWS; ++r) {
    const int y = y0 + r;
    __syncthreads();
    for (int i = tid; i < 4 * 3 * 66; i += 256) {
      const int ci = i / 198, rr = (i / 66) % 3, c = i % 66;
      const int yy = y - 1 + rr, xx = x0 - 1 + c;
      float v = 0.f;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        if (ci < 2) v = 2.f * x[(((size_t)b * 2 + ci) * H + yy) * W + xx] - 1.f;
        else if (ci == 2) v = linspace01_t(xx, W);
        else v = linspace01_t(yy, H);
      }
      sp[ci][rr][c] = v;
    }
    for (int i = tid; i < 64 * 32; i += 256) {
      const int px = i >> 5, c4 = i & 31;
      const float4 v = ldg4(dy, (((size_t)b * H + y) * W + x0 + px) * 128 + c4 * 4);
      sd[px][c4 * 4] = v.x; sd[px][c4 * 4 + 1] = v.y; sd[px][c4 * 4 + 2] = v.z; sd[px][c4 * 4 + 3] = v.w;
    }
    __syncthreads();
    // the thread's two input channels (2 half, 2 half + 1) x 3 rows x 3 columns in registers, one new column
    // per pixel: 6 LDS reads per 18 FMAs instead of 18 (the same FMAs in the same order)
    const int ci0 = half * 2;
    float wv[2][3][3];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        wv[c2][rr][0] = sp[ci0 + c2][rr][0];
        wv[c2][rr][1] = sp[ci0 + c2][rr][1];
      }
    for (int px = 0; px < 64; ++px) {
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) wv[c2][rr][2] = sp[ci0 + c2][rr][px + 2];
      const float g = sd[px][co];
      if (half == 0) db += g;
#pragma unroll
      for (int k = 0; k < 18; ++k) {
        const int c2 = k / 9, tap = k % 9;
        acc[k] = fmaf(g, wv[c2][tap / 3][tap % 3], acc[k]);
      }
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          wv[c2][rr][0] = wv[c2][rr][1];
          wv[c2][rr][1] = wv[c2][rr][2];
        }
    }
  }
  float* o = part + (size_t)blockIdx.x * (128 * 37);
#pragma unroll
  for (int k = 0; k < 18; ++k) o[co * 36 + half * 18 + k] = acc[k];
  if (half == 0) o[128 * 36 + co] = db;
}

hipError_t begin_conv_wgrad(const float* x, const float* dy, float* part, float* dw, float* db, int B, int H, int W,
                            hipStream_t st, bool h16) {
  if (H % BW_ROWS || W % 64) return hipErrorInvalidValue;
  const int nb = B * (H / BW_ROWS) * (W / 64);
  if (h16) hipLaunchKernelGGL(begin_wgrad_kernel<__bf16>, dim3(nb), dim3(256), 0, st, x, SDP_H16(dy), part, H, W);
  else hipLaunchKernelGGL(begin_wgrad_kernel<float>, dim3(nb), dim3(256), 0, st, x, dy, part, H, W);
  (void)sum_rows(part, nb, 128 * 36, 128 * 37, dw, st);
  return sum_rows(part + 128 * 36, nb, 128, 128 * 37, db, st);
}

// ---------------------------------------------------------------- end_conv backward
// Forward (ncsnv2.py:510-516): out[b][co] = (conv3x3_zero(ELU(IN++(o)), W) + bias) / sigmas[y_b].
// dend = dscore / sigmas[y_b].  Data gradient (to the ELU output) with the IN++/ELU derivative
// applied (g = da * elu'(o*scale + shift)); weight and bias gradients.
template <typename TA>
__global__ __launch_bounds__(256) void end_dgrad_kernel(const float* __restrict__ dscore, const float* __restrict__ sigmas,
                                                        const int64_t* __restrict__ labels, const float* __restrict__ w,
                                                        const TA* __restrict__ o, const float* __restrict__ ss,
                                                        TA* __restrict__ g, int H, int W) {
  constexpr int C = 128;
  __shared__ float sd[2][3][66];
  __shared__ float sw[2 * C * 9];
  const int tid = threadIdx.x;
  const int tiles_row = W / 64, per_img = H * tiles_row;
  const int b = blockIdx.x / per_img, t = blockIdx.x % per_img;
  const int y = t / tiles_row, x0 = (t % tiles_row) * 64;
  const float inv = 1.f / sigmas[labels[b]];
  for (int i = tid; i < 2 * 3 * 66; i += 256) {
    const int co = i / 198, rr = (i / 66) % 3, c = i % 66;
    const int yy = y - 1 + rr, xx = x0 - 1 + c;
    sd[co][rr][c] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? dscore[(((size_t)b * 2 + co) * H + yy) * W + xx] * inv : 0.f;
  }
  for (int i = tid; i < 2 * C * 9; i += 256) sw[i] = w[i];
  __syncthreads();
  const int c4 = tid & 31, pl = tid >> 5;
  const float* ssb = ss + ((size_t)b * C + c4 * 4) * 2;
  const float4 s0 = *reinterpret_cast<const float4*>(ssb), s1 = *reinterpret_cast<const float4*>(ssb + 4);
  for (int px = pl; px < 64; px += 8) {
    float da[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int co = 0; co < 2; ++co)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3;
        const float dv = sd[co][2 - kh][px + 2 - kw];
#pragma unroll
        for (int k = 0; k < 4; ++k) da[k] = fmaf(dv, sw[(co * C + c4 * 4 + k) * 9 + tap], da[k]);
      }
    const size_t idx = (((size_t)b * H + y) * W + x0 + px) * C + c4 * 4;
    const float4 h = ldg4(o, idx);
    const float z0 = fmaf(h.x, s0.x, s0.y), z1 = fmaf(h.y, s0.z, s0.w), z2 = fmaf(h.z, s1.x, s1.y), z3 = fmaf(h.w, s1.z, s1.w);
    stg4(g, idx, make_float4(da[0] * elu_grad(z0, 1), da[1] * elu_grad(z1, 1), da[2] * elu_grad(z2, 1), da[3] * elu_grad(z3, 1)));
  }
}

// 16 rows per block (1024 blocks at B=8); the transformed input rows sit in a 3-slot ring, each row is
// loaded and pushed through IN++ + ELU once (it was staged afresh for each of the 3 output rows that read it)
constexpr int EW_ROWS = 16;
template <typename TA>
__global__ __launch_bounds__(256) void end_wgrad_kernel(const float* __restrict__ dscore, const float* __restrict__ sigmas,
                                                        const int64_t* __restrict__ labels, const TA* __restrict__ o,
                                                        const float* __restrict__ ss, float* __restrict__ part, int H,
                                                        int W) {
  constexpr int C = 128;
  __shared__ float sp[3 * 34 * C];
  __shared__ float sd[2][32];
  const int tid = threadIdx.x, ci = tid >> 1, co = tid & 1;
  const int tiles_row = W / 32, per_img = (H / EW_ROWS) * tiles_row;
  const int b = blockIdx.x / per_img, t = blockIdx.x % per_img;
  const int y0 = (t / tiles_row) * EW_ROWS, x0 = (t % tiles_row) * 32;
  const float inv = 1.f / sigmas[labels[b]];
  const float* ssb = ss + (size_t)b * C * 2;
  float acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = 0.f;
  float db = 0.f;
  // input row yy (y0 - 1 <= yy <= y0 + EW_ROWS) lives in ring slot (yy - y0 + 1) % 3
  auto stage_row = [&](int yy) {
    const int slot = (yy - y0 + 1) % 3;
    for (int i = tid; i < 34 * 32; i += 256) {
      const int cc = i >> 5, c4 = i & 31;
      const int xx = x0 - 1 + cc;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const float4 h = ldg4(o, (((size_t)b * H + yy) * W + xx) * C + c4 * 4);
        const float4 s0 = *reinterpret_cast<const float4*>(ssb + c4 * 8), s1 = *reinterpret_cast<const float4*>(ssb + c4 * 8 + 4);
        v = make_float4(elu(fmaf(h.x, s0.x, s0.y)), elu(fmaf(h.y, s0.z, s0.w)), elu(fmaf(h.z, s1.x, s1.y)),
                        elu(fmaf(h.w, s1.z, s1.w)));
      }
      *reinterpret_cast<float4*>(&sp[(slot * 34 + cc) * C + c4 * 4]) = v;
    }
  };
  stage_row(y0 - 1);
  stage_row(y0);
  for (int r = 0; r < EW_ROWS; ++r) {
    const int y = y0 + r;
    stage_row(y + 1);                                // slot of row y - 2, read last by iteration r - 1
    if (tid < 64) {
      const int c2 = tid >> 5, px = tid & 31;
      sd[c2][px] = dscore[(((size_t)b * 2 + c2) * H + y) * W + x0 + px] * inv;
    }
    __syncthreads();
    const int sl[3] = {r % 3, (r + 1) % 3, (r + 2) % 3};   // slots of rows y - 1, y, y + 1
    // the thread's channel at 3 rows x 3 columns in registers, one new column per pixel (3 LDS reads per 9
    // FMAs instead of 9; the same FMAs in the same order)
    float wv[3][3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      wv[kh][0] = sp[(sl[kh] * 34 + 0) * C + ci];
      wv[kh][1] = sp[(sl[kh] * 34 + 1) * C + ci];
    }
    for (int px = 0; px < 32; ++px) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) wv[kh][2] = sp[(sl[kh] * 34 + px + 2) * C + ci];
      const float gv = sd[co][px];
      if (ci == 0) db += gv;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) acc[tap] = fmaf(gv, wv[tap / 3][tap % 3], acc[tap]);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        wv[kh][0] = wv[kh][1];
        wv[kh][1] = wv[kh][2];
      }
    }
    __syncthreads();                                 // the ring slot and sd are rewritten next iteration
  }
  float* op = part + (size_t)blockIdx.x * (2 * C * 9 + 2);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) op[(co * C + ci) * 9 + tap] = acc[tap];
  if (ci == 0) op[2 * C * 9 + co] = db;
}

hipError_t end_conv_backward(const float* dscore, const float* sigmas, const int64_t* labels, const float* w,
                             const float* o, const float* ss, float* g, float* part, float* dw, float* db, int B, int H,
                             int W, hipStream_t st, bool h16) {
  if (H % EW_ROWS || W % 64) return hipErrorInvalidValue;
  const int nb = B * (H / EW_ROWS) * (W / 32);
  if (h16) {
    hipLaunchKernelGGL(end_dgrad_kernel<__bf16>, dim3(B * H * (W / 64)), dim3(256), 0, st, dscore, sigmas, labels, w,
                       SDP_H16(o), ss, SDP_H16W(g), H, W);
    hipLaunchKernelGGL(end_wgrad_kernel<__bf16>, dim3(nb), dim3(256), 0, st, dscore, sigmas, labels, SDP_H16(o), ss, part, H, W);
  } else {
    hipLaunchKernelGGL(end_dgrad_kernel<float>, dim3(B * H * (W / 64)), dim3(256), 0, st, dscore, sigmas, labels, w, o, ss, g,
                       H, W);
    hipLaunchKernelGGL(end_wgrad_kernel<float>, dim3(nb), dim3(256), 0, st, dscore, sigmas, labels, o, ss, part, H, W);
  }
  (void)sum_rows(part, nb, 2 * 128 * 9, 2 * 128 * 9 + 2, dw, st);
  return sum_rows(part + 2 * 128 * 9, nb, 2, 2 * 128 * 9 + 2, db, st);
}

// floats of the partial-sum scratch the head weight gradients need (begin_conv_wgrad, end_conv_backward)
size_t head_wgrad_part_floats(int B, int H, int W) {
  const size_t bw = (size_t)B * (H / BW_ROWS) * (W / 64) * 128 * 37;
  const size_t ew = (size_t)B * (H / EW_ROWS) * (W / 32) * (2 * 128 * 9 + 2);
  return bw > ew ? bw : ew;
}

// ---------------------------------------------------------------- DSM loss (losses/dsm.py:67-119)
// target = -noise / sigma_b^2 ; r = mask * (score - target) ; numPixels = sum(mask) (whole batch)
// loss_b = 0.5 * sum(r^2) * CHW / numPixels * sigma_b^p ; loss = mean_b ; dscore = d loss / d score
constexpr int DSM_BLK = 64;   // blocks per image
__global__ __launch_bounds__(256) void dsm_mask_sum_kernel(const float* __restrict__ mask, int n_img, float* part) {
  __shared__ float red[4];
  const int b = blockIdx.y, tid = threadIdx.x;
  const float* m = mask + (size_t)b * n_img;
  float s = 0.f;
  for (int i = blockIdx.x * 256 + tid; i < n_img; i += DSM_BLK * 256) s += m[i];
  s = wsum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) part[b * DSM_BLK + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void dsm_grad_kernel(const float* __restrict__ score, const float* __restrict__ noise,
                                                       const float* __restrict__ mask, const float* __restrict__ used_sigma,
                                                       const float* __restrict__ mpart, int B, int n_img, float power,
                                                       float* __restrict__ dscore, float* __restrict__ lpart) {
  __shared__ double red[4];
  const int b = blockIdx.y, tid = threadIdx.x;
  double np = 0.0;
  for (int k = 0; k < B * DSM_BLK; ++k) np += mpart[k];
  const float sg = used_sigma[b];
  const float inv2 = 1.f / (sg * sg);
  const double scale = (double)n_img / np * pow((double)sg, (double)power) / B;
  const size_t base = (size_t)b * n_img;
  double s = 0.0;
  for (int i = blockIdx.x * 256 + tid; i < n_img; i += DSM_BLK * 256) {
    const float m = mask[base + i];
    const float tgt = -inv2 * noise[base + i];
    const float r = m * (score[base + i] - tgt);
    s += (double)r * r;
    dscore[base + i] = (float)(scale * (double)(m * r));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) lpart[b * DSM_BLK + blockIdx.x] = (float)(red[0] + red[1] + red[2] + red[3]);
}

__global__ void dsm_final_kernel(const float* __restrict__ mpart, const float* __restrict__ lpart,
                                 const float* __restrict__ used_sigma, int B, int n_img, float power, float* loss,
                                 float* loss_per) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double np = 0.0;
  for (int k = 0; k < B * DSM_BLK; ++k) np += mpart[k];
  double tot = 0.0;
  for (int b = 0; b < B; ++b) {
    double s = 0.0;
    for (int k = 0; k < DSM_BLK; ++k) s += lpart[b * DSM_BLK + k];
    const double lb = 0.5 * s * n_img / np * pow((double)used_sigma[b], (double)power);
    if (loss_per) loss_per[b] = (float)lb;
    tot += lb;
  }
  *loss = (float)(tot / B);
}

hipError_t dsm_loss(const float* score, const float* noise, const float* mask, const float* used_sigma, int B, int n_img,
                    float power, float* dscore, float* loss, float* loss_per, float* part, hipStream_t st) {
  float* mpart = part;
  float* lpart = part + B * DSM_BLK;
  hipLaunchKernelGGL(dsm_mask_sum_kernel, dim3(DSM_BLK, B), dim3(256), 0, st, mask, n_img, mpart);
  hipLaunchKernelGGL(dsm_grad_kernel, dim3(DSM_BLK, B), dim3(256), 0, st, score, noise, mask, used_sigma, mpart, B, n_img,
                     power, dscore, lpart);
  hipLaunchKernelGGL(dsm_final_kernel, dim3(1), dim3(64), 0, st, mpart, lpart, used_sigma, B, n_img, power, loss, loss_per);
  return hipGetLastError();
}

// ---------------------------------------------------------------- optimizer step + EMA
// get_optimizer (losses/__init__.py:3-13) -- the torch.optim update of every optimizer it builds, in
// torch's per-element evaluation order, then EMAHelper.update (ema.py:16-21):
//   Adam    : g += wd p ; m = m + (1-b1)(g - m) ; v = b2 v + (1-b2) g^2 ; [amsgrad: vmax = max(vmax, v)]
//             p -= step_size * m / (sqrt(v or vmax)/bc2_sqrt + eps)
//   RMSprop : g += wd p ; v = alpha v + (1-alpha) g^2 ; p -= lr * g / (sqrt(v) + eps)
//   SGD     : g += wd p ; buf = first step ? g : momentum buf + (1-dampening) g ; p -= lr * buf
//   EMA     : shadow = (1-mu) p + mu shadow
template <int KIND>
__global__ void optim_ema_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ s0,
                                 float* __restrict__ s1, float* __restrict__ s2, float* __restrict__ shadow, size_t n,
                                 OptimHyper h) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float pi = p[i];
    float gi = g[i];
    if (h.weight_decay != 0.f) gi = gi + h.weight_decay * pi;   // torch._foreach_add(grads, params, alpha=wd)
    if constexpr (KIND == OPT_ADAM) {
      float mi = s0[i];
      mi = mi + h.omb1 * (gi - mi);                              // lerp(m, g, 1-b1), weight < 0.5 branch
      const float vi = s1[i] * h.b2 + h.omb2 * gi * gi;
      s0[i] = mi;
      s1[i] = vi;
      float vd = vi;
      if (s2) {                                                   // amsgrad: max_exp_avg_sq
        vd = fmaxf(s2[i], vi);
        s2[i] = vd;
      }
      const float denom = sqrtf(vd) / h.bc2_sqrt + h.eps;
      pi = pi - h.step_size * (mi / denom);
    } else if constexpr (KIND == OPT_RMSPROP) {
      const float vi = s0[i] * h.b2 + h.omb2 * gi * gi;         // b2 = alpha
      s0[i] = vi;
      pi = pi - h.step_size * (gi / (sqrtf(vi) + h.eps));
    } else {                                                      // SGD with momentum b1, dampening 0
      // torch: _foreach_mul_(bufs, momentum) then _foreach_add_(bufs, grads): two roundings, no FMA
      const float bi = h.first ? gi : __fadd_rn(__fmul_rn(s0[i], h.b1), gi);
      s0[i] = bi;
      pi = pi - h.step_size * bi;
    }
    p[i] = pi;
    if (shadow) shadow[i] = h.ommu * pi + h.mu * shadow[i];
  }
}

hipError_t optim_ema(int kind, float* p, const float* g, float* s0, float* s1, float* s2, float* shadow, size_t n,
                     const OptimHyper& h, hipStream_t st) {
  const dim3 grid(grid_for(n)), block(256);
  switch (kind) {
    case OPT_ADAM: hipLaunchKernelGGL(optim_ema_kernel<OPT_ADAM>, grid, block, 0, st, p, g, s0, s1, s2, shadow, n, h); break;
    case OPT_RMSPROP: hipLaunchKernelGGL(optim_ema_kernel<OPT_RMSPROP>, grid, block, 0, st, p, g, s0, s1, s2, shadow, n, h); break;
    case OPT_SGD: hipLaunchKernelGGL(optim_ema_kernel<OPT_SGD>, grid, block, 0, st, p, g, s0, s1, s2, shadow, n, h); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace sdp
