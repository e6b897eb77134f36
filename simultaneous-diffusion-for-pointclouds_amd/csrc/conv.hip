// Implicit-GEMM convolution on MFMA for the NCSN/RefineNet score network (gfx950).
//
// Covers every 3x3 conv of NCSN_LiDAR_small except begin/end conv:
//   conv3x3 circular (LiDARGen/models/layers.py:37-44), dilated_conv3x3 circular
//   (layers.py:55-60), ConvMeanPool 3x3/1x1 zero-pad + 2x2 mean (layers.py:291-313).
//
// GEMM view: M = output pixels, N = Cout, K = taps x Cin.  One 256-thread workgroup owns
// a 128-pixel x 128-channel output tile; 4 waves each own 64 px x 64 ch = 2x2 blocks of a
// 32x32 MFMA tile.  Dilated convs are run on their d x d polyphase sub-grids, so a tile is
// always TR x TC pixels of one sub-grid and its input patch has a 1-pixel halo whatever d.
// Per 32-channel chunk the (TR+2)x(TC+2) input patch is staged once into LDS -- with the
// consumer-side prologue (ELU or InstanceNorm++ affine + ELU) applied on the way -- and
// reused by all 9 taps.  Weights are pre-arranged on the host in MFMA fragment order and
// streamed from L2 straight into VGPRs (one tap ahead).
//
// MODE_F32   : v_mfma_f32_32x32x2_f32 on fp32 operands (exact fp32 products).
// MODE_F32X3 : operands split x = hi + lo (bf16 each), acc += hi*hi + hi*lo + lo*hi on
//              v_mfma_f32_32x32x16_bf16 -- error ~2e-5 of max|out| on the full network
//              (fp32 alone ~2e-6), 16x the issue rate of the fp32 MFMA per pass.
// MODE_BF16  : hi*hi only.
//
// Epilogue (fused): +bias, 2x2 mean-pool, +residual, +bilinear upsample of a half-res
// tensor, ELU, a second output (value + res2), and per-tile InstanceNorm++ statistics.
#include <type_traits>

#include "common.h"

namespace sdp {

constexpr int PSTRIDE = 144;  // bytes per staged patch pixel: 32 ch x (hi,lo bf16) or 32 x f32, + 16 pad

template <int TC, int KS>
struct ConvTile {
  static constexpr int TR = 128 / TC;
  static constexpr int HALO = KS == 3 ? 1 : 0;
  static constexpr int PC = TC + 2 * HALO;
  static constexpr int PR = TR + 2 * HALO;
  static constexpr int NPIX = PR * PC;
  static constexpr int NU = (NPIX * 8 + 255) / 256;            // 16-B staging units per thread per chunk
  static constexpr int PATCH_BYTES = NPIX * PSTRIDE;            // transformed (hi|lo or f32) patch
  static constexpr int RAW_BYTES = NU * 256 * 16;               // raw fp32 patch landed by LDS-DMA
  static constexpr int LDS_BYTES = PATCH_BYTES + RAW_BYTES;
};

SDP_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int MODE, int TC, int KS, bool POOL>
__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
  using T = ConvTile<TC, KS>;
  constexpr int NT = KS * KS;
  __shared__ __attribute__((aligned(16))) char lds[T::LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int d = a.dil, Hs = a.H / d, Ws = a.W / d;
  const int tiles_c = Ws / TC, tiles_rc = (Hs / T::TR) * tiles_c;
  int t = blockIdx.x;
  const int b = t / a.tiles_per_img;
  const int tile = t - b * a.tiles_per_img;
  t = tile;
  const int ph = t / tiles_rc;
  t -= ph * tiles_rc;
  const int ph_r = ph / d, ph_c = ph - (ph / d) * d;
  const int sr0 = (t / tiles_c) * T::TR, sc0 = (t % tiles_c) * TC;
  const int n0 = blockIdx.y * 128;
  const int trow0 = (TC == 64) ? 0 : 2 * wm;      // wave's 2 output rows: trow0, trow0+1
  const int tcol0 = (TC == 64) ? 32 * wm : 0;     // wave's 32 output columns

  const int Cin = a.Cin, Cout = a.Cout;
  const int nchunks = Cin / 32;
  const int NB = Cout / 32;
  const int nbg0 = n0 / 32 + wn * 2;               // global 32-channel block of this wave's nb=0

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // weight fragments through a buffer resource: lane offset in a VGPR (fixed per nb), the
  // (chunk, tap) offset in an SGPR -> no per-load address arithmetic
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wf, 0, 0x7fffffff, 0x00020000);
  const int wv0 = ((nbg0 + 0) * 64 + lane) * 64, wv1 = ((nbg0 + 1) * 64 + lane) * 64;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  uint4 bq[2][2][4];
  auto load_b = [&](auto buf, int chunk, int tap) __attribute__((always_inline)) {
    constexpr int J = decltype(buf)::value;
    const int so = __builtin_amdgcn_readfirstlane(((chunk * NT + tap) * NB) * 4096);
    static_for<0, 4>([&](auto q) {
      const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(wrs, wv0 + q * 16, so, 0);
      const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(wrs, wv1 + q * 16, so, 0);
      bq[J][0][q] = make_uint4(v0.x, v0.y, v0.z, v0.w);
      bq[J][1][q] = make_uint4(v1.x, v1.y, v1.z, v1.w);
    });
  };
  load_b(std::integral_constant<int, 0>{}, 0, 0);

  const float* inb = a.in + (size_t)b * a.H * a.W * Cin;
  // scale/shift rows of this image; when there is no affine prologue point at any valid
  // memory (loads below are unconditional, their values unused)
  const float* ssb = a.pro_ss ? a.pro_ss + (size_t)b * Cin * 2 : a.in;

  // ---- patch staging, software-pipelined: the next chunk's global loads are issued into
  //      registers before this chunk's MFMA loop and written (prologue applied) after it ----
  constexpr int NU = T::NU;
  char* raw = lds + T::PATCH_BYTES;
  float4 ssv0 = make_float4(1.f, 0.f, 1.f, 0.f), ssv1 = ssv0;   // (scale, shift) of this thread's 4 channels
  const int my_cv = tid & 7;                                     // every unit of a thread has cv == tid % 8
  // Staging unit u = 16 B (4 channels) of one patch pixel.  Its byte offset inside the image
  // (clamped into range, so every load is unconditional) and its validity (zero padding)
  // depend only on the tile, so they are computed once; per chunk only the scalar channel
  // offset changes.
  const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc((void*)inb, 0, 0x7fffffff, 0x00020000);
  int uoff[NU];
  unsigned uvalid = 0;
  static_for<0, NU>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    int u = tid + k * 256;
    bool valid = u < T::NPIX * 8;
    u = valid ? u : 0;
    const int pix = u >> 3, cv = u & 7;
    const int pr = pix / T::PC, pc = pix - pr * T::PC;
    int sr = sr0 - T::HALO + pr, sc = sc0 - T::HALO + pc;
    if (a.circular) {
      sr = sr < 0 ? sr + Hs : (sr >= Hs ? sr - Hs : sr);
      sc = sc < 0 ? sc + Ws : (sc >= Ws ? sc - Ws : sc);
    } else {
      valid = valid && sr >= 0 && sr < Hs && sc >= 0 && sc < Ws;
      sr = min(max(sr, 0), Hs - 1);
      sc = min(max(sc, 0), Ws - 1);
    }
    const int y = sr * d + ph_r, x = sc * d + ph_c;
    uoff[k] = ((y * a.W + x) * Cin + cv * 4) * 4;   // bytes, < 2^31 for every admitted shape
    uvalid |= (valid ? 1u : 0u) << k;
  });
  // LDS-DMA of staging unit k (no VGPR destination): lane i of a wave lands 16 B at the
  // wave-uniform base + 16*i, i.e. unit u at raw + 16*u
  auto load_unit = [&](auto kc, int chunk) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if ((tid & ~63) + k * 256 >= T::NPIX * 8) return;   // whole wave past the patch (wave-uniform)
    const int base = __builtin_amdgcn_readfirstlane(((tid & ~63) + k * 256) * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        irs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(raw + base)), 16,
        uoff[k], chunk * 128, 0, 0);
  };
  auto load_ss = [&](int chunk) __attribute__((always_inline)) {
    ssv0 = ld4(ssb + (chunk * 32 + my_cv * 4) * 2);
    ssv1 = ld4(ssb + (chunk * 32 + my_cv * 4) * 2 + 4);
  };
  auto write_patch = [&]() __attribute__((always_inline)) {
    static_for<0, NU>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int u = tid + k * 256;
      if (u >= T::NPIX * 8) return;
      const int pix = u >> 3, cv = u & 7;
      float4 v = *reinterpret_cast<const float4*>(raw + u * 16);
      const bool valid = (uvalid >> k) & 1u;
      if (!valid) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid) {
        if (a.pro_mode == PRO_AFFINE_ELU) {
          v.x = elu(fmaf(v.x, ssv0.x, ssv0.y));
          v.y = elu(fmaf(v.y, ssv0.z, ssv0.w));
          v.z = elu(fmaf(v.z, ssv1.x, ssv1.y));
          v.w = elu(fmaf(v.w, ssv1.z, ssv1.w));
        } else if (a.pro_mode == PRO_ELU) {
          v.x = elu(v.x); v.y = elu(v.y); v.z = elu(v.z); v.w = elu(v.w);
        }
      }
      char* dst = lds + pix * PSTRIDE;
      if constexpr (MODE == MODE_F32) {
        *reinterpret_cast<float4*>(dst + cv * 16) = v;
      } else {
        bf16x4 hi, lo;
        hi[0] = (__bf16)v.x; hi[1] = (__bf16)v.y; hi[2] = (__bf16)v.z; hi[3] = (__bf16)v.w;
        *reinterpret_cast<bf16x4*>(dst + cv * 8) = hi;
        if constexpr (MODE == MODE_F32X3) {
          lo[0] = (__bf16)(v.x - (float)hi[0]);
          lo[1] = (__bf16)(v.y - (float)hi[1]);
          lo[2] = (__bf16)(v.z - (float)hi[2]);
          lo[3] = (__bf16)(v.w - (float)hi[3]);
          *reinterpret_cast<bf16x4*>(dst + 64 + cv * 8) = lo;
        }
      }
    });
  };

  load_ss(0);
  static_for<0, NU>([&](auto k) { load_unit(k, 0); });
  auto do_chunk = [&](auto parity, int chunk) __attribute__((always_inline)) {
    constexpr int P = decltype(parity)::value;
    __syncthreads();
    write_patch();
    __syncthreads();
    const bool more = chunk + 1 < nchunks;

    // ---- 9 (or 1) taps over the staged patch; per tap: prefetch the next tap's weight
    //      fragments, issue a slice of the next chunk's patch loads, then the MFMAs ----
    static_for<0, NT>([&](auto tap_c) {
      constexpr int tap = decltype(tap_c)::value;
      constexpr int CUR = (tap + P) & 1, NXT = (tap + 1 + P) & 1;
      if constexpr (tap + 1 < NT) load_b(std::integral_constant<int, NXT>{}, chunk, tap + 1);
      else if (more) load_b(std::integral_constant<int, NXT>{}, chunk + 1, 0);
      if (more) {
        if constexpr (tap == 0) load_ss(chunk + 1);
        static_for<0, NU>([&](auto kc) {
          if constexpr (decltype(kc)::value % NT == tap) load_unit(kc, chunk + 1);
        });
      }
      // keep the prefetches ahead of this tap's MFMAs (hipcc otherwise sinks them to the end
      // of the tap, exposing their latency at the next tap)
      __builtin_amdgcn_sched_barrier(0);
      const int kh = (KS == 3) ? tap / 3 : 0, kw = (KS == 3) ? tap % 3 : 0;
      if constexpr (MODE == MODE_F32) {
        float av[2][16];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
          const int pix = (trow0 + mb + kh) * T::PC + tcol0 + (lane & 31) + kw;
          const char* src = lds + pix * PSTRIDE + (lane >> 5) * 64;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 f = *reinterpret_cast<const float4*>(src + q * 16);
            av[mb][4 * q + 0] = f.x; av[mb][4 * q + 1] = f.y; av[mb][4 * q + 2] = f.z; av[mb][4 * q + 3] = f.w;
          }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            const uint4 bv = bq[CUR][nb][k >> 2];
            const uint32_t bw = (k & 3) == 0 ? bv.x : (k & 3) == 1 ? bv.y : (k & 3) == 2 ? bv.z : bv.w;
            const float bf = __uint_as_float(bw);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mb][k], bf, acc[mb][nb], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 ahi[2], alo[2];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            const int pix = (trow0 + mb + kh) * T::PC + tcol0 + (lane & 31) + kw;
            const char* src = lds + pix * PSTRIDE + s * 32 + (lane >> 5) * 16;
            ahi[mb] = *reinterpret_cast<const bf16x8*>(src);
            if constexpr (MODE == MODE_F32X3) alo[mb] = *reinterpret_cast<const bf16x8*>(src + 64);
          }
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            const uint4 h4 = bq[CUR][nb][2 * s], l4 = bq[CUR][nb][2 * s + 1];
            const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(&h4);
            const bf16x8 blo = *reinterpret_cast<const bf16x8*>(&l4);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
              if constexpr (MODE == MODE_F32X3) {
                acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[mb], bhi, acc[mb][nb], 0, 0, 0);
                acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mb], blo, acc[mb][nb], 0, 0, 0);
              }
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mb], bhi, acc[mb][nb], 0, 0, 0);
            }
          }
        }
      }
    });
  };
  static_assert(NT % 2 == 1, "parity bookkeeping assumes an odd tap count");
  for (int chunk = 0; chunk < nchunks; chunk += 2) {   // nchunks is even (Cin % 64 == 0)
    do_chunk(std::integral_constant<int, 0>{}, chunk);
    do_chunk(std::integral_constant<int, 1>{}, chunk + 1);
  }

  // ------------------------------------------------------------------ epilogue
  // C/D layout of 32x32 MFMA: col (N) = lane&31, row (M) = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int col_lane = lane & 31;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  constexpr int NV = POOL ? 8 : 32;  // values per lane per nb
  // per-lane Welford state over this lane's NV outputs of each channel (InstanceNorm++ stats)
  float wmean[2] = {0.f, 0.f}, wm2[2] = {0.f, 0.f};
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int co = n0 + wn * 64 + nb * 32 + col_lane;
    const float bias = a.bias ? a.bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float v;
      int y, x;
      if constexpr (POOL) {
        const int r = 2 * i;  // regs r, r+1 hold adjacent columns
        const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float o00 = acc[0][nb][r] + bias, o10 = acc[1][nb][r] + bias;
        const float o01 = acc[0][nb][r + 1] + bias, o11 = acc[1][nb][r + 1] + bias;
        v = (((o00 + o10) + o01) + o11) / 4.0f;  // layers.py:310-312 summation order
        y = (sr0 + trow0) >> 1;
        x = (sc0 + tcol0 + m) >> 1;
      } else {
        const int mb = i >> 4, r = i & 15;
        const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        v = acc[mb][nb][r] + bias;
        y = (sr0 + trow0 + mb) * d + ph_r;
        x = (sc0 + tcol0 + m) * d + ph_c;
      }
      const size_t oidx = (((size_t)b * Ho + y) * Wo + x) * Cout + co;
      if (a.up) {
        // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor at (y, x)
        const int Hi = a.H / 2, Wi = a.W / 2;
        const float sh = (float)(Hi - 1) / (float)(a.H - 1), sw = (float)(Wi - 1) / (float)(a.W - 1);
        const float fy = sh * (float)y, fx = sw * (float)x;
        const int y0 = (int)fy, x0 = (int)fx;
        const int yp = y0 < Hi - 1 ? 1 : 0, xp = x0 < Wi - 1 ? 1 : 0;
        const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
        const float* ub = a.up + (size_t)b * Hi * Wi * Cout + co;
        const float v00 = ub[((size_t)y0 * Wi + x0) * Cout], v01 = ub[((size_t)y0 * Wi + x0 + xp) * Cout];
        const float v10 = ub[((size_t)(y0 + yp) * Wi + x0) * Cout], v11 = ub[((size_t)(y0 + yp) * Wi + x0 + xp) * Cout];
        v = v + (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11));
      }
      if (a.res) v = a.res[oidx] + v;
      if (a.out2) a.out2[oidx] = v + a.res2[oidx];
      if (a.epi_elu) v = elu(v);
      a.out[oidx] = v;
      const float delta = v - wmean[nb];
      wmean[nb] = fmaf(delta, 1.0f / (float)(i + 1), wmean[nb]);
      wm2[nb] = fmaf(delta, v - wmean[nb], wm2[nb]);
      // keep the compiler from hoisting every epilogue load at once (VGPR spills)
      if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }

  if (a.stats) {
    // Chan merge of equal-count partials: lanes l/l+32 (NV each), then waves wm=0/1 via LDS.
    constexpr float CNT = POOL ? 32.f : 128.f;
    float* red = reinterpret_cast<float*>(lds);  // [wn][nb][wm][32][2]
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const float om = __shfl_xor(wmean[nb], 32), o2 = __shfl_xor(wm2[nb], 32);
      const float dm = om - wmean[nb];
      const float mean = 0.5f * (wmean[nb] + om);
      const float m2 = wm2[nb] + o2 + dm * dm * (0.5f * NV);
      if (lane < 32) {
        float* r = red + (((wn * 2 + nb) * 2 + wm) * 32 + lane) * 2;
        r[0] = mean;
        r[1] = m2;
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 32) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float* r0 = red + (((wn * 2 + nb) * 2 + 0) * 32 + lane) * 2;
        const float* r1 = red + (((wn * 2 + nb) * 2 + 1) * 32 + lane) * 2;
        const float dm = r1[0] - r0[0];
        const float mean = 0.5f * (r0[0] + r1[0]);
        const float m2 = r0[1] + r1[1] + dm * dm * (0.25f * CNT);
        const int co = n0 + wn * 64 + nb * 32 + lane;
        float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.tiles_per_img + tile) * Cout + co;
        *st = make_float2(mean, m2);
      }
    }
  }
#endif
}

// ----------------------------------------------------------------------------- launch
template <int MODE, int TC, int KS, bool POOL>
static hipError_t launch_t(const ConvArgs& a, hipStream_t st) {
  dim3 grid(a.B * a.tiles_per_img, a.Cout / 128);
  hipLaunchKernelGGL((conv_mfma_kernel<MODE, TC, KS, POOL>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_mode(const ConvArgs& a, int ks, bool pool, int tc, hipStream_t st) {
  if (ks == 1) return launch_t<MODE, 64, 1, true>(a, st);   // only the ConvMeanPool 1x1 shortcut
  if (pool) return tc == 64 ? launch_t<MODE, 64, 3, true>(a, st) : launch_t<MODE, 32, 3, true>(a, st);
  return tc == 64 ? launch_t<MODE, 64, 3, false>(a, st) : launch_t<MODE, 32, 3, false>(a, st);
}

// Host entry: validates the shape contract the kernel's indexing assumes, then launches.
hipError_t conv_mfma(int mode, ConvArgs a, int ks, bool pool, hipStream_t st, const char** why) {
  const int d = a.dil;
  if (a.Cin % 64 || a.Cout % 128) { *why = "conv: Cin%64 and Cout%128 required"; return hipErrorInvalidValue; }
  if (a.H % d || a.W % d) { *why = "conv: H,W must be multiples of the dilation"; return hipErrorInvalidValue; }
  const int Hs = a.H / d, Ws = a.W / d;
  int tc = (Ws % 64 == 0) ? 64 : 32;
  if (ks == 1) tc = 64;
  const int tr = 128 / tc;
  if (Ws % tc || Hs % tr) { *why = "conv: sub-grid not divisible by the 128-pixel tile"; return hipErrorInvalidValue; }
  if (ks == 1 && !pool) { *why = "conv: 1x1 only as the pooled shortcut"; return hipErrorInvalidValue; }
  if (pool && (d != 1 || (a.H & 1) || (a.W & 1))) { *why = "conv: pooling needs d=1, even H,W"; return hipErrorInvalidValue; }
  if (a.up && ((a.H & 1) || (a.W & 1) || a.H < 2 || a.W < 2)) { *why = "conv: upsample needs even H,W"; return hipErrorInvalidValue; }
  if (!a.circular && d != 1) { *why = "conv: zero padding only for d=1"; return hipErrorInvalidValue; }
  a.tiles_per_img = a.H * a.W / 128;
  switch (mode) {
    case MODE_F32: return launch_mode<MODE_F32>(a, ks, pool, tc, st);
    case MODE_F32X3: return launch_mode<MODE_F32X3>(a, ks, pool, tc, st);
    default: return launch_mode<MODE_BF16>(a, ks, pool, tc, st);
  }
}

}  // namespace sdp
