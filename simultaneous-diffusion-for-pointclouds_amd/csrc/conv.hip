// Shape dispatch of the forward convolutions of NCSN_LiDAR_small (kernel: conv_kernel.h;
// launchers: conv_launch.h, instantiated per shape in conv_inst.hip).
#include "conv_launch.h"

namespace sdp {

// The 16-wide 3x3 forward tiles on 32-Cout waves, two per SIMD (conv_launch_nj2): the 128-Cout layers
// in both bf16 modes (4-wave workgroups, two per CU: 128->128 @64x1024 203.7 -> 184.4 us per fp32x3 B=4
// launch in the network, line 333.7-336.1 -> 345.0-345.1 image-steps/s), the 256-Cout layers in bf16
// (8-wave workgroups: 87.4 -> 80.8-85.4 us per B=4 launch; in fp32x3 they measured slower, 163.0 ->
// 165.8 us, and keep one 64-Cout wave per SIMD) -- profiles/experiments/r05_nj2_ab.log.
// The fp32x3 256-Cout layers run as two of those 128-Cout workgroups per tile (the patch is staged
// twice, and 8 waves per CU hide each other's phases): line 348.6-348.9 -> 356.6-357.5
// image-steps/s, 256->256 160.9-162.4 -> 159.7-161.5 us per launch (profiles/experiments/
// r05_pair256_ab.log).  SDP_CONV_NJ2=0 (build-time A/B only, tools/lib_variant.sh) restores the
// 64-Cout waves; SDP_CONV_NJ2_BF16_W8 picks the 8-wave workgroups for the bf16 256-Cout layers.
#ifndef SDP_CONV_NJ2
#define SDP_CONV_NJ2 1
#endif
#ifndef SDP_CONV_NJ2_BF16_W8
#define SDP_CONV_NJ2_BF16_W8 1
#endif

template <int MODE, bool PELU>
static hipError_t launch_elu(const ConvArgs& a, int ks, bool pool, int wm, int tc, bool half, hipStream_t st) {
  if (ks == 1)   // the ConvMeanPool 1x1 shortcut: pooled epilogue (training), or on pre-pooled input (forward)
    return pool ? conv_launch<MODE, 1, 64, 1, true, PELU>(a, st) : conv_launch<MODE, 1, 64, 1, false, PELU>(a, st);
  if (pool) return conv_launch<MODE, 1, 64, 3, true, PELU>(a, st);
  if constexpr (MODE != MODE_F32) {   // 16-wide tiles: the 16x16 MFMA shape only
    if (half) return SDP_CONV_NJ2 ? conv_launch_nj2<MODE, PELU, 4>(a, st) : conv_launch_half<MODE, PELU>(a, st);
    if (tc == 16) {   // the 256-Cout layers: two 128-Cout workgroups per tile (fp32x3), one 8-wave one (bf16)
      if (!SDP_CONV_NJ2) return conv_launch<MODE, 1, 16, 3, false, PELU>(a, st);
      return (MODE == MODE_BF16 && SDP_CONV_NJ2_BF16_W8) ? conv_launch_nj2<MODE, PELU, 8>(a, st)
                                                         : conv_launch_nj2<MODE, PELU, 4>(a, st);
    }
  }
  if (wm == 2) return conv_launch<MODE, 2, 32, 3, false, PELU>(a, st);
  return tc == 64 ? conv_launch<MODE, 1, 64, 3, false, PELU>(a, st) : conv_launch<MODE, 1, 32, 3, false, PELU>(a, st);
}

template <int MODE>
static hipError_t launch_mode(const ConvArgs& a, int ks, bool pool, int wm, int tc, hipStream_t st, bool half = false) {
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench: only the 3x3 non-pooled ELU-prologue kernels
  if constexpr (MODE != MODE_F32) {
    if (half) return SDP_CONV_NJ2 ? conv_launch_nj2<MODE, true, 4>(a, st) : conv_launch_half<MODE, true>(a, st);
    if (!SDP_CONV_NJ2) return conv_launch<MODE, 1, 16, 3, false, true>(a, st);
    return (MODE == MODE_BF16 && SDP_CONV_NJ2_BF16_W8) ? conv_launch_nj2<MODE, true, 8>(a, st)
                                                       : conv_launch_nj2<MODE, true, 4>(a, st);
  }
  if (wm == 2) return conv_launch<MODE, 2, 32, 3, false, true>(a, st);
  return conv_launch<MODE, 1, 32, 3, false, true>(a, st);
#else
  return a.pro_mode == PRO_NONE ? launch_elu<MODE, false>(a, ks, pool, wm, tc, half, st)
                                : launch_elu<MODE, true>(a, ks, pool, wm, tc, half, st);
#endif
}

// Host entry: validates the shape contract the kernel's indexing assumes, then launches.
//
// Workgroup shapes (conv_kernel.h ConvTile):
//   bf16 modes (fp32x3, bf16; 16x16 MFMAs), 3x3 non-pooled layers whose sub-grid tiles into 8 x 16:
//     256-channel outputs: 128 px x 256 Cout, 8 x 16 pixel tiles (a 10 x 18 patch, 1.41x the pixels),
//       4 waves, one workgroup per CU (171.4 -> 167.0 -> ~164 us per 256->256 @32x512 launch against
//       4 x 32 / 2 x 64 tiles, profiles/experiments/r02_tile_width_ab.log);
//     128-channel outputs: 128 px x 128 Cout, 8 x 16 tiles, 2 waves, two workgroups per CU (one's
//       prologue and epilogue run under the other's MFMAs: 214.5 -> 211.0 us per 128->128 @64x1024
//       launch against 256 px x 128 Cout on 4 waves, profiles/experiments/r03_half_wg_128only.log);
//   exact fp32 (32x32 MFMAs, 32-pixel fragment rows): 4 x 32 tiles (2 x 64 where the sub-grid needs
//     it) of 128 px x 256 Cout, or 8 x 32 tiles of 256 px x 128 Cout;
//   pooled (ConvMeanPool) and 1x1 layers: 2 x 64 tiles of 128 px x 256 Cout.
hipError_t conv_mfma(int mode, ConvArgs a, int ks, bool pool, hipStream_t st, const char** why) {
  const int d = a.dil;
  if (a.Cin % 64 || a.Cout % 128) { *why = "conv: Cin%64 and Cout%128 required"; return hipErrorInvalidValue; }
  if (a.H % d || a.W % d) { *why = "conv: H,W must be multiples of the dilation"; return hipErrorInvalidValue; }
  const int Hs = a.H / d, Ws = a.W / d;
  const int wm = (a.Cout % 256 == 0) ? 1 : 2;
  const bool sh16 = mode != MODE_F32;
  int tc;
  if (sh16 && Ws % 16 == 0 && Hs % 8 == 0) tc = 16;
  else if (wm == 2) tc = 32;
  else tc = (Ws % 32 == 0 && Hs % 4 == 0) ? 32 : 64;
  if (!sh16 && tc == 16) tc = 32;
  if (ks == 1 || pool) tc = 64;
  // 16-wide tiles of 128-channel outputs: the 2-wave workgroups (128 px x 128 Cout)
  const bool half = sh16 && wm == 2 && tc == 16 && ks == 3 && !pool;
  const int tr = (half ? 128 : wm * 128) / tc;
  if (Ws % tc || Hs % tr) { *why = "conv: sub-grid not divisible by the pixel tile"; return hipErrorInvalidValue; }
  if (sh16 && !a.wf16) { *why = "conv: bf16 modes need the 16x16 weight packing (#frag16)"; return hipErrorInvalidValue; }
  if (!sh16 && !a.wf) { *why = "conv: exact fp32 needs the 32x32 weight packing (#frag)"; return hipErrorInvalidValue; }
  if (ks == 1 && !pool && (d != 1 || wm != 1)) { *why = "conv: 1x1 needs d=1 and 256-multiple Cout"; return hipErrorInvalidValue; }
  if (pool && (d != 1 || wm != 1 || (a.H & 1) || (a.W & 1))) {
    *why = "conv: pooling needs d=1, even H,W and 256-multiple Cout";
    return hipErrorInvalidValue;
  }
  if (a.up && ((a.H & 1) || (a.W & 1) || a.H < 2 || a.W < 2)) { *why = "conv: upsample needs even H,W"; return hipErrorInvalidValue; }
  if (!a.circular && d != 1) { *why = "conv: zero padding only for d=1"; return hipErrorInvalidValue; }
  if (!a.pro_ss) { *why = "conv: prologue scale/shift table missing"; return hipErrorInvalidValue; }
  if (a.Cin > 1024 && a.ss_bstride == 0) { *why = "conv: identity table holds 1024 channels"; return hipErrorInvalidValue; }
  if (a.io16) {   // the bf16 training tape: the shapes the training plan launches (conv_launch.h IO16)
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench io16: the 16-wide ELU-prologue tiles only
    if (mode == MODE_BF16 && ks == 3 && tc == 16 && !pool) return conv_launch_nj2<MODE_BF16, true, 4, true>(a, st);
#else
    if (mode != MODE_BF16) { *why = "conv: bf16 tensors (io16) need bf16 mode"; return hipErrorInvalidValue; }
    const bool pe = a.pro_mode != PRO_NONE;
    if (pool && ks == 1) return pe ? conv_launch<MODE_BF16, 1, 64, 1, true, true, true>(a, st)
                                   : conv_launch<MODE_BF16, 1, 64, 1, true, false, true>(a, st);
    if (pool) return pe ? conv_launch<MODE_BF16, 1, 64, 3, true, true, true>(a, st)
                        : conv_launch<MODE_BF16, 1, 64, 3, true, false, true>(a, st);
    // 16-wide tiles: 4-wave 128-Cout workgroups for both Cout widths (the 256-Cout layers as a pair per
    // tile): with 8-channel staging units an 8-wave workgroup leaves 29 % of its units empty (720 for 1024
    // slots) and ran the 256-class slower than the float32 tape (181 vs 168.5 us per B=8 launch)
    if (ks == 3 && tc == 16)
      return pe ? conv_launch_nj2<MODE_BF16, true, 4, true>(a, st) : conv_launch_nj2<MODE_BF16, false, 4, true>(a, st);
#endif
    *why = "conv: no bf16-tensor (io16) kernel for this shape";
    return hipErrorInvalidValue;
  }
  switch (mode) {
    case MODE_F32: return launch_mode<MODE_F32>(a, ks, pool, wm, tc, st);
    case MODE_F32X3: return launch_mode<MODE_F32X3>(a, ks, pool, wm, tc, st, half);
    default: return launch_mode<MODE_BF16>(a, ks, pool, wm, tc, st, half);
  }
}

}  // namespace sdp
