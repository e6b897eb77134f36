// Shape dispatch of the forward convolutions of NCSN_LiDAR_small (kernel: conv_kernel.h;
// launchers: conv_launch.h, instantiated per shape in conv_inst.hip).
#include <cstdlib>

#include "conv_launch.h"
#include "wino_launch.h"

// preferred tile width of the 128 px x 256 Cout workgroups (A/B knob): 32 = 4 x 32 tiles, 64 = 2 x 64,
// 16 = 8 x 16 (bf16 modes on the 16x16 shape only)
#ifndef SDP_TC_WM1
#define SDP_TC_WM1 16
#endif
// tile width of the 256 px x 128 Cout workgroups: 32 = 8 x 32 tiles, 16 = 16 x 16 (16x16 shape only)
#ifndef SDP_TC_WM2
#define SDP_TC_WM2 32
#endif

namespace sdp {

// 128-channel outputs on 2-wave workgroups (128 px x 128 Cout, two per CU) instead of 256 px x 128
// Cout (one per CU): SDP_HALF=0 turns it off
static int half_wg() {   // 0 = off, 1 = 128-channel outputs, 2 = also the 256-channel outputs
  static const int h = [] {
    const char* e = getenv("SDP_HALF");
    return e ? atoi(e) : 1;
  }();
  return h;
}

template <int MODE, bool PELU>
static hipError_t launch_elu(const ConvArgs& a, int ks, bool pool, int wm, int tc, bool half, hipStream_t st) {
  if (ks == 1)   // the ConvMeanPool 1x1 shortcut: pooled epilogue (training), or on pre-pooled input (forward)
    return pool ? conv_launch<MODE, 1, 64, 1, true, PELU>(a, st) : conv_launch<MODE, 1, 64, 1, false, PELU>(a, st);
  if (pool) return conv_launch<MODE, 1, 64, 3, true, PELU>(a, st);
  if constexpr (MODE != MODE_F32) {   // 16-wide tiles: the 16x16 MFMA shape only
#ifndef SDP_CONV_BENCH_ONLY
    if (half) return conv_launch_half<MODE, PELU>(a, st);
#endif
    if (tc == 16) return wm == 2 ? conv_launch<MODE, 2, 16, 3, false, PELU>(a, st) : conv_launch<MODE, 1, 16, 3, false, PELU>(a, st);
  }
  if (wm == 2) return conv_launch<MODE, 2, 32, 3, false, PELU>(a, st);
  return tc == 64 ? conv_launch<MODE, 1, 64, 3, false, PELU>(a, st) : conv_launch<MODE, 1, 32, 3, false, PELU>(a, st);
}

template <int MODE>
static hipError_t launch_mode(const ConvArgs& a, int ks, bool pool, int wm, int tc, hipStream_t st, bool half = false) {
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench: only the 3x3 non-pooled ELU-prologue kernels
  if constexpr (MODE != MODE_F32) {
    if (half) return conv_launch_half<MODE, true>(a, st);
  }
  if (wm == 2) return conv_launch<MODE, 2, 32, 3, false, true>(a, st);
  return tc == 64 ? conv_launch<MODE, 1, 64, 3, false, true>(a, st) : conv_launch<MODE, 1, 32, 3, false, true>(a, st);
#else
  return a.pro_mode == PRO_NONE ? launch_elu<MODE, false>(a, ks, pool, wm, tc, half, st)
                                : launch_elu<MODE, true>(a, ks, pool, wm, tc, half, st);
#endif
}

// Winograd F(2,3) path (wino_kernel.h): the circular 3x3 non-pooled forward convs in the bf16 modes
// whose sub-grid tiles into 8 x 16 pixels.  SDP_WINO (bit mask, default 3): 1 = 256-channel outputs
// (128 px x 256 Cout workgroups), 2 = 128-channel outputs (128 px x 128 Cout); 0 = direct only
// (default while the Winograd kernel is slower than the direct one).
#ifndef SDP_CONV_BENCH_ONLY
static int wino_mask() {
  static const int m = [] {
    const char* e = getenv("SDP_WINO");
    return e ? atoi(e) : 0;
  }();
  return m;
}

template <int MODE>
static hipError_t wino_mode(const ConvArgs& a, int wm, hipStream_t st) {
  if (wm == 1) return a.pro_mode == PRO_NONE ? wino_launch<MODE, 1, false>(a, st) : wino_launch<MODE, 1, true>(a, st);
  return a.pro_mode == PRO_NONE ? wino_launch<MODE, 2, false>(a, st) : wino_launch<MODE, 2, true>(a, st);
}
#endif

// Host entry: validates the shape contract the kernel's indexing assumes, then launches.
hipError_t conv_mfma(int mode, ConvArgs a, int ks, bool pool, hipStream_t st, const char** why) {
  const int d = a.dil;
#ifndef SDP_CONV_BENCH_ONLY   // (tools/conv_bench times the direct kernel; tools/wino_bench the Winograd one)
  if (a.wfw && mode != MODE_F32 && ks == 3 && !pool && a.circular && !a.dact && a.Cin % 64 == 0 && a.H % d == 0 &&
      a.W % d == 0 && (a.H / d) % 8 == 0 && (a.W / d) % 16 == 0 && a.pro_ss &&
      (a.Cin <= 1024 || a.ss_bstride != 0)) {
    const int wm = a.Cout % 256 == 0 ? 1 : (a.Cout % 128 == 0 ? 2 : 0);
    if (wm && (wino_mask() & wm)) return mode == MODE_F32X3 ? wino_mode<MODE_F32X3>(a, wm, st) : wino_mode<MODE_BF16>(a, wm, st);
  }
#endif
  if (a.Cin % 64 || a.Cout % 128) { *why = "conv: Cin%64 and Cout%128 required"; return hipErrorInvalidValue; }
  if (a.H % d || a.W % d) { *why = "conv: H,W must be multiples of the dilation"; return hipErrorInvalidValue; }
  const int Hs = a.H / d, Ws = a.W / d;
  // 256-channel outputs: 128 px x 256 Cout tiles; 128-channel outputs: 256 px x 128 Cout
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench: SDP_WM=1|2 forces the workgroup shape
  const char* wm_env = getenv("SDP_WM");
  const int wm = wm_env ? atoi(wm_env) : ((a.Cout % 256 == 0) ? 1 : 2);
#else
  const int wm = (a.Cout % 256 == 0) ? 1 : 2;
#endif
  // 128 px x 256 Cout workgroups: 4 x 32 tiles (6 x 34 patch, 1.59x the pixels) where the sub-grid
  // allows, else 2 x 64 (4 x 66 patch, 2.06x) -- 4 x 32 measured 171.4 -> 167.0 us per 256->256
  // @32x512 launch (profiles/experiments/r02_tile_width_ab.log)
  // 16-wide tiles exist for the 16x16 MFMA shape (bf16 modes) only
  const bool sh16 = mode != MODE_F32 && !getenv("SDP_MFMA_SHAPE");
  const int tpref = (SDP_TC_WM1 == 16 && !sh16) ? 32 : SDP_TC_WM1;
  const int talt = tpref == 32 ? 64 : 32;
  int tc = (wm == 2) ? ((SDP_TC_WM2 == 16 && sh16 && Ws % 16 == 0 && Hs % 16 == 0) ? 16 : 32)
                     : ((Ws % tpref == 0 && Hs % (128 / tpref) == 0) ? tpref
                                                                     : ((Ws % talt == 0 && Hs % (128 / talt) == 0) ? talt : 32));
#ifdef SDP_CONV_BENCH_ONLY   // SDP_TC=32|64 forces the tile width of the WM=1 shape
  if (wm == 1 && getenv("SDP_TC")) tc = atoi(getenv("SDP_TC"));
#endif
  if (ks == 1 || pool) tc = 64;
  const int tr = wm * 128 / tc;
  if (Ws % tc || Hs % tr) { *why = "conv: sub-grid not divisible by the pixel tile"; return hipErrorInvalidValue; }
  if (ks == 1 && !pool && (d != 1 || wm != 1)) { *why = "conv: 1x1 needs d=1 and 256-multiple Cout"; return hipErrorInvalidValue; }
  if (pool && (d != 1 || wm != 1 || (a.H & 1) || (a.W & 1))) {
    *why = "conv: pooling needs d=1, even H,W and 256-multiple Cout";
    return hipErrorInvalidValue;
  }
  if (a.up && ((a.H & 1) || (a.W & 1) || a.H < 2 || a.W < 2)) { *why = "conv: upsample needs even H,W"; return hipErrorInvalidValue; }
  if (!a.circular && d != 1) { *why = "conv: zero padding only for d=1"; return hipErrorInvalidValue; }
  if (!a.pro_ss) { *why = "conv: prologue scale/shift table missing"; return hipErrorInvalidValue; }
  if (a.Cin > 1024 && a.ss_bstride == 0) { *why = "conv: identity table holds 1024 channels"; return hipErrorInvalidValue; }
  // 128-channel outputs: 2-wave workgroups of 8 x 16 pixels (16x16 shape, 3x3 non-pooled)
  const bool half = (wm == 2 ? half_wg() >= 1 : half_wg() >= 2) && sh16 && ks == 3 && !pool && Ws % 16 == 0 &&
                    Hs % 8 == 0;
#ifdef SDP_CONV_BENCH_ONLY
  if (mode == MODE_BF16) return launch_mode<MODE_BF16>(a, ks, pool, wm, tc, st, half);
  if (mode == MODE_F32) return launch_mode<MODE_F32>(a, ks, pool, wm, tc, st);
  return launch_mode<MODE_F32X3>(a, ks, pool, wm, tc, st, half);
#endif
  switch (mode) {
    case MODE_F32: return launch_mode<MODE_F32>(a, ks, pool, wm, tc, st);
    case MODE_F32X3: return launch_mode<MODE_F32X3>(a, ks, pool, wm, tc, st, half);
    default: return launch_mode<MODE_BF16>(a, ks, pool, wm, tc, st, half);
  }
}

}  // namespace sdp
