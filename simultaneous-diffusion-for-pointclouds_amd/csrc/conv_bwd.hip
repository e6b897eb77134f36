// Data gradient of the score network's convolutions (DSM training, LiDARGen/losses/dsm.py:67-119
// through NCSN_LiDAR_small).  A stride-1 conv with circular or zero padding is adjoint to the
// same conv over the output gradient with the kernel flipped in both taps and transposed in
// (Cin, Cout) -- circular padding stays circular, zero padding stays zero, a dilation stays
// the same dilation -- so the data gradient is the forward implicit-GEMM kernel
// (conv_kernel.h) run on dy with the "dgrad" weight packing (train_aux.hip pack kernel),
// without prologue, and with the backward epilogue: *elu'(...) of the forward activation
// (ConvArgs::dact) and the residual add of the gradient already accumulated for its input.
#include "conv_launch.h"

// preferred tile width of the 128 px x 256 Cout data-gradient workgroups (A/B knob; the forward's is
// SDP_TC_WM1 in conv.hip)
#ifndef SDP_DGRAD_TC_WM1
#define SDP_DGRAD_TC_WM1 64
#endif


// The 8 x 16 circular data gradients on 32-Cout waves, two per SIMD (dgrad_launch_nj2), as the forward:
// the 128-Cout layers in both modes, the 256-Cout layers in bf16 (bf16 training step 151.2-151.8 ->
// 151.7-152.5 image-steps/s, profiles/experiments/r05_dgrad_nj2_ab.log); SDP_DGRAD_NJ2=0 (build-time
// A/B only) restores the 64-Cout waves
#ifndef SDP_DGRAD_NJ2
#define SDP_DGRAD_NJ2 1
#endif
// the bf16 256-Cout data gradients on one 8-wave workgroup per tile: training 159.3-159.8 against
// 157.8-158.5 image-steps/s for two 4-wave 128-Cout ones (SDP_DGRAD_NJ2_BF16_W8=0, build-time A/B only;
// profiles/experiments/r05_dgrad_w8_vs_w4_ab.log)
#ifndef SDP_DGRAD_NJ2_BF16_W8
#define SDP_DGRAD_NJ2_BF16_W8 1
#endif

namespace sdp {

// 8 x 16 pixel tiles (the forward's: a 10 x 18 patch, 1.41x the pixels, against 4 x 66 = 2.06x for
// the 2 x 64 tiles) with the transposed direct 16x16 epilogue (conv_kernel.h TRN: 16-B elu' operand,
// residual and output accesses) -- the 128-channel outputs on 2-wave workgroups -- wherever the
// sub-grid tiles into 8 x 16 (every circular 3x3 layer of the network): bf16 training step 132.8 ->
// 137.0 image-steps/s against the 2 x 64 tiles (profiles/experiments/r03_dgrad16_train_ab.log,
// r03_trans_ab.log).  The zero-padded and 1x1 layers keep 2 x 64 / 8 x 32 tiles with the LDS-staged
// epilogue.

template <int MODE>
static hipError_t launch_dgrad_mode(const ConvArgs& a, int ks, int wm, int tc, bool t16, hipStream_t st) {
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench: the 8 x 16 circular 3x3 data gradients only
  if (!t16) return hipErrorInvalidValue;
  return wm == 2 ? dgrad_launch_half<MODE>(a, st) : dgrad_launch<MODE, 1, 16, 3, false>(a, st);
#endif
  if (ks == 1) return dgrad_launch<MODE, 2, 32, 1, false>(a, st);
  if (!a.circular) return dgrad_launch<MODE, 2, 32, 3, true>(a, st);
  if (t16) {
    if (wm == 2) return SDP_DGRAD_NJ2 ? dgrad_launch_nj2<MODE, 4>(a, st) : dgrad_launch_half<MODE>(a, st);
    if (SDP_DGRAD_NJ2 && MODE == MODE_BF16)
      return SDP_DGRAD_NJ2_BF16_W8 ? dgrad_launch_nj2<MODE, 8>(a, st) : dgrad_launch_nj2<MODE, 4>(a, st);
    return dgrad_launch<MODE, 1, 16, 3, false>(a, st);
  }
  if (wm == 2) return dgrad_launch<MODE, 2, 32, 3, false>(a, st);
  return tc == 64 ? dgrad_launch<MODE, 1, 64, 3, false>(a, st) : dgrad_launch<MODE, 1, 32, 3, false>(a, st);
}

// a.in = dy [B][H][W][Cin = forward Cout], a.wf = dgrad-packed weights, a.out = dx
// [B][H][W][Cout = forward Cin].  Same shape contract as conv_mfma, no pooling, no prologue.
hipError_t conv_dgrad(int mode, ConvArgs a, int ks, hipStream_t st, const char** why) {
  const int d = a.dil;
  if (a.Cin % 64 || a.Cout % 128) { *why = "dgrad: Cin%64 and Cout%128 required"; return hipErrorInvalidValue; }
  if (a.H % d || a.W % d) { *why = "dgrad: H,W must be multiples of the dilation"; return hipErrorInvalidValue; }
  if (a.pro_mode != PRO_NONE || a.up || a.out2 || a.stats) { *why = "dgrad: plain input, no fused extras"; return hipErrorInvalidValue; }
  const int Hs = a.H / d, Ws = a.W / d;
  const int wm = (a.Cout % 256 == 0 && ks == 3 && a.circular) ? 1 : 2;
  const int tpref = SDP_DGRAD_TC_WM1, talt = tpref == 32 ? 64 : 32;
  const int tc = (wm == 2) ? 32
                           : ((Ws % tpref == 0 && Hs % (128 / tpref) == 0) ? tpref
                                                                           : ((Ws % talt == 0 && Hs % (128 / talt) == 0) ? talt : 32));
  const int tr = wm * 128 / tc;
  if (Ws % tc || Hs % tr) { *why = "dgrad: sub-grid not divisible by the pixel tile"; return hipErrorInvalidValue; }
  if (!a.circular && d != 1) { *why = "dgrad: zero padding only for d=1"; return hipErrorInvalidValue; }
  if (a.dact && !a.aux) { *why = "dgrad: dact needs aux"; return hipErrorInvalidValue; }
  if (a.dact == 3 && !a.epi_ss) { *why = "dgrad: dact 3 needs epi_ss"; return hipErrorInvalidValue; }
  if (!a.pro_ss) { *why = "dgrad: prologue identity table missing"; return hipErrorInvalidValue; }
  if (!a.wf16) { *why = "dgrad: weights in wf16 (the #dfrag16 packing)"; return hipErrorInvalidValue; }
  const bool t16 = ks == 3 && a.circular && Ws % 16 == 0 && Hs % 8 == 0;
  if (a.io16) {   // the bf16 training tape: the shapes the training plan launches (conv_launch.h IO16)
#ifdef SDP_CONV_BENCH_ONLY   // tools/conv_bench io16: the 16-wide circular data gradients only
    if (mode == MODE_BF16 && t16) return dgrad_launch_nj2<MODE_BF16, 4, true>(a, st);
#else
    if (mode != MODE_BF16) { *why = "dgrad: bf16 tensors (io16) need bf16 mode"; return hipErrorInvalidValue; }
    if (ks == 1) return dgrad_launch<MODE_BF16, 2, 32, 1, false, true>(a, st);
    if (!a.circular) return dgrad_launch<MODE_BF16, 2, 32, 3, true, true>(a, st);
    if (t16) return dgrad_launch_nj2<MODE_BF16, 4, true>(a, st);   // 128-Cout workgroups (see conv.hip's io16 forward)
#endif
    *why = "dgrad: no bf16-tensor (io16) kernel for this shape";
    return hipErrorInvalidValue;
  }
  switch (mode) {
    case MODE_F32X3: return launch_dgrad_mode<MODE_F32X3>(a, ks, wm, tc, t16, st);
    case MODE_BF16: return launch_dgrad_mode<MODE_BF16>(a, ks, wm, tc, t16, st);
    default: *why = "dgrad: training runs in fp32x3 or bf16"; return hipErrorInvalidValue;
  }
}

}  // namespace sdp
