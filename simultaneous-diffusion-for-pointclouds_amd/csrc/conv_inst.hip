// Definitions + explicit instantiations of the conv launchers (conv_launch.h).
//
// Built once per kernel shape (Makefile: conv_i_<code>.o with -DSDP_INST=<code>):
//   forward : code = 100 * (mode + 1) + 10 * pelu + shape   (shape = index into FwdShape; 7 = the
//             2-wave workgroups of conv_launch_half; 8 = the non-pooled 1x1; 9 / 6 = the 32-Cout waves
//             of conv_launch_nj2 on 4 / 8 waves)
//   dgrad 2-wave workgroups: code = 1000 + 10 * mode + 6; 32-Cout waves on 4 / 8 waves: + 7 / + 8
//   dgrad   : code = 1000 + 10 * mode + shape                (shape = index into DgradShape)
// Without SDP_INST (tools/conv_bench, -DSDP_CONV_BENCH_ONLY) it instantiates the 3x3 non-pooled
// ELU-prologue forward shapes of every mode, which is all that bench dispatches.
#include "conv_kernel.h"
#include "conv_launch.h"

namespace sdp {

// MFMA shapes: the bf16 modes (fp32x3, bf16) run every launch on v_mfma_f32_16x16x32_bf16 (SH = 16);
// exact fp32 on v_mfma_f32_32x32x2_f32 (SH = 32).  The 16x16 shape holds a higher clock under this
// power-limited load at the same cycles per FLOP (256->256 185 -> 171 us,
// 128->128 @64x1024 227 -> 214 us).

// SDP_FWD_TRN (diagnostic A/B builds only): the 16-wide forward tiles in the D = W x X orientation
// with the transposed direct epilogue (16-B accesses), as the data gradient runs
#ifndef SDP_FWD_TRN
#define SDP_FWD_TRN 0
#endif

// SDP_CONV_CPAIR=0 (build-time A/B only): the two Cout blocks of a tile on grid.y (dispatched a whole
// grid row apart, the second patch read from HBM)
#ifndef SDP_CONV_CPAIR
#define SDP_CONV_CPAIR 1
#endif

// SDP_NJ2_STRIP (build-time A/B): strip tile order (conv_strip_w) for the 4-wave 32-Cout-wave launches too --
// 1 = the paired 256-Cout layers, 2 = every 4-wave launch (the 128-channel layers as well)
#ifndef SDP_NJ2_STRIP
#define SDP_NJ2_STRIP 1
#endif

template <int MODE, int WM, int TC, int KS, bool POOL, bool PELU, bool IO16>
hipError_t conv_launch(ConvArgs a, hipStream_t st) {
  using T = ConvTile<WM, TC, KS, 4, 4, IO16>;
  a.tiles_per_img = a.H * a.W / (T::TR * TC);
  a.groups_per_img = a.H * a.W / 128;
  a.strip_w = conv_strip_w(a.H / a.dil / T::TR, a.W / a.dil / TC);
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  if constexpr (MODE != MODE_F32) {
    hipLaunchKernelGGL((conv_mfma_kernel<MODE, WM, TC, KS, POOL, POOL, PELU, 16, 4, (SDP_FWD_TRN && TC == 16 && !POOL), 4, IO16>),
                       grid, dim3(256), 0, st, a);
    return hipGetLastError();
  } else if constexpr (TC >= 32) {   // the 32x32 shape tiles rows in 32-pixel fragments
    hipLaunchKernelGGL((conv_mfma_kernel<MODE, WM, TC, KS, POOL, POOL, PELU>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;   // (not reached: conv.hip picks 16-wide tiles for the bf16 modes only)
}

template <int MODE, bool PELU>
hipError_t conv_launch_half(ConvArgs a, hipStream_t st) {
  using T = ConvTile<1, 16, 3, 2>;
  a.tiles_per_img = a.H * a.W / (T::TR * 16);
  a.groups_per_img = a.H * a.W / 128;
  a.strip_w = 0;   // row-major: strips cut this class's reads 229 -> 177 MB but cost 2.6 % of time
                   // (profiles/experiments/r03_strip_ab.log)
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  hipLaunchKernelGGL((conv_mfma_kernel<MODE, 1, 16, 3, false, false, PELU, 16, 2, (SDP_FWD_TRN != 0)>), grid,
                     dim3(T::NTH), 0, st, a);
  return hipGetLastError();
}

// 32-Cout waves, two per SIMD (conv_kernel.h ConvTile NJ = 2): 128 px x 128 Cout on 4 waves, two
// workgroups per CU (pair), or 128 px x 256 Cout on 8 waves, one per CU (oct)
template <int MODE, bool PELU, int NW, bool IO16>
hipError_t conv_launch_nj2(ConvArgs a, hipStream_t st) {
  using T = ConvTile<1, 16, 3, NW, 2, IO16>;
  a.tiles_per_img = a.H * a.W / (T::TR * 16);
  a.groups_per_img = a.H * a.W / 128;
  // two Cout blocks per tile (the fp32x3 256-Cout layers on 4-wave workgroups): dealt as adjacent pairs
  // of the XCD-ordered index, so a tile's second patch read comes from that XCD's L2
  a.cpair = (SDP_CONV_CPAIR && a.Cout == 2 * T::NTILE) ? 1 : 0;
  const bool strip = NW == 8 || SDP_NJ2_STRIP == 2 || (SDP_NJ2_STRIP == 1 && a.cpair);
  a.strip_w = strip ? conv_strip_w(a.H / a.dil / T::TR, a.W / a.dil / 16) : 0;
  dim3 grid(a.B * a.tiles_per_img * (a.cpair ? 2 : 1), a.cpair ? 1 : a.Cout / T::NTILE);
  hipLaunchKernelGGL((conv_mfma_kernel<MODE, 1, 16, 3, false, false, PELU, 16, NW, false, 2, IO16>), grid, dim3(T::NTH), 0,
                     st, a);
  return hipGetLastError();
}

template <int MODE, int WM, int TC, int KS, bool ZP, bool IO16>
hipError_t dgrad_launch(ConvArgs a, hipStream_t st) {
  using T = ConvTile<WM, TC, KS, 4, 4, IO16>;
  a.tiles_per_img = a.H * a.W / (T::TR * TC);
  a.groups_per_img = a.H * a.W / 128;
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  if constexpr (TC < 32) {   // 8 x 16 tiles: the transposed direct epilogue (conv_kernel.h TRN)
    hipLaunchKernelGGL((conv_mfma_kernel<MODE, WM, TC, KS, false, ZP, false, 16, 4, true, 4, IO16>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_mfma_kernel<MODE, WM, TC, KS, false, ZP, false, 16, 4, false, 4, IO16>), grid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

// the shapes conv.hip / conv_bwd.hip dispatch to
template <int S> struct FwdShape;
template <> struct FwdShape<0> { static constexpr int WM = 1, TC = 64, KS = 1; static constexpr bool POOL = true; };
template <> struct FwdShape<1> { static constexpr int WM = 1, TC = 64, KS = 3; static constexpr bool POOL = true; };
template <> struct FwdShape<2> { static constexpr int WM = 2, TC = 32, KS = 3; static constexpr bool POOL = false; };
template <> struct FwdShape<3> { static constexpr int WM = 1, TC = 64, KS = 3; static constexpr bool POOL = false; };
template <> struct FwdShape<4> { static constexpr int WM = 1, TC = 32, KS = 3; static constexpr bool POOL = false; };
template <> struct FwdShape<5> { static constexpr int WM = 1, TC = 16, KS = 3; static constexpr bool POOL = false; };  // 16x16 shape only
template <> struct FwdShape<8> { static constexpr int WM = 1, TC = 64, KS = 1; static constexpr bool POOL = false; };  // pool-first 1x1 shortcut
template <int MODE>
hipError_t dgrad_launch_half(ConvArgs a, hipStream_t st) {
  using T = ConvTile<1, 16, 3, 2>;
  a.tiles_per_img = a.H * a.W / (T::TR * 16);
  a.groups_per_img = a.H * a.W / 128;
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  hipLaunchKernelGGL((conv_mfma_kernel<MODE, 1, 16, 3, false, false, false, 16, 2, true>), grid, dim3(T::NTH), 0, st, a);
  return hipGetLastError();
}

// data gradient on 32-Cout waves, two per SIMD (conv_kernel.h ConvTile NJ = 2, transposed epilogue):
// 4 waves = 128 Cout per workgroup, two per CU; 8 waves = 256 Cout, one per CU
template <int MODE, int NW, bool IO16>
hipError_t dgrad_launch_nj2(ConvArgs a, hipStream_t st) {
  using T = ConvTile<1, 16, 3, NW, 2, IO16>;
  a.tiles_per_img = a.H * a.W / (T::TR * 16);
  a.groups_per_img = a.H * a.W / 128;
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  hipLaunchKernelGGL((conv_mfma_kernel<MODE, 1, 16, 3, false, false, false, 16, NW, true, 2, IO16>), grid, dim3(T::NTH), 0,
                     st, a);
  return hipGetLastError();
}

template <int S> struct DgradShape;
template <> struct DgradShape<0> { static constexpr int WM = 2, TC = 32, KS = 1; static constexpr bool ZP = false; };
template <> struct DgradShape<1> { static constexpr int WM = 2, TC = 32, KS = 3; static constexpr bool ZP = true; };
template <> struct DgradShape<2> { static constexpr int WM = 2, TC = 32, KS = 3; static constexpr bool ZP = false; };
template <> struct DgradShape<3> { static constexpr int WM = 1, TC = 64, KS = 3; static constexpr bool ZP = false; };
template <> struct DgradShape<4> { static constexpr int WM = 1, TC = 32, KS = 3; static constexpr bool ZP = false; };
template <> struct DgradShape<5> { static constexpr int WM = 1, TC = 16, KS = 3; static constexpr bool ZP = false; };  // 16x16 shape only

#if defined(SDP_INST) && SDP_INST >= 3000   // IO16 data gradients (bf16 tape): 0 = 1x1, 1 = zero-padded 3x3, 7 / 8 = 32-Cout waves on 4 / 8
constexpr int kS = SDP_INST % 10;
static_assert(kS == 0 || kS == 1 || kS == 7 || kS == 8, "SDP_INST: bad IO16 dgrad code");
#if SDP_INST % 10 == 0
template hipError_t dgrad_launch<MODE_BF16, 2, 32, 1, false, true>(ConvArgs, hipStream_t);
#elif SDP_INST % 10 == 1
template hipError_t dgrad_launch<MODE_BF16, 2, 32, 3, true, true>(ConvArgs, hipStream_t);
#else
template hipError_t dgrad_launch_nj2<MODE_BF16, kS == 7 ? 4 : 8, true>(ConvArgs, hipStream_t);
#endif
#elif defined(SDP_INST) && SDP_INST >= 2000   // IO16 forward (bf16 tape): 0 = pooled 1x1, 1 = pooled 3x3, 9 / 6 = nj2 on 4 / 8 waves
constexpr int kPelu = (SDP_INST / 10) % 10, kS = SDP_INST % 10;
static_assert(kPelu <= 1 && (kS == 0 || kS == 1 || kS == 6 || kS == 9), "SDP_INST: bad IO16 forward code");
#if SDP_INST % 10 == 0
template hipError_t conv_launch<MODE_BF16, 1, 64, 1, true, (kPelu != 0), true>(ConvArgs, hipStream_t);
#elif SDP_INST % 10 == 1
template hipError_t conv_launch<MODE_BF16, 1, 64, 3, true, (kPelu != 0), true>(ConvArgs, hipStream_t);
#else
template hipError_t conv_launch_nj2<MODE_BF16, (kPelu != 0), kS == 9 ? 4 : 8, true>(ConvArgs, hipStream_t);
#endif
#elif defined(SDP_INST) && SDP_INST < 1000 && (SDP_INST % 10 == 6 || SDP_INST % 10 == 9)
constexpr int kMode = SDP_INST / 100 - 1, kPelu = (SDP_INST / 10) % 10;
static_assert(kMode >= 1 && kMode <= 2 && kPelu <= 1, "SDP_INST: bad 32-Cout-wave forward code");
template hipError_t conv_launch_nj2<kMode, (kPelu != 0), SDP_INST % 10 == 9 ? 4 : 8>(ConvArgs, hipStream_t);
#elif defined(SDP_INST) && SDP_INST < 1000 && SDP_INST % 10 == 7
constexpr int kMode = SDP_INST / 100 - 1, kPelu = (SDP_INST / 10) % 10;
static_assert(kMode >= 1 && kMode <= 2 && kPelu <= 1, "SDP_INST: bad 2-wave forward code");
template hipError_t conv_launch_half<kMode, (kPelu != 0)>(ConvArgs, hipStream_t);
#elif defined(SDP_INST) && SDP_INST < 1000
constexpr int kMode = SDP_INST / 100 - 1, kPelu = (SDP_INST / 10) % 10, kShape = SDP_INST % 10;
static_assert(kMode >= 0 && kMode <= 2 && kPelu <= 1 && (kShape <= 5 || kShape == 8) &&
                  (kShape < 5 || kShape == 8 || kMode != MODE_F32),
              "SDP_INST: bad forward code");
using FS = FwdShape<kShape>;
template hipError_t conv_launch<kMode, FS::WM, FS::TC, FS::KS, FS::POOL, (kPelu != 0)>(ConvArgs, hipStream_t);
#elif defined(SDP_INST) && (SDP_INST % 10 == 7 || SDP_INST % 10 == 8)
constexpr int kMode = (SDP_INST / 10) % 10;
static_assert(SDP_INST / 100 == 10 && (kMode == MODE_F32X3 || kMode == MODE_BF16), "SDP_INST: bad dgrad code");
template hipError_t dgrad_launch_nj2<kMode, SDP_INST % 10 == 7 ? 4 : 8>(ConvArgs, hipStream_t);
#elif defined(SDP_INST) && SDP_INST % 10 == 6
constexpr int kMode = (SDP_INST / 10) % 10;
static_assert(SDP_INST / 100 == 10 && (kMode == MODE_F32X3 || kMode == MODE_BF16), "SDP_INST: bad dgrad code");
template hipError_t dgrad_launch_half<kMode>(ConvArgs, hipStream_t);
#elif defined(SDP_INST)
constexpr int kMode = (SDP_INST / 10) % 10, kShape = SDP_INST % 10;
static_assert(SDP_INST / 100 == 10 && (kMode == MODE_F32X3 || kMode == MODE_BF16) && kShape <= 5,
              "SDP_INST: bad dgrad code");
using DS = DgradShape<kShape>;
template hipError_t dgrad_launch<kMode, DS::WM, DS::TC, DS::KS, DS::ZP>(ConvArgs, hipStream_t);
#elif defined(SDP_CONV_BENCH_ONLY)
template hipError_t conv_launch<MODE_F32, 2, 32, 3, false, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch<MODE_F32, 1, 32, 3, false, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch<MODE_F32X3, 1, 16, 3, false, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch<MODE_BF16, 1, 16, 3, false, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch_half<MODE_F32X3, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch_half<MODE_BF16, true>(ConvArgs, hipStream_t);
template hipError_t conv_launch_nj2<MODE_F32X3, true, 4>(ConvArgs, hipStream_t);
template hipError_t conv_launch_nj2<MODE_F32X3, true, 8>(ConvArgs, hipStream_t);
template hipError_t conv_launch_nj2<MODE_BF16, true, 4>(ConvArgs, hipStream_t);
template hipError_t conv_launch_nj2<MODE_BF16, true, 8>(ConvArgs, hipStream_t);
template hipError_t conv_launch_nj2<MODE_BF16, true, 4, true>(ConvArgs, hipStream_t);   // the bf16 tape (io16)
template hipError_t dgrad_launch_nj2<MODE_BF16, 4, true>(ConvArgs, hipStream_t);
#else
#error "conv_inst.hip: build with -DSDP_INST=<code> (Makefile) or -DSDP_CONV_BENCH_ONLY (tools/conv_bench)"
#endif

}  // namespace sdp
