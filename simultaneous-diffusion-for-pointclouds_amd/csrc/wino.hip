// Launchers of the Winograd F(2,3) convolution (wino_kernel.h), one object per instantiation
// (Makefile: wino_i_<code>.o with -DSDP_WINST=<code>, code = 10 * (mode - 1) + 2 * (wm - 1) + pelu).
#include "wino_kernel.h"
#include "wino_launch.h"

namespace sdp {

template <int MODE, int WM, bool PELU>
hipError_t wino_launch(ConvArgs a, hipStream_t st) {
  using T = WinoTile<WM>;
  a.tiles_per_img = a.H * a.W / (T::TR * T::TC);
  a.groups_per_img = a.H * a.W / 128;
  dim3 grid(a.B * a.tiles_per_img, a.Cout / T::NTILE);
  hipLaunchKernelGGL((wino_conv_kernel<MODE, WM, PELU>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

#if defined(SDP_WINST)
constexpr int kMode = SDP_WINST / 10 + 1, kWm = (SDP_WINST % 10) / 2 + 1, kPelu = SDP_WINST % 2;
static_assert((kMode == MODE_F32X3 || kMode == MODE_BF16) && kWm <= 2, "SDP_WINST: bad code");
template hipError_t wino_launch<kMode, kWm, (kPelu != 0)>(ConvArgs, hipStream_t);
#else
#error "wino.hip: build with -DSDP_WINST=<code> (Makefile)"
#endif

}  // namespace sdp
