// Launchers of wino_conv_kernel (wino_kernel.h), instantiated per (mode, workgroup shape,
// prologue) in wino.hip.
#pragma once
#include "common.h"

namespace sdp {

template <int MODE, int WM, bool PELU>
hipError_t wino_launch(ConvArgs a, hipStream_t st);

}  // namespace sdp
