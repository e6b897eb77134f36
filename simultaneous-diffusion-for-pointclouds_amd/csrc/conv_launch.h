// Launchers of conv_mfma_kernel, one per kernel shape.  Declared here, defined and explicitly
// instantiated in conv_inst.hip, which the Makefile compiles once per (mode, prologue, shape) with
// -DSDP_INST=<code>: every object holds one or two kernels, so `make -j` builds the ~70 kernel
// instantiations in parallel instead of in two translation units (10 + 4 minutes serial).
#pragma once
#include "common.h"

namespace sdp {

// forward conv (conv.hip dispatch): shapes of the table in conv_inst.hip
template <int MODE, int WM, int TC, int KS, bool POOL, bool PELU, bool IO16 = false>
hipError_t conv_launch(ConvArgs a, hipStream_t st);

// forward conv of the 128-channel layers on 2-wave workgroups (128 px x 128 Cout, two per CU),
// bf16 modes on the 16x16 shape (conv_inst.hip shape 7)
template <int MODE, bool PELU>
hipError_t conv_launch_half(ConvArgs a, hipStream_t st);

// forward of the 16-wide 3x3 tiles on 32-Cout waves, two per SIMD (conv_inst.hip shapes 9 / 6): NW = 4
// (128 Cout per workgroup, two per CU) or 8 (256 Cout, one per CU)
template <int MODE, bool PELU, int NW, bool IO16 = false>
hipError_t conv_launch_nj2(ConvArgs a, hipStream_t st);

// data gradient of the 128-channel layers on 2-wave workgroups (conv_inst.hip dgrad shape 6)
template <int MODE>
hipError_t dgrad_launch_half(ConvArgs a, hipStream_t st);

// data gradient of the 16-wide 3x3 tiles on 32-Cout waves, two per SIMD (conv_inst.hip dgrad shapes 7 / 8)
template <int MODE, int NW, bool IO16 = false>
hipError_t dgrad_launch_nj2(ConvArgs a, hipStream_t st);

// data gradient (conv_bwd.hip dispatch)
template <int MODE, int WM, int TC, int KS, bool ZP, bool IO16 = false>
hipError_t dgrad_launch(ConvArgs a, hipStream_t st);

// IO16 (the bf16 training tape) launchers exist for MODE_BF16 and these shapes only (conv_inst.hip codes
// 2000 + 10 * pelu + {0, 1, 6, 9} forward, 3000 + {0, 1, 7, 8} data gradient)

}  // namespace sdp
