// Host-side launchers of the libsdp kernels (each validates its shape contract first).
#pragma once
#include "common.h"

namespace sdp {

hipError_t conv_mfma(int mode, ConvArgs a, int ks, bool pool, hipStream_t st, const char** why);
hipError_t begin_conv(const float* x, const float* w, const float* bias, float* out, float* stats, int B, int H, int W,
                      hipStream_t st);
hipError_t end_conv(const float* in, const float* ss, const float* w, const float* bias, const float* sigmas,
                    const int64_t* labels, float* out, int B, int H, int W, int Cin, hipStream_t st);
hipError_t inpp_finalize(const float* stats, int B, int T, float cnt, int C, const float* alpha, const float* gamma,
                         const float* beta, float* ss, hipStream_t st);
hipError_t maxpool5(const float* in, float* out, int B, int H, int W, int C, hipStream_t st);
hipError_t langevin_step(float* x, const float* g, const float* ref, const int32_t* mask, const float* noise,
                         uint64_t seed, uint64_t offset, float step, float nscale, float gref, int n2n, int B, int C,
                         int HW, float* lik_out, uint32_t* absmax, hipStream_t st);
hipError_t axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask, const float* ref, float b,
                     size_t n, hipStream_t st);

}  // namespace sdp
