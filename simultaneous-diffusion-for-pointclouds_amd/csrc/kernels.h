// Host-side launchers of the libsdp kernels (each validates its shape contract first).
#pragma once
#include "common.h"
#include "langevin.h"

namespace sdp {

hipError_t conv_mfma(int mode, ConvArgs a, int ks, bool pool, hipStream_t st, const char** why);
// h16: bf16 output (the training tape; bf16 mode)
hipError_t begin_conv(const float* x, const float* w, const float* bias, float* out, float* stats, int B, int H, int W,
                      hipStream_t st, int mode = MODE_F32, bool h16 = false);
// lg: fuse the Langevin update into the epilogue (out may then be null: scores not stored); mode: the
// conv arithmetic (MODE_F32: exact fp32 FMAs; bf16 modes: the MFMA partials form, fp32x3 / bf16)
hipError_t end_conv(const float* in, const float* ss, const float* w, const float* bias, const float* sigmas,
                    const int64_t* labels, float* out, int B, int H, int W, int Cin, hipStream_t st,
                    const LangevinArgs* lg = nullptr, int mode = MODE_F32, bool h16 = false);
// scratch: B*C*16 bytes (per-(b,c) float64 mean and variance)
hipError_t inpp_finalize(const float* stats, int B, int T, float cnt, int C, const float* alpha, const float* gamma,
                         const float* beta, float* ss, hipStream_t st, float* nst, void* scratch);
hipError_t maxpool5(const float* in, float* out, int B, int H, int W, int C, hipStream_t st, uint8_t* idx = nullptr,
                    bool h16 = false);
// 2x2 mean pool (the pool-first ConvMeanPool 1x1 shortcut): out [B][H/2][W/2][C]
hipError_t avgpool2(const float* in, float* out, int B, int H, int W, int C, hipStream_t st);
hipError_t langevin_step(float* x, const float* g, const float* ref, const int32_t* mask, const float* noise,
                         uint64_t seed, uint64_t offset, float step, float nscale, float gref, int n2n, int B, int C,
                         int HW, float* lik_out, uint32_t* absmax, hipStream_t st);
hipError_t axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask, const float* ref, float b,
                     size_t n, hipStream_t st);

// ---- training (DSM backward; train_aux.hip, wgrad.hip, conv_bwd.hip)
// one conv's weights for pack_weights_multi: output slots [begin, begin + Cout*Cin*NT)
struct PackDesc {
  const float* w;
  uint32_t* out;
  int Cout, Cin, NT, dgrad;
  size_t begin;
};
hipError_t pack_weights_multi(const PackDesc* d, int nd, size_t total, int mode, hipStream_t st);
hipError_t pack_weights(const float* w, uint32_t* out, int Cout, int Cin, int k, int mode, int dgrad, hipStream_t st);
// InstanceNorm++ backward: C a power of two in [32, 512], HW a multiple of 512 (else hipErrorInvalidValue)
hipError_t inpp_backward(const float* g, const float* h, const float* nst, const float* alpha, const float* gamma, int B,
                         int HW, int C, float* part, float* coef, float* ppart, float* dalpha, float* dgamma,
                         float* dbeta, const float* r1, const float* r2, float* out, hipStream_t st, bool h16 = false);
// h16 (the bf16 training tape, train.hip): the activation / gradient tensors (float* in the signatures)
// hold bf16 elements; parameters, statistics, coefficients and the images stay float32
hipError_t unpool(const float* dout, float* dst, int B, int H, int W, int C, hipStream_t st, bool h16 = false);
hipError_t maxpool5_backward(const uint8_t* idx, const float* dp, const float* res, float* dst, int B, int H, int W, int C,
                             hipStream_t st, bool h16 = false);
hipError_t upsample_backward(const float* g, float* dlow, int B, int H, int W, int C, int accumulate, hipStream_t st,
                             bool h16 = false);
hipError_t elu_backward_post(const float* dy, const float* y, const float* res, float* dst, size_t n, hipStream_t st,
                             bool h16 = false);
hipError_t add_tensors(const float* a, const float* b, float* dst, size_t n, hipStream_t st, bool h16 = false);
size_t head_wgrad_part_floats(int B, int H, int W);   // scratch of begin_conv_wgrad / end_conv_backward
hipError_t begin_conv_wgrad(const float* x, const float* dy, float* part, float* dw, float* db, int B, int H, int W,
                            hipStream_t st, bool h16 = false);
hipError_t end_conv_backward(const float* dscore, const float* sigmas, const int64_t* labels, const float* w,
                             const float* o, const float* ss, float* g, float* part, float* dw, float* db, int B, int H,
                             int W, hipStream_t st, bool h16 = false);
hipError_t dsm_loss(const float* score, const float* noise, const float* mask, const float* used_sigma, int B, int n_img,
                    float power, float* dscore, float* loss, float* loss_per, float* part, hipStream_t st);
// optimizer kinds of get_optimizer (losses/__init__.py:3-13); values = sdp.h SDP_OPTIM_*
enum { OPT_ADAM = 0, OPT_RMSPROP = 1, OPT_SGD = 2 };
struct OptimHyper {
  float b1, b2;          // Adam betas; RMSprop: b2 = alpha; SGD: b1 = momentum
  float eps, weight_decay;
  float step_size;       // Adam: lr / bias_correction1; RMSprop, SGD: lr
  float bc2_sqrt;        // Adam: sqrt(bias_correction2)
  float mu;              // EMA rate
  float omb1, omb2, ommu; // 1 - b1, 1 - b2, 1 - mu: computed from the double hyperparameters and
                         //   rounded once, as torch (Python float scalars) and EMAHelper do
  int first;             // SGD: first step (momentum buffer = g)
};
// s0, s1, s2: Adam exp_avg, exp_avg_sq, max_exp_avg_sq (amsgrad, else null); RMSprop square_avg; SGD momentum_buffer
hipError_t optim_ema(int kind, float* p, const float* g, float* s0, float* s1, float* s2, float* shadow, size_t n,
                     const OptimHyper& h, hipStream_t st);
hipError_t conv_dgrad(int mode, ConvArgs a, int ks, hipStream_t st, const char** why);
// weight-gradient workgroups per launch (pixel splits x Cin/32 x Cout/128): one round of
// two workgroups per CU (1024: +2% kernel time and a costlier reduce)
#ifndef SDP_WGRAD_BLOCKS   // weight-gradient workgroups aimed for per launch (pixel splits x channel blocks)
#define SDP_WGRAD_BLOCKS 512
#endif
constexpr int WGRAD_TARGET_BLOCKS = SDP_WGRAD_BLOCKS;
int wgrad_splits(int B, int H, int W, int d, int Cin, int Cout, int ks);
size_t wgrad_part_floats(int S, int Cin, int Cout, int ks);
// h16: a.in and a.dy hold bf16 elements (the training tape; bf16 mode)
hipError_t conv_wgrad(int mode, WgradArgs a, int ks, float* out, float* bias_out, int accumulate, hipStream_t st,
                      const char** why, bool h16 = false);

}  // namespace sdp
