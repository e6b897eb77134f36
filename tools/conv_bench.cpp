// Standalone timing of one conv_mfma launch shape (diagnostics; links a conv.o built with
// -DSDP_CONV_BENCH_ONLY [-DSDP_KO=mask]).  Usage: conv_bench Cin Cout H W B [dil] [iters] [mode]
// (mode: 0 fp32, 1 fp32x3 (default), 2 bf16) [dgrad]: with a 9th argument "dgrad", the data gradient
// (conv_dgrad: no prologue, epilogue * elu'(IN++ input, dact 3) + residual, as the training backward);
// a 10th argument "io16": the bf16-tape instantiation (bf16 tensors, mode 2 only; random bits serve)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../simultaneous-diffusion-for-pointclouds_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int Cin = atoi(argv[1]), Cout = atoi(argv[2]), H = atoi(argv[3]), W = atoi(argv[4]), B = atoi(argv[5]);
  const int dil = argc > 6 ? atoi(argv[6]) : 1, iters = argc > 7 ? atoi(argv[7]) : 20;
  const int mode = argc > 8 ? atoi(argv[8]) : sdp::MODE_F32X3;
  const size_t nin = (size_t)B * H * W * Cin, nout = (size_t)B * H * W * Cout, nw = (size_t)Cout * Cin * 9;
  std::vector<float> h(std::max(nin, nw));
  srand(1);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  float *in, *out, *ss, *stats, *bias;
  uint32_t* wf;
  CK(hipMalloc(&in, nin * 4));
  CK(hipMalloc(&out, nout * 4));
  CK(hipMalloc(&wf, nw * 4));
  CK(hipMalloc(&ss, (size_t)B * Cin * 2 * 4));
  CK(hipMalloc(&stats, (size_t)B * (H * W / 128) * Cout * 2 * 4));
  CK(hipMalloc(&bias, Cout * 4));
  CK(hipMemcpy(in, h.data(), nin * 4, hipMemcpyHostToDevice));
  // packed weight words: two bf16 halves of small random values (realistic bit toggling --
  // MFMA power, and so the clock, depends on the operand bits)
  std::vector<uint32_t> hw(nw);
  for (auto& v : hw) {
    float f0 = ((float)rand() / RAND_MAX - 0.5f) * 0.05f, f1 = ((float)rand() / RAND_MAX - 0.5f) * 0.05f;
    uint32_t b0, b1;
    memcpy(&b0, &f0, 4);
    memcpy(&b1, &f1, 4);
    v = (b0 >> 16) | (b1 & 0xffff0000u);
  }
  CK(hipMemcpy(wf, hw.data(), nw * 4, hipMemcpyHostToDevice));
  std::vector<float> sh((size_t)B * Cin * 2);
  for (size_t i = 0; i < sh.size(); i += 2) { sh[i] = 1.f; sh[i + 1] = 0.f; }
  CK(hipMemcpy(ss, sh.data(), sh.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, Cout * 4));
  sdp::ConvArgs a{};
  a.in = in; a.wf = reinterpret_cast<const uint4*>(wf);
  // the library's forward reads the coalesced 16x16 packing (#frag16); random words fit any layout
  a.wf16 = a.wf; a.bias = bias; a.out = out; a.pro_ss = ss;
  a.ss_bstride = 2 * Cin; a.stats = stats; a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.dil = dil; a.circular = 1; a.pro_mode = sdp::PRO_AFFINE_ELU; a.epi_elu = 0;
  unsigned long long* dbg;
  const int nwg_max = B * H * W / 128;
  CK(hipMalloc(&dbg, (size_t)nwg_max * 8 * 8));
  CK(hipMemset(dbg, 0, (size_t)nwg_max * 8 * 8));
  a.dbg = dbg;
  const char* why = "";
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool dg = argc > 9 && !strcmp(argv[9], "dgrad");
  if (dg) {   // the training data gradient: dy in, dx = conv^T(dy) * elu'(h * scale + shift) + res
    float *aux, *res, *ess;
    CK(hipMalloc(&aux, nout * 4));
    CK(hipMalloc(&res, nout * 4));
    CK(hipMalloc(&ess, (size_t)B * Cout * 2 * 4));
    CK(hipMemcpy(aux, h.data(), std::min(nin, nout) * 4, hipMemcpyHostToDevice));
    CK(hipMemset(res, 0, nout * 4));
    std::vector<float> e2((size_t)B * Cout * 2);
    for (size_t i = 0; i < e2.size(); i += 2) { e2[i] = 1.f; e2[i + 1] = 0.f; }
    CK(hipMemcpy(ess, e2.data(), e2.size() * 4, hipMemcpyHostToDevice));
    a.pro_mode = sdp::PRO_NONE; a.stats = nullptr; a.bias = nullptr;   // (wf16: the #dfrag16 layout; random words serve)
    a.dact = 3; a.aux = aux; a.epi_ss = ess; a.res = res;
  }
  if (argc > 10 && !strcmp(argv[10], "io16")) a.io16 = 1;   // (the fp32 buffers hold twice the bf16 elements needed)
  auto launch = [&]() { return dg ? sdp::conv_dgrad(mode, a, 3, 0, &why) : sdp::conv_mfma(mode, a, 3, false, 0, &why); };
  for (int i = 0; i < 3; ++i) CK(launch());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters, fl = 2.0 * B * H * W * (double)Cin * Cout * 9;
  printf("%s %d->%d @%dx%d B=%d d=%d mode %d: %.1f us  %.1f TF/s (algorithmic)\n", dg ? "dgrad" : "conv", Cin, Cout, H,
         W, B, dil, mode, us,
         fl / us * 1e-6);
#ifdef SDP_TIMING
  std::vector<unsigned long long> d((size_t)nwg_max * 8);
  CK(hipMemcpy(d.data(), dbg, d.size() * 8, hipMemcpyDeviceToHost));
  double s[7] = {0}; int n = 0; unsigned long long tmin = ~0ull, tmax = 0;
  for (int i = 0; i < nwg_max; ++i) {
    const unsigned long long* o = &d[(size_t)i * 8];
    if (!o[0]) continue;
    ++n;
    s[0] += o[1] - o[0]; s[1] += o[2] - o[1]; s[2] += o[3] - o[2]; s[3] += o[4] - o[3]; s[4] += o[5];
    s[5] += o[4] - o[0];
    s[6] += (double)(o[4] - o[0]) / (double)(o[7] > o[6] ? o[7] - o[6] : 1) * 0.1;   // GHz: memtime / memrealtime (100 MHz)
    tmin = std::min(tmin, o[0]); tmax = std::max(tmax, o[4]);
  }
  printf("  per-WG memtime ticks (n=%d): setup %.0f  prologue %.0f  loop %.0f (barrier %.0f)  epilogue %.0f  total %.0f ; "
         "span of last launch %llu ; in-kernel clock %.3f GHz\n", n, s[0] / n, s[1] / n, s[2] / n, s[4] / n, s[3] / n,
         s[5] / n, tmax - tmin, s[6] / n);
#endif
  return 0;
}
