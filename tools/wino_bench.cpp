// Standalone timing of the Winograd conv kernel (diagnostics; links wino.hip objects built with
// -DSDP_WINST=1 and 3 [-DSDP_WKO=mask]).  Usage: wino_bench Cin Cout H W B [dil] [iters]
// fp32x3, IN++ affine + ELU prologue; Cout 256 -> WM=1, Cout 128 -> WM=2.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../simultaneous-diffusion-for-pointclouds_amd/csrc/wino_launch.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int Cin = atoi(argv[1]), Cout = atoi(argv[2]), H = atoi(argv[3]), W = atoi(argv[4]), B = atoi(argv[5]);
  const int dil = argc > 6 ? atoi(argv[6]) : 1, iters = argc > 7 ? atoi(argv[7]) : 20;
  const size_t nin = (size_t)B * H * W * Cin, nout = (size_t)B * H * W * Cout, nw = (size_t)Cout * Cin * 12;
  std::vector<float> h(nin);
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
  std::vector<uint32_t> hw(nw);   // bf16 pairs of small random values (realistic operand bits)
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
  a.in = in; a.wfw = reinterpret_cast<const uint4*>(wf); a.bias = bias; a.out = out; a.pro_ss = ss;
  a.ss_bstride = 2 * Cin; a.stats = stats; a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.dil = dil; a.circular = 1; a.pro_mode = sdp::PRO_AFFINE_ELU; a.epi_elu = 0;
  unsigned long long* dbg;
  const int nwg = B * H * W / 128 * 2;
  CK(hipMalloc(&dbg, (size_t)nwg * 8 * 8));
  CK(hipMemset(dbg, 0, (size_t)nwg * 8 * 8));
  a.dbg = dbg;
  auto launch = [&]() {
    return Cout % 256 == 0 ? sdp::wino_launch<sdp::MODE_F32X3, 1, true>(a, 0) : sdp::wino_launch<sdp::MODE_F32X3, 2, true>(a, 0);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(launch());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters, fl = 2.0 * B * H * W * (double)Cin * Cout * 9;
  printf("wino %d->%d @%dx%d B=%d d=%d: %.1f us  %.1f TF/s (direct-equivalent)  %.1f TF/s (executed, 6 MAC/px)\n", Cin, Cout,
         H, W, B, dil, us, fl / us * 1e-6, fl * 6 / 9 / us * 1e-6);
#ifdef SDP_TIMING
  std::vector<unsigned long long> d((size_t)nwg * 8);
  CK(hipMemcpy(d.data(), dbg, d.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> clk;
  double loop = 0, tot = 0;
  int n = 0;
  for (int i = 0; i < nwg; ++i) {
    const unsigned long long* o = &d[(size_t)i * 8];
    if (!o[0]) continue;
    ++n;
    loop += o[1] - o[0];
    tot += o[3] - o[0];
    clk.push_back((double)(o[3] - o[0]) / (double)(o[4] - o[2]) * 0.1);   // memrealtime: 100 MHz
  }
  std::sort(clk.begin(), clk.end());
  printf("  per-WG shader cycles (n=%d): main loop %.0f, total %.0f; median clock %.2f GHz\n", n, loop / n, tot / n,
         clk[clk.size() / 2]);
#endif
  return 0;
}
