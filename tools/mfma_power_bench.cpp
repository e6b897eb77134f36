// Full-chip bare MFMA loop: v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16 at equal
// FLOPs per wave, operands re-read from LDS every step (as a conv main loop does), one wave
// per SIMD, every CU busy for ~0.2 s -- does the smaller instruction run at a higher clock
// when the chip is power-limited?  Usage: mfma_power_bench [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// 32x32x16: 8 accumulators (128 regs), per step 4 A reads + 2 B reads -> 8 MFMAs (like the conv)
__global__ __launch_bounds__(256, 1) void k32(float* out, int iters, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 256) reinterpret_cast<float*>(lds)[i] = (float)(i % 7) * 0.01f;
  __syncthreads();
  f32x16 acc[4][2] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    bf16x8 a[4], b[2];
#pragma unroll
    for (int m = 0; m < 4; ++m) a[m] = *reinterpret_cast<const bf16x8*>(lds + ((it * 4 + m) & 63) * 1024 + lane * 16);
#pragma unroll
    for (int n = 0; n < 2; ++n) b[n] = *reinterpret_cast<const bf16x8*>(lds + ((it * 2 + n + 32) & 63) * 1024 + lane * 16);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc[m][n][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// 16x16x32: 32 accumulators (128 regs), per step 8 A reads + 4 B reads -> 32 MFMAs = same FLOPs
__global__ __launch_bounds__(256, 1) void k16(float* out, int iters, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 256) reinterpret_cast<float*>(lds)[i] = (float)(i % 7) * 0.01f;
  __syncthreads();
  f32x4 acc[8][4] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    bf16x8 a[8], b[4];
#pragma unroll
    for (int m = 0; m < 8; ++m) a[m] = *reinterpret_cast<const bf16x8*>(lds + ((it * 8 + m) & 63) * 1024 + lane * 16);
#pragma unroll
    for (int n = 0; n < 4; ++n) b[n] = *reinterpret_cast<const bf16x8*>(lds + ((it * 4 + n + 32) & 63) * 1024 + lane * 16);
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[m][n][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int nwg = 256 * 2;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, nwg * 256 * 4));
  CK(hipMalloc(&clk, nwg * 8));
  unsigned long long hc[512];
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      if (v == 0) hipLaunchKernelGGL(k32, dim3(nwg), dim3(256), 0, 0, out, iters, clk);
      else hipLaunchKernelGGL(k16, dim3(nwg), dim3(256), 0, 0, out, iters, clk);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(hc, clk, nwg * 8, hipMemcpyDeviceToHost));
      double avg = 0;
      for (int i = 0; i < nwg; ++i) avg += (double)hc[i];
      avg /= nwg;
      // FLOPs: per wave per iter 8 x (32*32*16*2) = 262144 (both variants)
      const double fl = (double)nwg * 4 * iters * 262144.0;
      const double mf = (v == 0 ? 8.0 : 32.0) * iters;
      printf("%s rep %d: %.2f ms  %.0f TFLOP/s  ticks/WG %.0f  ticks per MFMA %.2f  implied clock %.2f GHz\n",
             v == 0 ? "32x32x16" : "16x16x32", rep, ms, fl / ms * 1e-9, avg, avg / mf, avg / (ms * 1e-3 / 2) * 1e-9);
    }
  }
  return 0;
}
