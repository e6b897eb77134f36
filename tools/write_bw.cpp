// Write-bandwidth ceiling of MI355X HBM for the begin_conv output shape (B=4 x 64 x 1024 x 128 fp32 =
// 134 MB): how fast can a kernel that only STORES that much go, per store pattern?
//   0: grid-stride float4 stores, whole 1 KiB per wave instruction (plain)
//   1: the same, nontemporal
//   2: 16 pixels x 64 B per instruction (the 16x16 MFMA C-fragment pattern), plain
//   3: the same, nontemporal
//   4: copy (read 134 MB + write 134 MB), float4, plain -- the read+write reference
// Usage: write_bw [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void wr(f4* __restrict__ out, const f4* __restrict__ in, size_t n4) {
  const size_t tid = blockIdx.x * 256 + threadIdx.x, nthr = (size_t)gridDim.x * 256;
  const f4 v = {1.f, 2.f, (float)threadIdx.x, 0.f};
  if constexpr (MODE <= 1) {
    for (size_t i = tid; i < n4; i += nthr) {
      if constexpr (MODE == 1) __builtin_nontemporal_store(v, out + i);
      else out[i] = v;
    }
  } else if constexpr (MODE <= 3) {
    // one "tile" = 64 pixels x 128 channels (32 f4 per pixel); a wave writes, per instruction,
    // 16 pixels x 4 f4 (64 B) -- lanes (q = l / 16, p = l % 16) -> pixel p, f4 column 4 f + q
    const int lane = threadIdx.x & 63, q = lane >> 4, p = lane & 15;
    const size_t nw = nthr / 64, wid = tid / 64;
    const size_t ntile = n4 / (16 * 32);   // 16-pixel groups
    for (size_t t = wid; t < ntile; t += nw) {
      f4* base = out + t * 16 * 32 + p * 32 + q;
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        if constexpr (MODE == 3) __builtin_nontemporal_store(v, base + 4 * f);
        else base[4 * f] = v;
      }
    }
  } else {
    for (size_t i = tid; i < n4; i += nthr) out[i] = in[i];
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const size_t bytes = (size_t)4 * 64 * 1024 * 128 * 4, n4 = bytes / 16;
  f4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"float4 grid-stride", "float4 grid-stride nt", "16px x 64B runs", "16px x 64B runs nt", "copy"};
  for (int grid : {1024, 2048, 8192}) {
    for (int m = 0; m < 5; ++m) {
      auto launch = [&]() {
        switch (m) {
          case 0: hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(256), 0, 0, a, b, n4); break;
          case 1: hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(256), 0, 0, a, b, n4); break;
          case 2: hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(256), 0, 0, a, b, n4); break;
          case 3: hipLaunchKernelGGL(wr<3>, dim3(grid), dim3(256), 0, 0, a, b, n4); break;
          default: hipLaunchKernelGGL(wr<4>, dim3(grid), dim3(256), 0, 0, a, b, n4); break;
        }
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters, moved = (m == 4 ? 2.0 : 1.0) * bytes;
      printf("grid %5d  %-24s %7.1f us  %6.2f TB/s\n", grid, names[m], us, moved / us / 1e6);
    }
  }
  return 0;
}
