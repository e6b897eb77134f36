// Small / memory-bound kernels of the score network (gfx950).
//   begin_conv : input prep (2x-1, coordinate channels; ncsnv2.py:485-496) fused with the
//                4->ngf zero-padded 3x3 conv + bias (ncsnv2.py:433,498) and IN++ tile stats.
//   end_conv   : final IN++ affine + ELU prologue, ngf->2 zero-padded 3x3 conv + bias,
//                / sigmas[y] (ncsnv2.py:510-516), NCHW output.
//   inpp_finalize : per-tile (mean, M2) -> per-(b,c) InstanceNorm2dPlus scale/shift
//                (normalization.py:163-176), in two small launches.
//   maxpool5   : MaxPool2d(5, stride 1, padding 2) of CRPBlock (layers.py:70), NHWC.
#include "common.h"
#include "langevin.h"

namespace sdp {

// torch.linspace(0, 1, steps=n)[i] (scalar form: start + step*i below halfway, else end - step*(n-1-i))
SDP_DEV float linspace01(int i, int n) {
  if (n == 1) return 0.f;
  const float step = 1.0f / (float)(n - 1);
  return i < n / 2 ? step * (float)i : 1.0f - step * (float)(n - 1 - i);
}

SDP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- begin conv (Cin=4 -> 128)
// Persistent; thread = (4 output channels, 16 consecutive pixels) of a 128-pixel row tile.  The
// 36 x 128 weights are staged in LDS once per workgroup ([tap][4-channel group]: one b128 per tap
// gives a thread its 4 output channels), so a thread holds only its 64 accumulators and the
// registers allow 4 workgroups per CU; the prepped 4 x 3 x 130 input patch is broadcast by b128
// reads (18 values per (channel, row) feed 3 taps x 16 px x 4 channels).  The next tile's patch is
// loaded into registers while the current one computes, by UNCONDITIONAL loads (clamped address,
// value selected after): a load under a branch makes the compiler wait vmcnt(0) at the join,
// which on gfx9 also waits for every output store still in flight.
// Output: every store instruction writes two whole 512-B pixel rows (nt: streamed past L2).
// Statistics of each 64-pixel half: two-pass (mean, M2) per thread, Chan merges across the
// 4 pixel groups (lane l ^ 32, then through LDS).  HBM-bound: 8 B in + 512 B out per pixel.
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int BC_TP = 128, BC_RS = 132;            // pixels per tile; staged patch row stride (floats)
#ifndef SDP_BC_KO   // diagnostic knock-outs (tools/lib_variant.sh only): 1 = no output stores, 2 = no FMAs
#define SDP_BC_KO 0
#endif
constexpr int BC_WG_PER_CU = 3;
__global__ __launch_bounds__(256, BC_WG_PER_CU) void begin_conv_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         float* __restrict__ stats, int B, int H, int W) {
  constexpr int CO = 128;
  __shared__ __attribute__((aligned(16))) float sp[12 * BC_RS];   // [ci*3 + row][col], cols -1 .. 128
  __shared__ __attribute__((aligned(16))) float4 swl[36 * 32];    // [tap][cg]: channels 4cg .. 4cg+3
  __shared__ float2 red[2][2][CO];                                   // [64-px half][pixel-group pair][channel]
  __shared__ __attribute__((aligned(16))) float rawb[4 * 256];      // DMA landing zone of the next patch
  const int tid = threadIdx.x, cg = tid & 31, pg = tid >> 5;       // channels 4cg.., pixels 16pg..
  for (int i = tid; i < 36 * 32; i += 256) {
    const int k = i >> 5, g4 = i & 31;
    swl[i] = make_float4(w[(4 * g4 + 0) * 36 + k], w[(4 * g4 + 1) * 36 + k], w[(4 * g4 + 2) * 36 + k],
                         w[(4 * g4 + 3) * 36 + k]);
  }
  const f32x2v b01 = {bias[4 * cg], bias[4 * cg + 1]}, b23 = {bias[4 * cg + 2], bias[4 * cg + 3]};
  const int tiles_row = W / BC_TP, tiles_per_img = H * tiles_row, ntiles = B * tiles_per_img;
  // patch rows cr = ci*3 + r: the 2 x 3 x 130 image values of the next tile are landed in rawb by
  // LDS-DMA (4 B per lane, clamped addresses: no branch, nothing the compiler must wait for) while
  // the current tile computes; the coordinate rows are computed when the patch is staged.  Unit
  // i = tid + 256k is landed and later read by the same thread, so it needs only the vmcnt wait:
  // after the DMA each thread issues exactly 17 stores (16 outputs + 1 statistic), and gfx9's
  // vector memory ops retire in order, so vmcnt <= 17 means the DMA has landed.
  constexpr int NI = 6 * 130, PE = (NI + 255) / 256;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, B * 2 * H * W * 4, 0x00020000);
  auto patch_dma = [&](int t) {
    const int b = t / tiles_per_img, tile = t % tiles_per_img;
    const int y = tile / tiles_row, x0 = (tile % tiles_row) * BC_TP;
#pragma unroll
    for (int k = 0; k < PE; ++k) {
      const int i = min(tid + k * 256, NI - 1);
      const int cr = i / 130, c = i % 130, ci = cr / 3, r = cr % 3;
      const int yy = min(max(y - 1 + r, 0), H - 1), xx = min(max(x0 - 1 + c, 0), W - 1);
      const int off = t < ntiles ? ((((b * 2 + ci) * H + yy) * W + xx) * 4) : 0;
      const int base = __builtin_amdgcn_readfirstlane(((tid & ~63) + k * 256) * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(rawb) + base), 4,
          off, 0, 0, 0);
    }
  };
  patch_dma(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int b = t / tiles_per_img, tile = t % tiles_per_img;
    const int y = tile / tiles_row, x0 = (tile % tiles_row) * BC_TP;
    if (t == (int)blockIdx.x) __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): no stores behind the first DMA
    else __builtin_amdgcn_s_waitcnt(0x4f71);                        // vmcnt(17)
    __syncthreads();                               // the previous tile's patch / red are consumed
#pragma unroll
    for (int k = 0; k < PE; ++k) {
      const int i = tid + k * 256;
      const int cr = i / 130, c = i % 130, r = cr % 3;
      const int yy = y - 1 + r, xx = x0 - 1 + c;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      if (i < NI) {
        sp[cr * BC_RS + c] = ok ? 2.f * rawb[i] - 1.f : 0.f;              // channels 0, 1: 2x - 1
        const float e = cr < 3 ? linspace01(xx, W) : linspace01(yy, H);   // rows 6..11: coordinates
        sp[(cr + 6) * BC_RS + c] = ok ? e : 0.f;
      }
    }
    __syncthreads();
    patch_dma(t + gridDim.x);                      // the next tile's patch lands meanwhile
    f32x2v acc[16][2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[i][0] = b01;
      acc[i][1] = b23;
    }
#pragma unroll
    for (int cr = 0; cr < ((SDP_BC_KO & 2) ? 0 : 12); ++cr) {   // (input channel, kernel row)
      float v[18];
      const float* row = sp + cr * BC_RS + 16 * pg;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 f = *reinterpret_cast<const float4*>(row + 4 * q);
        v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
      }
      v[16] = row[16];
      v[17] = row[17];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int k = (cr / 3) * 9 + (cr % 3) * 3 + kw;
        const float4 wk = swl[k * 32 + cg];
        const f32x2v w01 = {wk.x, wk.y}, w23 = {wk.z, wk.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const f32x2v vv = {v[i + kw], v[i + kw]};
          acc[i][0] = __builtin_elementwise_fma(vv, w01, acc[i][0]);
          acc[i][1] = __builtin_elementwise_fma(vv, w23, acc[i][1]);
        }
      }
    }
    float* o = out + (((size_t)b * H + y) * W + x0 + 16 * pg) * CO + 4 * cg;
#pragma unroll
    for (int i = 0; i < ((SDP_BC_KO & 1) ? 0 : 16); ++i)
      __builtin_nontemporal_store(f32x4v{acc[i][0].x, acc[i][0].y, acc[i][1].x, acc[i][1].y},
                                  reinterpret_cast<f32x4v*>(o + (size_t)i * CO));
    // statistics of channel 4cg+j over this thread's 16 pixels, then over 32 (lanes l, l^32 hold
    // pixel groups 2w, 2w+1), then over 64 (waves 2h, 2h+1 through LDS)
    float mean[4], m2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sm += (j & 1) ? acc[i][j >> 1].y : acc[i][j >> 1].x;
      mean[j] = sm * (1.f / 16.f);
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float dv = ((j & 1) ? acc[i][j >> 1].y : acc[i][j >> 1].x) - mean[j];
        q = fmaf(dv, dv, q);
      }
      m2[j] = q;
      const float mp = __shfl_xor(mean[j], 32), qp = __shfl_xor(m2[j], 32), d = mean[j] - mp;
      m2[j] = m2[j] + qp + d * d * 8.f;
      mean[j] = 0.5f * (mean[j] + mp);
    }
    const int wv = tid >> 6, half = wv >> 1;
    if ((tid & 63) < 32) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[half][wv & 1][4 * cg + j] = make_float2(mean[j], m2[j]);
    }
    __syncthreads();
    {
      const int hh = tid >> 7, c = tid & 127;       // 256 threads = 2 halves x 128 channels
      const float2 a = red[hh][0][c], q = red[hh][1][c];
      const float d = a.x - q.x;
      float2* st = reinterpret_cast<float2*>(stats) + ((size_t)b * (H * W / 64) + (y * W + x0) / 64 + hh) * CO + c;
      *st = make_float2(0.5f * (a.x + q.x), a.y + q.y + d * d * 16.f);
    }
  }
}

// ---------------------------------------------------------------- begin conv on MFMA (bf16 modes)
// The same 128-pixel row tiles, the 4 -> 128 contraction on v_mfma_f32_16x16x32_bf16 with
// M = 16 output channels, N = 16 pixels, K = (tap, channel) = 36 of 64 (two 32-deep steps;
// fp32x3 = lo*hi + hi*lo + hi*hi of the bf16 split).  C fragments then hold 4 consecutive channels
// of one pixel per lane: 16-B stores, a wave pair writes whole 128-B runs.  Wave w owns channels
// 64 (w & 1) .. +63 and pixels 64 (w >> 1) .. +63 of the tile, i.e. whole 64-pixel statistics
// groups: (mean, M2) per channel in registers, Chan merges across the 16 pixel lanes.  Persistent;
// the weight fragments are built once per workgroup, the next tile's image values are loaded into
// registers (unconditional, clamped loads) while the current tile computes.  The FMA work of the
// direct kernel (4608 per pixel on packed-f32 VALU) is what kept it off the HBM roofline.
#ifndef SDP_BM_WG         // workgroups per CU of the MFMA begin conv
#define SDP_BM_WG 2
#endif
constexpr int BM_WG_PER_CU = SDP_BM_WG, BM_TS = 68;   // workgroups per CU; transpose row stride (floats)
#ifndef SDP_BC_LDS_T      // 1: output stores through an LDS transpose (256-B runs); 0: straight from the C fragments
#define SDP_BC_LDS_T 1
#endif
#ifndef SDP_BM_KO         // diagnostic knock-outs (tools/lib_variant.sh only): 1 = no output stores, 2 = no
#define SDP_BM_KO 0       // statistics, 4 = no MFMAs
#endif
#ifndef SDP_BC_NT         // 1: nontemporal output stores.  tools/write_bw on MI355X: plain float4 stores of the
#define SDP_BC_NT 0       // 134 MB output reach 6.1-6.3 TB/s, nt ones 4.9-5.4 (whole rows) / 3.7 (64-B runs)
#endif
SDP_DEV void bm_store(f32x4v v, f32x4v* p) {
  if constexpr (SDP_BC_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
#ifndef SDP_HEAD_DIRECT   // A/B switch (tools/lib_variant.sh only): 1 = the direct fp32 begin/end conv in every mode
#define SDP_HEAD_DIRECT 0
#endif
SDP_DEV void bm_store(f32x4v v, __bf16* p) { *reinterpret_cast<uint2*>(p) = f4_to_bf4(make_float4(v[0], v[1], v[2], v[3])); }
SDP_DEV void bm_store(f32x4v v, float* p) { bm_store(v, reinterpret_cast<f32x4v*>(p)); }
// TO: the output's element type (__bf16 in the bf16 training tape, train.hip); statistics from the float values
template <int MODE, typename TO = float>
__global__ __launch_bounds__(256, BM_WG_PER_CU) void begin_conv_mfma_kernel(const float* __restrict__ x,
                                                                           const float* __restrict__ w,
                                                                           const float* __restrict__ bias,
                                                                           TO* __restrict__ out,
                                                                           float* __restrict__ stats, int B, int H, int W) {
  constexpr int CO = 128, NI = 6 * 130, PE = (NI + 255) / 256;
  __shared__ __attribute__((aligned(16))) float sp[12 * BC_RS];   // [ci*3 + row][col], cols -1 .. 128
#if SDP_BC_LDS_T
  __shared__ __attribute__((aligned(16))) float tbuf[4 * 64 * BM_TS];   // per wave: [64 px][64 ch + pad]
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, l16 = lane & 15;
  const int ch = wave & 1, ph = wave >> 1;
  const int tiles_row = W / BC_TP, tiles_per_img = H * tiles_row, ntiles = B * tiles_per_img;

  // A (weight) fragments: row co = 64 ch + 16 f + l16, k = 32 s + 8 q + j -> (tap k / 4, ci k % 4)
  bf16x8 ah[4][2], al[4][2];
  f32x4 bias4[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int co = 64 * ch + 16 * f + l16;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * q + j;
        const float v = k < 36 ? w[(co * 4 + (k & 3)) * 9 + (k >> 2)] : 0.f;
        ah[f][s][j] = (__bf16)v;
        al[f][s][j] = (__bf16)(v - (float)ah[f][s][j]);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) bias4[f][r] = bias[64 * ch + 16 * f + 4 * q + r];
  }
  // image values of a tile's patch rows (2 channels x 3 rows x 130 columns), clamped addresses
  float rv[PE];
  auto load_patch = [&](int t) __attribute__((always_inline)) {
    t = min(t, ntiles - 1);
    const int b = t / tiles_per_img, tile = t % tiles_per_img;
    const int y = tile / tiles_row, x0 = (tile % tiles_row) * BC_TP;
#pragma unroll
    for (int k = 0; k < PE; ++k) {
      const int i = min(tid + k * 256, NI - 1);
      const int cr = i / 130, c = i % 130, ci = cr / 3, r = cr % 3;
      const int yy = min(max(y - 1 + r, 0), H - 1), xx = min(max(x0 - 1 + c, 0), W - 1);
      rv[k] = x[(((size_t)b * 2 + ci) * H + yy) * W + xx];
    }
  };
  load_patch(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int b = t / tiles_per_img, tile = t % tiles_per_img;
    const int y = tile / tiles_row, x0 = (tile % tiles_row) * BC_TP;
    __syncthreads();                               // the previous tile's patch is consumed
#pragma unroll
    for (int k = 0; k < PE; ++k) {
      const int i = tid + k * 256;
      const int cr = i / 130, c = i % 130, r = cr % 3;
      const int yy = y - 1 + r, xx = x0 - 1 + c;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      if (i < NI) {
        sp[cr * BC_RS + c] = ok ? 2.f * rv[k] - 1.f : 0.f;                // channels 0, 1: 2x - 1
        const float e = cr < 3 ? linspace01(xx, W) : linspace01(yy, H);   // rows 6..11: coordinates
        sp[(cr + 6) * BC_RS + c] = ok ? e : 0.f;
      }
    }
    __syncthreads();
    load_patch(t + gridDim.x);                     // the next tile's values fly meanwhile
    f32x4 acc[4][4];                               // [pixel group g][channel fragment f]
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // B fragment (im2col): pixel 64 ph + 16 g + l16, k = 32 s + 8 q + j
      const int px = 64 * ph + 16 * g + l16;
      float v0[8], v1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * q + j, tap = k >> 2, ci = k & 3;
        v0[j] = sp[(ci * 3 + tap / 3) * BC_RS + px + tap % 3];
        const int tap1 = 8;                         // s = 1: only k = 32..35 (tap 8, q = 0, j < 4) are real
        v1[j] = (q == 0 && j < 4) ? sp[(j * 3 + tap1 / 3) * BC_RS + px + tap1 % 3] : 0.f;
      }
      bf16x8 bh0, bl0, bh1, bl1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bh0[j] = (__bf16)v0[j];
        bl0[j] = (__bf16)(v0[j] - (float)bh0[j]);
        bh1[j] = (__bf16)v1[j];
        bl1[j] = (__bf16)(v1[j] - (float)bh1[j]);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        f32x4 c = bias4[f];
        if constexpr (SDP_BM_KO & 4) { acc[g][f] = c + bh0[0] * (float)g; continue; }
        if constexpr (MODE == MODE_F32X3) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[f][0], bh0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f][0], bl0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[f][1], bh1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f][1], bl1, c, 0, 0, 0);
        }
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f][0], bh0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f][1], bh1, c, 0, 0, 0);
        acc[g][f] = c;
      }
    }
#if SDP_BC_LDS_T
    // stores through a wave-private LDS transpose: each instruction writes 4 pixels x 256 B (the
    // wave's 64 channels) instead of 16 pixels x 64 B.  The statistics come from the transposed
    // values: lane (pq, c4) holds channels 4 c4 .. +3 of pixels 4 i + pq, i < 16 -- a two-pass
    // (mean, M2) over its 16 pixels, then two equal-count Chan merges (lanes ^16, ^32) -- instead
    // of 4 levels of cross-lane merges of 16 channels on the C-fragment layout
    float* tw = tbuf + wave * 64 * BM_TS;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        *reinterpret_cast<f32x4v*>(tw + (16 * g + l16) * BM_TS + 16 * f + 4 * q) =
            f32x4v{acc[g][f][0], acc[g][f][1], acc[g][f][2], acc[g][f][3]};
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int pq = lane >> 4, c4 = lane & 15;
    f32x4v tv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) tv[i] = *reinterpret_cast<const f32x4v*>(tw + (4 * i + pq) * BM_TS + 4 * c4);
    if constexpr (!(SDP_BM_KO & 1)) {
      TO* o = out + (((size_t)b * H + y) * W + x0 + 64 * ph + pq) * CO + 64 * ch + 4 * c4;
#pragma unroll
      for (int i = 0; i < 16; ++i) bm_store(tv[i], o + (size_t)4 * i * CO);
    }
    if constexpr (SDP_BM_KO & 2) continue;
    f32x4v mean = tv[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mean += tv[i];
    mean *= (1.f / 16.f);
    f32x4v m2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const f32x4v dv = tv[i] - mean;
      m2 += dv * dv;
    }
    float2 res[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mj = mean[j], qj = m2[j], n = 16.f;
#pragma unroll
      for (int o2 = 16; o2 < 64; o2 <<= 1) {
        const float mp = __shfl_xor(mj, o2), qp = __shfl_xor(qj, o2), d = mj - mp;
        qj = qj + qp + d * d * (0.5f * n);
        mj = 0.5f * (mj + mp);
        n *= 2.f;
      }
      res[j] = make_float2(mj, qj);
    }
    if (pq == 0) {
      float4* st = reinterpret_cast<float4*>(reinterpret_cast<float2*>(stats) +
                                             ((size_t)b * (H * W / 64) + (y * W + x0) / 64 + ph) * CO + 64 * ch + 4 * c4);
      st[0] = make_float4(res[0].x, res[0].y, res[1].x, res[1].y);
      st[1] = make_float4(res[2].x, res[2].y, res[3].x, res[3].y);
    }
  }
}
#else
    if constexpr (!(SDP_BM_KO & 1)) {
    // stores: lane = 4 channels (64 ch + 16 f + 4 q ..) of pixel x0 + 64 ph + 16 g + l16
    TO* o = out + (((size_t)b * H + y) * W + x0 + 64 * ph + l16) * CO + 64 * ch + 4 * q;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        bm_store(f32x4v{acc[g][f][0], acc[g][f][1], acc[g][f][2], acc[g][f][3]}, o + (size_t)16 * g * CO + 16 * f);
    }
    if constexpr (SDP_BM_KO & 2) continue;
    // statistics of this wave's 64-pixel group: 4 values per lane and channel, then the 16 lanes
    float2* st = reinterpret_cast<float2*>(stats) + ((size_t)b * (H * W / 64) + (y * W + x0) / 64 + ph) * CO + 64 * ch + 4 * q;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float mean = 0.25f * (((acc[0][f][r] + acc[1][f][r]) + acc[2][f][r]) + acc[3][f][r]);
        float m2 = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float dv = acc[g][f][r] - mean;
          m2 = fmaf(dv, dv, m2);
        }
        float n = 4.f;
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) {     // equal-count Chan merges
          const float mp = __shfl_xor(mean, o2), qp = __shfl_xor(m2, o2), d = mean - mp;
          m2 = m2 + qp + d * d * (0.5f * n);
          mean = 0.5f * (mean + mp);
          n *= 2.f;
        }
        if (l16 == 0) st[16 * f + r] = make_float2(mean, m2);
      }
  }
}
#endif

// ---------------------------------------------------------------- end conv (128 -> 2), NCHW out
// block: 4 rows x 64 cols of output.  The image's IN++ (scale, shift) and the 2 x 128 x 9 weights
// (as (co0, co1) pairs per (tap, channel)) are staged in LDS once.  Per 32-channel chunk the
// (6 x 66) patch (IN++ affine + ELU applied on the way in) sits in LDS at a 36-float pixel stride
// (16-B aligned, conflict-free ds_read_b128 across consecutive pixels); the NEXT chunk's raw patch
// is loaded into registers while the current one is consumed, by unconditional loads (clamped
// address, zero selected after -- no vmcnt(0) at a branch join).  Wave g takes channels 8g..8g+7
// of the chunk, each thread one column: per kw a patch column of 6 rows x 4 channels (6 b128
// reads) feeds its 4 output rows x 3 taps x 4 channels of packed (co0, co1) FMAs -- the same
// per-output fma order as a scalar loop.  The 4 channel-group partials are summed through LDS.
// LGV: the Langevin update of sdp_net_forward_langevin in the epilogue (langevin.h): the block's
// 4 x 64 x 2 scores update x in place, write lik (and the scores when out is given) and feed
// max|x_new[:,0]|; the float4 groups are those of the stand-alone kernel, so are the Philox counters.
constexpr int EC_CIN = 128, EC_PS = 36, EC_NU = (6 * 66 * 8 + 255) / 256;   // pixel stride (floats); units per thread
template <bool LGV>
__global__ __launch_bounds__(256) void end_conv_kernel(const float* __restrict__ in, const float* __restrict__ ss,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       const float* __restrict__ sigmas, const int64_t* __restrict__ labels,
                                                       float* __restrict__ out, int H, int W, LangevinArgs lg) {
  constexpr int Cin = EC_CIN;
  __shared__ __attribute__((aligned(16))) float sp[6 * 66 * EC_PS];
  __shared__ __attribute__((aligned(16))) f32x2v sw[9 * Cin];     // [tap][ci] -> (w[co0], w[co1])
  __shared__ __attribute__((aligned(16))) float4 sss[Cin / 2];    // (scale, shift) of channels 2j, 2j+1
  __shared__ f32x2v red[4][4][64];
  const int tid = threadIdx.x;
  const int tiles_row = W / 64, tiles_per_img = (H / 4) * tiles_row;
  const int b = blockIdx.x / tiles_per_img, tile = blockIdx.x % tiles_per_img;
  const int y0 = (tile / tiles_row) * 4, x0 = (tile % tiles_row) * 64;
  const int c = tid & 63, g = tid >> 6;
  float4 raw[EC_NU];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int k = 0; k < EC_NU; ++k) {
      const int i = tid + k * 256;
      const int pix = i >> 3, cv = i & 7;
      const int pr = pix / 66, pc = pix % 66;
      const int yy = y0 - 1 + pr, xx = x0 - 1 + pc;
      const bool ok = i < 6 * 66 * 8 && yy >= 0 && yy < H && xx >= 0 && xx < W;
      raw[k] = *reinterpret_cast<const float4*>(in + (ok ? (((size_t)b * H + yy) * W + xx) * Cin + c0 + cv * 4 : 0));
    }
  };
  load_chunk(0);
  for (int i = tid; i < 9 * Cin; i += 256) {
    const int tap = i / Cin, ci = i % Cin;
    sw[i] = f32x2v{w[(size_t)ci * 9 + tap], w[((size_t)Cin + ci) * 9 + tap]};
  }
  if (tid < Cin / 2) sss[tid] = reinterpret_cast<const float4*>(ss + (size_t)b * Cin * 2)[tid];
  f32x2v acc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = f32x2v{0.f, 0.f};
  for (int c0 = 0; c0 < Cin; c0 += 32) {
    __syncthreads();                                 // the previous chunk's patch is consumed
#pragma unroll
    for (int k = 0; k < EC_NU; ++k) {              // transform (zero padding stays zero) -> LDS
      const int i = tid + k * 256;
      if (i >= 6 * 66 * 8) break;
      const int pix = i >> 3, cv = i & 7;
      const int pr = pix / 66, pc = pix % 66;
      const int yy = y0 - 1 + pr, xx = x0 - 1 + pc;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const int j = (c0 + cv * 4) >> 1;
        const float4 s01 = sss[j], s23 = sss[j + 1];
        const float4 f = raw[k];
        o.x = elu(fmaf(f.x, s01.x, s01.y));
        o.y = elu(fmaf(f.y, s01.z, s01.w));
        o.z = elu(fmaf(f.z, s23.x, s23.y));
        o.w = elu(fmaf(f.w, s23.z, s23.w));
      }
      *reinterpret_cast<float4*>(&sp[pix * EC_PS + cv * 4]) = o;
    }
    __syncthreads();
    if (c0 + 32 < Cin) load_chunk(c0 + 32);          // next chunk in flight during this one
#pragma unroll
    for (int cq = 0; cq < 2; ++cq) {
      const int ci = g * 8 + cq * 4;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float4 col[6];
#pragma unroll
        for (int pr = 0; pr < 6; ++pr) col[pr] = *reinterpret_cast<const float4*>(&sp[(pr * 66 + c + kw) * EC_PS + ci]);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const f32x2v* wt = &sw[(kh * 3 + kw) * Cin + c0 + ci];
          const f32x2v w0 = wt[0], w1 = wt[1], w2 = wt[2], w3 = wt[3];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float4 v = col[r + kh];
            acc[r] = __builtin_elementwise_fma(f32x2v{v.x, v.x}, w0, acc[r]);
            acc[r] = __builtin_elementwise_fma(f32x2v{v.y, v.y}, w1, acc[r]);
            acc[r] = __builtin_elementwise_fma(f32x2v{v.z, v.z}, w2, acc[r]);
            acc[r] = __builtin_elementwise_fma(f32x2v{v.w, v.w}, w3, acc[r]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[g][r][c] = acc[r];
  __syncthreads();
  const float sg = sigmas[labels[b]];
  if constexpr (!LGV) {
    for (int i = tid; i < 8 * 64; i += 256) {
      const int k = i >> 6, cc = i & 63, r = k >> 1, co = k & 1;
      const float v = ((red[0][r][cc][co] + red[1][r][cc][co]) + red[2][r][cc][co]) + red[3][r][cc][co];
      out[(((size_t)b * 2 + co) * H + y0 + r) * W + x0 + cc] = (v + bias[co]) / sg;
    }
  } else {
    uint32_t lmax = 0u;
    if (tid < 128) {                                 // (row, channel) x 16 float4 groups of 4 columns
      const int k = tid >> 4, r = k >> 1, co = k & 1, c4 = (tid & 15) * 4;
      float gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = ((red[0][r][c4 + q][co] + red[1][r][c4 + q][co]) + red[2][r][c4 + q][co]) + red[3][r][c4 + q][co];
        gv[q] = (v + bias[co]) / sg;
      }
      const float4 g4 = make_float4(gv[0], gv[1], gv[2], gv[3]);
      const size_t e = (((size_t)b * 2 + co) * H + y0 + r) * W + x0 + c4;
      if (out) *reinterpret_cast<float4*>(out + e) = g4;
      float4 l;
      const float4 o = langevin_group(lg, e / 4, g4, l);
      reinterpret_cast<float4*>(lg.x)[e / 4] = o;
      if (lg.lik) reinterpret_cast<float4*>(lg.lik)[e / 4] = l;
      if (co == 0) lmax = absmax4(o);
    }
    if (lg.absmax) block_absmax<4>(lmax, lg.absmax);
  }
}

// ---------------------------------------------------------------- end conv on MFMA (bf16 modes)
// The 128 -> 2 contraction as 18 partials per INPUT pixel, P[q][(tap, co)] = sum_ci e[q][ci] w[co][ci][tap]
// with e = ELU(IN++(a)), on v_mfma_f32_16x16x32_bf16 (M = 16 input pixels, N = the 18 (tap, co)
// columns in two 16-wide blocks, K = 32 channels per step; fp32x3 = lo*hi + hi*lo + hi*hi of the
// bf16 split, as conv_kernel.h), then out[p][co] = bias + sum_tap P[p + d_tap][(tap, co)] from LDS.
// Block: 16 x 32 output pixels; every pixel of its 18 x 34 input region (1.2x the outputs) is read
// and transformed ONCE, straight into A fragments (no LDS staging, no per-tap re-transform): the
// IN++/ELU transform of the direct kernel's 6 x 66 patches (1.55x, once per chunk) was its VALU
// bound.  Lane l holds pixel l % 16 of a 16-pixel group and the 8 channels {4q..4q+3, 16+4q..16+4q+3}
// (q = l / 16) of each 32-channel step -- two float4 loads; B uses the same channel order.
// The (scale, shift) of the lane's 32 channels and the B fragments stay in registers for the block.
#ifndef SDP_EC_TR         // output tile of the MFMA end conv (rows x columns)
#define SDP_EC_TR 16
#endif
#ifndef SDP_EC_TC
#define SDP_EC_TC 32
#endif
constexpr int E2_TR = SDP_EC_TR, E2_TC = SDP_EC_TC, E2_PR = E2_TR + 2, E2_PC = E2_TC + 2, E2_NP = E2_PR * E2_PC;
constexpr int E2_NG = (E2_NP + 15) / 16, E2_PS = 19;   // 16-pixel groups; P row stride (floats)
#ifndef SDP_EC_DEPTH      // groups in the load ring (2 or 3)
#define SDP_EC_DEPTH 2
#endif
#ifndef SDP_EC_KO         // diagnostic knock-outs (tools/lib_variant.sh only): 1 = no IN++/ELU transform,
#define SDP_EC_KO 0       // 2 = no MFMAs, 4 = no input loads
#endif
#ifndef SDP_EC_SS_LDS     // 1: IN++ (scale, shift) read from LDS per group; 0: held in registers
#define SDP_EC_SS_LDS 0
#endif
template <int MODE, bool LGV, typename TI = float>
__global__ __launch_bounds__(256, 2) void end_conv_mfma_kernel(const TI* __restrict__ in, const float* __restrict__ ss,
                                                               const float* __restrict__ w, const float* __restrict__ bias,
                                                               const float* __restrict__ sigmas,
                                                               const int64_t* __restrict__ labels, float* __restrict__ out,
                                                               int H, int W, LangevinArgs lg) {
  constexpr int Cin = EC_CIN;
  __shared__ float P[E2_NG * 16 * E2_PS];
  __shared__ float sw[2 * Cin * 9];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, l16 = lane & 15;
  const int tiles_row = W / E2_TC, tiles_per_img = (H / E2_TR) * tiles_row;
  const int b = blockIdx.x / tiles_per_img, tile = blockIdx.x % tiles_per_img;
  const int y0 = (tile / tiles_row) * E2_TR, x0 = (tile % tiles_row) * E2_TC;
  auto chan = [&](int ks, int j) { return 32 * ks + (j < 4 ? 4 * q + j : 12 + 4 * q + j); };

  // raw input of one 16-pixel group: clamped addresses, unconditional loads (validity applied later)
  auto load_group = [&](int g, float4 (&r)[8]) __attribute__((always_inline)) {
    const int p = 16 * g + l16, pr = p / E2_PC, pc = p - pr * E2_PC;
    const int yy = min(max(y0 - 1 + pr, 0), H - 1), xx = min(max(x0 - 1 + pc, 0), W - 1);
    const size_t src = (((size_t)b * H + yy) * W + xx) * Cin + 4 * q;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if constexpr (SDP_EC_KO & 4) {
        r[2 * ks] = make_float4((float)g, (float)ks, 0.f, 1.f);
        r[2 * ks + 1] = r[2 * ks];
        continue;
      }
      r[2 * ks] = ldg4(in, src + 32 * ks);
      r[2 * ks + 1] = ldg4(in, src + 32 * ks + 16);
    }
  };
  float4 ra[8], rb[8];
#if SDP_EC_DEPTH == 3
  float4 rc[8];
#endif
  load_group(wave, ra);
#if SDP_EC_DEPTH == 3
  load_group(min(wave + 4, E2_NG - 1), rb);
#endif

  for (int i = tid; i < 2 * Cin * 9; i += 256) sw[i] = w[i];
#if SDP_EC_SS_LDS
  // (scale, shift) of the image's channels in LDS, read per group (frees 64 VGPRs for the load ring)
  __shared__ __attribute__((aligned(16))) float4 ssl[Cin / 2];
  if (tid < Cin / 2) ssl[tid] = reinterpret_cast<const float4*>(ss + (size_t)b * Cin * 2)[tid];
  auto scale_shift = [&](int ks, int j) __attribute__((always_inline)) {
    const float4 v = ssl[chan(ks, j) >> 1];
    return (j & 1) ? make_float2(v.z, v.w) : make_float2(v.x, v.y);
  };
#else
  float2 sc[4][8];
  {
    const float2* ssb = reinterpret_cast<const float2*>(ss) + (size_t)b * Cin;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[ks][j] = ssb[chan(ks, j)];
  }
  auto scale_shift = [&](int ks, int j) __attribute__((always_inline)) { return sc[ks][j]; };
#endif
  __syncthreads();
  auto split8 = [](const float (&v)[8], bf16x8& hi, bf16x8& lo) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hi[j] = (__bf16)v[j];
      lo[j] = (__bf16)(v[j] - (float)hi[j]);
    }
  };
  bf16x8 bh[4][2], bl[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int n = 16 * nb + l16, tap = n >> 1, co = n & 1;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = n < 18 ? sw[(co * Cin + chan(ks, j)) * 9 + tap] : 0.f;
      split8(v, bh[ks][nb], bl[ks][nb]);
    }

  // ---- partials of the region's pixel groups (wave w takes groups w, w + 4, ...)
  auto do_group = [&](int g, const float4 (&r)[8]) __attribute__((always_inline)) {
    const int p = 16 * g + l16, pr = p / E2_PC, pc = p - pr * E2_PC;
    const int yy = y0 - 1 + pr, xx = x0 - 1 + pc;
    const bool ok = p < E2_NP && yy >= 0 && yy < H && xx >= 0 && xx < W;   // zero padding of the conv input
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float4 f0 = r[2 * ks], f1 = r[2 * ks + 1];
      const float raw[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 sv = scale_shift(ks, j);
        v[j] = ok ? ((SDP_EC_KO & 1) ? raw[j] : elu_max(fmaf(raw[j], sv.x, sv.y))) : 0.f;
      }
      bf16x8 ah, al;
      split8(v, ah, al);
      if constexpr (SDP_EC_KO & 2) {
        acc0[ks] += (float)ah[0] + (float)al[1];
        continue;
      }
      if constexpr (MODE == MODE_F32X3) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[ks][0], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[ks][0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[ks][1], acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[ks][1], acc1, 0, 0, 0);
      }
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[ks][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[ks][1], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {   // C[pixel 4q + rr][column l16]
      float* prow = P + (16 * g + 4 * q + rr) * E2_PS;
      prow[l16] = acc0[rr];
      if (l16 < 2) prow[16 + l16] = acc1[rr];
    }
  };
  // two groups per iteration, each computed while the other's loads fly; the loads are unconditional
  // (a clamped group index) so no branch join makes the compiler drain vmcnt
#if SDP_EC_DEPTH == 3
  for (int g = wave; g < E2_NG; g += 12) {   // ring of three: two groups' loads fly behind each compute
    load_group(min(g + 8, E2_NG - 1), rc);
    do_group(g, ra);
    load_group(min(g + 12, E2_NG - 1), ra);
    if (g + 4 < E2_NG) do_group(g + 4, rb);
    load_group(min(g + 16, E2_NG - 1), rb);
    if (g + 8 < E2_NG) do_group(g + 8, rc);
  }
#else
  for (int g = wave; g < E2_NG; g += 8) {
    load_group(min(g + 4, E2_NG - 1), rb);
    do_group(g, ra);
    load_group(min(g + 8, E2_NG - 1), ra);
    if (g + 4 < E2_NG) do_group(g + 4, rb);
  }
#endif
  __syncthreads();

  // ---- out[r][c4 .. c4+3][co] = bias + sum over the 9 taps of the partials, / sigma; one float4
  // group (4 columns of one row and channel) per thread and pass
  constexpr int G4R = E2_TC / 4, NG4 = E2_TR * 2 * G4R, NPASS = (NG4 + 255) / 256;
  const float sg = sigmas[labels[b]];
  uint32_t lmax = 0u;
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    const int gi = tid + 256 * pass;
    if (NG4 % 256 == 0 || gi < NG4) {
      const int r = gi / (2 * G4R), co = (gi / G4R) & 1, c4 = (gi % G4R) * 4;
      const float bco = bias[co];
      float gv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float s = 0.f;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) s += P[((r + tap / 3) * E2_PC + c4 + k + tap % 3) * E2_PS + 2 * tap + co];
        gv[k] = (s + bco) / sg;
      }
      const float4 g4 = make_float4(gv[0], gv[1], gv[2], gv[3]);
      const size_t e = (((size_t)b * 2 + co) * H + y0 + r) * W + x0 + c4;
      if constexpr (!LGV) {
        *reinterpret_cast<float4*>(out + e) = g4;
      } else {
        if (out) *reinterpret_cast<float4*>(out + e) = g4;
        float4 l;
        const float4 o = langevin_group(lg, e / 4, g4, l);
        reinterpret_cast<float4*>(lg.x)[e / 4] = o;
        if (lg.lik) reinterpret_cast<float4*>(lg.lik)[e / 4] = l;
        if (co == 0) lmax = max(lmax, absmax4(o));
      }
    }
  }
  if constexpr (LGV) {
    if (lg.absmax) block_absmax<4>(lmax, lg.absmax);
  }
}

// ---------------------------------------------------------------- IN++ finalize
// stats [B][T][C] of float2 (tile mean, tile M2) with `cnt` values per tile -> ss [B][C] of
// float2 (scale, shift) such that IN++(x) = x*scale + shift.  Two launches:
//   inpp_moments : B * C/8 blocks of 1024 threads = 8 channels x 128 tile groups; Chan merge of
//                  the equal-count tile partials in float64, fixed-order tree (deterministic,
//                  batch invariant) -> (mean, biased var) per (b, c)
//   inpp_ss      : one block per image over its C channels: m = mean_c(mean), v = unbiased
//                  var_c(mean) (normalization.py:164-166), then the affine of every channel.
// (One launch with a last-block ticket measured slower: the device-scope fences each block needs
// to publish its moments across XCDs cost more than the second launch.)
constexpr int INPP_CPB = 8, INPP_G = 1024 / INPP_CPB;
__global__ __launch_bounds__(1024) void inpp_moments_kernel(const float2* __restrict__ stats, int T, float cnt, int C,
                                                            double2* __restrict__ mv) {
  __shared__ double red[1024];
  const int tid = threadIdx.x, l = tid % INPP_CPB, g = tid / INPP_CPB;
  const int nb = C / INPP_CPB;
  const int b = blockIdx.x / nb, c = (blockIdx.x % nb) * INPP_CPB + l;
  const float2* st = stats + (size_t)b * T * C + c;
  auto group_sum = [&](double v) {   // sum over the 128 tile groups of each channel, fixed tree order
    red[tid] = v;
    __syncthreads();
    for (int s = INPP_G / 2; s > 0; s >>= 1) {
      if (g < s) red[tid] += red[tid + s * INPP_CPB];
      __syncthreads();
    }
    const double r = red[l];
    __syncthreads();
    return r;
  };
  double sm = 0.0;
  for (int t = g; t < T; t += INPP_G) sm += st[(size_t)t * C].x;
  const double mean = group_sum(sm) / T;
  double m2 = 0.0;
  for (int t = g; t < T; t += INPP_G) {
    const float2 v = st[(size_t)t * C];
    const double dm = (double)v.x - mean;
    m2 += (double)v.y + dm * dm * cnt;
  }
  m2 = group_sum(m2);
  if (g == 0) mv[(size_t)b * C + c] = make_double2(mean, m2 / ((double)T * cnt));   // biased (nn.InstanceNorm2d)
}

__global__ __launch_bounds__(1024) void inpp_ss_kernel(const double2* __restrict__ mv, int C,
                                                       const float* __restrict__ alpha, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float2* __restrict__ ss,
                                                       float4* __restrict__ nst) {
  __shared__ double red[1024];
  const int b = blockIdx.x, c = threadIdx.x;
  const double2 m_v = mv[(size_t)b * C + c];
  const double mean = m_v.x, var = m_v.y;
  red[c] = mean;
  __syncthreads();
  for (int s = C / 2; s > 0; s >>= 1) {
    if (c < s) red[c] += red[c + s];
    __syncthreads();
  }
  const double m = red[0] / C;
  __syncthreads();
  red[c] = (mean - m) * (mean - m);
  __syncthreads();
  for (int s = C / 2; s > 0; s >>= 1) {
    if (c < s) red[c] += red[c + s];
    __syncthreads();
  }
  const double v = red[0] / (C - 1);
  const double inv = 1.0 / sqrt(var + 1e-5);
  const double mn = (mean - m) / sqrt(v + 1e-5);
  const double gm = gamma[c];
  const double scale = gm * inv;
  const double shift = gm * (-mean * inv + mn * (double)alpha[c]) + (double)beta[c];
  ss[(size_t)b * C + c] = make_float2((float)scale, (float)shift);
  // training: the per-(b,c) statistics the backward needs (mean, rstd, mhat, 1/sqrt(v + eps))
  if (nst) nst[(size_t)b * C + c] = make_float4((float)mean, (float)inv, (float)mn, (float)(1.0 / sqrt(v + 1e-5)));
}

// ---------------------------------------------------------------- maxpool 5x5 s1 p2 (NHWC)
// Block = a strip of MP_COLS columns x 128 channels (32 float4 lanes per pixel, so a wave reads
// two whole 512-B pixel rows) over `rows` output rows.  Each input row of the strip plus its 2+2
// halo columns is landed in LDS ONCE by LDS-DMA, MP_D rows ahead of its use in a ring of MP_NS
// row slots; every thread takes the 5-wide horizontal max of its (column, 4 channels) from LDS and
// slides a 5-row window of those maxima in registers -> per output (MP_COLS+4)/MP_COLS x
// (rows+4)/rows global reads.  One barrier per row.  The DMA has no register result, so the
// compiler places no wait for it: each thread waits for its own DMA of a row with an explicit
// vmcnt (vector memory ops retire in order on gfx9, and exactly P DMAs + S stores per row follow).
// Out-of-image rows/columns are read at the clamped (edge) position: a copy of a value that is
// inside the same 5x5 window, so the max is the one -inf padding gives.
// idx (training): window position 0..24 of the max in row-major window order, the first one
// on ties (strict > along the row, then strict > down the rows) -- the index torch's
// max_pool2d keeps for its backward.  For it the edge copies are overwritten with -inf (an edge
// copy sits earlier in window order than its original and would take the tie), so -inf padding
// never wins.
// output rows per block: 32 while the grid keeps >= MP_MIN_BLOCKS blocks, else 16 -- 256 @32x512
// (512 blocks either way) 35.5 -> 27.3 us, 128 @64x1024 58.4 -> 57 us; 128 @32x512 would drop to 256
// blocks and run 19.1 -> 23.2 us, so it keeps 16 (profiles/experiments/r02_maxpool_rows_ab.log)
#ifndef SDP_MP_MIN_BLOCKS
#define SDP_MP_MIN_BLOCKS 512
#endif
constexpr int MP_COLS = 8, MP_NS = 6, MP_D = 2, MP_MIN_BLOCKS = SDP_MP_MIN_BLOCKS;
template <bool IDX>
__global__ __launch_bounds__(256) void maxpool5_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                       uchar4* __restrict__ idx, int B, int H, int W, int C,
                                                       int rows) {
  constexpr int SC = MP_COLS + 4;                  // staged columns
  constexpr int NUNIT = SC * 32;                   // float4 units per staged row: 384 = waves 0..3 + waves 0..1
  static_assert(NUNIT == 384 && MP_NS >= MP_D + 1 && 4 + MP_D <= MP_NS, "maxpool5 ring layout");
  __shared__ __attribute__((aligned(16))) float4 row_buf[MP_NS][NUNIT];
  const int tid = threadIdx.x, c4 = tid & 31, xl = tid >> 5;   // (column in strip, float4 channel group)
  const int wave = tid >> 6;
  const int C4 = C / 4, CG = C4 / 32;              // 128-channel groups
  const int strips = W / MP_COLS, RB = (H + rows - 1) / rows;
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so give each XCD a contiguous
  // range -- the strips on either side of a strip (its halo columns) then sit in the same L2
  const int nwg = gridDim.x;
  int t = (nwg & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (nwg >> 3) + ((int)blockIdx.x >> 3);
  const int cg = t % CG;
  t /= CG;
  const int strip = t % strips;
  t /= strips;
  const int rb = t % RB, b = t / RB;
  const int x0 = strip * MP_COLS, y0 = rb * rows, y1 = min(H, y0 + rows);
  const int x = x0 + xl;
  const float NEG = -INFINITY;
  const i32x4 rs = buffer_desc(in + (size_t)b * H * W * C, (uint32_t)H * W * C * 4);
  const uint32_t ring = (uint32_t)reinterpret_cast<uintptr_t>(&row_buf[0][0]);
  // unit k of this thread: i = tid + 256k (k = 1 only on waves 0, 1), staged column i >> 5
  int colo[2];
  bool colok[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + k * 256, xx = x0 - 2 + (i >> 5);
    colok[k] = xx >= 0 && xx < W;
    colo[k] = ((min(max(xx, 0), W - 1) * C4) + cg * 32 + (i & 31)) * 16;
  }
  auto dma_row = [&](int yy, int slot) {
    const int rowo = min(max(yy, 0), H - 1) * W * C4 * 16;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && wave >= 2) break;              // wave-uniform: units 256..383 are waves 0, 1
      dma16_lds_opaque(rs, ring + (slot * NUNIT + (tid & ~63) + k * 256) * 16, colo[k], rowo);
    }
  };
  auto pad_row = [&](int yy, int slot) {           // IDX: the edge copies of this thread's units -> -inf
    if constexpr (IDX) {
      const bool rowok = yy >= 0 && yy < H;
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if ((k == 0 || wave < 2) && !(rowok && colok[k])) row_buf[slot][tid + k * 256] = make_float4(NEG, NEG, NEG, NEG);
    }
  };
  auto hmax = [&](int slot, float4& m, uchar4& c) {
    m = make_float4(NEG, NEG, NEG, NEG);
    c = make_uchar4(2, 2, 2, 2);
#pragma unroll
    for (int dx = 0; dx < 5; ++dx) {
      const float4 v = row_buf[slot][(xl + dx) * 32 + c4];
      const unsigned char k = (unsigned char)dx;
      if (v.x > m.x) { m.x = v.x; c.x = k; }
      if (v.y > m.y) { m.y = v.y; c.y = k; }
      if (v.z > m.z) { m.z = v.z; c.z = k; }
      if (v.w > m.w) { m.w = v.w; c.w = k; }
    }
  };
  float4 hm[5];
  uchar4 hc[5];
  // row y0 - 2 + ri sits in slot ri % MP_NS.  Prologue: rows ri = 0 .. 3 + MP_D in flight at once;
  // rows 0..3 prime the window
#pragma unroll
  for (int ri = 0; ri < 4 + MP_D; ++ri) dma_row(y0 - 2 + ri, ri);
  __builtin_amdgcn_s_waitcnt(0x0f70);              // vmcnt(0)
#pragma unroll
  for (int ri = 0; ri < 4 + MP_D; ++ri) pad_row(y0 - 2 + ri, ri);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) hmax(k, hm[k], hc[k]);
  // iteration j (output row y0 + j) reads row ri = j + 4 and lands row ri = j + 4 + MP_D.  Row
  // j + 4 was landed at iteration j - MP_D (or in the prologue); after that DMA this thread issued
  // S stores, then P DMAs + S stores in each of the MP_D - 1 iterations between
  constexpr int S = IDX ? 2 : 1;
  constexpr int WAIT01 = S + (MP_D - 1) * (2 + S), WAIT23 = S + (MP_D - 1) * (1 + S);
  static_assert(WAIT01 < 64, "vmcnt field");
  for (int y = y0; y < y1; ++y) {
    const int j = y - y0;
    const int slot = (j + 4) % MP_NS;
    if (wave < 2) __builtin_amdgcn_s_waitcnt(0x0f70 | (WAIT01 & 15) | ((WAIT01 >> 4) << 14));
    else __builtin_amdgcn_s_waitcnt(0x0f70 | (WAIT23 & 15) | ((WAIT23 >> 4) << 14));
    if (j >= MP_D) pad_row(y + 2, slot);           // rows past the prologue were landed in the loop
    __syncthreads();                               // row y+2 landed everywhere; row j+4+MP_D-MP_NS consumed
    hmax(slot, hm[4], hc[4]);
    dma_row(y + 2 + MP_D, (j + 4 + MP_D) % MP_NS);
    float4 m = hm[0];
    uchar4 bi = hc[0];                             // row 0 of the window
#pragma unroll
    for (int r = 1; r < 5; ++r) {
      const unsigned char ro = (unsigned char)(5 * r);
      if (hm[r].x > m.x) { m.x = hm[r].x; bi.x = ro + hc[r].x; }
      if (hm[r].y > m.y) { m.y = hm[r].y; bi.y = ro + hc[r].y; }
      if (hm[r].z > m.z) { m.z = hm[r].z; bi.z = ro + hc[r].z; }
      if (hm[r].w > m.w) { m.w = hm[r].w; bi.w = ro + hc[r].w; }
    }
    const size_t o = (((size_t)b * H + y) * W + x) * C4 + cg * 32 + c4;
    reinterpret_cast<float4*>(out)[o] = m;
    if constexpr (IDX) idx[o] = bi;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hm[r] = hm[r + 1];
      hc[r] = hc[r + 1];
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);              // the rows landed past the strip's end
}

// maxpool 5x5 s1 p2 with the argmax indices on a bf16 tensor (the bf16 training tape, train.hip): the
// same window order, tie rule and -inf padding as maxpool5_kernel<true>.  Block = 32 columns x 128
// channels over `rows` output rows; thread (column xl, 8-channel group c8) owns column xl.
// Each input row of the strip (+2 halo columns each side, out-of-image positions -inf) is read once into
// an LDS slot (the next row's loads fly in registers while the current row is reduced), the horizontal
// 5-max comes from LDS and slides down a 5-row register window
constexpr int MPH_COLS = 16, MPH_SC = MPH_COLS + 4, MPH_U = MPH_SC * 16;   // staged 16-B units per row: 320
__global__ __launch_bounds__(256) void maxpool5_h16_kernel(const __bf16* __restrict__ in, __bf16* __restrict__ out,
                                                           unsigned char* __restrict__ idx, int B, int H, int W, int C,
                                                           int rows) {
  __shared__ uint4 srow[2][MPH_U];
  const int tid = threadIdx.x, c8 = tid & 15, xl = tid >> 4;
  const int CG = C / 128, strips = W / MPH_COLS, RB = (H + rows - 1) / rows;
  int t = blockIdx.x;
  const int cg = t % CG;
  t /= CG;
  const int strip = t % strips;
  t /= strips;
  const int rb = t % RB, b = t / RB;
  const int x0 = strip * MPH_COLS, y0 = rb * rows, y1 = min(H, y0 + rows);
  constexpr uint32_t NEG2 = 0xff80ff80u;           // two bf16 -inf
  uint4 pre[2];
  auto fetch = [&](int yy) {                        // row yy's units of this thread -> registers
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k, col = i >> 4, cc = i & 15, xx = x0 - 2 + col;
      pre[k] = make_uint4(NEG2, NEG2, NEG2, NEG2);
      if (i < MPH_U && yy >= 0 && yy < H && xx >= 0 && xx < W)
        pre[k] = *reinterpret_cast<const uint4*>(in + (((size_t)b * H + yy) * W + xx) * C + cg * 128 + cc * 8);
    }
  };
  auto put = [&](int slot) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k;
      if (i < MPH_U) srow[slot][i] = pre[k];
    }
  };
  // horizontal 5-max (first max on ties) of column xl from LDS slot
  auto hmax = [&](int slot, float (&m)[8], unsigned char (&c)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      m[e] = -INFINITY;
      c[e] = 2;
    }
#pragma unroll
    for (int dx = 0; dx < 5; ++dx) {
      const uint4 u = srow[slot][(xl + dx) * 16 + c8];
      const float4 lo = bf4_to_f4(make_uint2(u.x, u.y)), hi = bf4_to_f4(make_uint2(u.z, u.w));
      const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (v[e] > m[e]) {
          m[e] = v[e];
          c[e] = (unsigned char)dx;
        }
    }
  };
  float hm[5][8];
  unsigned char hc[5][8];
  fetch(y0 - 2);
#pragma unroll
  for (int r = 0; r < 5; ++r) {                     // rows y0-2 .. y0+1 into the window, y0+2 fetched
    __syncthreads();
    put(r & 1);
    fetch(y0 - 1 + r);
    __syncthreads();
    if (r < 4) hmax(r & 1, hm[r], hc[r]);
  }
  // slot 0 holds row y0 + 2 (r = 4), pre holds row y0 + 3
  int slot = 0;
  for (int y = y0; y < y1; ++y) {
    hmax(slot, hm[4], hc[4]);
    __syncthreads();                                 // the slot about to be refilled has been read
    slot ^= 1;
    put(slot);                                       // row y + 3
    fetch(y + 4);
    float m[8];
    unsigned char bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      m[e] = hm[0][e];
      bi[e] = hc[0][e];
#pragma unroll
      for (int r = 1; r < 5; ++r)
        if (hm[r][e] > m[e]) {
          m[e] = hm[r][e];
          bi[e] = (unsigned char)(5 * r) + hc[r][e];
        }
    }
    const size_t o = (((size_t)b * H + y) * W + x0 + xl) * C + cg * 128 + c8 * 8;
    *reinterpret_cast<uint4*>(out + o) =
        make_uint4(pack_bf2(m[0], m[1]), pack_bf2(m[2], m[3]), pack_bf2(m[4], m[5]), pack_bf2(m[6], m[7]));
    if (idx) {
      uint2 kk;
      kk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      kk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *reinterpret_cast<uint2*>(idx + o) = kk;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        hm[r][e] = hm[r + 1][e];
        hc[r][e] = hc[r + 1][e];
      }
    __syncthreads();                                 // the new slot is complete
  }
}

// ---------------------------------------------------------------- host launchers
hipError_t begin_conv(const float* x, const float* w, const float* bias, float* out, float* stats, int B, int H, int W,
                      hipStream_t st, int mode, bool h16) {
  if (W % BC_TP) return hipErrorInvalidValue;
  const int ntiles = B * H * (W / BC_TP);
  if (h16) {   // bf16 output (training tape): bf16 mode, MFMA form
    if (mode != MODE_BF16) return hipErrorInvalidValue;
    const dim3 grid(std::min(ntiles, 256 * BM_WG_PER_CU));
    hipLaunchKernelGGL((begin_conv_mfma_kernel<MODE_BF16, __bf16>), grid, dim3(256), 0, st, x, w, bias,
                       reinterpret_cast<__bf16*>(out), stats, B, H, W);
    return hipGetLastError();
  }
  if (mode != MODE_F32 && !SDP_HEAD_DIRECT) {   // bf16 modes: the MFMA form
    const dim3 grid(std::min(ntiles, 256 * BM_WG_PER_CU));
    if (mode == MODE_F32X3)
      hipLaunchKernelGGL(begin_conv_mfma_kernel<MODE_F32X3>, grid, dim3(256), 0, st, x, w, bias, out, stats, B, H, W);
    else
      hipLaunchKernelGGL(begin_conv_mfma_kernel<MODE_BF16>, grid, dim3(256), 0, st, x, w, bias, out, stats, B, H, W);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(begin_conv_kernel, dim3(std::min(ntiles, 256 * BC_WG_PER_CU)), dim3(256), 0, st, x, w, bias, out,
                     stats, B, H, W);
  return hipGetLastError();
}

hipError_t end_conv(const float* in, const float* ss, const float* w, const float* bias, const float* sigmas,
                    const int64_t* labels, float* out, int B, int H, int W, int Cin, hipStream_t st,
                    const LangevinArgs* lg, int mode, bool h16) {
  if (Cin != EC_CIN) return hipErrorInvalidValue;
  if (h16) {   // bf16 input (training tape): bf16 mode, scores only
    if (mode != MODE_BF16 || lg || H % E2_TR || W % E2_TC) return hipErrorInvalidValue;
    hipLaunchKernelGGL((end_conv_mfma_kernel<MODE_BF16, false, __bf16>), dim3(B * (H / E2_TR) * (W / E2_TC)), dim3(256), 0, st,
                       reinterpret_cast<const __bf16*>(in), ss, w, bias, sigmas, labels, out, H, W, LangevinArgs{});
    return hipGetLastError();
  }
  if (mode != MODE_F32 && !SDP_HEAD_DIRECT && H % E2_TR == 0 && W % E2_TC == 0) {   // bf16 modes: the MFMA form
    const dim3 grid(B * (H / E2_TR) * (W / E2_TC));
    const LangevinArgs la = lg ? *lg : LangevinArgs{};
    if (mode == MODE_F32X3) {
      if (lg) hipLaunchKernelGGL((end_conv_mfma_kernel<MODE_F32X3, true>), grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W, la);
      else hipLaunchKernelGGL((end_conv_mfma_kernel<MODE_F32X3, false>), grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W, la);
    } else {
      if (lg) hipLaunchKernelGGL((end_conv_mfma_kernel<MODE_BF16, true>), grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W, la);
      else hipLaunchKernelGGL((end_conv_mfma_kernel<MODE_BF16, false>), grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W, la);
    }
    return hipGetLastError();
  }
  if (H % 4 || W % 64) return hipErrorInvalidValue;
  const dim3 grid(B * (H / 4) * (W / 64));
  if (lg)
    hipLaunchKernelGGL(end_conv_kernel<true>, grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W, *lg);
  else
    hipLaunchKernelGGL(end_conv_kernel<false>, grid, dim3(256), 0, st, in, ss, w, bias, sigmas, labels, out, H, W,
                       LangevinArgs{});
  return hipGetLastError();
}

hipError_t inpp_finalize(const float* stats, int B, int T, float cnt, int C, const float* alpha, const float* gamma,
                         const float* beta, float* ss, hipStream_t st, float* nst, void* scratch) {
  if (C % 64 || C > 1024 || (C & (C - 1))) return hipErrorInvalidValue;
  double2* mv = reinterpret_cast<double2*>(scratch);
  hipLaunchKernelGGL(inpp_moments_kernel, dim3(B * (C / INPP_CPB)), dim3(1024), 0, st,
                     reinterpret_cast<const float2*>(stats), T, cnt, C, mv);
  hipLaunchKernelGGL(inpp_ss_kernel, dim3(B), dim3(C), 0, st, mv, C, alpha, gamma, beta, reinterpret_cast<float2*>(ss),
                     reinterpret_cast<float4*>(nst));
  return hipGetLastError();
}

// 2x2 mean pool of the ConvMeanPool 1x1 shortcut's input (layers.py:291-313 with the mean taken before the
// 1x1 conv instead of after it: the conv is linear per pixel, so the two orders differ only in float
// rounding, and the conv then runs on a quarter of the pixels).  Summation order of layers.py:311-312:
// ((x[::2, ::2] + x[1::2, ::2]) + x[::2, 1::2]) + x[1::2, 1::2], then / 4.
__global__ __launch_bounds__(256) void avgpool2_kernel(const float4* __restrict__ in, float4* __restrict__ out, int H,
                                                       int W, int C4, size_t n4) {
  const int Ho = H / 2, Wo = W / 2;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    size_t p = i / C4;
    const int x = (int)(p % Wo);
    p /= Wo;
    const int y = (int)(p % Ho);
    const size_t b = p / Ho;
    const size_t r0 = ((b * H + 2 * y) * W + 2 * x) * C4 + c, r1 = r0 + (size_t)W * C4;
    const float4 a00 = in[r0], a01 = in[r0 + C4], a10 = in[r1], a11 = in[r1 + C4];
    out[i] = make_float4((((a00.x + a10.x) + a01.x) + a11.x) / 4.0f, (((a00.y + a10.y) + a01.y) + a11.y) / 4.0f,
                         (((a00.z + a10.z) + a01.z) + a11.z) / 4.0f, (((a00.w + a10.w) + a01.w) + a11.w) / 4.0f);
  }
}

hipError_t avgpool2(const float* in, float* out, int B, int H, int W, int C, hipStream_t st) {
  if ((H & 1) || (W & 1) || (C & 3)) return hipErrorInvalidValue;
  const size_t n4 = (size_t)B * (H / 2) * (W / 2) * (C / 4);
  const int grid = (int)std::min<size_t>((n4 + 255) / 256, 256 * 32);
  hipLaunchKernelGGL(avgpool2_kernel, dim3(grid), dim3(256), 0, st, reinterpret_cast<const float4*>(in),
                     reinterpret_cast<float4*>(out), H, W, C / 4, n4);
  return hipGetLastError();
}

hipError_t maxpool5(const float* in, float* out, int B, int H, int W, int C, hipStream_t st, uint8_t* idx, bool h16) {
  if (C % 128 || W % MP_COLS) return hipErrorInvalidValue;
  if (h16) {
    if (W % MPH_COLS) return hipErrorInvalidValue;
    auto hb = [&](int rows) { return B * ((H + rows - 1) / rows) * (W / MPH_COLS) * (C / 128); };
    const int rows = hb(32) >= 1024 ? 32 : (hb(16) >= 1024 ? 16 : 8), grid = hb(rows);
    hipLaunchKernelGGL(maxpool5_h16_kernel, dim3(grid), dim3(256), 0, st, reinterpret_cast<const __bf16*>(in),
                       reinterpret_cast<__bf16*>(out), idx, B, H, W, C, rows);
    return hipGetLastError();
  }
  auto blocks = [&](int rows) { return B * ((H + rows - 1) / rows) * (W / MP_COLS) * (C / 128); };
  const int rows = blocks(32) >= MP_MIN_BLOCKS ? 32 : 16, grid = blocks(rows);
  if (idx)
    hipLaunchKernelGGL(maxpool5_kernel<true>, dim3(grid), dim3(256), 0, st, in, out, reinterpret_cast<uchar4*>(idx), B, H,
                       W, C, rows);
  else
    hipLaunchKernelGGL(maxpool5_kernel<false>, dim3(grid), dim3(256), 0, st, in, out, nullptr, B, H, W, C, rows);
  return hipGetLastError();
}

}  // namespace sdp
