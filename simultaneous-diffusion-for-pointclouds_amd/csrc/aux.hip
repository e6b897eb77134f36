// Small / memory-bound kernels of the score network (gfx950).
//   begin_conv : input prep (2x-1, coordinate channels; ncsnv2.py:485-496) fused with the
//                4->ngf zero-padded 3x3 conv + bias (ncsnv2.py:433,498) and IN++ tile stats.
//   end_conv   : final IN++ affine + ELU prologue, ngf->2 zero-padded 3x3 conv + bias,
//                / sigmas[y] (ncsnv2.py:510-516), NCHW output.
//   inpp_finalize : per-tile (mean, M2) -> per-(b,c) InstanceNorm2dPlus scale/shift
//                (normalization.py:163-176), in two small launches.
//   maxpool5   : MaxPool2d(5, stride 1, padding 2) of CRPBlock (layers.py:70), NHWC.
#include "common.h"

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
// block: 64 output pixels of one row x 128 channels; thread = (pixel, 32-channel quarter).
// The 64 x 128 result goes through LDS so the stores are whole 512-B pixel rows and the
// per-(b, c) statistics of the 64-pixel tile are a two-pass column sum (no wave shuffles).
__global__ __launch_bounds__(256) void begin_conv_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         float* __restrict__ stats, int H, int W) {
  constexpr int CO = 128, OS = CO + 4;   // staged row stride (floats)
  __shared__ float sw[36 * CO];          // [ci*9 + tap][co]
  __shared__ float sp[4][3][66];         // prepped input patch [ci][row][col]
  __shared__ float so[64 * OS];          // staged output [px][co]
  const int tid = threadIdx.x;
  const int tiles_row = W / 64;
  const int tiles_per_img = H * tiles_row;
  const int b = blockIdx.x / tiles_per_img, tile = blockIdx.x % tiles_per_img;
  const int y = tile / tiles_row, x0 = (tile % tiles_row) * 64;
  for (int i = tid; i < 36 * CO; i += 256) {
    const int co = i % CO, k = i / CO;          // k = ci*9 + tap ; w is [co][ci][3][3]
    sw[i] = w[co * 36 + k];
  }
  for (int i = tid; i < 4 * 3 * 66; i += 256) {
    const int ci = i / 198, r = (i / 66) % 3, c = i % 66;
    const int yy = y - 1 + r, xx = x0 - 1 + c;
    float v = 0.f;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      if (ci < 2) v = 2.f * x[(((size_t)b * 2 + ci) * H + yy) * W + xx] - 1.f;
      else if (ci == 2) v = linspace01(xx, W);
      else v = linspace01(yy, H);
    }
    sp[ci][r][c] = v;
  }
  __syncthreads();
  const int px = tid & 63, cq = tid >> 6;
  float acc[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) acc[j] = bias[cq * 32 + j];
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float v = sp[ci][tap / 3][px + tap % 3];
      const float* wr = sw + (ci * 9 + tap) * CO + cq * 32;
#pragma unroll
      for (int j = 0; j < 32; ++j) acc[j] = fmaf(v, wr[j], acc[j]);
    }
#pragma unroll
  for (int j = 0; j < 32; j += 4)
    *reinterpret_cast<float4*>(&so[px * OS + cq * 32 + j]) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
  __syncthreads();
  // rows: 32 threads per pixel row (16 B each), 8 rows per pass
  float* o = out + (((size_t)b * H + y) * W + x0) * CO;
  for (int i = tid; i < 64 * 32; i += 256) {
    const int p = i >> 5, c4 = i & 31;
    *reinterpret_cast<float4*>(o + (size_t)p * CO + c4 * 4) = *reinterpret_cast<const float4*>(&so[p * OS + c4 * 4]);
  }
  // statistics: thread (channel, half) sums 32 pixels, two passes, Chan merge of the halves
  const int c = tid & 127, hf = tid >> 7;
  float sm = 0.f;
  for (int p = hf * 32; p < hf * 32 + 32; ++p) sm += so[p * OS + c];
  const float mh = sm * (1.f / 32.f);
  float m2 = 0.f;
  for (int p = hf * 32; p < hf * 32 + 32; ++p) {
    const float dv = so[p * OS + c] - mh;
    m2 = fmaf(dv, dv, m2);
  }
  __syncthreads();
  float2* red = reinterpret_cast<float2*>(sw);
  red[tid] = make_float2(mh, m2);
  __syncthreads();
  if (hf == 0) {
    const float2 q = red[tid + 128];
    const float dm = mh - q.x;
    float2* st = reinterpret_cast<float2*>(stats) + ((size_t)b * tiles_per_img + tile) * CO + c;
    *st = make_float2(0.5f * (mh + q.x), m2 + q.y + dm * dm * 16.f);
  }
}

// ---------------------------------------------------------------- end conv (128 -> 2), NCHW out
// block: 4 rows x 64 cols of output.  Per 32-channel chunk the (6 x 66) patch (IN++ affine +
// ELU applied on the way in) sits in LDS; wave g (warp-uniform) takes channels 8g..8g+7 of
// the chunk, each thread one column: a patch column of 6 rows feeds its 4 output rows x 3
// taps x 2 channels, so every LDS read serves 4 FMAs.  The 4 channel-group partials are
// summed through LDS at the end.
__global__ __launch_bounds__(256) void end_conv_kernel(const float* __restrict__ in, const float* __restrict__ ss,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       const float* __restrict__ sigmas, const int64_t* __restrict__ labels,
                                                       float* __restrict__ out, int H, int W, int Cin) {
  constexpr int PS = 33;
  __shared__ float sp[6 * 66 * PS];
  __shared__ float sw[2 * 32 * 9];   // [co][ci][tap] of the chunk
  __shared__ float red[4][8][64];
  const int tid = threadIdx.x;
  const int tiles_row = W / 64, tiles_per_img = (H / 4) * tiles_row;
  const int b = blockIdx.x / tiles_per_img, tile = blockIdx.x % tiles_per_img;
  const int y0 = (tile / tiles_row) * 4, x0 = (tile % tiles_row) * 64;
  const int c = tid & 63, g = tid >> 6;
  const float* ssb = ss + (size_t)b * Cin * 2;
  float acc[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = 0.f;
  for (int c0 = 0; c0 < Cin; c0 += 32) {
    __syncthreads();
    for (int i = tid; i < 6 * 66 * 8; i += 256) {
      const int pix = i >> 3, cv = i & 7;
      const int pr = pix / 66, pc = pix % 66;
      const int yy = y0 - 1 + pr, xx = x0 - 1 + pc;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const int ch = c0 + cv * 4;
        const float4 f = *reinterpret_cast<const float4*>(in + (((size_t)b * H + yy) * W + xx) * Cin + ch);
        const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = elu(fmaf(fv[k], ssb[(ch + k) * 2], ssb[(ch + k) * 2 + 1]));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) sp[pix * PS + cv * 4 + k] = v[k];
    }
    for (int i = tid; i < 2 * 32 * 9; i += 256) {
      const int co = i / 288, rem = i % 288, ci = rem / 9, tap = rem % 9;
      sw[i] = w[((size_t)co * Cin + c0 + ci) * 9 + tap];
    }
    __syncthreads();
    for (int cj = 0; cj < 8; ++cj) {
      const int ci = g * 8 + cj;
      float wv[2][9];
#pragma unroll
      for (int co = 0; co < 2; ++co)
#pragma unroll
        for (int t = 0; t < 9; ++t) wv[co][t] = sw[co * 288 + ci * 9 + t];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float col[6];
#pragma unroll
        for (int pr = 0; pr < 6; ++pr) col[pr] = sp[(pr * 66 + c + kw) * PS + ci];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            acc[r][0] = fmaf(col[r + kh], wv[0][kh * 3 + kw], acc[r][0]);
            acc[r][1] = fmaf(col[r + kh], wv[1][kh * 3 + kw], acc[r][1]);
          }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[g][2 * r][c] = acc[r][0];
    red[g][2 * r + 1][c] = acc[r][1];
  }
  __syncthreads();
  const float sg = sigmas[labels[b]];
  for (int i = tid; i < 8 * 64; i += 256) {
    const int k = i >> 6, cc = i & 63, r = k >> 1, co = k & 1;
    const float v = ((red[0][k][cc] + red[1][k][cc]) + red[2][k][cc]) + red[3][k][cc];
    out[(((size_t)b * 2 + co) * H + y0 + r) * W + x0 + cc] = (v + bias[co]) / sg;
  }
}

// ---------------------------------------------------------------- IN++ finalize
// stats [B][T][C] of float2 (tile mean, tile M2) with `cnt` values per tile -> ss [B][C] of
// float2 (scale, shift) such that IN++(x) = x*scale + shift.  Two launches:
//   inpp_moments : one 1024-thread block per (image, 64 channels), 16 tile groups; Chan merge
//                  of the equal-count partials in float64 -> (mean, biased var) per (b, c)
//   inpp_ss      : one block per image over its C channels: m = mean_c(mean), v = unbiased
//                  var_c(mean) (normalization.py:164-166), then the affine of every channel
constexpr int INPP_G = 16;   // tile groups (one wave each) per inpp_moments block of 64 channels
__global__ __launch_bounds__(64 * INPP_G) void inpp_moments_kernel(const float2* __restrict__ stats, int T, float cnt,
                                                                   int C, double2* __restrict__ mv) {
  __shared__ double red[64 * INPP_G];
  const int cb = C / 64, l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int b = blockIdx.x / cb, c = (blockIdx.x % cb) * 64 + l;
  const float2* st = stats + (size_t)b * T * C + c;
  auto block_sum = [&](double v) {
    red[threadIdx.x] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < INPP_G; ++k) s += red[k * 64 + l];   // fixed order: deterministic
    __syncthreads();
    return s;
  };
  double sm = 0.0;
#pragma unroll 4
  for (int t = g; t < T; t += INPP_G) sm += st[(size_t)t * C].x;
  const double mean = block_sum(sm) / T;
  double m2 = 0.0;
#pragma unroll 4
  for (int t = g; t < T; t += INPP_G) {
    const float2 v = st[(size_t)t * C];
    const double dm = (double)v.x - mean;
    m2 += (double)v.y + dm * dm * cnt;
  }
  m2 = block_sum(m2);
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
// Separable: a thread owns 4 channels of one column over MP_ROWS output rows; it takes the
// 5-wide horizontal max of every input row it needs (MP_ROWS + 4 of them) once and slides a
// 5-row window over them -> 5*(MP_ROWS+4)/MP_ROWS loads per output instead of 25.
// idx (training): window position 0..24 of the max in row-major window order, the first one
// on ties (strict > along the row, then strict > down the rows) -- the index torch's
// max_pool2d keeps for its backward.  -inf padding never wins.
constexpr int MP_ROWS = 16;
__global__ __launch_bounds__(256) void maxpool5_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                       uchar4* __restrict__ idx, int B, int H, int W, int C) {
  const int C4 = C / 4, RB = (H + MP_ROWS - 1) / MP_ROWS;
  const size_t n = (size_t)B * RB * W * C4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    size_t p = i / C4;
    const int x = p % W;
    p /= W;
    const int rb = p % RB;
    const int b = p / RB;
    const int y0 = rb * MP_ROWS, y1 = min(H, y0 + MP_ROWS);
    float4 hm[5];          // horizontal maxima of rows y-2 .. y+2 (ring)
    uchar4 hc[5];          // their column positions dx+2
    auto hrow = [&](int yy, float4& m, uchar4& c) {
      m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      c = make_uchar4(2, 2, 2, 2);
      if (yy < 0 || yy >= H) return;
      const float* row = in + (((size_t)b * H + yy) * W) * C + c4 * 4;
#pragma unroll
      for (int dx = -2; dx <= 2; ++dx) {
        const int xx = x + dx;
        if (xx < 0 || xx >= W) continue;
        const float4 v = *reinterpret_cast<const float4*>(row + (size_t)xx * C);
        const unsigned char k = (unsigned char)(dx + 2);
        if (v.x > m.x) { m.x = v.x; c.x = k; }
        if (v.y > m.y) { m.y = v.y; c.y = k; }
        if (v.z > m.z) { m.z = v.z; c.z = k; }
        if (v.w > m.w) { m.w = v.w; c.w = k; }
      }
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) hrow(y0 - 2 + k, hm[k], hc[k]);
    for (int y = y0; y < y1; ++y) {
      hrow(y + 2, hm[4], hc[4]);
      float4 m = hm[0];
      uchar4 bi = make_uchar4(hc[0].x, hc[0].y, hc[0].z, hc[0].w);   // row 0 of the window
#pragma unroll
      for (int r = 1; r < 5; ++r) {
        const unsigned char ro = (unsigned char)(5 * r);
        if (hm[r].x > m.x) { m.x = hm[r].x; bi.x = ro + hc[r].x; }
        if (hm[r].y > m.y) { m.y = hm[r].y; bi.y = ro + hc[r].y; }
        if (hm[r].z > m.z) { m.z = hm[r].z; bi.z = ro + hc[r].z; }
        if (hm[r].w > m.w) { m.w = hm[r].w; bi.w = ro + hc[r].w; }
      }
      const size_t o = (((size_t)b * H + y) * W + x) * C4 + c4;
      reinterpret_cast<float4*>(out)[o] = m;
      if (idx) idx[o] = bi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hm[r] = hm[r + 1];
        hc[r] = hc[r + 1];
      }
    }
  }
}

// ---------------------------------------------------------------- host launchers
hipError_t begin_conv(const float* x, const float* w, const float* bias, float* out, float* stats, int B, int H, int W,
                      hipStream_t st) {
  hipLaunchKernelGGL(begin_conv_kernel, dim3(B * H * (W / 64)), dim3(256), 0, st, x, w, bias, out, stats, H, W);
  return hipGetLastError();
}

hipError_t end_conv(const float* in, const float* ss, const float* w, const float* bias, const float* sigmas,
                    const int64_t* labels, float* out, int B, int H, int W, int Cin, hipStream_t st) {
  hipLaunchKernelGGL(end_conv_kernel, dim3(B * (H / 4) * (W / 64)), dim3(256), 0, st, in, ss, w, bias, sigmas, labels,
                     out, H, W, Cin);
  return hipGetLastError();
}

hipError_t inpp_finalize(const float* stats, int B, int T, float cnt, int C, const float* alpha, const float* gamma,
                         const float* beta, float* ss, hipStream_t st, float* nst, void* scratch) {
  if (C % 64 || C > 1024 || (C & (C - 1))) return hipErrorInvalidValue;
  double2* mv = reinterpret_cast<double2*>(scratch);
  hipLaunchKernelGGL(inpp_moments_kernel, dim3(B * (C / 64)), dim3(64 * INPP_G), 0, st, reinterpret_cast<const float2*>(stats), T,
                     cnt, C, mv);
  hipLaunchKernelGGL(inpp_ss_kernel, dim3(B), dim3(C), 0, st, mv, C, alpha, gamma, beta, reinterpret_cast<float2*>(ss),
                     reinterpret_cast<float4*>(nst));
  return hipGetLastError();
}

hipError_t maxpool5(const float* in, float* out, int B, int H, int W, int C, hipStream_t st, uint8_t* idx) {
  const size_t n = (size_t)B * ((H + MP_ROWS - 1) / MP_ROWS) * W * (C / 4);
  const int grid = (int)std::min<size_t>((n + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(maxpool5_kernel, dim3(grid), dim3(256), 0, st, in, out, reinterpret_cast<uchar4*>(idx), B, H, W, C);
  return hipGetLastError();
}

}  // namespace sdp
