// Winograd F(2,3)-along-W convolution on MFMA for the circular 3x3 convs of NCSN_LiDAR_small
// (conv3x3 LiDARGen/models/layers.py:37-44, dilated_conv3x3 layers.py:55-60; gfx950, bf16 modes).
//
// The 3x3 conv is a direct 3-tap sum along H and a Winograd F(2,3) along W: every pair of
// output columns (2p, 2p+1) of a row is
//   Y0 = M0 + M1 + M2,  Y1 = M1 - M2 - M3,   M_j = sum_kh sum_ci V_j[row + kh][p][ci] * U_j[kh][ci][co]
// with the input transform over the 4 input columns d0..d3 = x[2p-1 .. 2p+2]
//   V0 = d0 - d2,  V1 = d1 + d2,  V2 = d2 - d1,  V3 = d1 - d3
// and the weight transform over the 3 taps g0..g2 of a row of the kernel
//   U0 = g0,  U1 = (g0 + g1 + g2) / 2,  U2 = (g0 - g1 + g2) / 2,  U3 = g2.
// 12 (kh, j) "taps" of 2 pixels each replace the 9 taps of 1 pixel: 6 MACs per output pixel
// instead of 9 (1.5x fewer MFMAs).  fp32x3 splits V and U into bf16 hi + lo exactly as the
// direct kernel splits its operands (CPU emulation of the whole network: 2.10e-5 of max|out|,
// direct 2.10e-5; tools/winograd_numerics.py).
//
// Workgroup = 4 waves, one per SIMD; output tile = TR x TC = 8 x 16 pixels of one d x d
// polyphase sub-grid (so the halo is 1 pixel whatever d), i.e. 8 rows x 8 column pairs.
//   WM = 1: 128 px x 256 Cout, every wave all 64 pairs x 64 Cout (4 M x 4 N fragments per tap)
//   WM = 2: 128 px x 128 Cout, waves 2 (rows 0-3 / 4-7) x 2 (64 Cout each)
// Accumulators: [position j][M fragment][N fragment] of v_mfma_f32_16x16x32_bf16 = 256 (WM=1)
// or 128 AGPRs; the output transform is register arithmetic in the epilogue (the 4 positions of
// a pair are the same register of 4 fragments in one lane).
//
// K loop per 32-channel chunk c (one barrier per chunk):
//   raw[2]: fp32 (TR+2) x (TC+2) x 32 patch, landed by LDS-DMA; chunk c+2's DMA is issued at the
//           start of chunk c into raw[c&1] and waited for at the end of chunk c
//   V[2]  : 4 x (TR+2) x 8 "V pixels" of 32 channels (hi | lo bf16); while the 12 taps of chunk c
//           run on V[c&1], the taps 1..NI transform raw[(c+1)&1] -> V[(c+1)&1]: every thread owns
//           (row, pair, 4-channel) items -- 4 raw pixels through the consumer prologue (IN++
//           affine, ELU), the 4 V values, the hi/lo split -- interleaved between the MFMAs
//   weights: Winograd-transformed on the device (train_aux.hip pack_slot_wino) into 16x16
//           fragment order, streamed from L2 into VGPRs two taps ahead
// Epilogue: straight from the accumulators (output transform, bias, bilinear upsample-add,
// residual, CRP second output, ELU, InstanceNorm++ statistics of 128-pixel groups).
#pragma once
#include "common.h"

namespace sdp {

// Diagnostic knock-outs for tools/wino_bench (never set in the library build):
// 1 = no patch DMA, 2 = no transform, 4 = no weight loads, 8 = no end-of-chunk wait + barrier,
// 16 = no epilogue, 32 = no A-fragment reads
#ifndef SDP_WKO
#define SDP_WKO 0
#endif

constexpr int WPSTRIDE = 144;   // bytes per V pixel: 32 ch x (hi, lo) bf16 + 16 pad (conflict-free A reads)

// acc += a * b on v_mfma_f32_32x32x16_bf16 with the accumulator tied in place ("+a"): with all 256
// AGPRs holding accumulators, the builtin's register allocation rotates every chain through
// temporaries and parks accumulators in VGPRs (hundreds of v_accvgpr moves per chunk).  The
// 32x32 shape leaves 24 of its 32 issue cycles to the vector ALU (the 16x16x32 shape 8 of 16):
// room for the input transform between the MFMAs
SDP_DEV void mfma32(f32x16& c, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int WM>
struct WinoTile {
  static constexpr int TR = 8, TC = 16;           // output pixels of one sub-grid per workgroup
  static constexpr int NP = TC / 2;               // column pairs per row
  static constexpr int PR = TR + 2, PC = TC + 2;  // raw patch (1-pixel halo)
  static constexpr int NPIX = PR * PC;
  static constexpr int NU = (NPIX * 8 + 255) / 256;          // 16-B DMA units per thread
  static constexpr int RAW_BYTES = NU * 256 * 16;
  static constexpr int NVPIX = 4 * PR * NP;                  // V pixels [j][row][pair]
  static constexpr int V_BYTES = NVPIX * WPSTRIDE;
  static constexpr int NITEM = PR * NP * 8;                  // (row, pair, 4-channel group) items
  static constexpr int NI = (NITEM + 255) / 256;             // items per thread (the last partial)
  static constexpr int WN = 4 / WM;                          // waves along N
  static constexpr int WROWS = TR / WM;                      // output rows per wave
  static constexpr int MF = WROWS / 4;                       // 32-pair (4-row) M fragments per wave
  static constexpr int NTILE = WN * 64;                      // output channels per workgroup
  static constexpr int UOFF_BYTES = NU * 256 * 4;             // per-thread DMA offsets (kept out of VGPRs)
  static constexpr int LDS_BYTES = 2 * V_BYTES + 2 * RAW_BYTES + UOFF_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int MODE, int WM, bool PELU>
__global__ __launch_bounds__(256, 1) void wino_conv_kernel(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(MODE == MODE_F32X3 || MODE == MODE_BF16, "Winograd path: bf16 modes only");
  using T = WinoTile<WM>;
  constexpr bool X3 = MODE == MODE_F32X3;
  __shared__ __attribute__((aligned(16))) char lds[T::LDS_BYTES];
  char* const vbuf = lds;                           // V[2]
  char* const rawb = lds + 2 * T::V_BYTES;          // raw[2]
  const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(rawb);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef SDP_TIMING   // tools/wino_bench: shader clock and wall clock of wave 0 around the workgroup
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t1 = 0;
#endif
  const int wm = WM == 1 ? 0 : (wave & 1), wn = WM == 1 ? wave : (wave >> 1);
  const int d = a.dil, Hs = a.H / d, Ws = a.W / d;
  const int tiles_c = Ws / T::TC, tiles_rc = (Hs / T::TR) * tiles_c;
  // XCD-aware order (as conv_mfma_kernel): each XCD gets a contiguous range of tiles
  const int nwg = gridDim.x;
  int t = (nwg & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (nwg >> 3) + ((int)blockIdx.x >> 3);
  const int b = t / a.tiles_per_img;
  const int tile = t - b * a.tiles_per_img;
  t = tile;
  const int ph = t / tiles_rc;
  t -= ph * tiles_rc;
  const int ph_r = ph / d, ph_c = ph - (ph / d) * d;
  const int sr0 = (t / tiles_c) * T::TR, sc0 = (t % tiles_c) * T::TC;
  const int n0 = blockIdx.y * T::NTILE;
  const int wrow0 = wm * T::WROWS;

  const int Cin = a.Cin, Cout = a.Cout;
  const int nchunks = Cin / 32;
  const int NB32 = Cout / 32;

  f32x16 acc[4][T::MF][2];                          // [position j][M fragment][32-Cout fragment]
  static_for<0, 4>([&](auto j) {
    static_for<0, T::MF>([&](auto f) {
      static_for<0, 2>([&](auto n) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][f][n][r] = 0.f;
      });
    });
  });

  // ---- weights: [chunk][tap 12][32-Cout fragment][q = (s0 hi, s0 lo, s1 hi, s1 lo)][lane][16 B]
  // (train_aux.hip pack_slot_wino: every fragment load of a wave is 1 KiB contiguous); lane offset
  // in a VGPR, the (chunk, tap) offset in an SGPR
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wfw, 0, 0x7fffffff, 0x00020000);
  int wvo[2];
  static_for<0, 2>([&](auto nc) {
    constexpr int nb = decltype(nc)::value;
    wvo[nb] = ((n0 / 32 + wn * 2 + nb) * 256 + lane) * 16;
  });
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  uint4 bq[3][2][4];                                // ring of 3 taps: [slot][nb][(s, hi/lo)]
  auto load_b = [&](auto slot_c, int chunk, int tap) __attribute__((always_inline)) {
    constexpr int J = decltype(slot_c)::value;
    if constexpr (SDP_WKO & 4) return;
    const int so = __builtin_amdgcn_readfirstlane((chunk * 12 + tap) * NB32 * 4096);
    static_for<0, 2>([&](auto nc) {
      constexpr int nb = decltype(nc)::value;
      static_for<0, 4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if constexpr (X3 || (q & 1) == 0) {
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, wvo[nb] + q * 1024, so, 0);
          bq[J][nb][q] = make_uint4(v.x, v.y, v.z, v.w);
        }
      });
    });
  };

  // ---- raw patch DMA: unit u = tid + 256 k = 16 B (4 channels) of patch pixel u / 8, at byte
  // 16 u of raw[buf]; offsets (circular wrap on the sub-grid) fixed per tile, the chunk is the
  // scalar offset; units past the patch re-load pixel 0 into the slack
  const float* inb = a.in + (size_t)b * a.H * a.W * Cin;
  const i32x4 irs = buffer_desc(inb, (uint32_t)a.H * a.W * Cin * 4);
  // their byte offsets live in LDS: read once per chunk, they would otherwise hold NU VGPRs
  // through the MFMA loop (where the register file is full)
  int* const uoff_lds = reinterpret_cast<int*>(lds + 2 * T::V_BYTES + 2 * T::RAW_BYTES);
  static_for<0, T::NU>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    int u = tid + k * 256;
    u = u < T::NPIX * 8 ? u : 0;
    const int pix = u >> 3, cv = u & 7;
    const int pr = pix / T::PC, pc = pix - pr * T::PC;
    int sr = sr0 - 1 + pr, sc = sc0 - 1 + pc;
    sr = sr < 0 ? sr + Hs : (sr >= Hs ? sr - Hs : sr);
    sc = sc < 0 ? sc + Ws : (sc >= Ws ? sc - Ws : sc);
    const int y = sr * d + ph_r, x = sc * d + ph_c;
    uoff_lds[k * 256 + tid] = ((y * a.W + x) * Cin + cv * 4) * 4;
  });
  const uint32_t wave_raw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(raw_lds + (tid & ~63) * 16));   // SGPR
  auto dma_chunk = [&](int chunk, int buf) __attribute__((always_inline)) {
    if constexpr (SDP_WKO & 1) return;
    static_for<0, T::NU>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      dma16_lds_opaque(irs, wave_raw + buf * T::RAW_BYTES + k * 4096, uoff_lds[k * 256 + tid], chunk * 128);
    });
  };

  // ---- transform items: i = tid + 256 k -> (row r, pair p, channel group cv = tid % 8)
  const int cv = tid & 7;
  const float* ssb = a.pro_ss + (size_t)b * a.ss_bstride;
  float4 ssv0, ssv1;                                // (scale, shift) of channels 4cv .. 4cv+3
  auto load_ss = [&](int chunk) __attribute__((always_inline)) {
    ssv0 = *reinterpret_cast<const float4*>(ssb + (chunk * 32 + cv * 4) * 2);
    ssv1 = *reinterpret_cast<const float4*>(ssb + (chunk * 32 + cv * 4) * 2 + 4);
  };
  // Byte offsets of item k in raw[] and V[], fixed per thread.  Items past the end (k = NI-1 on
  // waves 2, 3 when NITEM is not a multiple of 256) redo item k-1 of the same thread: the same
  // values to the same place, so the transform needs no branch
  int it_raw[T::NI], it_v[T::NI];
  static_for<0, T::NI>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int i = (tid + k * 256 < T::NITEM) ? tid + k * 256 : tid + (k - 1) * 256;
    const int rp = i >> 3, r = rp / T::NP, p = rp - r * T::NP;
    it_raw[k] = ((r * T::PC + 2 * p) * 8 + cv) * 16;
    it_v[k] = rp * WPSTRIDE + cv * 8;
  });
  // the 4 raw pixels of item k (patch row r, columns 2p .. 2p+3) from raw[buf]
  auto item_load = [&](auto kc, int buf, float4* dv) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    const char* src = rawb + buf * T::RAW_BYTES + it_raw[k];
#pragma unroll
    for (int c = 0; c < 4; ++c) dv[c] = *reinterpret_cast<const float4*>(src + c * 128);
  };
  auto pro1 = [&](float4 v) __attribute__((always_inline)) {
    v.x = fmaf(v.x, ssv0.x, ssv0.y);
    v.y = fmaf(v.y, ssv0.z, ssv0.w);
    v.z = fmaf(v.z, ssv1.x, ssv1.y);
    v.w = fmaf(v.w, ssv1.z, ssv1.w);
    if constexpr (PELU) {
      v.x = elu_max(v.x); v.y = elu_max(v.y); v.z = elu_max(v.z); v.w = elu_max(v.w);
    }
    return v;
  };
  // V_j of item k (4 channels) -> hi/lo bf16 at V pixel (j, r, p) of V[buf]
  auto item_store = [&](auto kc, auto jc, int buf, float4 v) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value, j = decltype(jc)::value;
    char* dst = vbuf + buf * T::V_BYTES + it_v[k] + j * T::PR * T::NP * WPSTRIDE;
    bf16x4 hi;
    hi[0] = (__bf16)v.x; hi[1] = (__bf16)v.y; hi[2] = (__bf16)v.z; hi[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(dst) = hi;
    if constexpr (X3) {
      bf16x4 lo;
      lo[0] = (__bf16)(v.x - (float)hi[0]);
      lo[1] = (__bf16)(v.y - (float)hi[1]);
      lo[2] = (__bf16)(v.z - (float)hi[2]);
      lo[3] = (__bf16)(v.w - (float)hi[3]);
      *reinterpret_cast<bf16x4*>(dst + 64) = lo;
    }
  };
  auto vsub = [](float4 p, float4 q) { return make_float4(p.x - q.x, p.y - q.y, p.z - q.z, p.w - q.w); };
  auto vadd = [](float4 p, float4 q) { return make_float4(p.x + q.x, p.y + q.y, p.z + q.z, p.w + q.w); };
  auto vpos = [&](auto jc, const float4* dv) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (j == 0) return vsub(dv[0], dv[2]);
    else if constexpr (j == 1) return vadd(dv[1], dv[2]);
    else if constexpr (j == 2) return vsub(dv[2], dv[1]);
    else return vsub(dv[1], dv[3]);
  };
  auto item_full = [&](auto kc, int rbuf, int vb) __attribute__((always_inline)) {
    float4 dv[4];
    item_load(kc, rbuf, dv);
#pragma unroll
    for (int c = 0; c < 4; ++c) dv[c] = pro1(dv[c]);
    static_for<0, 4>([&](auto jc) { item_store(kc, jc, vb, vpos(jc, dv)); });
  };

  // ---- prologue: chunks 0 and 1 landed, chunk 0 transformed into V[0]
  load_b(std::integral_constant<int, 0>{}, 0, 0);
  load_b(std::integral_constant<int, 1>{}, 0, 1);
  dma_chunk(0, 0);
  if (nchunks > 1) dma_chunk(1, 1);
  load_ss(0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  static_for<0, T::NI>([&](auto kc) { item_full(kc, 0, 0); });
  load_ss(nchunks > 1 ? 1 : 0);
  __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0)
  __syncthreads();

  // A fragment (tap (kh, j), fragment f, k step s): lane l = pair m = l % 32 of the fragment,
  // channels 16 s + 8 (l / 32) .. ; fragment f covers wave rows 4f .. 4f + 3 (m / 8)
  // -> V pixel (j, wrow0 + 4f + m/8 + kh, m % 8)
  const int a_lane = (wrow0 * T::NP + (lane & 31)) * WPSTRIDE + (lane >> 5) * 16;
  auto read_a = [&](const char* vb, auto g_c, bf16x8& hi, bf16x8& lo) __attribute__((always_inline)) {
    constexpr int g = decltype(g_c)::value;         // fragment sequence number: (tap * MF + f) * 2 + s
    constexpr int s = g % 2, tap = g / 2 / T::MF, f = (g / 2) % T::MF, kh = tap / 4, j = tap % 4;
    if constexpr (SDP_WKO & 32) return;
    const char* src = vb + ((j * T::PR + 4 * f + kh) * T::NP) * WPSTRIDE + a_lane + s * 32;
    hi = *reinterpret_cast<const bf16x8*>(src);
    if constexpr (X3) lo = *reinterpret_cast<const bf16x8*>(src + 64);
  };

  // items of the next chunk's transform: item k on taps 1 + 2k (its 4 raw pixels loaded, then the
  // prologue in 8 pieces of 2 channels) and 2 + 2k (the 4 positions' V, hi/lo split and store in 8
  // pieces), one piece after every (MF*4*2/8)-th MFMA block, so the VALU issues in the MFMA shadow
  auto pro_half = [&](float4& v, auto hc) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    const float4 sv = h ? ssv1 : ssv0;
    float x0 = h ? v.z : v.x, x1 = h ? v.w : v.y;
    x0 = fmaf(x0, sv.x, sv.y);
    x1 = fmaf(x1, sv.z, sv.w);
    if constexpr (PELU) {
      x0 = elu_max(x0);
      x1 = elu_max(x1);
    }
    if constexpr (h) { v.z = x0; v.w = x1; } else { v.x = x0; v.y = x1; }
  };
  auto store_half = [&](auto kc, auto jc, auto hc, int buf, const float4* dv) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value, j = decltype(jc)::value, h = decltype(hc)::value;
    const float4 vv = vpos(jc, dv);
    const float x0 = h ? vv.z : vv.x, x1 = h ? vv.w : vv.y;
    char* dst = vbuf + buf * T::V_BYTES + it_v[k] + j * T::PR * T::NP * WPSTRIDE + h * 4;
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    bf16x2 hi;
    hi[0] = (__bf16)x0;
    hi[1] = (__bf16)x1;
    *reinterpret_cast<bf16x2*>(dst) = hi;
    if constexpr (X3) {
      bf16x2 lo;
      lo[0] = (__bf16)(x0 - (float)hi[0]);
      lo[1] = (__bf16)(x1 - (float)hi[1]);
      *reinterpret_cast<bf16x2*>(dst + 64) = lo;
    }
  };
  auto do_chunk = [&](auto parity, int chunk) __attribute__((always_inline)) {
    constexpr int P = decltype(parity)::value;
    const char* vb = vbuf + P * T::V_BYTES;
    if (chunk + 2 < nchunks) dma_chunk(chunk + 2, P);   // raw[P] held chunk `chunk`: transformed last chunk
    // A fragments two (f) block groups ahead, in a ring of 3: fragment sequence g = tap * MF + f
    bf16x8 ahi[3], alo[3];
    read_a(vb, std::integral_constant<int, 0>{}, ahi[0], alo[0]);
    read_a(vb, std::integral_constant<int, 1>{}, ahi[1], alo[1]);
    float4 dv[4];
    static_for<0, 12>([&](auto tap_c) {
      constexpr int tap = decltype(tap_c)::value;
      constexpr int CUR = tap % 3, NXT = (tap + 2) % 3;
      if constexpr (tap + 2 < 12) load_b(std::integral_constant<int, NXT>{}, chunk, tap + 2);
      else load_b(std::integral_constant<int, NXT>{}, min(chunk + 1, nchunks - 1), tap - 10);
      if constexpr (tap == 11) load_ss(min(chunk + 2, nchunks - 1));
      // item K = tap / 4 of the next chunk: its raw pixels loaded at tap 4K, the prologue of pixels
      // 0, 1 on tap 4K+1 and of 2, 3 on 4K+2 (4 pieces each), the 4 positions' V on 4K+3 (8 pieces)
      constexpr int K = tap / 4, PH = tap % 4;
      constexpr bool XF = K < T::NI && !(SDP_WKO & 2);
      constexpr int NPC = PH == 0 ? 0 : (PH == 3 ? 8 : 4);   // pieces on this tap
      if constexpr (XF && PH == 0) item_load(std::integral_constant<int, K>{}, 1 - P, dv);
      // blocks (f, s, pass): the 2 N fragments of fragment f at k step s, one operand pass each
      // (fp32x3: lo*hi, hi*lo, hi*hi), so consecutive MFMAs feed different accumulators
      constexpr int NPASS = X3 ? 3 : 1;
      constexpr int NBLK = T::MF * 2 * NPASS;
      static_for<0, NBLK>([&](auto blk_c) {
        constexpr int blk = decltype(blk_c)::value;
        constexpr int fs = blk / NPASS, pass = blk % NPASS, f = fs / 2, sk = fs % 2;
        constexpr int g = (tap * T::MF + f) * 2 + sk, AS = g % 3;
        if constexpr (pass == 0 && g + 2 < 24 * T::MF)   // two fragments ahead
          read_a(vb, std::integral_constant<int, g + 2>{}, ahi[(g + 2) % 3], alo[(g + 2) % 3]);
        static_for<0, 2>([&](auto nbc) {
          constexpr int nb = decltype(nbc)::value;
          const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(&bq[CUR][nb][2 * sk]);
          if constexpr (X3 && pass == 0) {
            mfma32(acc[tap % 4][f][nb], alo[AS], bhi);
          } else if constexpr (X3 && pass == 1) {
            const bf16x8 blo = *reinterpret_cast<const bf16x8*>(&bq[CUR][nb][2 * sk + 1]);
            mfma32(acc[tap % 4][f][nb], ahi[AS], blo);
          } else {
            mfma32(acc[tap % 4][f][nb], ahi[AS], bhi);
          }
        });
        // piece i of this tap after block floor(i * NBLK / NPC)
        static_for<0, NPC>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          if constexpr (XF && (i * NBLK) / NPC == blk) {
            if constexpr (PH == 1 || PH == 2) {
              constexpr int px = (PH - 1) * 2 + i / 2;
              pro_half(dv[px], std::integral_constant<int, i % 2>{});
            } else {
              store_half(std::integral_constant<int, K>{}, std::integral_constant<int, i / 2>{},
                         std::integral_constant<int, i % 2>{}, 1 - P, dv);
            }
          }
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    // V[1-P] complete and raw[1-P] (chunk+1, transformed) free; chunk+2 landed in raw[P]
    if constexpr (!(SDP_WKO & 8)) {
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_s_barrier();
    }
  };
  static_assert(4 * T::NI <= 12, "transform items fit the taps");
  for (int chunk = 0; chunk < nchunks; chunk += 2) {   // nchunks is even (Cin % 64 == 0)
    do_chunk(std::integral_constant<int, 0>{}, chunk);
    do_chunk(std::integral_constant<int, 1>{}, chunk + 1);
  }

#ifdef SDP_TIMING
  t1 = __builtin_amdgcn_s_memtime();
#endif
  // the last MFMAs were inline asm: cover the MFMA-write -> VALU/accvgpr-read latency explicitly
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 15");
  asm volatile("s_nop 15");
  asm volatile("s_nop 15");
  __builtin_amdgcn_sched_barrier(0);
#ifdef SDP_TIMING
  if (tid == 0) {
    unsigned long long* o = a.dbg + blockIdx.x * 8 + blockIdx.y * gridDim.x * 8;
    o[0] = t0; o[1] = t1; o[2] = r0; o[3] = __builtin_amdgcn_s_memtime(); o[4] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if constexpr (SDP_WKO & 16) {   // knock-out: one store per lane keeps the accumulators live
    float sm = 0.f;
    static_for<0, 4>([&](auto jj) {
      static_for<0, T::MF>([&](auto f) {
        static_for<0, 2>([&](auto n) { sm += acc[jj][f][n][0] + acc[jj][f][n][15]; });
      });
    });
    a.out[(size_t)blockIdx.x * 256 + tid] = sm;
    return;
  }
  // ------------------------------------------------------------------ epilogue
  // Register r of fragment (j, f, nb) of lane l: pair m = (r & 3) + 8 (r >> 2) + 4 (l >> 5) of the
  // fragment, i.e. wave row 4f + (r >> 2), pair (r & 3) + 4 (l >> 5), Cout 32 nb + l % 32.  Per
  // (f, row rr = r >> 2) the lane holds output columns 8 (l >> 5) .. +7: value i = 32 f + 8 rr + 2 (r & 3) + e,
  // and every wave store instruction writes 32 consecutive channels (128 B) of 2 pixels.
  {
    const int Wo = a.W;
    const size_t bo = (size_t)b * a.H * Wo * Cout;
    const int img_bytes = a.H * Wo * Cout * 4;
    auto rs = [&](const float* p) { return __builtin_amdgcn_make_buffer_rsrc((void*)(p ? p + bo : a.out + bo), 0, img_bytes, 0x00020000); };
    const __amdgpu_buffer_rsrc_t ors = rs(a.out), rrs = rs(a.res), o2rs = rs(a.out2), r2rs = rs(a.res2);
    const int lcol = lane & 31, lhalf = lane >> 5;
    constexpr int NR = T::MF * 4;                     // output rows per lane
    constexpr int NV = NR * 8;
    const int xs = d * Cout * 4;                     // bytes between consecutive output pixels of a run
    static_for<0, 2>([&](auto nbc) {
      constexpr int nb = decltype(nbc)::value;
      const int co = n0 + wn * 64 + nb * 32 + lcol;
      const float bias = a.bias ? a.bias[co] : 0.f;
      int vbase[NR];
      static_for<0, NR>([&](auto rc) {
        constexpr int rw = decltype(rc)::value;      // = 4 f + rr
        const int y = (sr0 + wrow0 + rw) * d + ph_r, x = (sc0 + 8 * lhalf) * d + ph_c;
        vbase[rw] = ((y * Wo + x) * Cout + co) * 4;
      });
      float v[NV];
      static_for<0, T::MF>([&](auto fc) {
        constexpr int f = decltype(fc)::value;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float m0 = acc[0][f][nb][r], m1 = acc[1][f][nb][r], m2 = acc[2][f][nb][r], m3 = acc[3][f][nb][r];
          const int i = f * 32 + (r >> 2) * 8 + (r & 3) * 2;
          v[i] = ((m0 + m1) + m2) + bias;
          v[i + 1] = ((m1 - m2) - m3) + bias;
        }
      });
      if (a.up) {   // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor
        const int Hi = a.H / 2, Wi = a.W / 2;
        const float shh = (float)(Hi - 1) / (float)(a.H - 1), sww = (float)(Wi - 1) / (float)(a.W - 1);
        const float* ub = a.up + (size_t)b * Hi * Wi * Cout + co;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int rw = i / 8, k = i % 8;
          const int y = (sr0 + wrow0 + rw) * d + ph_r, x = (sc0 + 8 * lhalf + k) * d + ph_c;
          const float fy = shh * (float)y, fx = sww * (float)x;
          const int y0 = (int)fy, x0 = (int)fx;
          const int yp = y0 < Hi - 1 ? 1 : 0, xp = x0 < Wi - 1 ? 1 : 0;
          const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
          const float v00 = ub[((size_t)y0 * Wi + x0) * Cout], v01 = ub[((size_t)y0 * Wi + x0 + xp) * Cout];
          const float v10 = ub[((size_t)(y0 + yp) * Wi + x0) * Cout];
          const float v11 = ub[((size_t)(y0 + yp) * Wi + x0 + xp) * Cout];
          v[i] = v[i] + (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11));
        }
      }
#define SDP_WEPI_OFF(i) vbase[(i) / 8], __builtin_amdgcn_readfirstlane(((i) % 8) * xs)
      if (a.res) {
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, SDP_WEPI_OFF(i), 0)) + v[i];
      }
      if (a.out2) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const float r2 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r2rs, SDP_WEPI_OFF(i), 0));
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i] + r2), o2rs, SDP_WEPI_OFF(i), 0);
        }
      }
      if (a.epi_elu) {
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = elu(v[i]);
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), ors, SDP_WEPI_OFF(i), 2);
#undef SDP_WEPI_OFF
      if (a.stats) {
        // two-pass (mean, M2) over the lane's NV values, a Chan merge of equal-count partials with
        // lane l ^ 32 (the other 8 columns) -> the wave's WROWS x 16 pixels of channel co
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) sum += v[i];
        float mean = sum * (1.0f / NV);
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const float dv = v[i] - mean;
          m2 = fmaf(dv, dv, m2);
        }
        const float mp = __shfl_xor(mean, 32), qp = __shfl_xor(m2, 32), dm = mean - mp;
        m2 = m2 + qp + dm * dm * (0.5f * NV);
        mean = 0.5f * (mean + mp);
        if constexpr (WM == 1) {
          if (lane < 32) {
            float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.groups_per_img + tile) * Cout + co;
            *st = make_float2(mean, m2);
          }
        } else {
          // the 128-pixel group is the whole tile: the two row waves merge through LDS (free now)
          float2* xch = reinterpret_cast<float2*>(lds) + (wn * 2 + nb) * 32;
          if (wm == 1 && lane < 32) xch[lane] = make_float2(mean, m2);
          __syncthreads();
          if (wm == 0 && lane < 32) {
            const float2 o = xch[lane];
            const float dd = mean - o.x;
            m2 = m2 + o.y + dd * dd * (float)NV;
            mean = 0.5f * (mean + o.x);
            float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.groups_per_img + tile) * Cout + co;
            *st = make_float2(mean, m2);
          }
        }
      }
    });
  }
#endif
}

}  // namespace sdp
