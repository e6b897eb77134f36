// Implicit-GEMM convolution kernel on MFMA for the NCSN/RefineNet score network (gfx950).
//
// Covers every 3x3 conv of NCSN_LiDAR_small except begin/end conv:
//   conv3x3 circular (LiDARGen/models/layers.py:37-44), dilated_conv3x3 circular
//   (layers.py:55-60), ConvMeanPool 3x3/1x1 zero-pad + 2x2 mean (layers.py:291-313).
//
// GEMM view: M = output pixels, N = Cout, K = taps x Cin.  One workgroup = 4 waves, ONE wave
// per SIMD (512-register budget, accumulators in AGPRs); each wave owns 128 px x 64 Cout =
// 4 x 2 blocks of the 32x32 MFMA tile, so per (tap, 16-wide k step) it reads 8 A fragments
// from LDS and 4 B fragments from L2 for 24 MFMAs (fp32x3).  Workgroup shapes:
//   WM=1: 128 px x 256 Cout (4 waves side by side in N; the patch serves 256 channels)
//   WM=2: 256 px x 128 Cout (2 x 2 waves; for the 128-channel layers)
// Dilated convs run on their d x d polyphase sub-grids, so a tile is always TR x TC pixels
// of one sub-grid and its input patch has a 1-pixel halo whatever d.
//
// K loop, per 32-channel chunk, fully software-pipelined (one barrier per chunk):
//   raw   : the fp32 (TR+2) x (TC+2) x 32 input patch of chunk k+1, landed by LDS-DMA
//           (buffer_load ... lds) during chunk k-1
//   patch : two buffers; while the 9 taps of chunk k run their MFMAs on patch[k&1], the
//           taps 0..3 transform raw -> patch[(k+1)&1] (consumer prologue: InstanceNorm++
//           affine and/or ELU, zero padding, bf16 hi/lo split) and the taps 4..8 issue the
//           LDS-DMA of chunk k+2 into raw.
//   weights: pre-arranged on the host in MFMA fragment order, streamed from L2 into VGPRs
//           one tap ahead (buffer_load_b128 with a scalar per-(chunk, tap) offset).
//
// MODE_F32   : v_mfma_f32_32x32x2_f32 on fp32 operands (exact fp32 products).
// MODE_F32X3 : operands split x = hi + lo (bf16 each), acc += hi*hi + hi*lo + lo*hi on
//              v_mfma_f32_32x32x16_bf16 -- error ~2e-5 of max|out| on the full network.
// MODE_BF16  : hi*hi only.
//
// Epilogue (fused): +bias, 2x2 mean-pool, +residual, +bilinear upsample of a half-res
// tensor, ELU, a second output (value + res2), and per-128-pixel InstanceNorm++ statistics
// (mean, M2) of every output channel.
#pragma once
#include <type_traits>

#include "common.h"

namespace sdp {

// Diagnostic knock-outs for tools/conv_bench (never set in the library build):
// 1 = no patch DMA, 2 = no transform, 4 = no weight loads, 8 = no chunk barrier, 16 = no epilogue
#ifndef SDP_KO
#define SDP_KO 0
#endif

// cache-policy bits (aux) of the patch LDS-DMA loads and of the forward epilogue stores
#ifndef SDP_DMA_AUX
#define SDP_DMA_AUX 0
#endif
#ifndef SDP_STORE_AUX     // plain (write-back) stores: each epilogue store instruction writes 64-B runs (fp32) or 32-B
#define SDP_STORE_AUX 0   // runs (bf16 tape) of a pixel's channels, which L2 merges into whole lines before they leave
#endif                    // for HBM; nt (2) sent them as partial lines.  Round 6 A/Bs (one box each, interleaved):
                          // fp32x3 line 348.9-349.3 -> 361.8-363.1 image-steps/s (profiles/experiments/
                          // r06_store_policy_ab.log); bf16-tape training 183.7-184.3 -> 200.6-201.6 (r06_store16_ab.log).
                          // (Round 2 had measured no difference on the kernel of that time, 172.4 vs 172.6 us.)
#ifndef SDP_STORE_AUX16   // the bf16-tape (IO16) epilogues
#define SDP_STORE_AUX16 SDP_STORE_AUX
#endif

#ifdef SDP_TIMING   // tools/conv_bench: per-workgroup phase clocks of wave 0 into a.dbg
#define SDP_T(i) do { if (tid == 0) tclk[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define SDP_T(i) do { } while (0)
#endif

constexpr int PSTRIDE = 144;  // bytes per staged patch pixel: 32 ch x (hi,lo bf16) or 32 x f32, + 16 pad

// NW = waves per workgroup: 4 (one workgroup per CU), or 2 (128-pixel x 128-Cout workgroups, two
// per CU: one's prologue and epilogue run under the other's MFMAs).
// NJ = 16-Cout fragments per wave: 4 (128 px x 64 Cout per wave, one wave per SIMD, 512 registers), or
// 2 (128 px x 32 Cout, two waves per SIMD at 256 registers: one wave's prologue, epilogue and waits run
// under its partner's MFMAs) -- NW = 4 with two workgroups per CU (128 Cout), or NW = 8 (256 Cout).
// IO16: activations stored as bf16 (the training tape, train.hip): a 16-B staging unit holds 8 channels
template <int WM, int TC, int KS, int NW = 4, int NJ = 4, bool IO16 = false>
struct ConvTile {
  static constexpr int NTH = 64 * NW;              // threads per workgroup
  static constexpr int WN = NW / WM;               // waves along N
  static constexpr int RW = 128 / TC;              // pixel rows per wave
  static constexpr int TR = WM * RW;               // tile rows
  static constexpr int NTILE = WN * 16 * NJ;       // output channels per workgroup
  static constexpr int WPC = 4 * (NJ == 2 ? 2 : 1) / NW;   // workgroups per CU the kernel is sized for
  static constexpr int HALO = KS == 3 ? 1 : 0;
  static constexpr int PC = TC + 2 * HALO;
  static constexpr int PR = TR + 2 * HALO;
  static constexpr int NPIX = PR * PC;
  static constexpr int UPP = IO16 ? 4 : 8;                      // 16-B staging units per pixel and 32-channel chunk
  static constexpr int NU = (NPIX * UPP + NTH - 1) / NTH;      // 16-B staging units per thread per chunk
  static constexpr int PATCH_BYTES = NU * (NTH / UPP) * PSTRIDE;  // one transformed patch (+ slack: every
                                                                  //   staging unit has a pixel slot)
  static constexpr int RAW_BYTES = NU * NTH * 16;               // raw fp32 patch landed by LDS-DMA
  static constexpr int PIPE_BYTES = 2 * PATCH_BYTES + RAW_BYTES;
  static constexpr int EPI_BYTES = WM * 64 * (NTILE + 8) * 4;   // LDS-staged epilogue (one half)
  static constexpr int LDS_BYTES = PIPE_BYTES > EPI_BYTES ? PIPE_BYTES : EPI_BYTES;
  static_assert(LDS_BYTES * WPC <= 160 * 1024, "LDS budget (WPC workgroups per CU)");
};

SDP_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// The 16x16 3x3 tap schedule (bf16 modes): each of the NT taps of a chunk is 32 MFMA blocks, and the
// tap's other work -- the next taps' weight loads, the A-fragment LDS reads, the next chunk's patch
// transform and the chunk after next's LDS-DMA -- is dealt out to the blocks one small filler at a
// time, so every block's VALU/LDS/VMEM issue fits beside its MFMAs (an MFMA leaves 8 of its 16
// issue cycles to other instructions, MI355X_MICROARCH.md constants).  Staging unit k (16 B of one
// patch pixel) is transformed in tap tap_of(k): the units spread over all taps, and each unit's next
// DMA follows its own transform, so it has a whole chunk to land.
template <int NU, int NT, int NSTG_ = 5>
struct XformPlan {
  static constexpr int tap_of(int k) { return k * NT / NU; }
  static constexpr int first(int tap) {
    int k = 0;
    while (k < NU && tap_of(k) < tap) ++k;
    return k;
  }
  static constexpr int count(int tap) {
    int n = 0;
    for (int k = 0; k < NU; ++k) n += tap_of(k) == tap ? 1 : 0;
    return n;
  }
  static constexpr int max_count() {
    int m = 0;
    for (int t = 0; t < NT; ++t) m = count(t) > m ? count(t) : m;
    return m;
  }
  // transform stages of one piece (2 channels of a unit): 5 in fp32x3 (both values per stage; its 3
  // MFMAs per block leave 24 issue cycles), 8 in bf16 (one value per stage where it costs; 8 cycles)
  static constexpr int NSTG = NSTG_;
  // block of stage slot q of Q in a tap of NBLK blocks: blocks 2 .. NBLK-1, evenly
  static constexpr int stage_blk(int q, int Q, int NBLK) { return 2 + q * (NBLK - 2) / (Q > 0 ? Q : 1); }
};

// SH: MFMA shape of the bf16 modes -- 32 = v_mfma_f32_32x32x16_bf16 (wave tile = 4 x 2 fragments
// of 32 px x 32 Cout, two 16-deep k steps per 32-channel chunk), 16 = v_mfma_f32_16x16x32_bf16
// (8 x 4 fragments of 16 px x 16 Cout, one 32-deep k step per chunk).  Same cycles per FLOP; the
// chip holds a higher clock on the 16x16 shape under this load (MI355X_MICROARCH.md 'DVFS
// give-back' item 7).  SH = 16 is forward-only (direct epilogue, no dact) and reads the SAME packed
// weights: a lane fetches the (cout, 8-channel group) its 16x16 fragment needs from the 32x32
// packing by its own buffer offset.
// TRN (data-gradient launches on the 16x16 shape): the MFMAs compute D = W x X (weights as the A
// operand, the patch as B -- the same fragment registers), so a lane's 4 accumulators are 4
// consecutive output channels of ONE pixel and every epilogue load/store is 16 B per lane (32 per
// wave and tensor instead of 128 of 4 B).  The forward keeps D = X x W: measured in the network,
// D = W x X made the fp32x3 forward convs 2-3 % slower (256->256 165 -> 170 us, 128->128 @64x1024
// 209 -> 213 us) while the bf16 training step ran 132.8 -> 137.0 image-steps/s with the transposed
// direct epilogue on the data gradient (profiles/experiments/r03_trans_ab.log).
// IO16 (the bf16 training tape, bf16 mode only): every activation tensor of the launch -- in, out, res, res2,
// out2, up, aux -- holds bf16 elements: 16-B staging units of 8 channels (half the patch DMA bytes), bf16
// epilogue loads and stores; statistics, bias and accumulation stay float32.
template <int MODE, int WM, int TC, int KS, bool POOL, bool ZP, bool PELU, int SH = 32, int NW = 4, bool TRN = false,
          int NJ = 4, bool IO16 = false>
__global__ __launch_bounds__(64 * NW, NJ == 2 ? 2 : 1) void conv_mfma_kernel(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
  static_assert(!IO16 || MODE == MODE_BF16, "the bf16 tape runs in bf16 mode");
  constexpr int ES = IO16 ? 2 : 4;                 // bytes per activation element
  constexpr int CPU = IO16 ? 8 : 4;                // channels per 16-B staging unit
  constexpr int USH = IO16 ? 2 : 3;                // log2(staging units per pixel-chunk)
  constexpr int PPU = CPU / 2;                     // 2-channel transform pieces per unit
  // IO16 without an ELU prologue (the data gradient, the CRP / MSF / shortcut convs: the identity (1, 0)
  // table): the transform is a copy of the unit's 16 B (zero padding aside)
  constexpr bool COPY = IO16 && !PELU;
  static_assert((SH == 32) == (MODE == MODE_F32), "bf16 modes: 16x16 shape; exact fp32: 32x32");
  static_assert(NW == 4 || (SH == 16 && !POOL), "2-wave workgroups: the 16x16 non-pooled forward only");
  static_assert(NJ == 4 || (SH == 16 && !POOL && KS == 3 && WM == 1), "32-Cout waves: the 16x16 3x3 tiles only");
  using T = ConvTile<WM, TC, KS, NW, NJ, IO16>;
  constexpr int NTH = T::NTH;
  constexpr int NT = KS * KS;
  constexpr bool TRANS = TRN && SH == 16 && !POOL;
  constexpr int NU = T::NU;
  constexpr int XT = NT >= 4 ? 4 : NT;            // taps that carry the transform of the next chunk
  __shared__ __attribute__((aligned(16))) char lds[T::LDS_BYTES];
  char* const raw = lds + 2 * T::PATCH_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef SDP_TIMING
  unsigned long long tclk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tbar = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz: the in-kernel clock
#endif
  SDP_T(0);
  const int wm = WM == 1 ? 0 : (wave & 1), wn = WM == 1 ? wave : (wave >> 1);
  const int d = a.dil, Hs = a.H / d, Ws = a.W / d;
  const int tiles_c = Ws / TC, tiles_rc = (Hs / T::TR) * tiles_c;
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so give each XCD a
  // contiguous range of tiles -- vertically adjacent tiles share their halo rows in its L2
  const int nwg = gridDim.x;
  int t = (nwg & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (nwg >> 3) + ((int)blockIdx.x >> 3);
  const int cblk = a.cpair ? (t & 1) : (int)blockIdx.y;
  if (a.cpair) t >>= 1;
  const int b = t / a.tiles_per_img;
  const int tile = t - b * a.tiles_per_img;
  t = tile;
  const int ph = t / tiles_rc;
  t -= ph * tiles_rc;
  const int ph_r = ph / d, ph_c = ph - (ph / d) * d;
  int trow, tcol;
  if (a.strip_w) {   // strips of strip_w tile columns x all tile rows (common.h conv_strip_w)
    const int R = Hs / T::TR, sw = a.strip_w;
    const int strip = t / (R * sw), w_ = t - strip * (R * sw);
    trow = w_ / sw;
    tcol = strip * sw + (w_ - trow * sw);
  } else {
    trow = t / tiles_c;
    tcol = t % tiles_c;
  }
  const int sr0 = trow * T::TR, sc0 = tcol * TC;
  const int n0 = cblk * T::NTILE;
  const int wrow0 = wm * T::RW;                    // wave's first tile row

  const int Cin = a.Cin, Cout = a.Cout;
  const int nchunks = Cin / 32;
  const int NB = Cout / 32;
  const int f0 = n0 / 16 + wn * NJ;                // global 16-channel fragment of this wave's nj = 0
  const int nbg0 = f0 / 2;                         // global 32-channel block of this wave's nb=0

  f32x16 acc[4][2];
  f32x4 acc4[8][NJ];                               // SH == 16: [16-px group][16-Cout group]
  if constexpr (SH == 32) {
    static_for<0, 4>([&](auto i) {
      static_for<0, 2>([&](auto j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      });
    });
  } else {
    static_for<0, 8>([&](auto i) {
      static_for<0, NJ>([&](auto j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc4[i][j][r] = 0.f;
      });
    });
  }

  // weight fragments through a buffer resource: lane offset in a VGPR (fixed per nb), the
  // (chunk, tap) offset in an SGPR -> no per-load address arithmetic
  // SH 16 forward: the 16x16-native packing "#frag16" in wf16 (every fragment load of a wave reads
  // 1 KiB contiguous) -- the forward's "#frag16", the data gradient's "#dfrag16"; with wf16 null the 32x32 "#frag"
  // packing in wf in 16-B pieces per lane
  const bool c16 = SH == 16 && a.wf16 != nullptr;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(c16 ? a.wf16 : a.wf), 0, 0x7fffffff, 0x00020000);
  const int wv0 = ((nbg0 + 0) * 64 + lane) * 64, wv1 = ((nbg0 + 1) * 64 + lane) * 64;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  // weight fragment ring: 3 taps deep (prefetch distance 2) when the tap count is a multiple
  // of 3, so the slot of (chunk, tap) is tap % 3 in every chunk; 2 deep for the 1x1 conv (a 9-slot
  // ring for the hi-only bf16 fragments measured 135.5 -> 134.4 image-steps/s in the bf16 training
  // step, profiles/experiments/r03_train_ring_wgrad_ab.log)
  constexpr int NBUF = (NT % 3 == 0) ? 3 : 2;
  uint4 bq[NBUF][NJ / 2][4];   // SH 32: [slot][nb][(s, hi/lo)]; SH 16: [slot][nj / 2][(nj % 2, hi/lo)]
  // SH 16: fragment nj (Couts 16 nj .. of the wave's 64) lane l needs Cout 16 nj + l % 16 and
  // channel group g = l / 16 (channels 8g .. 8g+7 of the chunk); the 32x32 packing stores Cout c,
  // channels 16 s + 8 h at lane c % 32 + 32 h, slot s -- so the lane reads from there
  int wq16[NJ];
  const int wlo16 = __builtin_amdgcn_readfirstlane(c16 ? 1024 : 16);   // byte offset of the lo part
  {
    const int g = lane >> 4, h = g & 1, sg = g >> 1;
    static_for<0, NJ>([&](auto njc) {
      constexpr int nj = decltype(njc)::value;
      const int L = 16 * (nj & 1) + (lane & 15) + 32 * h;
      // "#frag16": [chunk][tap][16-Cout fragment][hi, lo][lane][16 B]
      wq16[nj] = c16 ? ((f0 + nj) * 128 + lane) * 16 : ((nbg0 + (nj >> 1)) * 64 + L) * 64 + sg * 32;
    });
  }
  auto load_b = [&](auto buf, int chunk, int tap) __attribute__((always_inline)) {
    constexpr int J = decltype(buf)::value;
    if constexpr (SDP_KO & 4) return;
    const int so = __builtin_amdgcn_readfirstlane(((chunk * NT + tap) * NB) * 4096);
    // (the lo halves only in fp32x3: MODE_BF16 multiplies the hi parts alone)
    if constexpr (SH == 32) {   // exact fp32: 16 fp32 k values of a 32-Cout block per lane
      static_for<0, 4>([&](auto q) {
        const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(wrs, wv0 + q * 16, so, 0);
        const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(wrs, wv1 + q * 16, so, 0);
        bq[J][0][q] = make_uint4(v0.x, v0.y, v0.z, v0.w);
        bq[J][1][q] = make_uint4(v1.x, v1.y, v1.z, v1.w);
      });
    } else {
      static_for<0, NJ>([&](auto njc) {
        constexpr int nj = decltype(njc)::value;
        const u32x4 vh = __builtin_amdgcn_raw_buffer_load_b128(wrs, wq16[nj], so, 0);
        bq[J][nj >> 1][2 * (nj & 1)] = make_uint4(vh.x, vh.y, vh.z, vh.w);
        if constexpr (MODE != MODE_BF16) {
          const u32x4 vl = __builtin_amdgcn_raw_buffer_load_b128(wrs, wq16[nj] + wlo16, so, 0);
          bq[J][nj >> 1][2 * (nj & 1) + 1] = make_uint4(vl.x, vl.y, vl.z, vl.w);
        }
      });
    }
  };

  const char* inb = reinterpret_cast<const char*>(a.in) + (size_t)b * a.H * a.W * Cin * ES;
  // (scale, shift) rows of this image (the identity table when there is no affine prologue):
  // consumed only by the next chunk's transform, so the loads stay in flight across a chunk
  const float* ssb = a.pro_ss + (size_t)b * a.ss_bstride;
  const int my_cv = tid & (T::UPP - 1);            // every unit of a thread has cv == tid % UPP
  // (scale, shift) of this thread's CPU channels, double-buffered by chunk parity: chunk c's rows live
  // in ssv[c & 1][..] (the transform of chunk c writes patch buffer c & 1 too); float4 k = channels 2k, 2k+1
  float4 ssv[2][PPU];
  auto load_ss = [&](auto buf, int chunk) __attribute__((always_inline)) {
    constexpr int SB = decltype(buf)::value;
    static_for<0, PPU>([&](auto kc) { ssv[SB][kc] = ld4(ssb + (chunk * 32 + my_cv * CPU) * 2 + 4 * decltype(kc)::value); });
  };

  // Staging unit u = 16 B (4 channels) of one patch pixel.  Its byte offset inside the image
  // (clamped into range, so every load is unconditional) and its validity (zero padding)
  // depend only on the tile, so they are computed once; per chunk only the scalar channel
  // offset changes.  Unit u is landed by lane u%64 of wave (u%256)/64 -- the same thread
  // that transforms it, so raw needs no barrier, only the DMA's vmcnt.
  // num_records = the image's bytes: the (unconditional) DMA of a chunk past the last one
  // reads zeros instead of running off the tensor
  const __amdgpu_buffer_rsrc_t irs =
      __builtin_amdgcn_make_buffer_rsrc((void*)inb, 0, a.H * a.W * Cin * ES, 0x00020000);
  int uoff[NU];
  unsigned uvalid = 0;
  static_for<0, NU>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    int u = tid + k * NTH;
    bool valid = u < T::NPIX * T::UPP;
    u = valid ? u : 0;
    const int pix = u >> USH, cv = u & (T::UPP - 1);
    const int pr = pix / T::PC, pc = pix - pr * T::PC;
    int sr = sr0 - T::HALO + pr, sc = sc0 - T::HALO + pc;
    if (a.circular) {
      sr = sr < 0 ? sr + Hs : (sr >= Hs ? sr - Hs : sr);
      sc = sc < 0 ? sc + Ws : (sc >= Ws ? sc - Ws : sc);
    } else {
      valid = valid && sr >= 0 && sr < Hs && sc >= 0 && sc < Ws;
      sr = min(max(sr, 0), Hs - 1);
      sc = min(max(sc, 0), Ws - 1);
    }
    const int y = sr * d + ph_r, x = sc * d + ph_c;
    uoff[k] = ((y * a.W + x) * Cin + cv * CPU) * ES;   // bytes, < 2^31 for every admitted shape
    uvalid |= (valid ? 1u : 0u) << k;
  });
  // LDS-DMA of staging unit k: lane i of a wave lands 16 B at the wave-uniform base + 16*i
  auto load_unit = [&](auto kc, int chunk) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if constexpr (SDP_KO & 1) return;
    const int base = __builtin_amdgcn_readfirstlane(((tid & ~63) + k * NTH) * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        irs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(raw + base)), 16,
        uoff[k], chunk * 32 * ES, 0, SDP_DMA_AUX);
  };
  // the same DMA as inline asm (common.h dma16_lds_opaque), for the main loop of the 3x3 tap schedule:
  // the compiler cannot tell the raw slots apart and would wait for every DMA in flight (vmcnt(0))
  // before the next raw read.  Ordering without that wait: unit k's slot is read again one chunk
  // later, and the weight loads issued after its DMA -- which complete in issue order with it --
  // are waited for two taps later, before their MFMAs
  const i32x4 irs_o = buffer_desc(inb, (uint32_t)(a.H * a.W * Cin * ES));
  auto load_unit_o = [&](auto kc, int chunk) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if constexpr (SDP_KO & 1) return;
    const uint32_t base = (uint32_t)(uintptr_t)(raw + ((tid & ~63) + k * NTH) * 16);
    dma16_lds_opaque(irs_o, base, uoff[k], chunk * 32 * ES);
  };
  // transform staging unit k of raw into patch buffer PB
  // transform of staging unit k: raw (fp32, landed by this thread's own DMA) -> patch buffer PB
  auto xform_load = [&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    return *reinterpret_cast<const float4*>(raw + (tid + k * NTH) * 16);
  };
  auto xform_store = [&](auto kc, auto pb, float4 v) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr int PB = decltype(pb)::value;
    const int pix = (tid + k * NTH) >> USH;   // units past the patch land in its slack: no branch
    if constexpr (COPY) {
      uint4 u = __builtin_bit_cast(uint4, v);
      if constexpr (ZP) {
        if (!((uvalid >> k) & 1u)) u = make_uint4(0u, 0u, 0u, 0u);
      }
      *reinterpret_cast<uint4*>(lds + PB * T::PATCH_BYTES + pix * PSTRIDE + my_cv * 16) = u;
      return;
    }
    if constexpr (IO16) {   // 8 bf16 channels -> prologue -> 8 bf16 (one 16-B LDS write)
      const uint4 u = __builtin_bit_cast(uint4, v);
      const float4 lo = bf4_to_f4(make_uint2(u.x, u.y)), hi = bf4_to_f4(make_uint2(u.z, u.w));
      float x8[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float4 sv = ssv[PB][e >> 1];
        x8[e] = fmaf(x8[e], (e & 1) ? sv.z : sv.x, (e & 1) ? sv.w : sv.y);
        if constexpr (PELU) x8[e] = elu_max(x8[e]);
        if constexpr (ZP) {
          if (!((uvalid >> k) & 1u)) x8[e] = 0.f;
        }
      }
      *reinterpret_cast<uint4*>(lds + PB * T::PATCH_BYTES + pix * PSTRIDE + my_cv * 16) =
          make_uint4(pack_bf2(x8[0], x8[1]), pack_bf2(x8[2], x8[3]), pack_bf2(x8[4], x8[5]), pack_bf2(x8[6], x8[7]));
      return;
    }
    const float4 ssv0 = ssv[PB][0], ssv1 = ssv[PB][1];
    v.x = fmaf(v.x, ssv0.x, ssv0.y);
    v.y = fmaf(v.y, ssv0.z, ssv0.w);
    v.z = fmaf(v.z, ssv1.x, ssv1.y);
    v.w = fmaf(v.w, ssv1.z, ssv1.w);
    if constexpr (PELU) {
      v.x = elu_max(v.x); v.y = elu_max(v.y); v.z = elu_max(v.z); v.w = elu_max(v.w);
    }
    if constexpr (ZP) {   // zero padding (ConvMeanPool, layers.py:291-313, and its data gradient)
      if (!((uvalid >> k) & 1u)) v = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    char* dst = lds + PB * T::PATCH_BYTES + pix * PSTRIDE;
    if constexpr (MODE == MODE_F32) {
      *reinterpret_cast<float4*>(dst + my_cv * 16) = v;
    } else {
      bf16x4 hi;
      hi[0] = (__bf16)v.x; hi[1] = (__bf16)v.y; hi[2] = (__bf16)v.z; hi[3] = (__bf16)v.w;
      *reinterpret_cast<bf16x4*>(dst + my_cv * 8) = hi;
      if constexpr (MODE == MODE_F32X3) {
        bf16x4 lo;
        lo[0] = (__bf16)(v.x - (float)hi[0]);
        lo[1] = (__bf16)(v.y - (float)hi[1]);
        lo[2] = (__bf16)(v.z - (float)hi[2]);
        lo[3] = (__bf16)(v.w - (float)hi[3]);
        *reinterpret_cast<bf16x4*>(dst + 64 + my_cv * 8) = lo;
      }
    }
  };
  auto xform_unit = [&](auto kc, auto pb) __attribute__((always_inline)) { xform_store(kc, pb, xform_load(kc)); };
  // half of unit k (channels 2h, 2h+1 of its 4): prologue + bf16 hi/lo split + one ds_write2
  auto xform_piece = [&](auto kc, auto hc, auto pb, float4 v4) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value, h = decltype(hc)::value, PB = decltype(pb)::value;
    if constexpr (SDP_KO & 2) return;
    const int pix = (tid + k * NTH) >> USH;
    float x0, x1;
    if constexpr (IO16) {   // piece h = channels 2h, 2h+1 = the two bf16 halves of word h
      const uint32_t w = __float_as_uint(h == 0 ? v4.x : h == 1 ? v4.y : h == 2 ? v4.z : v4.w);
      x0 = __uint_as_float(w << 16);
      x1 = __uint_as_float(w & 0xffff0000u);
    } else {
      x0 = h ? v4.z : v4.x;
      x1 = h ? v4.w : v4.y;
    }
    const float4 sv = ssv[PB][h];
    x0 = fmaf(x0, sv.x, sv.y);
    x1 = fmaf(x1, sv.z, sv.w);
    if constexpr (PELU) {
      x0 = elu_max(x0);
      x1 = elu_max(x1);
    }
    if constexpr (ZP) {
      const bool ok = (uvalid >> k) & 1u;
      x0 = ok ? x0 : 0.f;
      x1 = ok ? x1 : 0.f;
    }
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    bf16x2 hi;
    hi[0] = (__bf16)x0;
    hi[1] = (__bf16)x1;
    char* dst = lds + PB * T::PATCH_BYTES + pix * PSTRIDE + my_cv * (2 * CPU) + h * 4;
    *reinterpret_cast<bf16x2*>(dst) = hi;
    if constexpr (MODE == MODE_F32X3) {
      bf16x2 lo;
      lo[0] = (__bf16)(x0 - (float)hi[0]);
      lo[1] = (__bf16)(x1 - (float)hi[1]);
      *reinterpret_cast<bf16x2*>(dst + 64) = lo;
    }
  };

  SDP_T(1);
  // ---- prologue: chunk 0 staged + transformed, chunk 1 in flight ----
  load_b(std::integral_constant<int, 0>{}, 0, 0);
  static_for<1, NBUF - 1>([&](auto j) { load_b(j, 0, decltype(j)::value); });
  load_ss(std::integral_constant<int, 0>{}, 0);
  static_for<0, NU>([&](auto k) { load_unit(k, 0); });
  static_for<0, NU>([&](auto k) { xform_unit(k, std::integral_constant<int, 0>{}); });
  if (nchunks > 1) {
    load_ss(std::integral_constant<int, 1>{}, 1);
    static_for<0, NU>([&](auto k) { load_unit(k, 1); });
  }
  __syncthreads();
  SDP_T(2);

  // A fragments of (tap, s) for the bf16 modes: lane reads 16 B = 8 channels of one patch pixel;
  // s = which half of the 8 16-px fragments (mb 4s .. 4s+3), lane l = pixel l % 16, channels 8 (l / 16) ..
  const int a_lane_off16 = (lane & 15) * PSTRIDE + (lane >> 4) * 16;
  auto read_a = [&](const char* pat, auto tap_c, auto s_c, bf16x8* hi, bf16x8* lo) __attribute__((always_inline)) {
    constexpr int tap = decltype(tap_c)::value, s = decltype(s_c)::value;
    constexpr int kh = (KS == 3) ? tap / 3 : 0, kw = (KS == 3) ? tap % 3 : 0;
    static_for<0, 4>([&](auto mbc) {
      constexpr int i = decltype(mbc)::value, mb = 4 * s + i;
      constexpr int mr = mb / (TC / 16), mc = (mb % (TC / 16)) * 16;
      const char* src = pat + ((wrow0 + mr + kh) * T::PC + mc + kw) * PSTRIDE + a_lane_off16;
      hi[i] = *reinterpret_cast<const bf16x8*>(src);
      if constexpr (MODE == MODE_F32X3) lo[i] = *reinterpret_cast<const bf16x8*>(src + 64);
    });
  };

  auto do_chunk = [&](auto parity, int chunk) __attribute__((always_inline)) {
    constexpr int P = decltype(parity)::value;
    // The transform of chunk+1 and the DMA of chunk+2 run unconditionally (branch-free
    // regions schedule across the MFMAs); past the last chunk they touch only dead buffers.
    const char* pat = lds + P * T::PATCH_BYTES;
    bf16x8 pre_hi[4], pre_lo[4];   // s=0 fragments of the next tap, read one region ahead
    if constexpr (MODE != MODE_F32) read_a(pat, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},
                                           pre_hi, pre_lo);
    static_for<0, NT>([&](auto tap_c) {
      constexpr int tap = decltype(tap_c)::value;
      constexpr int DIST = NBUF - 1;                       // prefetch distance in taps
      constexpr int CUR = NBUF >= 3 ? tap % NBUF : (tap + P) & 1;
      constexpr int NXT = NBUF >= 3 ? (tap + DIST) % NBUF : (tap + 1 + P) & 1;
      if constexpr (tap + DIST < NT) load_b(std::integral_constant<int, NXT>{}, chunk, tap + DIST);
      else load_b(std::integral_constant<int, NXT>{}, min(chunk + 1, nchunks - 1), tap + DIST - NT);
      __builtin_amdgcn_sched_barrier(0);
      // next chunk's transform on taps [0, XT), then the chunk after next's DMA on the rest
      // this tap's share of the next chunk's transform (units k with k % XT == tap)
      constexpr int NX = (tap < XT) ? (NU - tap + XT - 1) / XT : 0;
      float4 xv[NX > 0 ? NX : 1];
      auto xform_loads = [&]() __attribute__((always_inline)) {
        static_for<0, NX>([&](auto j) { xv[j] = xform_load(std::integral_constant<int, tap + XT * j>{}); });
      };
      auto xform_stores = [&]() __attribute__((always_inline)) {
        static_for<0, NX>([&](auto j) {
          xform_store(std::integral_constant<int, tap + XT * j>{}, std::integral_constant<int, 1 - P>{}, xv[j]);
        });
      };
      auto dmas = [&]() __attribute__((always_inline)) {
        if constexpr (tap == NT - 1) load_ss(std::integral_constant<int, P>{}, min(chunk + 2, nchunks - 1));
        static_for<0, NU>([&](auto kc) {
          constexpr int dt = NT > XT ? XT : 0;   // all at the first free tap: the longest flight
          if constexpr (dt == tap) load_unit(kc, chunk + 2);
        });
      };
      if constexpr (MODE == MODE_F32) {
        xform_loads();
        xform_stores();
        if constexpr (NT == 1) __builtin_amdgcn_sched_barrier(0);
        dmas();
        const int kh = (KS == 3) ? tap / 3 : 0, kw = (KS == 3) ? tap % 3 : 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {   // k steps [8*half, 8*half+8)
          float av[4][8];
          static_for<0, 4>([&](auto mbc) {
            constexpr int mb = decltype(mbc)::value;
            constexpr int mr = mb / (TC / 32), mc = (mb % (TC / 32)) * 32;
            const int pix = (wrow0 + mr + kh) * T::PC + mc + (lane & 31) + kw;
            const char* src = pat + pix * PSTRIDE + (lane >> 5) * 64 + half * 32;
            const float4 f0 = *reinterpret_cast<const float4*>(src);
            const float4 f1 = *reinterpret_cast<const float4*>(src + 16);
            av[mb][0] = f0.x; av[mb][1] = f0.y; av[mb][2] = f0.z; av[mb][3] = f0.w;
            av[mb][4] = f1.x; av[mb][5] = f1.y; av[mb][6] = f1.z; av[mb][7] = f1.w;
          });
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const int k = half * 8 + kk;
            static_for<0, 2>([&](auto nbc) {
              constexpr int nb = decltype(nbc)::value;
              const uint4 bv = bq[CUR][nb][k >> 2];
              const uint32_t bw = (k & 3) == 0 ? bv.x : (k & 3) == 1 ? bv.y : (k & 3) == 2 ? bv.z : bv.w;
              const float bf = __uint_as_float(bw);
              static_for<0, 4>([&](auto mbc) {
                constexpr int mb = decltype(mbc)::value;
                acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mb][kk], bf, acc[mb][nb], 0, 0, 0);
              });
            });
          }
        }
      } else {
        // Explicitly interleaved: 16 blocks of (s, nb, mb) -> 3 MFMAs (fp32x3) each, every
        // block its own scheduling region carrying one piece (2 channels) of the next chunk's
        // transform, so the VALU issues in the MFMA shadow.  Reads: this tap's raw units
        // first (their lgkmcnt retires first), then A(tap, s=1), then A(tap+1, s=0).
        float4 xv[NX > 0 ? NX : 1];
        static_for<0, NX>([&](auto j) { xv[j] = xform_load(std::integral_constant<int, tap + XT * j>{}); });
        bf16x8 c0_hi[4], c0_lo[4], c1_hi[4], c1_lo[4];
        static_for<0, 4>([&](auto mb) {
          c0_hi[mb] = pre_hi[mb];
          if constexpr (MODE == MODE_F32X3) c0_lo[mb] = pre_lo[mb];
        });
        read_a(pat, tap_c, std::integral_constant<int, 1>{}, c1_hi, c1_lo);
        if constexpr (tap + 1 < NT)
          read_a(pat, std::integral_constant<int, tap + 1>{}, std::integral_constant<int, 0>{}, pre_hi, pre_lo);
        if constexpr (NT > 1) dmas();   // 1x1: after the blocks, behind this tap's raw reads
        constexpr int NBLK = 8 * NJ;
        static_for<0, NBLK>([&](auto blk_c) {
          constexpr int blk = decltype(blk_c)::value;
          {
            // block = (half s of the px groups, Cout group nj, px group i of the half)
            constexpr int s = blk / (4 * NJ), nj = (blk / 4) % NJ, i = blk & 3, mb = 4 * s + i;
            const uint4 h4 = bq[CUR][nj >> 1][2 * (nj & 1)], l4 = bq[CUR][nj >> 1][2 * (nj & 1) + 1];
            const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(&h4);
            const bf16x8 blo = *reinterpret_cast<const bf16x8*>(&l4);
            const bf16x8 ahi = s == 0 ? c0_hi[i] : c1_hi[i];
            if constexpr (TRANS) {   // D = W x X: rows = Cout, columns = pixels (same fragment registers)
              if constexpr (MODE == MODE_F32X3) {
                const bf16x8 alo = s == 0 ? c0_lo[i] : c1_lo[i];
                acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi, alo, acc4[mb][nj], 0, 0, 0);
                acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(blo, ahi, acc4[mb][nj], 0, 0, 0);
              }
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi, ahi, acc4[mb][nj], 0, 0, 0);
            } else {
              if constexpr (MODE == MODE_F32X3) {
                const bf16x8 alo = s == 0 ? c0_lo[i] : c1_lo[i];
                acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc4[mb][nj], 0, 0, 0);
                acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc4[mb][nj], 0, 0, 0);
              }
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc4[mb][nj], 0, 0, 0);
            }
          }
          if constexpr (COPY) {
            if constexpr (blk < NX) xform_store(std::integral_constant<int, tap + XT * blk>{}, std::integral_constant<int, 1 - P>{},
                                                xv[blk]);
          } else if constexpr (blk < PPU * NX) {
            xform_piece(std::integral_constant<int, tap + XT * (blk / PPU)>{}, std::integral_constant<int, blk % PPU>{},
                        std::integral_constant<int, 1 - P>{}, xv[blk / PPU]);
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (NT == 1) dmas();
      }
    });
    // patch[P] free for chunk+2's transform, patch[1-P] complete.  A raw barrier: only the
    // LDS writes must have landed; the DMA of chunk+2 and the weight loads stay in flight.
#ifdef SDP_TIMING
    const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
#endif
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    if constexpr (!(SDP_KO & 8)) __builtin_amdgcn_s_barrier();
#ifdef SDP_TIMING
    tbar += __builtin_amdgcn_s_memtime() - tb0;
#endif
  };
  // ---- the 16x16 3x3 tap schedule (XformPlan): 32 blocks of (s, nj, i) per tap, each 3 MFMAs
  // (fp32x3) or 1 (bf16) plus at most a filler or two:
  //   blocks 0 .. NQ-1       : the A fragments of this tap's half s = 1 (cb), one LDS read each
  //   odd blocks 1 .. 2NQ-1  : the weight fragments of tap + 2 (ring slot (tap + 2) % 3), one load each
  //   blocks 16 .. 16+NQ-1   : the half-0 fragments of tap + 1 (into ca: free after block 15)
  //   blocks 0, 1            : the raw values of the units this tap transforms (XformPlan::tap_of)
  //   blocks 2 .. 31         : their transform, 5 stages per 2-channel piece
  //   blocks 30, 31          : the LDS-DMA of those units for the chunk after next (raw slot free)
  using XP = XformPlan<NU, NT, (MODE == MODE_BF16 && !IO16) ? 8 : 5>;   // (IO16: 4 pieces per unit)
  constexpr int NQ = MODE == MODE_F32X3 ? 8 : 4;   // A reads per half tap
  constexpr int NWL = NJ * (MODE == MODE_F32X3 ? 2 : 1);   // weight loads per tap
  constexpr int NBLK = 8 * NJ;                     // MFMA blocks per tap: (half s, Cout fragment nj, px group i)
  static_assert(NQ <= NBLK / 2 && 2 * NWL <= NBLK, "the tap's fillers fit its blocks");
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // one A fragment: pixel group i of half s of tap `tap`, hi (LO = 0) or lo part
  auto read_a1 = [&](const char* pat, auto tap_c, auto s_c, auto i_c, auto lo_c) __attribute__((always_inline)) {
    constexpr int tap = decltype(tap_c)::value, s = decltype(s_c)::value, i = decltype(i_c)::value;
    constexpr int kh = tap / 3, kw = tap % 3, mb = 4 * s + i;
    constexpr int mr = mb / (TC / 16), mc = (mb % (TC / 16)) * 16;
    return *reinterpret_cast<const bf16x8*>(pat + ((wrow0 + mr + kh) * T::PC + mc + kw) * PSTRIDE + a_lane_off16 +
                                            (decltype(lo_c)::value ? 64 : 0));
  };
  // weight load q of (chunk, tap) into ring slot J: q = 2 nj + part (fp32x3) or nj (bf16)
  auto load_b1 = [&](auto buf, auto q_c, int chunk, int tap) __attribute__((always_inline)) {
    constexpr int J = decltype(buf)::value, q = decltype(q_c)::value;
    constexpr int nj = MODE == MODE_F32X3 ? (q >> 1) : q, part = MODE == MODE_F32X3 ? (q & 1) : 0;
    if constexpr (SDP_KO & 4) return;
    const int so = __builtin_amdgcn_readfirstlane(((chunk * NT + tap) * NB) * 4096 + (part ? wlo16 : 0));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, wq16[nj], so, 0);
    bq[J][nj >> 1][2 * (nj & 1) + part] = make_uint4(v.x, v.y, v.z, v.w);
  };
  auto do_chunk9 = [&](auto parity, int chunk) __attribute__((always_inline)) {
    constexpr int P = decltype(parity)::value;
    const char* pat = lds + P * T::PATCH_BYTES;
    bf16x8 ca[2][4], cb[2][4];   // [hi, lo][i]: half s = 0 / s = 1 of the current tap
    static_for<0, 4>([&](auto i) {
      ca[0][i] = read_a1(pat, I0{}, I0{}, i, I0{});
      if constexpr (MODE == MODE_F32X3) ca[1][i] = read_a1(pat, I0{}, I0{}, i, I1{});
    });
    load_ss(std::integral_constant<int, P>{}, min(chunk + 2, nchunks - 1));   // buffer P: chunk-1's, free
    static_for<0, NT>([&](auto tap_c) {
      constexpr int tap = decltype(tap_c)::value;
      constexpr int CUR = tap % 3, NXT = (tap + 2) % 3;
      constexpr int U0 = XP::first(tap), UN = XP::count(tap), Q = COPY ? UN : UN * PPU * XP::NSTG;
      constexpr int UNA = UN > 0 ? UN : 1;
      const int wchunk = tap + 2 < NT ? chunk : min(chunk + 1, nchunks - 1);
      constexpr int wtap = tap + 2 < NT ? tap + 2 : tap + 2 - NT;
      float4 xr[UNA];                                  // raw values of this tap's units
      float py0[PPU * UNA], py1[PPU * UNA], pe0[PPU * UNA], pe1[PPU * UNA];
      uint32_t phi[PPU * UNA], plo[PPU * UNA];
      // stage st of piece pc (unit U0 + pc / 2, channels 2 (pc % 2) ..): the xform_piece arithmetic,
      // split so that each stage fits one block's free issue cycles
      auto stage = [&](auto pc_c, auto st_c) __attribute__((always_inline)) {
        constexpr int pc = decltype(pc_c)::value, st = decltype(st_c)::value;
        constexpr int j = pc / PPU, h = pc % PPU, k = U0 + j, PB = 1 - P;
        if constexpr (SDP_KO & 2) return;
        if constexpr (COPY) {   // one stage per unit: the 16-B copy (stage q = unit q of the tap)
          xform_store(std::integral_constant<int, U0 + decltype(pc_c)::value>{}, std::integral_constant<int, PB>{},
                      xr[decltype(pc_c)::value]);
          return;
        }
        // the piece's two raw values (IO16: the bf16 halves of word h of the unit)
        auto raw2 = [&](float& r0, float& r1) __attribute__((always_inline)) {
          const float4 v = xr[j];
          if constexpr (IO16) {
            const uint32_t w = __float_as_uint(h == 0 ? v.x : h == 1 ? v.y : h == 2 ? v.z : v.w);
            r0 = __uint_as_float(w << 16);
            r1 = __uint_as_float(w & 0xffff0000u);
          } else {
            r0 = h ? v.z : v.x;
            r1 = h ? v.w : v.y;
          }
        };
        if constexpr (XP::NSTG == 8) {   // bf16: the same arithmetic one value at a time
          const float4 v = xr[j];
          const float4 sv = ssv[PB][h];
          if constexpr (st == 0) {
            py0[pc] = fmaf(h ? v.z : v.x, sv.x, sv.y);
            if constexpr (PELU) pe0[pc] = fminf(py0[pc], 0.f);
          } else if constexpr (st == 1) {
            py1[pc] = fmaf(h ? v.w : v.y, sv.z, sv.w);
            if constexpr (PELU) pe1[pc] = fminf(py1[pc], 0.f);
          } else if constexpr (st == 2) {
            if constexpr (PELU) pe0[pc] = __expf(pe0[pc]);
          } else if constexpr (st == 3) {
            if constexpr (PELU) pe1[pc] = __expf(pe1[pc]);
          } else if constexpr (st == 4) {
            if constexpr (PELU) py0[pc] = fmaxf(py0[pc], pe0[pc] - 1.0f);
            if constexpr (ZP) py0[pc] = ((uvalid >> k) & 1u) ? py0[pc] : 0.f;
          } else if constexpr (st == 5) {
            if constexpr (PELU) py1[pc] = fmaxf(py1[pc], pe1[pc] - 1.0f);
            if constexpr (ZP) py1[pc] = ((uvalid >> k) & 1u) ? py1[pc] : 0.f;
          } else if constexpr (st == 6) {
            typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
            bf16x2 hi;
            hi[0] = (__bf16)py0[pc];
            hi[1] = (__bf16)py1[pc];
            phi[pc] = *reinterpret_cast<const uint32_t*>(&hi);
          } else {
            const int pix = (tid + k * NTH) >> 3;
            *reinterpret_cast<uint32_t*>(lds + PB * T::PATCH_BYTES + pix * PSTRIDE + my_cv * 8 + h * 4) = phi[pc];
          }
          return;
        }
        if constexpr (st == 0) {
          float r0, r1;
          raw2(r0, r1);
          const float4 sv = ssv[PB][h];
          py0[pc] = fmaf(r0, sv.x, sv.y);
          py1[pc] = fmaf(r1, sv.z, sv.w);
          if constexpr (PELU) {
            pe0[pc] = fminf(py0[pc], 0.f);
            pe1[pc] = fminf(py1[pc], 0.f);
          }
        } else if constexpr (st == 1) {
          if constexpr (PELU) {
            pe0[pc] = __expf(pe0[pc]);
            pe1[pc] = __expf(pe1[pc]);
          }
        } else if constexpr (st == 2) {
          if constexpr (PELU) {   // elu_max (common.h)
            py0[pc] = fmaxf(py0[pc], pe0[pc] - 1.0f);
            py1[pc] = fmaxf(py1[pc], pe1[pc] - 1.0f);
          }
          if constexpr (ZP) {
            const bool ok = (uvalid >> k) & 1u;
            py0[pc] = ok ? py0[pc] : 0.f;
            py1[pc] = ok ? py1[pc] : 0.f;
          }
        } else if constexpr (st == 3) {
          typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
          bf16x2 hi;
          hi[0] = (__bf16)py0[pc];
          hi[1] = (__bf16)py1[pc];
          phi[pc] = *reinterpret_cast<const uint32_t*>(&hi);
          if constexpr (MODE == MODE_F32X3) {
            bf16x2 lo;
            lo[0] = (__bf16)(py0[pc] - (float)hi[0]);
            lo[1] = (__bf16)(py1[pc] - (float)hi[1]);
            plo[pc] = *reinterpret_cast<const uint32_t*>(&lo);
          }
        } else {
          const int pix = (tid + k * NTH) >> USH;
          char* dst = lds + PB * T::PATCH_BYTES + pix * PSTRIDE + my_cv * (2 * CPU) + h * 4;
          *reinterpret_cast<uint32_t*>(dst) = phi[pc];
          if constexpr (MODE == MODE_F32X3) *reinterpret_cast<uint32_t*>(dst + 64) = plo[pc];
        }
      };
      static_for<0, NBLK>([&](auto blk_c) {
        constexpr int blk = decltype(blk_c)::value;
        constexpr int s = blk / (4 * NJ), nj = (blk / 4) % NJ, i = blk & 3, mb = 4 * s + i;
        // ---- fillers that feed this tap: raw reads first (the transform waits on them)
        if constexpr (blk < UN) xr[blk] = xform_load(std::integral_constant<int, U0 + blk>{});
        // ---- the block's MFMAs
        {
          const uint4 h4 = bq[CUR][nj >> 1][2 * (nj & 1)], l4 = bq[CUR][nj >> 1][2 * (nj & 1) + 1];
          const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(&h4);
          const bf16x8 blo = *reinterpret_cast<const bf16x8*>(&l4);
          const bf16x8 ahi = s == 0 ? ca[0][i] : cb[0][i];
          if constexpr (TRANS) {   // D = W x X: rows = Cout, columns = pixels (same fragment registers)
            if constexpr (MODE == MODE_F32X3) {
              const bf16x8 alo = s == 0 ? ca[1][i] : cb[1][i];
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi, alo, acc4[mb][nj], 0, 0, 0);
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(blo, ahi, acc4[mb][nj], 0, 0, 0);
            }
            acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi, ahi, acc4[mb][nj], 0, 0, 0);
          } else {
            if constexpr (MODE == MODE_F32X3) {
              const bf16x8 alo = s == 0 ? ca[1][i] : cb[1][i];
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc4[mb][nj], 0, 0, 0);
              acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc4[mb][nj], 0, 0, 0);
            }
            acc4[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc4[mb][nj], 0, 0, 0);
          }
        }
        // ---- fillers for later taps
        if constexpr (blk < NQ) {   // this tap's half-1 fragments (used from block NBLK / 2)
          constexpr int q = blk, ii = MODE == MODE_F32X3 ? (q >> 1) : q, lo = MODE == MODE_F32X3 ? (q & 1) : 0;
          cb[lo][ii] = read_a1(pat, tap_c, I1{}, std::integral_constant<int, ii>{}, std::integral_constant<int, lo>{});
        }
        if constexpr ((blk & 1) && (blk >> 1) < NWL)   // tap + 2's weights
          load_b1(std::integral_constant<int, NXT>{}, std::integral_constant<int, (blk >> 1)>{}, wchunk, wtap);
        if constexpr (tap + 1 < NT && blk >= NBLK / 2 && blk < NBLK / 2 + NQ) {   // tap + 1's half-0 fragments
          constexpr int q = blk - NBLK / 2, ii = MODE == MODE_F32X3 ? (q >> 1) : q, lo = MODE == MODE_F32X3 ? (q & 1) : 0;
          ca[lo][ii] = read_a1(pat, std::integral_constant<int, tap + 1>{}, I0{}, std::integral_constant<int, ii>{},
                               std::integral_constant<int, lo>{});
        }
        static_for<0, Q>([&](auto q_c) {   // transform stages dealt to this block
          constexpr int q = decltype(q_c)::value;
          if constexpr (XP::stage_blk(q, Q, NBLK) == blk) {
            if constexpr (COPY) stage(std::integral_constant<int, q>{}, std::integral_constant<int, 0>{});
            else stage(std::integral_constant<int, q / XP::NSTG>{}, std::integral_constant<int, q % XP::NSTG>{});
          }
        });
        if constexpr (UN > 0 && blk >= NBLK - UN)   // the DMA of a transformed unit (its raw slot was read)
          load_unit_o(std::integral_constant<int, U0 + blk - (NBLK - UN)>{}, chunk + 2);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    // patch[P] free for chunk+2's transform, patch[1-P] complete (see do_chunk)
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    if constexpr (!(SDP_KO & 8)) __builtin_amdgcn_s_barrier();
  };
  static_assert(NT % 2 == 1, "parity bookkeeping assumes an odd tap count");
  // (the data-gradient launches keep do_chunk: in bf16 training the tap schedule measured 3-5 % slower
  // on them, profiles/experiments/r05_train_kernel_stats_ab.log)
#ifndef SDP_DGRAD16_TAPS   // A/B (build-time): the IO16 data gradient on the tap schedule -- measured slower,
#define SDP_DGRAD16_TAPS 0    // bf16-tape training 181.0-181.5 -> 177.6-177.8 image-steps/s (profiles/experiments/r06_dgrad16_taps_ab.log)
#endif
  if constexpr (MODE != MODE_F32 && NT == 9 && (!TRANS || (IO16 && SDP_DGRAD16_TAPS))) {
    static_assert(XP::max_count() * PPU * XP::NSTG <= 2 * (NBLK - 2), "at most two transform stages per block");
    for (int chunk = 0; chunk < nchunks; chunk += 2) {   // nchunks is even (Cin % 64 == 0)
      do_chunk9(std::integral_constant<int, 0>{}, chunk);
      do_chunk9(std::integral_constant<int, 1>{}, chunk + 1);
    }
  } else {
    for (int chunk = 0; chunk < nchunks; chunk += 2) {
      do_chunk(std::integral_constant<int, 0>{}, chunk);
      do_chunk(std::integral_constant<int, 1>{}, chunk + 1);
    }
  }

  SDP_T(3);
  // the direct 16x16 epilogue: every forward, and the data-gradient launches of the 16-wide tiles
  // and 2-wave workgroups (the LDS-staged epilogue below needs TC >= 32 and 4 waves)
  if (TRANS && (!a.dact || TC < 32 || NW != 4)) {
    if constexpr (TRANS) {
    // ------------------------------------------------------------------ epilogue, 16x16 D = W x X
    // Register r of fragment (mb, nj) of lane l holds Cout 16 nj + 4 (l / 16) + r of the wave's 64 at
    // pixel l % 16 of the fragment's 16-px row segment: every load/store below moves 16 B per lane
    // (a wave instruction covers 16 pixels x 64 B).  InstanceNorm++ statistics: the lane holds 8
    // values (one per fragment mb) of each of its 16 channels; the 128-pixel group of a channel spans
    // the 16 lanes of a DPP row -> per-lane two-pass (mean, M2), then Chan merges over the row by
    // quad_perm / row_half_mirror / row_mirror moves.
    __builtin_amdgcn_s_waitcnt(0);   // the last (dead) DMA may still be landing in raw
    const int Ho = a.H, Wo = a.W;
    const size_t bo = (size_t)b * Ho * Wo * Cout;
    const int img_bytes = Ho * Wo * Cout * ES;
    auto rs = [&](const float* p) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(reinterpret_cast<const char*>(p) + bo * ES), 0, img_bytes, 0x00020000);
    };
    const int lq = lane >> 4, lcol = lane & 15;
    constexpr int CB = TC / 16;                      // 16-px fragments per tile row
    const int voff = (lcol * d * Cout + 4 * lq) * ES; // lane part of every byte offset
    auto soff = [&](int mb, int nj) {                // wave-uniform part: fragment mb's first pixel, channel block nj
      const int mr = mb / CB, mc = (mb % CB) * 16;
      const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc) * d + ph_c;
      return __builtin_amdgcn_readfirstlane(((y * Wo + x) * Cout + n0 + wn * 16 * NJ + nj * 16) * ES);
    };
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int so) {
      if constexpr (IO16) {   // 4 bf16 channels: 8 B per lane
        typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
        const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(r, voff, so, 0);
        return bf4_to_f4(make_uint2(q.x, q.y));
      } else {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, voff, so, 0);
        return make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w));
      }
    };
    auto st = [&](float4 v, __amdgpu_buffer_rsrc_t r, int so, auto aux_c) {
      constexpr int AUX = decltype(aux_c)::value;
      if constexpr (IO16) {
        typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
        const uint2 w = f4_to_bf4(v);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{w.x, w.y}, r, voff, so, AUX);
      } else {
        const u32x4 q = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(q, r, voff, so, AUX);
      }
    };
    auto rs_or_out = [&](const float* p) { return rs(p ? p : a.out); };
    const __amdgpu_buffer_rsrc_t ors = rs(a.out), xrs = rs_or_out(a.aux), rrs = rs_or_out(a.res), o2rs = rs_or_out(a.out2),
                                 r2rs = rs_or_out(a.res2);
    static_for<0, NJ>([&](auto njc) {
      constexpr int nj = decltype(njc)::value;
      __builtin_amdgcn_sched_barrier(0);              // one channel block at a time (register pressure)
      const int co0 = n0 + wn * 16 * NJ + nj * 16 + 4 * lq;   // the lane's 4 channels
      // every read of the block first -- the elu' operand, its (scale, shift), the residual -- so they
      // share one HBM round trip: issued where they are used, the residual's loads waited behind the
      // elu' math (data gradient 310 -> 260 us per 256->256 B=8 launch, bf16 training step 136.1 ->
      // 142.2 image-steps/s, profiles/experiments/r04_dgrad_epilogue_ab.log)
      float4 hq[8], rq[8], s0 = make_float4(1.f, 0.f, 1.f, 0.f), s1 = s0;
      if (a.dact) static_for<0, 8>([&](auto mb) { hq[mb] = ld(xrs, soff(mb, nj)); });
      if (a.dact == 3) {
        s0 = ld4(a.epi_ss + ((size_t)b * Cout + co0) * 2);
        s1 = ld4(a.epi_ss + ((size_t)b * Cout + co0) * 2 + 4);
      }
      if (a.res) static_for<0, 8>([&](auto mb) { rq[mb] = ld(rrs, soff(mb, nj)); });
      const float4 bias4 = a.bias ? ld4(a.bias + co0) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 esc = make_float4(s0.x, s0.z, s1.x, s1.z), esh = make_float4(s0.y, s0.w, s1.y, s1.w);
      float4 v[8];
      static_for<0, 8>([&](auto mbc) {
        constexpr int mb = decltype(mbc)::value;
        const f32x4 q = acc4[mb][nj];
        v[mb] = make_float4(q[0] + bias4.x, q[1] + bias4.y, q[2] + bias4.z, q[3] + bias4.w);
      });
      if (a.up) {   // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor
        const int Hi = a.H / 2, Wi = a.W / 2;
        const float shh = (float)(Hi - 1) / (float)(a.H - 1), sww = (float)(Wi - 1) / (float)(a.W - 1);
        const size_t ub = (size_t)b * Hi * Wi * Cout + co0;
        auto lup = [&](size_t e) { return IO16 ? ldg4(reinterpret_cast<const __bf16*>(a.up), e) : ldg4(a.up, e); };
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) {
          const int mr = mb / CB, mc = (mb % CB) * 16;
          const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc + lcol) * d + ph_c;
          const float fy = shh * (float)y, fx = sww * (float)x;
          const int y0 = (int)fy, x0 = (int)fx;
          const int yp = y0 < Hi - 1 ? 1 : 0, xp = x0 < Wi - 1 ? 1 : 0;
          const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
          const float4 v00 = lup(ub + ((size_t)y0 * Wi + x0) * Cout), v01 = lup(ub + ((size_t)y0 * Wi + x0 + xp) * Cout);
          const float4 v10 = lup(ub + ((size_t)(y0 + yp) * Wi + x0) * Cout);
          const float4 v11 = lup(ub + ((size_t)(y0 + yp) * Wi + x0 + xp) * Cout);
          auto bil = [&](float a00, float a01, float a10, float a11) {
            return ly0 * (lx0 * a00 + lx1 * a01) + ly1 * (lx0 * a10 + lx1 * a11);
          };
          v[mb].x = v[mb].x + bil(v00.x, v01.x, v10.x, v11.x);
          v[mb].y = v[mb].y + bil(v00.y, v01.y, v10.y, v11.y);
          v[mb].z = v[mb].z + bil(v00.z, v01.z, v10.z, v11.z);
          v[mb].w = v[mb].w + bil(v00.w, v01.w, v10.w, v11.w);
        }
      }
      if (a.dact) {   // backward: * the derivative of the ELU that followed this tensor (ConvArgs::dact)
        static_for<0, 8>([&](auto mbc) {
          constexpr int mb = decltype(mbc)::value;
          float4 h = hq[mb];
          if (a.dact == 3) h = make_float4(fmaf(h.x, esc.x, esh.x), fmaf(h.y, esc.y, esh.y), fmaf(h.z, esc.z, esh.z),
                                           fmaf(h.w, esc.w, esh.w));
          v[mb] = make_float4(v[mb].x * elu_grad(h.x, a.dact), v[mb].y * elu_grad(h.y, a.dact),
                              v[mb].z * elu_grad(h.z, a.dact), v[mb].w * elu_grad(h.w, a.dact));
        });
      }
      if (a.res) {
        static_for<0, 8>([&](auto mbc) {
          constexpr int mb = decltype(mbc)::value;
          const float4 r = rq[mb];
          v[mb] = make_float4(r.x + v[mb].x, r.y + v[mb].y, r.z + v[mb].z, r.w + v[mb].w);
        });
      }
      if (a.out2) {
        static_for<0, 8>([&](auto mbc) {
          constexpr int mb = decltype(mbc)::value;
          const float4 r2 = ld(r2rs, soff(mb, nj));
          st(make_float4(v[mb].x + r2.x, v[mb].y + r2.y, v[mb].z + r2.z, v[mb].w + r2.w), o2rs, soff(mb, nj),
             std::integral_constant<int, 0>{});
        });
      }
      if (a.epi_elu) {
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) v[mb] = make_float4(elu(v[mb].x), elu(v[mb].y), elu(v[mb].z), elu(v[mb].w));
      }
      if constexpr (!(SDP_KO & 16)) {
        static_for<0, 8>([&](auto mbc) {
          constexpr int mb = decltype(mbc)::value;
          st(v[mb], ors, soff(mb, nj), std::integral_constant<int, IO16 ? SDP_STORE_AUX16 : SDP_STORE_AUX>{});
        });
      }
      if (a.stats) {
        float mean[4], m2[4];
        static_for<0, 4>([&](auto rc) {
          constexpr int r = decltype(rc)::value;
          auto comp = [&](const float4& q) { return r == 0 ? q.x : r == 1 ? q.y : r == 2 ? q.z : q.w; };
          float s = 0.f;
#pragma unroll
          for (int mb = 0; mb < 8; ++mb) s += comp(v[mb]);
          mean[r] = s * 0.125f;
          float q2 = 0.f;
#pragma unroll
          for (int mb = 0; mb < 8; ++mb) {
            const float dv = comp(v[mb]) - mean[r];
            q2 = fmaf(dv, dv, q2);
          }
          m2[r] = q2;
        });
        // Chan merges of equal-count partials over the 16 lanes of the row: partners by lane ^ 1,
        // lane ^ 2 (quad_perm), the mirrored quad (row_half_mirror), the mirrored half-row (row_mirror)
        auto merge = [&](auto ctl_c, float n) {
          constexpr int CTL = decltype(ctl_c)::value;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float mp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mean[r]), CTL, 0xf, 0xf, false));
            const float qp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m2[r]), CTL, 0xf, 0xf, false));
            const float dm = mean[r] - mp;
            m2[r] = m2[r] + qp + dm * dm * (0.5f * n);
            mean[r] = 0.5f * (mean[r] + mp);
          }
        };
        merge(std::integral_constant<int, 0xB1>{}, 8.f);     // quad_perm [1,0,3,2]
        merge(std::integral_constant<int, 0x4E>{}, 16.f);    // quad_perm [2,3,0,1]
        merge(std::integral_constant<int, 0x141>{}, 32.f);   // row_half_mirror
        merge(std::integral_constant<int, 0x140>{}, 64.f);   // row_mirror
        if (lcol == 0) {
          float4* sp = reinterpret_cast<float4*>(reinterpret_cast<float2*>(a.stats) +
                                                 ((size_t)b * a.groups_per_img + tile * WM + wm) * Cout + co0);
          sp[0] = make_float4(mean[0], m2[0], mean[1], m2[1]);
          sp[1] = make_float4(mean[2], m2[2], mean[3], m2[3]);
        }
      }
    });
    }  // if constexpr (TRANS)
  } else if (SH == 16 && !TRANS && (!a.dact || TC < 32 || NW != 4)) {
    if constexpr (SH == 16 && !TRANS) {
    // ------------------------------------------------------------------ epilogue, 16x16 fragments
    // Register r of fragment (mb, nj) of lane l holds pixel 4 (l / 16) + r of the fragment's 16-px
    // row segment and Cout 16 nj + l % 16 of the wave's 64: every wave store writes four 64-B runs
    // of channels.  ConvMeanPool pairs registers r, r+1 (columns) and fragments mb, mb + TC/16
    // (rows); the 128-pixel InstanceNorm++ group of a channel spans the 4 lanes l % 16 + 16q.
    __builtin_amdgcn_s_waitcnt(0);   // the last (dead) DMA may still be landing in raw
    const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
    const size_t bo = (size_t)b * Ho * Wo * Cout;
    const int img_bytes = Ho * Wo * Cout * ES;
    auto rs = [&](const float* p) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(reinterpret_cast<const char*>(p ? p : a.out) + bo * ES), 0, img_bytes,
                                               0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ors = rs(a.out), rrs = rs(a.res), o2rs = rs(a.out2), r2rs = rs(a.res2), xrs = rs(a.aux);
    const int lq = lane >> 4, lcol = lane & 15;
    constexpr int CB = TC / 16;                      // 16-px fragments per tile row
    constexpr int NF = POOL ? CB : 8;                // fragments (pooled: row-0 fragments) per lane
    constexpr int PER = POOL ? 2 : 4;                // values per fragment and lane
    constexpr int NV = NF * PER;
    const int xs = (POOL ? 1 : d) * Cout * ES;       // bytes between consecutive output pixels of a run
    // byte offset of value i of channel block nj: a per-fragment VGPR base (channel block 0) and a
    // wave-uniform SGPR part (the value's pixel step, the block's 64-B channel offset)
    int vbase[NF];
    static_for<0, NF>([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      const int co = n0 + wn * 16 * NJ + lcol;
      if constexpr (POOL) {
        vbase[f] = (((sr0 >> 1) * Wo + ((sc0 + f * 16) >> 1) + 2 * lq) * Cout + co) * ES;
      } else {
        constexpr int mr = f / CB, mc = (f % CB) * 16;
        const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc + 4 * lq) * d + ph_c;
        vbase[f] = ((y * Wo + x) * Cout + co) * ES;
      }
    });
#define SDP_EPI16_OFF(i, nj) vbase[(i) / PER], __builtin_amdgcn_readfirstlane(((i) % PER) * xs + (nj) * 16 * ES)
    // one value of a tensor (IO16: a bf16 element, widened)
    auto ld1 = [&](__amdgpu_buffer_rsrc_t r, int vo, int so) __attribute__((always_inline)) {
      if constexpr (IO16) return __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0) << 16);
      else return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
    };
    // the NV values of channel block nj: float per value, or (IO16) bf16 pairs of adjacent channels --
    // lanes l and l ^ 1 hold channels c, c ^ 1 of the same pixels: each swaps half its values with its
    // partner (DPP quad_perm [1,0,3,2]) so that a lane stores 4 B = both channels of PER / 2 pixels
    auto store_vals = [&](const float (&w)[NV], __amdgpu_buffer_rsrc_t r, auto nj_c, auto aux_c) __attribute__((always_inline)) {
      constexpr int NJC = decltype(nj_c)::value, AUX = decltype(aux_c)::value;
      if constexpr (IO16) {
        constexpr int HP = PER / 2;
        const bool odd = lane & 1;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const int vb = vbase[f] + (odd ? HP * xs - 2 : 0);
#pragma unroll
          for (int k = 0; k < HP; ++k) {
            const float mine = odd ? w[f * PER + HP + k] : w[f * PER + k];
            const float send = odd ? w[f * PER + k] : w[f * PER + HP + k];
            const float got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0xB1, 0xf, 0xf, false));
            const uint32_t pk = odd ? pack_bf2(got, mine) : pack_bf2(mine, got);
            __builtin_amdgcn_raw_buffer_store_b32(pk, r, vb, __builtin_amdgcn_readfirstlane(k * xs + NJC * 16 * ES), AUX);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NV; ++i) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w[i]), r, SDP_EPI16_OFF(i, NJC), AUX);
      }
    };
    // The bias and the addend of every channel block (the residual, else the CRP second output's res2)
    // are loaded before the first store: loads and stores retire through one in-order counter on gfx9,
    // so a block's loads issued after the previous block's stores would wait for their acknowledgement
    // too (line 328.2 -> 335.1 image-steps/s, profiles/experiments/r04_epilogue_preload_ab.log)
    float pre[NJ][NV], biasv[NJ];
    static_for<0, NJ>([&](auto nj) { biasv[nj] = a.bias ? a.bias[n0 + wn * 16 * NJ + nj * 16 + lcol] : 0.f; });
    if (a.res || a.out2) {
      const __amdgpu_buffer_rsrc_t prs = a.res ? rrs : r2rs;
      static_for<0, NJ>([&](auto njc) {
#pragma unroll
        for (int i = 0; i < NV; ++i) pre[njc][i] = ld1(prs, SDP_EPI16_OFF(i, decltype(njc)::value));
      });
    }
    static_for<0, NJ>([&](auto njc) {
      constexpr int nj = decltype(njc)::value;
      const int co = n0 + wn * 16 * NJ + nj * 16 + lcol;
      const float bias = biasv[nj];
      float v[NV];
      if constexpr (POOL) {
        static_for<0, CB>([&](auto fc) {
          constexpr int f = decltype(fc)::value;
          static_for<0, 2>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const float a00 = acc4[f][nj][2 * k], a01 = acc4[f][nj][2 * k + 1];
            const float a10 = acc4[f + CB][nj][2 * k], a11 = acc4[f + CB][nj][2 * k + 1];
            v[f * 2 + k] = ((((a00 + bias) + (a10 + bias)) + (a01 + bias)) + (a11 + bias)) / 4.0f;  // layers.py:310-312
          });
        });
      } else {
        static_for<0, 8>([&](auto fc) {
          constexpr int f = decltype(fc)::value;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[f * 4 + r] = acc4[f][nj][r] + bias;
        });
      }
      if (a.up) {   // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor (non-pooled)
        const int Hi = a.H / 2, Wi = a.W / 2;
        const float shh = (float)(Hi - 1) / (float)(a.H - 1), sww = (float)(Wi - 1) / (float)(a.W - 1);
        const size_t ub = (size_t)b * Hi * Wi * Cout + co;
        auto lu = [&](size_t e) { return IO16 ? ldg1(reinterpret_cast<const __bf16*>(a.up), e) : ldg1(a.up, e); };
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int f = i / PER, k = i % PER;
          const int mr = f / CB, mc = (f % CB) * 16;
          const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc + 4 * lq + k) * d + ph_c;
          const float fy = shh * (float)y, fx = sww * (float)x;
          const int y0 = (int)fy, x0 = (int)fx;
          const int yp = y0 < Hi - 1 ? 1 : 0, xp = x0 < Wi - 1 ? 1 : 0;
          const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
          const float v00 = lu(ub + ((size_t)y0 * Wi + x0) * Cout), v01 = lu(ub + ((size_t)y0 * Wi + x0 + xp) * Cout);
          const float v10 = lu(ub + ((size_t)(y0 + yp) * Wi + x0) * Cout);
          const float v11 = lu(ub + ((size_t)(y0 + yp) * Wi + x0 + xp) * Cout);
          v[i] = v[i] + (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11));
        }
      }
      if (a.dact) {   // backward: * the derivative of the ELU that followed this tensor (ConvArgs::dact)
        float esc = 1.f, esh = 0.f;
        if (a.dact == 3) {
          esc = a.epi_ss[((size_t)b * Cout + co) * 2];
          esh = a.epi_ss[((size_t)b * Cout + co) * 2 + 1];
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          float h = ld1(xrs, SDP_EPI16_OFF(i, nj));
          if (a.dact == 3) h = fmaf(h, esc, esh);
          v[i] = v[i] * elu_grad(h, a.dact);
        }
      }
      if (a.res) {
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = pre[nj][i] + v[i];
      }
      if (a.out2) {
        float r2[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i)   // (a residual and a second output together: loaded here, all before the stores)
          r2[i] = a.res ? ld1(r2rs, SDP_EPI16_OFF(i, nj)) : pre[nj][i];
#pragma unroll
        for (int i = 0; i < NV; ++i) r2[i] = v[i] + r2[i];
        store_vals(r2, o2rs, njc, std::integral_constant<int, 0>{});
      }
      if (a.epi_elu) {
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = elu(v[i]);
      }
      if constexpr (!(SDP_KO & 16))
        store_vals(v, ors, njc, std::integral_constant<int, IO16 ? SDP_STORE_AUX16 : SDP_STORE_AUX>{});
      if (a.stats) {
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
        // Chan merges of equal-count partials: lanes l ^ 16 (NV values each), then l ^ 32 (2 NV each)
        float mp = __shfl_xor(mean, 16), qp = __shfl_xor(m2, 16), dm = mean - mp;
        m2 = m2 + qp + dm * dm * (0.5f * NV);
        mean = 0.5f * (mean + mp);
        mp = __shfl_xor(mean, 32);
        qp = __shfl_xor(m2, 32);
        dm = mean - mp;
        m2 = m2 + qp + dm * dm * (float)NV;
        mean = 0.5f * (mean + mp);
        if (lq == 0) {
          float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.groups_per_img + tile * WM + wm) * Cout + co;
          *st = make_float2(mean, m2);
        }
      }
    });
#undef SDP_EPI16_OFF
    }  // if constexpr (SH == 16 && !TRANS)
  } else if (a.dact) {
    if constexpr (TC >= 32 && NW == 4 && SH == 16) {   // (the data gradient runs in the bf16 modes only)
    // data-gradient launches (training): the LDS-staged epilogue -- its 16-B pixel-row
    // accesses of the elu' operand and the residual gradient beat per-channel 4-B accesses
    // ------------------------------------------------------------------ epilogue
    // The accumulators go through LDS (the patch/raw buffers are free now) in two halves of
    // 64 pixels per wave, so the output is written as whole pixel rows -- every thread owns 4
    // consecutive channels of a pixel, every store/load is 16 B and a wave instruction covers
    // 1 KiB (Cout 256) or two 512-B rows -- with bias, 2x2 mean-pool, residual, bilinear
    // upsample-add, the CRP second output, ELU and the InstanceNorm++ statistics applied on
    // the way.
    __builtin_amdgcn_s_waitcnt(0);   // the last (dead) DMA may still be landing in raw
    __syncthreads();
    constexpr int SROW = T::NTILE + 8;               // staged row stride (floats): conflict-free writes
    constexpr int SP = WM * 64;                      // staged pixels per half
    constexpr int CG = T::NTILE / 4;                 // 16-B channel groups per pixel
    constexpr int PL = 256 / CG;                     // threads per channel group
    constexpr int NPO = POOL ? SP / 4 : SP;          // output pixels per half
    static_assert(SP * SROW * 4 <= T::LDS_BYTES, "epilogue staging fits the LDS");
    float* stage = reinterpret_cast<float*>(lds);
    const int cg = tid % CG, pl = tid / CG;
    const int co0 = n0 + cg * 4;                     // this thread's 4 output channels
    const float4 bias4 = a.bias ? ld4(a.bias + co0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 es0 = make_float4(1.f, 0.f, 1.f, 0.f), es1 = es0;   // (scale, shift) of the thread's 4 channels (dact 3)
    if (a.dact == 3) {
      es0 = ld4(a.epi_ss + ((size_t)b * Cout + co0) * 2);
      es1 = ld4(a.epi_ss + ((size_t)b * Cout + co0) * 2 + 4);
    }
    const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
    using TA = std::conditional_t<IO16, __bf16, float>;   // activation element type
    auto tp = [](const float* p) { return reinterpret_cast<const TA*>(p); };
    TA* const outb = reinterpret_cast<TA*>(a.out) + (size_t)b * Ho * Wo * Cout;
    // shifted sums per (stats group, channel): K = the thread's first value
    float4 sK[WM], s1[WM], s2[WM];
    int sn[WM];
    static_for<0, WM>([&](auto g) {
      sK[g] = make_float4(0.f, 0.f, 0.f, 0.f); s1[g] = sK[g]; s2[g] = sK[g]; sn[g] = 0;
    });
    static_for<0, 2>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      // ---- stage this half's accumulators: wave (wm, wn), fragments mb of the half
      {
        // 16x16 fragments 4h .. 4h+3 of the wave hold the same 64 pixels as the 32x32 ones
        // 2h, 2h+1: fragment i, lane pixel 4 (l / 16) + r is staged pixel q = 16 i + 4 (l / 16) + r
        // (non-pooled only: the data-gradient launches; a pooled forward never takes this path)
        if constexpr (!POOL && TRANS) {   // lane l holds pixel l % 16, Couts 4 (l / 16) .. + 3: one 16-B write
          static_for<0, 4>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            static_for<0, 4>([&](auto njc) {
              constexpr int nj = decltype(njc)::value;
              float* dst = stage + (wm * 64 + 16 * i + (lane & 15)) * SROW + wn * 64 + nj * 16 + 4 * (lane >> 4);
              const f32x4 q = acc4[4 * h + i][nj];
              *reinterpret_cast<float4*>(dst) = make_float4(q[0], q[1], q[2], q[3]);
            });
          });
        } else if constexpr (!POOL) {
          static_for<0, 4>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            static_for<0, 4>([&](auto njc) {
              constexpr int nj = decltype(njc)::value;
              float* dst = stage + (wm * 64 + 16 * i + 4 * (lane >> 4)) * SROW + wn * 64 + nj * 16 + (lane & 15);
  #pragma unroll
              for (int r = 0; r < 4; ++r) dst[r * SROW] = acc4[4 * h + i][nj][r];
            });
          });
        }
      }
      __syncthreads();
      // ---- row phase: output pixels j = pl, pl + PL, ... of this half
      auto pix = [&](int j, int& y, int& x, int& g) __attribute__((always_inline)) {
        if constexpr (POOL) {   // staged pixel s = row*32 + col over rows 0/1 and columns [32h, 32h+32)
          y = (sr0 + wrow0) >> 1;
          x = (sc0 + 32 * h + 2 * j) >> 1;
          g = 0;
        } else {
          const int ws = j >> 6, q = j & 63;                 // staged pixel -> (wave row block, pixel)
          const int mb = 2 * h + (q >> 5);
          const int row = ws * T::RW + mb / (TC / 32), col = (mb % (TC / 32)) * 32 + (q & 31);
          y = (sr0 + row) * d + ph_r;
          x = (sc0 + col) * d + ph_c;
          g = ws;
        }
      };
      const size_t bo = (size_t)b * Ho * Wo * Cout;
      // the elu' operand, the residual and res2 of the NEXT pixel are loaded before this pixel's
      // stores: loads and stores retire in order (vmcnt), so loads issued after the stores would wait
      // for their acknowledgement -- a store + load round trip per pixel
      struct Ops { float4 h, r, q; };
      auto fetch = [&](int j) __attribute__((always_inline)) {
        Ops o;
        int y, x, g;
        pix(min(j, NPO - 1), y, x, g);
        const size_t oi = bo + ((size_t)y * Wo + x) * Cout + co0;
        o.h = a.aux ? ldg4(tp(a.aux), oi) : make_float4(0.f, 0.f, 0.f, 0.f);
        o.r = a.res ? ldg4(tp(a.res), oi) : make_float4(0.f, 0.f, 0.f, 0.f);
        o.q = a.out2 ? ldg4(tp(a.res2), oi) : make_float4(0.f, 0.f, 0.f, 0.f);
        return o;
      };
      Ops nx = fetch(pl);
      for (int j = pl; j < NPO; j += PL) {
        const Ops cu = nx;
        nx = fetch(j + PL);
        float4 v;
        int y, x, g;
        pix(j, y, x, g);
        if constexpr (POOL) {
          const float* s0 = stage + (2 * j) * SROW + cg * 4;
          const float4 o00 = ld4(s0), o01 = ld4(s0 + SROW), o10 = ld4(s0 + 32 * SROW), o11 = ld4(s0 + 33 * SROW);
          auto pool1 = [&](float a00, float a10, float a01, float a11, float bb) {
            return ((((a00 + bb) + (a10 + bb)) + (a01 + bb)) + (a11 + bb)) / 4.0f;  // layers.py:310-312
          };
          v.x = pool1(o00.x, o10.x, o01.x, o11.x, bias4.x);
          v.y = pool1(o00.y, o10.y, o01.y, o11.y, bias4.y);
          v.z = pool1(o00.z, o10.z, o01.z, o11.z, bias4.z);
          v.w = pool1(o00.w, o10.w, o01.w, o11.w, bias4.w);
        } else {
          const float4 o = ld4(stage + j * SROW + cg * 4);
          v = make_float4(o.x + bias4.x, o.y + bias4.y, o.z + bias4.z, o.w + bias4.w);
        }
        const size_t oidx = ((size_t)y * Wo + x) * Cout + co0;
        if (a.up) {
          // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor at (y, x)
          const int Hi = a.H / 2, Wi = a.W / 2;
          const float sh = (float)(Hi - 1) / (float)(a.H - 1), sw = (float)(Wi - 1) / (float)(a.W - 1);
          const float fy = sh * (float)y, fx = sw * (float)x;
          const int y0 = (int)fy, x0 = (int)fx;
          const int yp = y0 < Hi - 1 ? 1 : 0, xp = x0 < Wi - 1 ? 1 : 0;
          const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
          const TA* ub = tp(a.up) + (size_t)b * Hi * Wi * Cout + co0;
          const float4 v00 = ldg4(ub, ((size_t)y0 * Wi + x0) * Cout), v01 = ldg4(ub, ((size_t)y0 * Wi + x0 + xp) * Cout);
          const float4 v10 = ldg4(ub, ((size_t)(y0 + yp) * Wi + x0) * Cout);
          const float4 v11 = ldg4(ub, ((size_t)(y0 + yp) * Wi + x0 + xp) * Cout);
          auto bil = [&](float a00, float a01, float a10, float a11) {
            return ly0 * (lx0 * a00 + lx1 * a01) + ly1 * (lx0 * a10 + lx1 * a11);
          };
          v.x = v.x + bil(v00.x, v01.x, v10.x, v11.x);
          v.y = v.y + bil(v00.y, v01.y, v10.y, v11.y);
          v.z = v.z + bil(v00.z, v01.z, v10.z, v11.z);
          v.w = v.w + bil(v00.w, v01.w, v10.w, v11.w);
        }
        if (a.dact) {
          // backward: scale by the derivative of the ELU that followed this tensor in the forward
          //   1: aux = pre-activation h          elu'(h) = h > 0 ? 1 : e^h
          //   2: aux = post-activation ELU(h)    elu'    = y > 0 ? 1 : y + 1
          //   3: aux = InstanceNorm++ input h, z = h*scale + shift (epi_ss)  elu'(z)
          float4 h4 = cu.h;
          if (a.dact == 3)
            h4 = make_float4(fmaf(h4.x, es0.x, es0.y), fmaf(h4.y, es0.z, es0.w), fmaf(h4.z, es1.x, es1.y),
                             fmaf(h4.w, es1.z, es1.w));
          v = make_float4(v.x * elu_grad(h4.x, a.dact), v.y * elu_grad(h4.y, a.dact), v.z * elu_grad(h4.z, a.dact),
                          v.w * elu_grad(h4.w, a.dact));
        }
        if (a.res) v = make_float4(cu.r.x + v.x, cu.r.y + v.y, cu.r.z + v.z, cu.r.w + v.w);
        if (a.out2)
          stg4(reinterpret_cast<TA*>(a.out2), bo + oidx, make_float4(v.x + cu.q.x, v.y + cu.q.y, v.z + cu.q.z, v.w + cu.q.w));
        if (a.epi_elu) v = make_float4(elu(v.x), elu(v.y), elu(v.z), elu(v.w));
        if constexpr (!(SDP_KO & 16)) stg4(outb, oidx, v);
        static_for<0, WM>([&](auto gc) {
          constexpr int gg = decltype(gc)::value;
          if (gg == g) {
            if (sn[gg] == 0) sK[gg] = v;
            const float4 dv = make_float4(v.x - sK[gg].x, v.y - sK[gg].y, v.z - sK[gg].z, v.w - sK[gg].w);
            s1[gg] = make_float4(s1[gg].x + dv.x, s1[gg].y + dv.y, s1[gg].z + dv.z, s1[gg].w + dv.w);
            s2[gg] = make_float4(fmaf(dv.x, dv.x, s2[gg].x), fmaf(dv.y, dv.y, s2[gg].y), fmaf(dv.z, dv.z, s2[gg].z),
                                 fmaf(dv.w, dv.w, s2[gg].w));
            ++sn[gg];
          }
        });
      }
      __syncthreads();   // staging buffer reused by the next half / the statistics
    });

    if (a.stats) {
      // per-thread partials -> (mean, M2) in LDS, then a Chan merge over the PL threads of a
      // channel group; one 128-pixel statistics group per wave row block (WM)
      float2* part = reinterpret_cast<float2*>(lds);   // [WM][PL][NTILE]
      static_for<0, WM>([&](auto gc) {
        constexpr int gg = decltype(gc)::value;
        const float n = (float)sn[gg], inv = sn[gg] ? 1.f / n : 0.f;
        const float k4[4] = {sK[gg].x, sK[gg].y, sK[gg].z, sK[gg].w};
        const float a4[4] = {s1[gg].x, s1[gg].y, s1[gg].z, s1[gg].w};
        const float q4[4] = {s2[gg].x, s2[gg].y, s2[gg].z, s2[gg].w};
  #pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float mean = k4[c] + a4[c] * inv;
          const float m2 = fmaxf(q4[c] - a4[c] * a4[c] * inv, 0.f);
          part[(gg * PL + pl) * T::NTILE + cg * 4 + c] = make_float2(mean, m2);
        }
      });
      __syncthreads();
      constexpr int PER = (POOL ? 32 : 128) / PL;      // values per thread per statistics group
      for (int i = tid; i < WM * T::NTILE; i += 256) {
        const int gg = i / T::NTILE, co = i % T::NTILE;
        float mean = 0.f;
        for (int k = 0; k < PL; ++k) mean += part[(gg * PL + k) * T::NTILE + co].x;
        mean *= 1.f / PL;
        float m2 = 0.f;
        for (int k = 0; k < PL; ++k) {
          const float2 pk = part[(gg * PL + k) * T::NTILE + co];
          const float dm = pk.x - mean;
          m2 += pk.y + (float)PER * dm * dm;
        }
        float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.groups_per_img + tile * WM + gg) * Cout + n0 + co;
        *st = make_float2(mean, m2);
      }
    }
    }  // if constexpr (TC >= 32)
  } else {
    if constexpr (SH == 32) {   // the 32x32 direct epilogue (the 16x16 forward takes the first branch)
    // ------------------------------------------------------------------ epilogue
    // Straight from the accumulators, no LDS round trip: register r of fragment (mb, nb) of
    // lane l holds pixel m = (r&3) + 8(r>>2) + 4(l>>5) of the fragment's 32-pixel row segment
    // and output channel l&31 of its 32-channel block, so every wave store writes two 128-B
    // runs of channels.  ConvMeanPool's 2x2 mean pairs registers r, r+1 (columns) and fragments
    // mb, mb + TC/32 (rows) inside a lane.  Bias, bilinear upsample-add, the backward elu'
    // factor, residual, the CRP second output and ELU are applied on the way; InstanceNorm++
    // statistics: each wave holds the whole 128-pixel statistics group of its channels, so a
    // two-pass (mean, M2) over the lane's values + a Chan merge with lane l^32 gives them.
    __builtin_amdgcn_s_waitcnt(0);   // the last (dead) DMA may still be landing in raw
    {
      const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
      const size_t bo = (size_t)b * Ho * Wo * Cout;
      const int img_bytes = Ho * Wo * Cout * 4;
      // buffer resources over this image of every epilogue tensor: per-element byte offsets are
      // a per-fragment VGPR base + a wave-uniform (SGPR) register offset
      auto rs = [&](const float* p) { return __builtin_amdgcn_make_buffer_rsrc((void*)(p ? p + bo : a.out + bo), 0, img_bytes, 0x00020000); };
      const __amdgpu_buffer_rsrc_t ors = rs(a.out), rrs = rs(a.res), xrs = rs(a.aux), o2rs = rs(a.out2), r2rs = rs(a.res2);
      const int lhalf = lane >> 5, lcol = lane & 31;
      constexpr int CB = TC / 32;                      // fragments per tile row
      constexpr int NV = POOL ? 16 : 64;               // values per lane per channel block
      // value i: fragment f = i / PER, register step k = i % PER
      constexpr int PER = POOL ? 8 : 16;
      // byte offset step between consecutive output pixels of a fragment row (wave-uniform)
      const int xs = (POOL ? 1 : d) * Cout * 4;
      int vbase[POOL ? CB : 4];                          // byte offset of the fragment's pixel m = 4*lhalf (block nb = 0)
      static_for<0, (POOL ? CB : 4)>([&](auto fc) {
        constexpr int f = decltype(fc)::value;
        const int co = n0 + wn * 64 + lcol;
        if constexpr (POOL) {
          vbase[f] = (((sr0 >> 1) * Wo + ((sc0 + f * 32) >> 1) + 2 * lhalf) * Cout + co) * 4;
        } else {
          constexpr int mr = f / CB, mc = (f % CB) * 32;
          const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc + 4 * lhalf) * d + ph_c;
          vbase[f] = ((y * Wo + x) * Cout + co) * 4;
        }
      });
      // pixel index (within the fragment row, relative to 4*lhalf) of value step k
      auto mstep = [](int k) { return POOL ? ((((k & 1) * 2 + (k >> 1) * 4) & 3) + 8 * (((k & 1) * 2 + (k >> 1) * 4) >> 2)) / 2
                                           : (k & 3) + 8 * (k >> 2); };
  #define SDP_EPI_OFF(i, nb) vbase[(i) / PER], __builtin_amdgcn_readfirstlane(mstep((i) % PER) * xs + (nb) * 128)
      // the addend of both channel blocks (residual, else res2) loaded before the first store (see
      // the 16x16 epilogue: loads and stores retire in one in-order counter)
      float pre[2][NV], biasv[2];
      static_for<0, 2>([&](auto nb) { biasv[nb] = a.bias ? a.bias[n0 + wn * 64 + nb * 32 + lcol] : 0.f; });
      if (a.res || a.out2) {
        const __amdgpu_buffer_rsrc_t prs = a.res ? rrs : r2rs;
        static_for<0, 2>([&](auto nbc) {
  #pragma unroll
          for (int i = 0; i < NV; ++i)
            pre[nbc][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, SDP_EPI_OFF(i, decltype(nbc)::value), 0));
        });
      }
      static_for<0, 2>([&](auto nbc) {
        constexpr int nb = decltype(nbc)::value;
        const int co = n0 + wn * 64 + nb * 32 + lcol;
        const float bias = biasv[nb];
        float v[NV];
        if constexpr (POOL) {
          static_for<0, CB>([&](auto mbc) {
            constexpr int mb = decltype(mbc)::value;
            static_for<0, 8>([&](auto kc) {
              constexpr int k = decltype(kc)::value;
              constexpr int r = (k & 1) * 2 + (k >> 1) * 4;          // r & 3 in {0, 2}
              const float a00 = acc[mb][nb][r], a01 = acc[mb][nb][r + 1];
              const float a10 = acc[mb + CB][nb][r], a11 = acc[mb + CB][nb][r + 1];
              v[mb * 8 + k] = ((((a00 + bias) + (a10 + bias)) + (a01 + bias)) + (a11 + bias)) / 4.0f;  // layers.py:310-312
            });
          });
        } else {
          static_for<0, 4>([&](auto mbc) {
            constexpr int mb = decltype(mbc)::value;
  #pragma unroll
            for (int r = 0; r < 16; ++r) v[mb * 16 + r] = acc[mb][nb][r] + bias;
          });
        }
        if (a.up) {   // F.interpolate(bilinear, align_corners=True) of a [H/2][W/2] tensor (non-pooled)
          const int Hi = a.H / 2, Wi = a.W / 2;
          const float shh = (float)(Hi - 1) / (float)(a.H - 1), sww = (float)(Wi - 1) / (float)(a.W - 1);
          const float* ub = a.up + (size_t)b * Hi * Wi * Cout + co;
  #pragma unroll
          for (int i = 0; i < NV; ++i) {
            const int f = i / PER, k = i % PER;
            const int mr = f / CB, mc = (f % CB) * 32;
            const int y = (sr0 + wrow0 + mr) * d + ph_r, x = (sc0 + mc + 4 * lhalf + mstep(k)) * d + ph_c;
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
        if (a.dact) {
          float esc = 1.f, esh = 0.f;
          if (a.dact == 3) {
            esc = a.epi_ss[((size_t)b * Cout + co) * 2];
            esh = a.epi_ss[((size_t)b * Cout + co) * 2 + 1];
          }
  #pragma unroll
          for (int i = 0; i < NV; ++i) {
            float h = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, SDP_EPI_OFF(i, nb), 0));
            if (a.dact == 3) h = fmaf(h, esc, esh);
            v[i] = v[i] * elu_grad(h, a.dact);
          }
        }
        if (a.res) {
  #pragma unroll
          for (int i = 0; i < NV; ++i) v[i] = pre[nb][i] + v[i];
        }
        if (a.out2) {
          float r2[NV];
  #pragma unroll
          for (int i = 0; i < NV; ++i)
            r2[i] = a.res ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r2rs, SDP_EPI_OFF(i, nb), 0)) : pre[nb][i];
  #pragma unroll
          for (int i = 0; i < NV; ++i) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i] + r2[i]), o2rs, SDP_EPI_OFF(i, nb), 0);
        }
        if (a.epi_elu) {
  #pragma unroll
          for (int i = 0; i < NV; ++i) v[i] = elu(v[i]);
        }
        if constexpr (!(SDP_KO & 16)) {
  #pragma unroll
          for (int i = 0; i < NV; ++i) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), ors, SDP_EPI_OFF(i, nb), SDP_STORE_AUX);
        }
        if (a.stats) {
          float sum = 0.f;
  #pragma unroll
          for (int i = 0; i < NV; ++i) sum += v[i];
          const float mean_l = sum * (1.0f / NV);
          float m2_l = 0.f;
  #pragma unroll
          for (int i = 0; i < NV; ++i) {
            const float dv = v[i] - mean_l;
            m2_l = fmaf(dv, dv, m2_l);
          }
          const float mean_p = __shfl_xor(mean_l, 32), m2_p = __shfl_xor(m2_l, 32);
          const float dm = mean_l - mean_p;
          const float mean = 0.5f * (mean_l + mean_p);
          const float m2 = m2_l + m2_p + dm * dm * (0.5f * NV);
          if (lhalf == 0) {
            float2* st = reinterpret_cast<float2*>(a.stats) + ((size_t)b * a.groups_per_img + tile * WM + wm) * Cout + co;
            *st = make_float2(mean, m2);
          }
        }
      });
  #undef SDP_EPI_OFF
    }
    }  // if constexpr (SH == 32)
  }
#ifdef SDP_TIMING
  SDP_T(4);
  if (tid == 0) {
    unsigned long long* o = a.dbg + blockIdx.x * 8;
    o[0] = tclk[0]; o[1] = tclk[1]; o[2] = tclk[2]; o[3] = tclk[3]; o[4] = tclk[4]; o[5] = tbar;
    o[6] = rt0; o[7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
#endif
}

}  // namespace sdp
