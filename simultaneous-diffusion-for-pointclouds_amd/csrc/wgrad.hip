// Weight gradient of the score network's 3x3 / dilated / 1x1 convolutions on MFMA (gfx950),
// for the DSM training backward (LiDARGen/losses/dsm.py:67-119 -> loss.backward(),
// runners/ncsn_runner_kitti_simultaneous.py:229-232).
//
//   dW[co][ci][kh][kw] = sum_{b,y,x} dy[b][y][x][co] * a[b][y + (kh-1)d][x + (kw-1)d][ci]
//   a = prologue(in): the forward conv's input transform (InstanceNorm++ affine + ELU, ELU,
//       or none), zero or circular padding.
//
// GEMM view per tap: M = Cout, N = Cin, K = pixels.  Both operands sit in HBM as NHWC
// (channel-contiguous), but an MFMA lane needs 8 consecutive K (= pixels) of one channel, so
// the tiles are staged in LDS as [pixel][32 channels] bf16 rows (64 B, conflict-free) and read
// with ds_read_b64_tr_b16, the CDNA4 transposing LDS read: a tap's pixel shift is then just a
// row offset, and the 9 taps reuse one staged input patch.
//
// Workgroup (4 waves, one per SIMD): 128 Cout x 32 Cin x all taps; wave w owns Cout
// [32w, 32w+32) -> 9 accumulators of 32x32.  Grid split x Cin/32 x Cout/128 (1-D, the channel blocks
// of a split together on one XCD, see the kernel): the pixels are
// split S ways, every workgroup walks its range of TR x TC pixel tiles (polyphase sub-grid
// for dilated convs, like the forward) with the next tile's global loads in registers, and
// writes its partial sums to part[split][tap][Cout][Cin]; conv_wgrad_reduce sums the splits
// in a fixed order (deterministic) into the state_dict layout [Cout][Cin][k][k].
#include "common.h"
#include "kernels.h"

// SDP_WGRAD_KO (diagnostic builds only, wrong results): 1 = the B operand read once per k step (no per-tap
// LDS reads), 2 = no staging (the MFMAs run on whatever the LDS holds), 4 = OCC 3 without the input patch's
// loads, 8 = OCC 3 without the dy DMAs
#ifndef SDP_WGRAD_KO
#define SDP_WGRAD_KO 0
#endif

namespace sdp {

typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 vbf16x4;
typedef __attribute__((address_space(3))) vbf16x4 lds_vbf16x4;

SDP_DEV bf16x4 ds_read_tr(const char* p) {
  const vbf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      reinterpret_cast<lds_vbf16x4*>(reinterpret_cast<uintptr_t>(p)));
  return __builtin_bit_cast(bf16x4, v);
}

// two transposed reads -> one 8-element operand: a register-pair concatenation, no VALU
// (element-wise inserts cost ~14 VALU per MFMA here)
SDP_DEV bf16x8 cat8(bf16x4 a, bf16x4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

template <int TC, int KS>
struct WgTile {
  static constexpr int TR = 128 / TC;
  static constexpr int HALO = KS == 3 ? 1 : 0;
  static constexpr int PC = TC + 2 * HALO, PR = TR + 2 * HALO, NPIX = PR * PC;
  static constexpr int NUA = (NPIX * 8 + 255) / 256;   // a-patch float4 units per thread
  static constexpr int NUD = 16;                        // dy tile: 128 px x 128 co / 4 / 256
  static constexpr int DY_PLANE = 4 * 128 * 64;         // [wave][px][32 co] bf16
  static constexpr int A_PLANE = NPIX * 64;             // [px][32 ci] bf16
  static constexpr int RAW_DY = 64 * 128 * 4;           // OCC 3: one half of the fp32 dy tile, landed by LDS-DMA
};

// OCC: 1 = one workgroup per CU, next tile's loads in registers (fp32x3); 2 = two workgroups per CU
// taking turns, chunked staging (bf16: 134.4 image-steps/s in the bf16 training step against 119.2
// for OCC 1 and for one workgroup per CU with the next two tiles' loads in flight,
// profiles/experiments/r03_train_ring_wgrad_ab.log); 3 = two workgroups per CU, the dy tile landed by
// LDS-DMA in two 32-KB halves (no registers), the next tile's first half issued before this tile's
// MFMAs -- one exposed global round trip per tile (the second half, with the input patch's loads)
// instead of four
template <int MODE, int TC, int KS, int OCC>
__global__ __launch_bounds__(256, OCC >= 2 ? 2 : 1) void conv_wgrad_kernel(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  using T = WgTile<TC, KS>;
  constexpr int NT = KS * KS;
  constexpr int NPL = MODE == MODE_F32X3 ? 2 : 1;      // bf16 planes: hi (+ lo)
  constexpr int RAWB = OCC == 3 ? T::RAW_DY : 0;
  static_assert(OCC != 3 || 2 * (NPL * (T::DY_PLANE + T::A_PLANE) + RAWB) <= 160 * 1024, "OCC 3: two workgroups per CU");
  __shared__ __attribute__((aligned(16))) char lds[NPL * (T::DY_PLANE + T::A_PLANE) + RAWB];
  char* const dyL = lds;                                // plane pl at + pl * DY_PLANE
  char* const aL = lds + NPL * T::DY_PLANE;             // plane pl at + pl * A_PLANE
  char* const rawL = lds + NPL * (T::DY_PLANE + T::A_PLANE);   // OCC 3

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // OCC 3: values derived from the thread index are recomputed where they are used (from an opaque copy
  // of it): hoisted they are tens of loop-invariant VGPRs, spilled at two waves per SIMD, and a scratch
  // reload before the MFMA loop would make it wait for the next tile's DMA (one vmcnt)
  auto tidx = [&]() __attribute__((always_inline)) {
    int t = tid;
    if constexpr (OCC == 3) asm volatile("" : "+v"(t));
    return t;
  };
  const int d = a.dil, Hs = a.H / d, Ws = a.W / d;
  const int tiles_c = Ws / TC, tiles_rc = (Hs / T::TR) * tiles_c, tiles_img = tiles_rc * d * d;
  const int total = a.B * tiles_img;
  // 1-D grid of (pixel split, Cin block, Cout block), the channel blocks fastest, dealt to the XCDs in
  // contiguous ranges: the Cin/32 workgroups that read the same dy tile (and the Cout/128 that read the
  // same input patch) run together on one XCD and share it through its L2 (PMC reads 514 -> 378 MB per
  // launch against the splits-fastest order; time unchanged, profiles/experiments/r05_wgrad_occ_ab.log)
  const int ncb = (a.Cin / 32) * (a.Cout / 128), G = gridDim.x;
  const int q = (G & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (G >> 3) + ((int)blockIdx.x >> 3);
  const int S = G / ncb;
  const int cb = q % ncb, cib = cb % (a.Cin / 32), cob = cb / (a.Cin / 32);
  const int split = q / ncb;
  const int t_begin = (int)((long long)total * split / S), t_end = (int)((long long)total * (split + 1) / S);
  const int ci0 = cib * 32, co0 = cob * 128;
  const int Cin = a.Cin, Cout = a.Cout;

  f32x16 acc[NT];
  static_for<0, NT>([&](auto i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  });

  static_assert(OCC >= 1 && OCC <= 3, "OCC: 1, 2 or 3");
  float4 rdS[1][T::NUD], raS[1][T::NUA];
  int tb = 0, tph_r = 0, tph_c = 0, tsr0 = 0, tsc0 = 0;
  auto decode = [&](int t) {
    tb = t / tiles_img;
    int r = t - tb * tiles_img;
    const int ph = r / tiles_rc;
    r -= ph * tiles_rc;
    tph_r = ph / d;
    tph_c = ph - tph_r * d;
    tsr0 = (r / tiles_c) * T::TR;
    tsc0 = (r % tiles_c) * TC;
  };
  // Per-unit byte offsets inside a tile are tile-independent (the polyphase sub-grid makes
  // every tile the same shape), so they are computed once; a tile then costs one wave-uniform
  // base per tensor and the loads go through buffer resources (base in SGPRs, unit offset in a
  // VGPR) -- no per-load address arithmetic.  Tiles whose input patch touches the image border
  // (circular wrap / zero padding) take the general path.
  // dy unit k = lane pixel (tid >> 5) + 8k of the tile: one VGPR offset plus a wave-uniform
  // per-unit step (8 columns, or a row every TC / 8 units) in the SGPR offset
  const int voff_dy0 = (((tid >> 5) * d) * Cout + (tid & 31) * 4) * 4;
  const int dy_col8 = 8 * d * Cout * 4, dy_row = d * a.W * Cout * 4;
  int voff_a[T::NUA];
#pragma unroll
  for (int k = 0; k < T::NUA; ++k) {
    int u = tid + k * 256;
    u = u < T::NPIX * 8 ? u : 0;
    const int pix = u >> 3, cv = u & 7;
    voff_a[k] = (((pix / T::PC) * d * a.W + (pix % T::PC) * d) * Cin + cv * 4) * 4;
  }
  const int img_dy_bytes = a.H * a.W * Cout * 4, img_in_bytes = a.H * a.W * Cin * 4;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  // per-tile buffer resources / wave-uniform bases (tile decoded into tb, tph_*, tsr0, tsc0)
  __amdgpu_buffer_rsrc_t drs, irs;
  int dbase = 0, ibase = 0;
  bool interior = false;
  auto prep_tile = [&]() {
    drs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.dy + (size_t)tb * a.H * a.W * Cout), 0, img_dy_bytes, 0x00020000);
    dbase = __builtin_amdgcn_readfirstlane((((tsr0 * d + tph_r) * a.W + tsc0 * d + tph_c) * Cout + co0) * 4);
    interior = tsr0 >= T::HALO && tsr0 + T::TR + T::HALO <= Hs && tsc0 >= T::HALO && tsc0 + TC + T::HALO <= Ws;
    irs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.in + (size_t)tb * a.H * a.W * Cin), 0, img_in_bytes, 0x00020000);
    ibase = __builtin_amdgcn_readfirstlane(
        ((((tsr0 - T::HALO) * d + tph_r) * a.W + (tsc0 - T::HALO) * d + tph_c) * Cin + ci0) * 4);
  };
  // global -> registers, units [KB, KE) of the dy tile / the input patch
  auto load_dy = [&](auto kb_, auto ke_, auto set_) {
    constexpr int KB = decltype(kb_)::value, KE = decltype(ke_)::value, SET = decltype(set_)::value;
    float4* rd = rdS[SET];
#pragma unroll
    for (int k = KB; k < KE; ++k) {
      constexpr int KPR = TC / 8;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(drs, voff_dy0, dbase + (k % KPR) * dy_col8 + (k / KPR) * dy_row, 0);
      rd[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
    }
  };
  // OCC 3: the prologue's (scale, shift) of the thread's channel group, loaded beside the patch (a load of
  // their own after the patch's wait would be one more round trip per tile)
  float4 ssa0 = make_float4(1.f, 0.f, 1.f, 0.f), ssa1 = ssa0;
  auto load_a = [&](auto kb_, auto ke_, auto set_) {
    constexpr int KB = decltype(kb_)::value, KE = decltype(ke_)::value, SET = decltype(set_)::value;
    float4* ra = raS[SET];
    if constexpr (OCC == 3 && KB == 0) {
      if (a.pro_mode != PRO_NONE) {
        const float* ssb = a.pro_ss + (size_t)tb * a.ss_bstride + ci0 * 2 + (tidx() & 7) * 8;
        ssa0 = *reinterpret_cast<const float4*>(ssb);
        ssa1 = *reinterpret_cast<const float4*>(ssb + 4);
      }
    }
    if (interior) {
      int tidv = tid;
      if constexpr (OCC == 3) asm volatile("" : "+v"(tidv));
#pragma unroll
      for (int k = KB; k < KE; ++k) {
        int vo = voff_a[k];
        if constexpr (OCC == 3) {   // recomputed per tile (7 loop-invariant VGPRs fewer)
          int u = tidv + k * 256;
          u = u < T::NPIX * 8 ? u : 0;
          const int pix = u >> 3, cv = u & 7;
          vo = (((pix / T::PC) * d * a.W + (pix % T::PC) * d) * Cin + cv * 4) * 4;
        }
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(irs, vo, ibase, 0);
        ra[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
      }
      return;
    }
    const float* inb = a.in + (size_t)tb * a.H * a.W * Cin + ci0;
    // OCC 3: recompute the unit coordinates per tile (an opaque copy of tid): hoisted out of the tile
    // loop they are ~30 loop-invariant VGPRs, spilled at two waves per SIMD
    int tidv = tid;
    if constexpr (OCC == 3) asm volatile("" : "+v"(tidv));
#pragma unroll
    for (int k = KB; k < KE; ++k) {
      int u = tidv + k * 256;
      u = u < T::NPIX * 8 ? u : 0;
      const int pix = u >> 3, cv = u & 7;
      int sr = tsr0 - T::HALO + pix / T::PC, sc = tsc0 - T::HALO + pix % T::PC;
      if (a.circular) {
        sr = sr < 0 ? sr + Hs : (sr >= Hs ? sr - Hs : sr);
        sc = sc < 0 ? sc + Ws : (sc >= Ws ? sc - Ws : sc);
      } else {
        sr = min(max(sr, 0), Hs - 1);
        sc = min(max(sc, 0), Ws - 1);
      }
      const int y = sr * d + tph_r, x = sc * d + tph_c;
      if constexpr (OCC == 3) {   // through the image's buffer resource: 32-bit offsets, no 64-bit addresses
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(irs, ((y * a.W + x) * Cin + ci0 + cv * 4) * 4, 0, 0);
        ra[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
      } else {
        ra[k] = *reinterpret_cast<const float4*>(inb + ((size_t)y * a.W + x) * Cin + cv * 4);
      }
    }
  };
  auto put_bf16 = [&](char* base, int plane, int off, float4 v) {
    bf16x4 hi;
    hi[0] = (__bf16)v.x; hi[1] = (__bf16)v.y; hi[2] = (__bf16)v.z; hi[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(base + off) = hi;
    if constexpr (MODE == MODE_F32X3) {
      bf16x4 lo;
      lo[0] = (__bf16)(v.x - (float)hi[0]);
      lo[1] = (__bf16)(v.y - (float)hi[1]);
      lo[2] = (__bf16)(v.z - (float)hi[2]);
      lo[3] = (__bf16)(v.w - (float)hi[3]);
      *reinterpret_cast<bf16x4*>(base + plane + off) = lo;
    }
  };
  // registers -> LDS (prologue transform on the input patch, zero padding, bf16 split)
  float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);   // bias gradient: sum of dy over this thread's pixels
  auto store_dy = [&](auto kb_, auto ke_, auto set_) {
    constexpr int KB = decltype(kb_)::value, KE = decltype(ke_)::value, SET = decltype(set_)::value;
    const float4* rd = rdS[SET];
#pragma unroll
    for (int k = KB; k < KE; ++k) {
      const int u = tid + k * 256, px = u >> 5, cv = u & 31;
      put_bf16(dyL, T::DY_PLANE, (cv >> 3) * (128 * 64) + px * 64 + (cv & 7) * 8, rd[k]);
      bsum = make_float4(bsum.x + rd[k].x, bsum.y + rd[k].y, bsum.z + rd[k].z, bsum.w + rd[k].w);
    }
    // keep the bias sums here: sunk past the k loop they hold the previous tile's registers
    // alive beside the next tile's loads (64 VGPRs of copies)
    asm volatile("" : "+v"(bsum.x), "+v"(bsum.y), "+v"(bsum.z), "+v"(bsum.w));
  };
  auto store_a = [&](auto kb_, auto ke_, auto set_) {
    constexpr int KB = decltype(kb_)::value, KE = decltype(ke_)::value, SET = decltype(set_)::value;
    const float4* ra = raS[SET];
    const int sb = tb, sr0_ = tsr0, sc0_ = tsc0;
    int tidv = tid;
    if constexpr (OCC == 3) asm volatile("" : "+v"(tidv));
    const float* ssb = a.pro_ss + (size_t)sb * a.ss_bstride + ci0 * 2;
    // every unit of a thread has channel group cv = tid % 8: its (scale, shift) loaded once
    float4 s0 = make_float4(1.f, 0.f, 1.f, 0.f), s1 = s0;
    if constexpr (OCC == 3) {
      s0 = ssa0;
      s1 = ssa1;
    } else if (a.pro_mode != PRO_NONE) {
      s0 = *reinterpret_cast<const float4*>(ssb + (tid & 7) * 8);
      s1 = *reinterpret_cast<const float4*>(ssb + (tid & 7) * 8 + 4);
    }
#pragma unroll
    for (int k = KB; k < KE; ++k) {
      const int u = tidv + k * 256;
      if (u >= T::NPIX * 8) break;
      const int pix = u >> 3, cv = u & 7;
      float4 v = ra[k];
      if (a.pro_mode != PRO_NONE) {
        v = make_float4(fmaf(v.x, s0.x, s0.y), fmaf(v.y, s0.z, s0.w), fmaf(v.z, s1.x, s1.y), fmaf(v.w, s1.z, s1.w));
        v = make_float4(elu(v.x), elu(v.y), elu(v.z), elu(v.w));
      }
      if (!a.circular && KS == 3) {
        const int sr = sr0_ - 1 + pix / T::PC, sc = sc0_ - 1 + pix % T::PC;
        if (sr < 0 || sr >= Hs || sc < 0 || sc >= Ws) v = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      put_bf16(aL, T::A_PLANE, pix * 64 + cv * 8, v);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using IND = std::integral_constant<int, T::NUD>;
  using INA = std::integral_constant<int, T::NUA>;
  // OCC 2: two workgroups per CU take turns (one stages while the other's MFMAs run), so a
  // tile is staged in chunks of CH units straight through registers, no cross-tile prefetch
  // (8 units = 32 VGPRs of loads: with the 144 accumulators at two waves per SIMD, 11 units spill
  // 3 VGPRs, a whole tile (22 units) 75)
  constexpr int CH = 8;
  auto stage_chunked = [&]() {

    static_for<0, (T::NUD + CH - 1) / CH>([&](auto c) {
      using KB = std::integral_constant<int, decltype(c)::value * CH>;
      using KE = std::integral_constant<int, (decltype(c)::value * CH + CH < T::NUD ? decltype(c)::value * CH + CH : T::NUD)>;
      load_dy(KB{}, KE{}, I0{});
      store_dy(KB{}, KE{}, I0{});
    });
    static_for<0, (T::NUA + CH - 1) / CH>([&](auto c) {
      using KB = std::integral_constant<int, decltype(c)::value * CH>;
      using KE = std::integral_constant<int, (decltype(c)::value * CH + CH < T::NUA ? decltype(c)::value * CH + CH : T::NUA)>;
      load_a(KB{}, KE{}, I0{});
      store_a(KB{}, KE{}, I0{});
    });
  };

  // OCC 3: half h of the dy tile (tile pixels 64h .. 64h+63) lands in rawL by LDS-DMA.  Unit u =
  // (wave * 8 + j) * 64 + lane, j < 8, is 16 B = 4 channels (u & 31) of tile pixel 64h + (u >> 5); it
  // lands at rawL + 16u and is converted by the thread that issued it (its own vmcnt, no barrier)
  // wave w's units are half pixels 16w + 2j + (lane >> 5): one tile row (TC >= 32), so unit j is unit
  // 0 plus a wave-uniform 2j columns (SGPR offset) -- one VGPR offset per thread
  static_assert(OCC != 3 || TC % 32 == 0, "OCC 3: a wave's 16 pixels inside one tile row");
  auto dma_dy_half = [&](int h) __attribute__((always_inline)) {
    if constexpr (OCC == 3) {
      const int tl = tidx();
      const int p = (tl >> 6) * 16 + ((tl & 63) >> 5);
      const int dyo = (((p / TC) * d * a.W + (p % TC) * d) * Cout + (tl & 31) * 4) * 4;
      const i32x4 rs = buffer_desc(a.dy + (size_t)tb * a.H * a.W * Cout, (uint32_t)img_dy_bytes);
      const int hoff = ((((64 / TC) * h) * d) * a.W) * Cout * 4;   // 64 tile pixels = 64 / TC tile rows
      const uint32_t l0 = (uint32_t)(uintptr_t)rawL + (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6) * 8 * 1024;
      if constexpr (!(SDP_WGRAD_KO & 8))
#pragma unroll
        for (int j = 0; j < 8; ++j) dma16_lds_opaque(rs, l0 + j * 1024, dyo, dbase + hoff + j * 2 * d * Cout * 4);
    }
  };
  // convert the thread's own 8 landed units of half h (fp32 -> bf16 [wave][px][32 co] rows, bias sums)
  // unit j of the thread: raw + rb + 1024 j -> dyL + wb + 4096 h + 128 j (pixel 64h + 16 wave + 2j + lane / 32,
  // channel quad lane % 32): two base VGPRs, the rest in the instructions' offset fields
  auto convert_dy_half = [&](auto h_) __attribute__((always_inline)) {
    if constexpr (OCC == 3) {
      constexpr int h = decltype(h_)::value;
      const int tl = tidx();
      const int rb = tl * 16 + (tl >> 6) * 7 * 1024;
      const int wb = ((tl & 31) >> 3) * (128 * 64) + ((tl >> 6) * 16 + ((tl & 63) >> 5)) * 64 + (tl & 7) * 8;
      // two batches of four (16 VGPRs of reads in flight beside the input patch's loads)
      static_for<0, 2>([&](auto g) {
        static_for<0, 4>([&](auto jj) {
          constexpr int j = decltype(g)::value * 4 + decltype(jj)::value;
          const float4 v = *reinterpret_cast<const float4*>(rawL + rb + j * 1024);
          put_bf16(dyL + wb, T::DY_PLANE, h * 4096 + j * 128, v);
          bsum = make_float4(bsum.x + v.x, bsum.y + v.y, bsum.z + v.z, bsum.w + v.w);
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  };

  // transposed-read lane roles (ds_read_b64_tr_b16, 32x32x16 operand): lane l of 16-lane
  // group G supplies row q = (l & 15) >> 2 (K), columns 4p .. 4p+3, p = l & 3 (M or N)
  // the MFMAs of the staged tile: 8 k steps of 16 pixels x all taps
  auto compute = [&]() __attribute__((always_inline)) {
    const int tl = tidx(), ln = tl & 63;
    const int G = ln >> 4, q = (ln & 15) >> 2, p = ln & 3;
    const int kq = 8 * (G >> 1) + q;                      // K of this lane's address, read r adds 4r
    const int mcol = 16 * (G & 1) + 4 * p;                 // channel of this lane's address
    const char* dy_rd = dyL + __builtin_amdgcn_readfirstlane(tl >> 6) * (128 * 64) + mcol * 2;
    const char* a_rd = aL + mcol * 2;
#pragma unroll 1
    for (int s = 0; s < 8; ++s) {   // 16 pixels per k step
      const int k0 = 16 * s + kq, k1 = k0 + 4;
      bf16x8 ahi = cat8(ds_read_tr(dy_rd + k0 * 64), ds_read_tr(dy_rd + k1 * 64)), alo;
      if constexpr (MODE == MODE_F32X3)
        alo = cat8(ds_read_tr(dy_rd + T::DY_PLANE + k0 * 64), ds_read_tr(dy_rd + T::DY_PLANE + k1 * 64));
      // patch pixel of tile pixel k at tap (0, 0)
      const int p0 = (k0 / TC) * T::PC + k0 % TC, p1 = (k1 / TC) * T::PC + k1 % TC;
      const char* b0 = a_rd + p0 * 64;
      const char* b1 = a_rd + p1 * 64;
      auto rd_b = [&](int toff, int plane) { return cat8(ds_read_tr(b0 + plane + toff), ds_read_tr(b1 + plane + toff)); };
      // B operands one tap ahead, so an MFMA never waits on the LDS read issued just before it
      bf16x8 bhi_n = rd_b(0, 0), blo_n;
      if constexpr (MODE == MODE_F32X3) blo_n = rd_b(0, T::A_PLANE);
      static_for<0, NT>([&](auto tc_) {
        constexpr int tap = decltype(tc_)::value;
        const bf16x8 bhi = bhi_n;
        bf16x8 blo;
        if constexpr (MODE == MODE_F32X3) blo = blo_n;
        if constexpr (tap + 1 < NT && !(SDP_WGRAD_KO & 1)) {
          constexpr int toff = (KS == 3 ? ((tap + 1) / 3) * T::PC + (tap + 1) % 3 : 0) * 64;
          bhi_n = rd_b(toff, 0);
          if constexpr (MODE == MODE_F32X3) blo_n = rd_b(toff, T::A_PLANE);
        }
        if constexpr (MODE == MODE_F32X3) {
          acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, bhi, acc[tap], 0, 0, 0);
          acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, blo, acc[tap], 0, 0, 0);
        }
        acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bhi, acc[tap], 0, 0, 0);
      });
    }
  };
  if constexpr (OCC == 3) {
    // raw holds the first half of tile t's dy (issued before the previous tile's MFMAs) at the loop top
    if (t_begin < t_end) {
      decode(t_begin);
      prep_tile();
      dma_dy_half(0);
    }
    for (int t = t_begin; t < t_end; ++t) {
      if constexpr (SDP_WGRAD_KO & 2) {
        __syncthreads();
        compute();
        continue;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's half-0 units have landed
      convert_dy_half(I0{});
      __builtin_amdgcn_s_waitcnt(0xc07f);                  // lgkmcnt(0): raw read before it is refilled
      dma_dy_half(1);
      if constexpr (!(SDP_WGRAD_KO & 4)) load_a(I0{}, INA{}, I0{});   // the input patch, beside the second half
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::NUA) : "memory");   // the half-1 DMA (older than the loads)
      convert_dy_half(std::integral_constant<int, 1>{});
      store_a(I0{}, INA{}, I0{});
      // vmcnt(0) + lgkmcnt(0) as a real s_waitcnt: the compiler then counts nothing in flight (a patch unit
      // past the patch has no use, so its load would stay pending and the MFMA loop's first register
      // reuse would wait on it -- behind the next tile's DMA)
      __builtin_amdgcn_s_waitcnt(0x0070);
      __syncthreads();                                     // dyL / aL complete, raw free
      if (t + 1 < t_end) {
        decode(t + 1);
        prep_tile();
        dma_dy_half(0);                                    // lands under this tile's MFMAs
      }
      compute();
      __syncthreads();                                     // dyL / aL read before the next tile rewrites them
    }
  } else {
    if (OCC == 1 && t_begin < t_end) {
      decode(t_begin);
      prep_tile();
      load_dy(I0{}, IND{}, I0{});
      load_a(I0{}, INA{}, I0{});
    }
    for (int t = t_begin; t < t_end; ++t) {
      __syncthreads();
      if constexpr (OCC == 1) {
        store_dy(I0{}, IND{}, I0{});
        store_a(I0{}, INA{}, I0{});
        __syncthreads();
        if (t + 1 < t_end) {
          decode(t + 1);
          prep_tile();
          load_dy(I0{}, IND{}, I0{});
          load_a(I0{}, INA{}, I0{});
        }
      } else {
        decode(t);
        prep_tile();
        stage_chunked();
        __syncthreads();
      }
      compute();
    }
  }
  // bias partials (the ci-block-0 workgroups): bpart[split][Cout]; every thread's channel
  // group is tid & 31, its pixels tid >> 5 -> combine the 8 threads of a group through LDS
  if (a.bpart && cib == 0) {
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(lds);
    red[tid] = bsum;
    __syncthreads();
    if (tid < 32) {
      float4 t = red[tid];
      for (int k = 1; k < 8; ++k) {
        const float4 v = red[tid + 32 * k];
        t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
      }
      *reinterpret_cast<float4*>(a.bpart + (size_t)split * Cout + co0 + tid * 4) = t;
    }
  }
  // partials: part[split][tap][Cout][Cin]; accumulator register r of lane l is
  // row (co) (r & 3) + 8 (r >> 2) + 4 (l >> 5), column (ci) l & 31
  static_for<0, NT>([&](auto tc_) {
    constexpr int tap = decltype(tc_)::value;
    float* dst = a.part + (((size_t)split * NT + tap) * Cout + co0 + wave * 32) * Cin + ci0 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(size_t)((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * Cin] = acc[tap][r];
  });
#endif
}

// The bf16 training tape (train.hip): input and dy stored as bf16 [pixel][C].  bf16 mode, two workgroups
// per CU as OCC 3, but the dy tile needs no conversion: wave w lands its own operand plane [px][32 Cout]
// (64-B rows) straight from the bf16 tensor by LDS-DMA (8 instructions of 16 pixels x 64 B), into a
// double buffer, so tile t+1's dy lands under tile t's MFMAs; the input patch travels as 16-B units of
// 8 channels (half the bytes of the fp32 patch) through registers for the prologue.  The bias gradient
// sums each wave's own plane back from LDS (bf16 values, float sums).
template <int TC, int KS>
__global__ __launch_bounds__(256, 2) void conv_wgrad_h16_kernel(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  using T = WgTile<TC, KS>;
  constexpr int NT = KS * KS;
  constexpr int NUA = (T::NPIX * 4 + 255) / 256;        // 16-B input units (8 bf16 channels) per thread
  static_assert(2 * (2 * T::DY_PLANE + T::A_PLANE) <= 160 * 1024, "two workgroups per CU");
  static_assert(TC % 16 == 0, "a 16-pixel dy group inside one tile row");
  __shared__ __attribute__((aligned(16))) char lds[2 * T::DY_PLANE + T::A_PLANE];
  char* const aL = lds + 2 * T::DY_PLANE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto tidx = [&]() __attribute__((always_inline)) {   // an opaque copy: thread-derived values recomputed per use
    int t = tid;
    asm volatile("" : "+v"(t));
    return t;
  };
  const int d = a.dil, Hs = a.H / d, Ws = a.W / d;
  const int tiles_c = Ws / TC, tiles_rc = (Hs / T::TR) * tiles_c, tiles_img = tiles_rc * d * d;
  const int total = a.B * tiles_img;
  const int ncb = (a.Cin / 32) * (a.Cout / 128), G = gridDim.x;   // as conv_wgrad_kernel: channel blocks per XCD
  const int q = (G & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (G >> 3) + ((int)blockIdx.x >> 3);
  const int S = G / ncb;
  const int cb = q % ncb, cib = cb % (a.Cin / 32), cob = cb / (a.Cin / 32);
  const int split = q / ncb;
  const int t_begin = (int)((long long)total * split / S), t_end = (int)((long long)total * (split + 1) / S);
  const int ci0 = cib * 32, co0 = cob * 128;
  const int Cin = a.Cin, Cout = a.Cout;
  const __bf16* in16 = reinterpret_cast<const __bf16*>(a.in);
  const __bf16* dy16 = reinterpret_cast<const __bf16*>(a.dy);
  const uint32_t img_dy_bytes = (uint32_t)a.H * a.W * Cout * 2, img_in_bytes = (uint32_t)a.H * a.W * Cin * 2;

  f32x16 acc[NT];
  static_for<0, NT>([&](auto i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  });
  int tb = 0, tph_r = 0, tph_c = 0, tsr0 = 0, tsc0 = 0;
  auto decode = [&](int t) {
    tb = t / tiles_img;
    int r = t - tb * tiles_img;
    const int ph = r / tiles_rc;
    r -= ph * tiles_rc;
    tph_r = ph / d;
    tph_c = ph - tph_r * d;
    tsr0 = (r / tiles_c) * T::TR;
    tsc0 = (r % tiles_c) * TC;
  };
  // dy tile of the decoded tile -> plane buffer `buf`: wave w lands Cout [co0 + 32w, +32) of the 128 pixels
  auto dma_dy = [&](int buf) __attribute__((always_inline)) {
    const int tl = tidx(), l = tl & 63, w = tl >> 6;
    const int voff = ((((l >> 2) * d) * Cout) + 32 * w + (l & 3) * 8) * 2;
    const i32x4 rs = buffer_desc(dy16 + (size_t)tb * a.H * a.W * Cout, img_dy_bytes);
    const int base = (((tsr0 * d + tph_r) * a.W + tsc0 * d + tph_c) * Cout + co0) * 2;
    const uint32_t l0 = (uint32_t)(uintptr_t)(lds + buf * T::DY_PLANE) + (uint32_t)__builtin_amdgcn_readfirstlane(w) * 8192u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int px0 = 16 * j, row = px0 / TC, col = px0 % TC;
      dma16_lds_opaque(rs, l0 + j * 1024, voff, base + ((row * d) * a.W + col * d) * Cout * 2);
    }
  };
  // input patch of the decoded tile -> registers (16 B = 8 channels per unit) + the prologue's (scale, shift)
  uint4 ra[NUA];
  float4 ssv[4];
  bool interior = false;
  auto load_a = [&]() __attribute__((always_inline)) {
    const int tl = tidx();
    if (a.pro_mode != PRO_NONE) {
      const float* ssb = a.pro_ss + (size_t)tb * a.ss_bstride + (ci0 + (tl & 3) * 8) * 2;
#pragma unroll
      for (int k = 0; k < 4; ++k) ssv[k] = *reinterpret_cast<const float4*>(ssb + 4 * k);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) ssv[k] = make_float4(1.f, 0.f, 1.f, 0.f);
    }
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(in16 + (size_t)tb * a.H * a.W * Cin), 0, img_in_bytes, 0x00020000);
    interior = tsr0 >= T::HALO && tsr0 + T::TR + T::HALO <= Hs && tsc0 >= T::HALO && tsc0 + TC + T::HALO <= Ws;
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    if (interior) {
      const int ibase = __builtin_amdgcn_readfirstlane(
          ((((tsr0 - T::HALO) * d + tph_r) * a.W + (tsc0 - T::HALO) * d + tph_c) * Cin + ci0) * 2);
#pragma unroll
      for (int k = 0; k < NUA; ++k) {
        int u = tl + k * 256;
        u = u < T::NPIX * 4 ? u : 0;
        const int pix = u >> 2, cv = u & 3;
        const int vo = (((pix / T::PC) * d * a.W + (pix % T::PC) * d) * Cin + cv * 8) * 2;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(irs, vo, ibase, 0);
        ra[k] = make_uint4(v.x, v.y, v.z, v.w);
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < NUA; ++k) {
      int u = tl + k * 256;
      u = u < T::NPIX * 4 ? u : 0;
      const int pix = u >> 2, cv = u & 3;
      int sr = tsr0 - T::HALO + pix / T::PC, sc = tsc0 - T::HALO + pix % T::PC;
      if (a.circular) {
        sr = sr < 0 ? sr + Hs : (sr >= Hs ? sr - Hs : sr);
        sc = sc < 0 ? sc + Ws : (sc >= Ws ? sc - Ws : sc);
      } else {
        sr = min(max(sr, 0), Hs - 1);
        sc = min(max(sc, 0), Ws - 1);
      }
      const int y = sr * d + tph_r, x = sc * d + tph_c;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(irs, ((y * a.W + x) * Cin + ci0 + cv * 8) * 2, 0, 0);
      ra[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // registers -> aL [px][32 ci] bf16: prologue (IN++ affine + ELU, ELU), zero padding
  auto store_a = [&]() __attribute__((always_inline)) {
    const int tl = tidx();
#pragma unroll
    for (int k = 0; k < NUA; ++k) {
      const int u = tl + k * 256;
      if (u >= T::NPIX * 4) break;
      const int pix = u >> 2, cv = u & 3;
      const float4 lo = bf4_to_f4(make_uint2(ra[k].x, ra[k].y)), hi = bf4_to_f4(make_uint2(ra[k].z, ra[k].w));
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      if (a.pro_mode != PRO_NONE) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float4 sv = ssv[e >> 1];
          v[e] = elu(fmaf(v[e], (e & 1) ? sv.z : sv.x, (e & 1) ? sv.w : sv.y));
        }
      }
      if (!a.circular && KS == 3) {
        const int sr = tsr0 - 1 + pix / T::PC, sc = tsc0 - 1 + pix % T::PC;
        if (sr < 0 || sr >= Hs || sc < 0 || sc >= Ws) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
      }
      *reinterpret_cast<uint4*>(aL + pix * 64 + cv * 16) =
          make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
    }
  };
  // bias gradient: this lane's 8 channels ((lane & 3) * 8 of the wave's 32) summed over its pixels
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bpart && cib == 0;
  auto bias_sum = [&](int buf) __attribute__((always_inline)) {
    const char* p = lds + buf * T::DY_PLANE + wave * 8192 + lane * 16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 u = *reinterpret_cast<const uint4*>(p + j * 1024);
      const float4 lo = bf4_to_f4(make_uint2(u.x, u.y)), hi = bf4_to_f4(make_uint2(u.z, u.w));
      bs[0] += lo.x; bs[1] += lo.y; bs[2] += lo.z; bs[3] += lo.w;
      bs[4] += hi.x; bs[5] += hi.y; bs[6] += hi.z; bs[7] += hi.w;
    }
  };
  // the MFMAs of the staged tile (as conv_wgrad_kernel, bf16 mode)
  auto compute = [&](const char* dyb) __attribute__((always_inline)) {
    const int tl = tidx(), ln = tl & 63;
    const int Gq = ln >> 4, qq = (ln & 15) >> 2, p = ln & 3;
    const int kq = 8 * (Gq >> 1) + qq;
    const int mcol = 16 * (Gq & 1) + 4 * p;
    const char* dy_rd = dyb + __builtin_amdgcn_readfirstlane(tl >> 6) * (128 * 64) + mcol * 2;
    const char* a_rd = aL + mcol * 2;
#pragma unroll 1
    for (int s = 0; s < 8; ++s) {
      const int k0 = 16 * s + kq, k1 = k0 + 4;
      const bf16x8 ahi = cat8(ds_read_tr(dy_rd + k0 * 64), ds_read_tr(dy_rd + k1 * 64));
      const int p0 = (k0 / TC) * T::PC + k0 % TC, p1 = (k1 / TC) * T::PC + k1 % TC;
      const char* b0 = a_rd + p0 * 64;
      const char* b1 = a_rd + p1 * 64;
      auto rd_b = [&](int toff) { return cat8(ds_read_tr(b0 + toff), ds_read_tr(b1 + toff)); };
      bf16x8 bhi_n = rd_b(0);
      static_for<0, NT>([&](auto tc_) {
        constexpr int tap = decltype(tc_)::value;
        const bf16x8 bhi = bhi_n;
        if constexpr (tap + 1 < NT) {
          constexpr int toff = (KS == 3 ? ((tap + 1) / 3) * T::PC + (tap + 1) % 3 : 0) * 64;
          bhi_n = rd_b(toff);
        }
        acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bhi, acc[tap], 0, 0, 0);
      });
    }
  };
  // tile t+1's dy (LDS-DMA into the other plane buffer) and input patch (registers) are both issued
  // before tile t's MFMAs, so a tile's only exposed wait is the one at the top of its iteration
  int buf = 0;
  if (t_begin < t_end) {
    decode(t_begin);
    dma_dy(0);
    load_a();
  }
  for (int t = t_begin; t < t_end; ++t) {
    __builtin_amdgcn_s_waitcnt(0x0070);                  // vmcnt(0) + lgkmcnt(0): dy landed, patch in registers
    store_a();
    if (do_bias) bias_sum(buf);                          // this wave's own plane (its own DMA, waited above)
    __syncthreads();                                     // aL complete
    if (t + 1 < t_end) {
      decode(t + 1);
      dma_dy(buf ^ 1);                                   // lands under this tile's MFMAs
      load_a();                                          // in flight under them too
    }
    compute(lds + buf * T::DY_PLANE);
    __syncthreads();                                     // aL and this plane buffer read before they are rewritten
    buf ^= 1;
  }
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = bs[e];
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      bs[e] = v;
    }
    if (lane < 4) {
      float* bp = a.bpart + (size_t)split * Cout + co0 + wave * 32 + lane * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) bp[e] = bs[e];
    }
  }
  static_for<0, NT>([&](auto tc_) {
    constexpr int tap = decltype(tc_)::value;
    float* dst = a.part + (((size_t)split * NT + tap) * Cout + co0 + wave * 32) * Cin + ci0 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(size_t)((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * Cin] = acc[tap][r];
  });
#endif
}

// out[co][ci][tap] (+)= sum_s part[s][tap][co][ci] (fixed order over s); grid.y = tap, and
// grid.y == NT reduces the bias partials bpart[s][co] into bias_out
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                const float* __restrict__ bpart, float* __restrict__ out,
                                                                float* __restrict__ bias_out, int S, int NT, int Cout,
                                                                int Cin, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // co * Cin + ci
  const int tap = blockIdx.y;
  if (tap == NT) {
    if (!bpart || i >= Cout) return;
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += bpart[(size_t)k * Cout + i];
    bias_out[i] = accumulate ? bias_out[i] + s : s;
    return;
  }
  if (i >= Cout * Cin) return;
  const size_t plane = (size_t)Cout * Cin, step = (size_t)NT * plane;
  const float* p = part + (size_t)tap * plane + i;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 4 <= S; k += 4) {
    s0 += p[(size_t)k * step];
    s1 += p[(size_t)(k + 1) * step];
    s2 += p[(size_t)(k + 2) * step];
    s3 += p[(size_t)(k + 3) * step];
  }
  for (; k < S; ++k) s0 += p[(size_t)k * step];
  const float s = (s0 + s1) + (s2 + s3);
  float* o = out + (size_t)i * NT + tap;
  *o = accumulate ? *o + s : s;
}

int wgrad_splits(int B, int H, int W, int d, int Cin, int Cout, int ks) {
  const int tc = ((W / d) % 64 == 0) ? 64 : 32;
  const int total = B * (H / d) * (W / d) / 128 * d * d;
  (void)tc;
  const int blocks = (Cin / 32) * (Cout / 128);
  int S = (WGRAD_TARGET_BLOCKS + blocks - 1) / blocks;
  S = S < total ? S : total;
  return S < 1 ? 1 : S;
}

size_t wgrad_part_floats(int S, int Cin, int Cout, int ks) { return (size_t)S * ks * ks * Cin * Cout; }

// tc: the tile width of the 3x3 launches (64 -> 2 x 64 tiles, 32 -> 4 x 32).  OCC 3 has no 2 x 64
// instantiation (its double-buffered dy tile does not fit twice per CU), so it runs 4 x 32 tiles
// whatever tc says -- wgrad_mode passes 32 for it.
template <int MODE, int OCC>
static hipError_t wgrad_occ(const WgradArgs& a, int ks, int tc, dim3 grid, hipStream_t st) {
  static_assert(OCC >= 1 && OCC <= 3, "wgrad: OCC 1, 2 or 3");
  if (ks == 1) hipLaunchKernelGGL((conv_wgrad_kernel<MODE, 64, 1, OCC>), grid, dim3(256), 0, st, a);
  else if constexpr (OCC != 3) {
    if (tc == 64) hipLaunchKernelGGL((conv_wgrad_kernel<MODE, 64, 3, OCC>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<MODE, 32, 3, OCC>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_wgrad_kernel<MODE, 32, 3, OCC>), grid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

// bf16: the dy tile by LDS-DMA (OCC 3) wherever its LDS fits twice per CU -- the 1x1 tiles and the
// 4 x 32 tiles of the 3x3 convs (the 2 x 64 tiles' 66 x 4 patch does not: 161 KB); SDP_WGRAD_OCC3=0
// (build-time A/B only) restores the chunked register staging (bf16 training step 151.0-151.4 against
// 152.0-152.5 image-steps/s with OCC 3, profiles/experiments/r05_wgrad_occ_ab.log, which also holds the
// rejected stagings: the whole next tile by LDS-DMA on one workgroup per CU, 303 against 195 us per
// launch, and part of the input patch prefetched in registers under the MFMAs, 214 against 200 us)
#ifndef SDP_WGRAD_OCC3
#define SDP_WGRAD_OCC3 1
#endif

template <int MODE>
static hipError_t wgrad_mode(const WgradArgs& a, int ks, int tc, int S, hipStream_t st) {
  dim3 grid(S * (a.Cin / 32) * (a.Cout / 128));
  if constexpr (MODE == MODE_BF16) {
    if (SDP_WGRAD_OCC3) {   // OCC 3 always runs 4 x 32 tiles for the 3x3 convs (the caller's tc is not used)
      const int Ws = a.W / a.dil, Hs = a.H / a.dil;
      if (ks == 1) return wgrad_occ<MODE, 3>(a, ks, tc, grid, st);
      if (Ws % 32 == 0 && Hs % 4 == 0) return wgrad_occ<MODE, 3>(a, ks, 32, grid, st);
    }
    return wgrad_occ<MODE, 2>(a, ks, tc, grid, st);
  }
  return wgrad_occ<MODE, 1>(a, ks, tc, grid, st);
}

hipError_t conv_wgrad(int mode, WgradArgs a, int ks, float* out, float* bias_out, int accumulate, hipStream_t st,
                      const char** why, bool h16) {
  const int d = a.dil;
  if (a.Cin % 32 || a.Cout % 128) { *why = "wgrad: Cin%32 and Cout%128 required"; return hipErrorInvalidValue; }
  if (a.H % d || a.W % d) { *why = "wgrad: H,W must be multiples of the dilation"; return hipErrorInvalidValue; }
  const int Ws = a.W / d, Hs = a.H / d;
  const int tc = (Ws % 64 == 0) ? 64 : 32;
  if (ks == 1 && (d != 1 || Ws % 64 || Hs % 2)) { *why = "wgrad: 1x1 needs d=1 and W%64"; return hipErrorInvalidValue; }
  if (Ws % tc || Hs % (128 / tc)) { *why = "wgrad: sub-grid not divisible by the pixel tile"; return hipErrorInvalidValue; }
  if (!a.circular && d != 1) { *why = "wgrad: zero padding only for d=1"; return hipErrorInvalidValue; }
  if (!a.pro_ss) { *why = "wgrad: prologue table missing"; return hipErrorInvalidValue; }
  const int S = wgrad_splits(a.B, a.H, a.W, d, a.Cin, a.Cout, ks);
  if (bias_out && !a.bpart) { *why = "wgrad: bias gradient needs bpart"; return hipErrorInvalidValue; }
  if (!bias_out) a.bpart = nullptr;
  if (!a.part || a.part_floats < wgrad_part_floats(S, a.Cin, a.Cout, ks)) {
    *why = "wgrad: partial buffer too small";
    return hipErrorInvalidValue;
  }
  hipError_t e;
  if (h16) {   // the bf16 tape: 4 x 32 tiles (3x3) or 2 x 64 (1x1)
    if (mode != MODE_BF16) { *why = "wgrad: the bf16 tape runs in bf16 mode"; return hipErrorInvalidValue; }
    const dim3 grid(S * (a.Cin / 32) * (a.Cout / 128));
    if (ks == 1) hipLaunchKernelGGL((conv_wgrad_h16_kernel<64, 1>), grid, dim3(256), 0, st, a);
    else if (Ws % 32 == 0 && Hs % 4 == 0) hipLaunchKernelGGL((conv_wgrad_h16_kernel<32, 3>), grid, dim3(256), 0, st, a);
    else { *why = "wgrad: the bf16 tape needs 4 x 32 tiles"; return hipErrorInvalidValue; }
    e = hipGetLastError();
  } else switch (mode) {
    case MODE_F32X3: e = wgrad_mode<MODE_F32X3>(a, ks, tc, S, st); break;
    case MODE_BF16: e = wgrad_mode<MODE_BF16>(a, ks, tc, S, st); break;
    default: *why = "wgrad: training runs in fp32x3 or bf16"; return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  const int n = a.Cout * a.Cin;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((n + 255) / 256, ks * ks + 1), dim3(256), 0, st, a.part, a.bpart,
                     out, bias_out, S, ks * ks, a.Cout, a.Cin, accumulate);
  return hipGetLastError();
}

}  // namespace sdp
