// Shared device helpers and launch-argument structs for libsdp (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#define SDP_DEV __device__ __forceinline__

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace sdp {

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E) -- keeps register
// arrays indexed by literals (runtime-indexed arrays are placed in scratch by hipcc)
template <int B, int E, class F>
SDP_DEV void static_for(F&& f) {  // SDP_DEV = __forceinline__
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

enum { MODE_F32 = 0, MODE_F32X3 = 1, MODE_BF16 = 2 };
enum { PRO_NONE = 0, PRO_ELU = 1, PRO_AFFINE_ELU = 2 };

// nn.ELU(alpha=1) (LiDARGen/models/layers.py:11-13)
// LDS-DMA of 16 B per lane (lane i lands at lds_byte + 16 i) issued as inline asm, so the compiler
// does not see it as an LDS write: it inserts no wait for it before later LDS reads (through one
// shared array it cannot tell the ring slots apart and would wait for every DMA in flight).  The
// caller waits for it with an explicit s_waitcnt vmcnt.  rsrc: a wave-uniform buffer descriptor
// (words: base lo, base hi, num_records, 0x00020000).
typedef __attribute__((ext_vector_type(4))) int i32x4;
SDP_DEV i32x4 buffer_desc(const void* base, uint32_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  return i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)p), __builtin_amdgcn_readfirstlane((int)((p >> 32) & 0xffff)),
               __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
SDP_DEV void dma16_lds_opaque(i32x4 rsrc, uint32_t lds_byte, int voff, int soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane((int)lds_byte)), "v"(voff), "s"(rsrc),
                 "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory");   // m0 is reserved (not a clobber): nothing else in these kernels uses it
}

// ---- element access of activation tensors stored as float32 or, in the bf16 training tape
// (train.hip), as bf16: 4 consecutive elements (i a multiple of 4) or one, always widened to float
SDP_DEV float4 ldg4(const float* p, size_t i) { return *reinterpret_cast<const float4*>(p + i); }
SDP_DEV float4 bf4_to_f4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
SDP_DEV float4 ldg4(const __bf16* p, size_t i) { return bf4_to_f4(*reinterpret_cast<const uint2*>(p + i)); }
SDP_DEV uint32_t pack_bf2(float a, float b) {   // round-to-nearest-even, a in the low half
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
SDP_DEV uint2 f4_to_bf4(float4 v) { return make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)); }
SDP_DEV void stg4(float* p, size_t i, float4 v) { *reinterpret_cast<float4*>(p + i) = v; }
SDP_DEV void stg4(__bf16* p, size_t i, float4 v) { *reinterpret_cast<uint2*>(p + i) = f4_to_bf4(v); }
SDP_DEV float ldg1(const float* p, size_t i) { return p[i]; }
SDP_DEV float ldg1(const __bf16* p, size_t i) { return (float)p[i]; }

SDP_DEV float elu(float x) { return x > 0.f ? x : (__expf(x) - 1.0f); }
// the same values without a compare/select (e^x - 1 >= x, and e^min(x,0) - 1 = 0 for x > 0):
// no VCC round trip, so it schedules freely between MFMAs
SDP_DEV float elu_max(float x) { return fmaxf(x, __expf(fminf(x, 0.f)) - 1.0f); }
// d ELU / d h, from the pre-activation h (form 1, 3) or from the output y = ELU(h) (form 2)
SDP_DEV float elu_grad(float t, int form) {
  if (form == 2) return t > 0.f ? 1.f : t + 1.f;
  return t > 0.f ? 1.f : __expf(t);
}

// Arguments of one implicit-GEMM 3x3 / 1x1 convolution launch (activations NHWC float32).
struct ConvArgs {
  const float* in;         // [B][H][W][Cin]
  const uint4* wf;         // 32x32 fragment-ordered weights (train_aux.hip pack_slot): the exact-fp32 forward "#frag"
  const uint4* wf16;       // weights in 16x16 fragment order (train_aux.hip pack_slot16): the bf16-mode forward
                           //   "#frag16" and the data gradient "#dfrag16"
  const float* bias;       // [Cout] or null
  float* out;              // [B][Ho][Wo][Cout]  (Ho,Wo = H,W or H/2,W/2 when pooled)
  const float* res;        // residual, layout of out, or null
  float* out2;             // optional second output: value + res2 (CRP running sum)
  const float* res2;
  const float* up;         // [B][H/2][W/2][Cout]: bilinear(align_corners) upsample-add, or null
  const float* pro_ss;     // [B][Cin][2] (scale, shift) of the prologue: InstanceNorm++ affine, or the
                           // identity (1, 0) table with ss_bstride = 0
  int ss_bstride;          // floats between the rows of consecutive images
  float* stats;            // [B][groups_per_img][Cout][2] per-128-pixel (mean, M2) or null
  int B, H, W, Cin, Cout;
  int dil, circular, pro_mode, epi_elu;
  int tiles_per_img;       // workgroup tiles per image (set by the launcher)
  int strip_w;             // tile order inside a phase sub-grid: 0 = row-major, else strips of strip_w tile
                           //   columns x all tile rows (set by the launcher, conv_strip_w)
  int groups_per_img;      // 128-pixel statistics groups per image (H*W/128)
  int cpair;               // 1: grid.x deals (tile, Cout block) pairs, the block in bit 0 of the XCD-ordered index
                           //   (both Cout halves of a tile on one XCD, back to back: the second patch read
                           //   hits its L2); 0: Cout block = blockIdx.y (set by the launcher)
  unsigned long long* dbg; // diagnostics builds only (SDP_TIMING): per-workgroup phase clocks
  // backward epilogue (data gradient): out *= elu'(...) of `aux` (layout of out) before +res;
  // dact 0 = off, 1 = aux is the pre-activation, 2 = aux is the ELU output, 3 = aux is the
  // InstanceNorm++ input and epi_ss [B][Cout][2] its (scale, shift)
  const float* aux;
  const float* epi_ss;
  int dact;
  // 1: every activation tensor of the launch (in, out, res, res2, out2, up, aux) holds bf16 elements
  // (the bf16 training tape, train.hip; bf16 mode); the launchers pick the IO16 instantiation
  int io16;
};

// Arguments of one weight-gradient launch (wgrad.hip).
struct WgradArgs {
  const float* in;         // forward input [B][H][W][Cin] (before the prologue)
  const float* pro_ss;     // prologue (scale, shift) table, as ConvArgs
  int ss_bstride;
  int pro_mode;            // PRO_NONE / PRO_ELU / PRO_AFFINE_ELU
  const float* dy;         // gradient of the conv output (before any pooling) [B][H][W][Cout]
  float* part;             // split partials [S][k*k][Cout][Cin]
  size_t part_floats;
  float* bpart;            // bias-gradient partials [S][Cout] (S <= 1024) or null
  int B, H, W, Cin, Cout, dil, circular;
};

// Tile order of the implicit-GEMM convs: every XCD runs a contiguous range of tiles (the kernels'
// XCD-aware blockIdx mapping), ~32 at a time (one per CU).  Ordering the tiles of a phase sub-grid in
// strips of strip_w tile columns x all R tile rows, with R * strip_w ~ 32, makes the tiles that run
// together on an XCD a full-height block: their halos (and the circular wrap of the top and bottom
// rows) are each other's pixels, read once into that XCD's L2, instead of re-read by the next
// round's row of tiles: 256 -> 256 @32x512 reads 125 -> 108 MB per launch (HBM traffic 1.40 -> 1.25x
// the algorithmic bytes), time unchanged (profiles/experiments/r03_strip_ab.log).
inline int conv_strip_w(int tile_rows, int tile_cols) {
  int sw = 1;
  while (sw * 2 * tile_rows <= 32 && tile_cols % (sw * 2) == 0) sw *= 2;
  return sw;
}

}  // namespace sdp
