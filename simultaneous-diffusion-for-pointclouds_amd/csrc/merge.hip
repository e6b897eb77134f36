// Cross-view reprojection / consistency merge (gfx950).
//
// Restates KITTISampling.py:160-490 (pose matrices) and models/__init__.py:263-579 (origin
// offsets) without the reference's per-view argsort / stable sorts / unique_consecutive /
// sparse->dense: every (output view, source point) pair of a megabatch is projected once
// (float64, as the reference's numpy-derived angles promote) and scattered with atomics
// into a [114 x W] "big" grid per output view:
//     cnt (u32), sum of log-depth codes (f64), sum of intensities (f64),
//     nearest code (u64 atomicMin on the f64 bits; codes are >= 0 so the order is the
//     unsigned order), then the lowest source index among the nearest (second pass).
// The accumulation bins the pairs by destination row so each cell is summed in LDS and
// written once (global atomics run at the memory side, ≈10 G/s for scattered lanes).
// A resolve pass turns a cell into the reference's controlled average (mean depth unless
// it exceeds the nearest depth + allowance), applies the negative-depth flip/roll and crop
// to the output view, and an apply pass adds cc * (-mask*(x - new)) on unknown pixels
// unless tooHigh.  Tie rule: equal nearest codes keep the lowest source index (the
// reference's unstable argsort leaves it unspecified).
#include <mutex>
#include "merge.h"

// reference evaluation order: no FMA contraction in this file (HIP __fmul_rn is a plain `*`)
#pragma clang fp contract(off)

namespace sdp {

// ---------------------------------------------------------------- K0: prep
// One launch: the output views' grids reset (counts and sums 0, nearest code and index all-ones), the
// snapshot of the sources' intensities that the fused resolve+apply pass reads while it corrects x in place,
// and the (cos, sin) table of the W column azimuths and H row elevations (KITTISampling.py:101-102,
// float64) that the count pass's world points use.  (Until round 6 this kernel also wrote every source's
// float64 world point, 32 B each, which the count pass read back: the count pass now computes them itself,
// once per source point -- profiles/experiments/r06_merge_fused_world_ab.log.)
constexpr int MERGE_PREP_WG = 1024;
__global__ __launch_bounds__(256) void merge_prep_kernel(MergeArgs a) {
  const int H = a.g.H, W = a.g.W, HW = H * W;
  const size_t n = (size_t)a.n_src * HW;
  const size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  if (i0 < (size_t)W) {
    const double az = (double)(W - 1 - (int)i0) * a.g.hA + a.g.hMin;
    a.trig[i0] = make_double2(cos(az), sin(az));
  } else if (i0 < (size_t)(W + H)) {
    const double el = (double)(H - 1 - (int)(i0 - W)) * a.g.vA + a.g.vMin;
    a.trig[i0] = make_double2(cos(el), sin(el));
  }
  const size_t ncell = (size_t)a.n_out * a.g.big * W;
  for (size_t c = i0; c < ncell; c += stride) {
    a.cnt[c] = 0u;
    a.sumL[c] = 0.0;
    a.sumI[c] = 0.0;
    a.minkey[c] = ~0ull;
    a.minidx[c] = ~0u;
  }
  for (size_t i = i0; i < n; i += stride) {
    const int v = i / HW, p = i % HW;
    a.isnap[i] = a.x[(size_t)v * 2 * HW + HW + p];
  }
}

// world point of source view v, pixel p (+ the source-valid flag in .w), from the prep kernel's trig table
__device__ __forceinline__ double4 world_point(const MergeArgs& a, int v, int p) {
  const int HW = a.g.H * a.g.W, W = a.g.W;
  const int r = p / W, c = p - r * W;
  const float x0 = a.x[(size_t)v * 2 * HW + p];
  // realDistance = (2^(|x|*6/smod) - 1) * (+-1), float32 (KITTISampling.py:164-166)
  const float e = __fdiv_rn(__fmul_rn(fabsf(x0), 6.0f), a.smod);
  float rd = __fsub_rn(exp2f(e), 1.0f);
  if (x0 < 0.f) rd = -rd;
  const double2 tz = a.trig[c], te = a.trig[W + r];
  const double cz = tz.x, sz = tz.y, ce = te.x, se = te.y;
  const double rdd = (double)rd;
  double px = __dmul_rn(__dmul_rn(rdd, cz), ce);
  double py = __dmul_rn(__dmul_rn(rdd, sz), ce);
  double pz = __dmul_rn(rdd, se);
  const int vl = v % a.aB;
  double flag = a.exist[(size_t)vl * HW + p] ? 1.0 : 0.0;
  double4 w;
  if (a.variant == 0) {
    const double* T = a.toWorld + (size_t)v * 16;
    w.x = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[0], px), __dmul_rn(T[1], py)), __dmul_rn(T[2], pz)), T[3]);
    w.y = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[4], px), __dmul_rn(T[5], py)), __dmul_rn(T[6], pz)), T[7]);
    w.z = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[8], px), __dmul_rn(T[9], py)), __dmul_rn(T[10], pz)), T[11]);
  } else {
    w.x = __dadd_rn(px, (double)a.origins[vl * 3 + 0]);
    w.y = __dadd_rn(py, (double)a.origins[vl * 3 + 1]);
    w.z = __dadd_rn(pz, (double)a.origins[vl * 3 + 2]);
    if (!a.sky[(size_t)v * HW + p]) flag = 0.0;   // source sky gate (models/__init__.py:356-359)
  }
  w.w = flag;
  return w;
}

struct Proj {
  int cell;     // -1 if not valid
  double code;  // log2(d+1)/6*smod
};

// project world point w into output view o (global index); K1 keeps the result for K3 (pcell, pcode)
// project() inlined into the count pass: merge 450 -> 398 us at a 32-view megabatch (one config-4
// rank), 170 -> 156 us at 4 views (profiles/experiments/r03_merge_inline_ab.log); 0 = a call
#ifndef SDP_MERGE_INLINE
#define SDP_MERGE_INLINE 1
#endif
#if SDP_MERGE_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
Proj project(const MergeArgs& a, double4 w, int o) {
  Proj pr;
  pr.cell = -1;
  pr.code = 0.0;
  double qx, qy, qz;
  if (a.variant == 0) {
    const double* F = a.fromWorld + (size_t)o * 16;
    qx = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[0], w.x), __dmul_rn(F[1], w.y)), __dmul_rn(F[2], w.z)), F[3]);
    qy = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[4], w.x), __dmul_rn(F[5], w.y)), __dmul_rn(F[6], w.z)), F[7]);
    qz = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(F[8], w.x), __dmul_rn(F[9], w.y)), __dmul_rn(F[10], w.z)), F[11]);
  } else {
    const int ol = o % a.aB;
    qx = __dsub_rn(w.x, (double)a.origins[ol * 3 + 0]);
    qy = __dsub_rn(w.y, (double)a.origins[ol * 3 + 1]);
    qz = __dsub_rn(w.z, (double)a.origins[ol * 3 + 2]);
  }
  const double xy = __dadd_rn(__dmul_rn(qx, qx), __dmul_rn(qy, qy));
  const double dist = sqrt(__dadd_rn(xy, __dmul_rn(qz, qz)));
  const double code = __dmul_rn(__ddiv_rn(log2(__dadd_rn(dist, 1.0)), 6.0), (double)a.smod);
  const double h = atan2(qy, qx);
  const double e = atan2(qz, sqrt(xy));
  const double fc = rint(__ddiv_rn(__dsub_rn(h, a.g.hMin), a.g.hA));
  const double fr = rint(__ddiv_rn(__dsub_rn(e, a.g.bigMin), a.g.vA));
  const int col = a.g.W - 1 - (int)fc;
  const int row = a.g.big - 1 - (int)fr;
  // a NaN bin (a NaN or infinite world point) fails the reference's range test (numpy comparisons with NaN
  // are false); (int) of NaN is 0 here, so it is excluded explicitly
  bool ok = w.w != 0.0 && fc == fc && fr == fr && col > -1 && col < a.g.W && row > -1 && row < a.g.big;
  // setting 5 (kitti) / always (AllForOne): min-depth filter code > log2(1.2)/6*smod
  if (a.variant == 1 || a.setting == 5) ok = ok && code > (double)a.min_code;
  if (ok) pr.cell = row * a.g.W + col;
  pr.code = code;
  return pr;
}

// ---------------------------------------------------------------- K1-K4: binned accumulation
// Global atomics execute at the memory side at one chip-wide rate (≈10 G/s for lanes that hit
// scattered addresses), and every pair needs four (count, two sums, nearest code): a 32-view
// megabatch spent 3.8 ms of an 18.8-ms step there.  Instead the pairs are binned by
// destination tile = (output view, big-grid row):
//   K1 bin_count  : each chunk (a range of source points x every output view) projects its points,
//                   counts them per tile (LDS) and keeps
//                   every pair's (cell, code) -- the float64 projection (two atan2, log2, sqrt)
//                   is the costly part of both binning passes;
//   scan          : exclusive offsets over [tile][chunk] (tile-major);
//   K3 bin_scatter: the chunks read the kept projections back and write one 16-B record per pair
//                   into their tile's range (LDS cursors);
//   K4 tile passes: workgroups take parts of <= MERGE_TSEG records of ONE tile, sum them per cell in
//                   LDS (ds atomics) and store (one-part tile) or add once per touched cell (larger
//                   tiles) to the grids; a second sweep finds the lowest source index among the
//                   nearest.  (One workgroup per whole tile was 5.9 ms: the horizon rows hold most
//                   records -- 8 % of a 32-view megabatch's records land in one row.)
// Tile passes: the records of one destination tile (output view, big row) are summed by workgroups that each
// own a part of at most MERGE_TSEG of that tile's records and nothing else; a tile of one part (most tiles)
// also finds its nearest indices and writes its row of cells with plain stores -- no global atomics.  They
// replace round 5's segment passes (4096 consecutive records per workgroup across tile boundaries, records of
// a third tile onward straight to global atomics): 32-view megabatch merge 360-363 -> 301-305 us, 4 views
// 113-115 -> 84-85 us (profiles/experiments/r06_merge_tile_ab.log).
#ifndef SDP_MERGE_TSEG      // records per part
#define SDP_MERGE_TSEG 2048
#endif
#ifndef SDP_MERGE_TNT       // threads per tile-pass workgroup
#define SDP_MERGE_TNT 256
#endif
constexpr uint32_t MERGE_TSEG = SDP_MERGE_TSEG;
constexpr int MERGE_TNT = SDP_MERGE_TNT;

__global__ __launch_bounds__(256) void merge_bin_count_kernel(MergeArgs a, size_t per_chunk) {
  extern __shared__ uint32_t hist[];
  const int HW = a.g.H * a.g.W, T = a.n_out * a.g.big;
  for (int t = threadIdx.x; t < T; t += 256) hist[t] = 0u;
  __syncthreads();
  // chunk = a range of source points, each projected into every output view in turn (the view loop is
  // wave-uniform, so the view's pose is a scalar load): a source's world point is computed once (since
  // the fused prep: from x and the trig table; before, read from a 32-B world array) and projected into
  // every view, not read once per output view (a config-4 rank read 268 MB of world points).  Count 126 -> 111 us and merge 289-291 -> 277-279
  // us at a 32-view megabatch, bit-identical (profiles/experiments/r06_merge_srcmajor_ab.log); round 5's
  // source-major numbering had put a different view in every lane (per-lane pose gathers) and was slower.
  const size_t per_out = (size_t)a.aB * HW;
  const size_t s0 = blockIdx.x * per_chunk, s1 = s0 + per_chunk < per_out ? s0 + per_chunk : per_out;
  for (size_t sp = s0 + threadIdx.x; sp < s1; sp += 256) {
    int m0p = -1;
    double4 wv = make_double4(0.0, 0.0, 0.0, 0.0);
    for (int ol = 0; ol < a.n_out; ++ol) {
      const int o = a.o_begin + ol, m0 = (o / a.aB) * a.aB;
      if (m0 != m0p) {
        const uint32_t s32 = (uint32_t)sp;   // < aB * HW < 2^22 (checked by the launcher)
        wv = world_point(a, m0 + (int)(s32 / (uint32_t)HW), (int)(s32 % (uint32_t)HW));
        m0p = m0;
      }
      const Proj pr = project(a, wv, o);
      const size_t ii = (size_t)ol * per_out + sp;
      a.pcell[ii] = pr.cell;
      if (pr.cell >= 0) {
        a.pcode[ii] = pr.code;
        atomicAdd(&hist[ol * a.g.big + pr.cell / a.g.W], 1u);
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += 256) a.tcount[(size_t)t * a.nchunk + blockIdx.x] = hist[t];
}

// The top level of the offset scan rides here (one launch less): every workgroup scans the nb block
// totals of merge_scan_block_kernel in LDS; workgroup 0 also publishes every tile's first record and
// the total (toff) and the part table (pstart) for the tile passes, which run after this launch.  The scan is redundant work:
// each of the nchunk workgroups reads all nb totals from L2 (nchunk * nb loads, at most 1024 x 8192) --
// cheaper than the launch it replaces at the measured sizes (4 views: 156 -> 110 us for the whole chain,
// a 32-view config-4 rank 401 -> 352 us; profiles/experiments/r05_merge_chain_ab.log).
__global__ __launch_bounds__(256) void merge_bin_scatter_kernel(MergeArgs a, size_t per_chunk, int nb) {
  extern __shared__ uint32_t cur[];                // [T] tile cursors, then [nb + 1] scanned block totals
  const int HW = a.g.H * a.g.W, T = a.n_out * a.g.big, tid = threadIdx.x;
  uint32_t* sb = cur + T;
  constexpr int SB = 2048;   // scan block (merge_scan_block_kernel)
  {
    __shared__ uint32_t part[256];
    const int per = (nb + 255) / 256, b0 = tid * per;
    uint32_t t = 0;
    for (int k = 0; k < per; ++k) t += b0 + k < nb ? a.bsum[b0 + k] : 0u;
    part[tid] = t;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const uint32_t y = tid >= off ? part[tid - off] : 0u;
      __syncthreads();
      part[tid] += y;
      __syncthreads();
    }
    uint32_t run = part[tid] - t;
    for (int k = 0; k < per; ++k)
      if (b0 + k < nb) {
        const uint32_t x = a.bsum[b0 + k];
        sb[b0 + k] = run;
        run += x;
      }
    if (tid == 255) sb[nb] = part[255];
    __syncthreads();
  }
  for (int t = tid; t < T; t += 256) {
    const size_t k = (size_t)t * a.nchunk + blockIdx.x;
    cur[t] = a.tcount[k] + sb[k / SB];
  }
  __syncthreads();
  if (blockIdx.x == 0) {   // chunk 0's cursors are the tiles' first records
    for (int t = tid; t < T; t += 256) a.toff[t] = cur[t];
    if (tid == 0) a.toff[T] = sb[nb];
    // the tile passes' part table: tile t is cut into max(1, ceil(n_t / MERGE_TSEG)) parts of consecutive
    // records; pstart = their exclusive scan (+ the part count at [T])
    __shared__ uint32_t ps[256];
    const int per = (T + 255) / 256, t0 = tid * per;
    auto parts = [&](int t) {
      const uint32_t n = (t + 1 < T ? cur[t + 1] : sb[nb]) - cur[t];
      return n == 0u ? 1u : (n + MERGE_TSEG - 1) / MERGE_TSEG;
    };
    uint32_t loc = 0;
    for (int k = 0; k < per; ++k) loc += t0 + k < T ? parts(t0 + k) : 0u;
    ps[tid] = loc;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const uint32_t y = tid >= off ? ps[tid - off] : 0u;
      __syncthreads();
      ps[tid] += y;
      __syncthreads();
    }
    uint32_t run = ps[tid] - loc;
    for (int k = 0; k < per; ++k)
      if (t0 + k < T) {
        a.pstart[t0 + k] = run;
        run += parts(t0 + k);
      }
    if (tid == 255) a.pstart[T] = ps[255];
  }
  __syncthreads();
  const size_t per_out = (size_t)a.aB * HW;
  const size_t s0 = blockIdx.x * per_chunk, s1 = s0 + per_chunk < per_out ? s0 + per_chunk : per_out;
  for (int olc = 0; olc < a.n_out; ++olc)           // view by view: consecutive lanes, consecutive pairs
  for (size_t i = (size_t)olc * per_out + s0 + tid; i < (size_t)olc * per_out + s1; i += 256) {
    const int cell = a.pcell[i];
    if (cell < 0) continue;
    const int ol = olc, s = (int)(i - (size_t)olc * per_out), o = a.o_begin + ol, m0 = (o / a.aB) * a.aB;
    Proj pr;
    pr.cell = cell;
    pr.code = a.pcode[i];
    const int row = pr.cell / a.g.W, col = pr.cell % a.g.W;
    const uint32_t pos = atomicAdd(&cur[ol * a.g.big + row], 1u);
    const float inten = a.x[((size_t)m0 * 2 + 1) * HW + (size_t)(s / HW) * 2 * HW + (s % HW)];
    const unsigned long long cb = (unsigned long long)__double_as_longlong(pr.code);
    a.rec[pos] = make_float4(__uint_as_float((uint32_t)cb), __uint_as_float((uint32_t)(cb >> 32)), inten,
                             __uint_as_float(((uint32_t)s << 10) | (uint32_t)col));
  }
}

// exclusive scan of v[0..n) in blocks of 2048 (block totals -> bsum; their scan is done by the
// consumer, merge_bin_scatter_kernel); consumers add the scanned bsum[k / 2048] to v[k]
__global__ __launch_bounds__(256) void merge_scan_block_kernel(uint32_t* __restrict__ v, size_t n,
                                                               uint32_t* __restrict__ bsum) {
  __shared__ uint32_t sh[256];
  const int tid = threadIdx.x;
  const size_t base = blockIdx.x * 2048ull + tid * 8;
  uint32_t x[8], t = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x[k] = base + k < n ? v[base + k] : 0u;
    t += x[k];
  }
  sh[tid] = t;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const uint32_t y = tid >= off ? sh[tid - off] : 0u;
    __syncthreads();
    sh[tid] += y;
    __syncthreads();
  }
  uint32_t run = sh[tid] - t;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (base + k < n) v[base + k] = run;
    run += x[k];
  }
  if (tid == 255) bsum[blockIdx.x] = sh[255];
}

// K4 (tile passes): workgroup = part k of tile t (pstart table, written by merge_bin_scatter_kernel).  The
// 1024 threads sum the part's records per cell in LDS (count, two float64 sums, nearest code).  A tile of one
// part then sweeps its records again for the lowest source index among the nearest and stores its whole row
// of cells (the grid reset of merge_world_kernel is overwritten); a part of a larger tile adds its touched
// cells to the grids with atomics, and merge_tile_minidx_kernel finds those tiles' nearest indices.
__device__ __forceinline__ int part_tile(const uint32_t* sps, uint32_t p, int T) {   // largest t: sps[t] <= p
  int lo = 0, hi = T - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sps[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ void rec_fields(const float4 r, unsigned long long& cb, uint32_t& w) {
  cb = (unsigned long long)__float_as_uint(r.x) | ((unsigned long long)__float_as_uint(r.y) << 32);
  w = __float_as_uint(r.w);
}
// Each thread takes a contiguous run of the part's records (not lane-interleaved ones): consecutive records are
// consecutive source pixels, which mostly land in the same cell (in the 32-view bench megabatch 64 consecutive
// records of the largest tile hit one cell 23 times on average), so the thread sums a run of equal cells in
// registers and issues the LDS atomics once per run -- lane-interleaved records made those atomics collide.
// With few sources per megabatch (the 4-view line) the collisions are rarer and lane-interleaved (coalesced)
// records measured faster: RUNS = false walks the part with a stride of the workgroup (every record then
// closes its own run).  Merge at 4 views 80 vs 93 us, at a 32-view megabatch 300 vs 343 us for runs
// (profiles/experiments/r06_merge_tile_ab.log); the launcher picks RUNS for aB >= 16 sources.
template <bool RUNS, typename F>
__device__ __forceinline__ void for_runs(const MergeArgs& a, uint32_t r0, uint32_t r1, F&& f) {
  constexpr int U = 4;                              // records in flight per thread
  if constexpr (RUNS) {
    const uint32_t per = (r1 - r0 + MERGE_TNT - 1) / MERGE_TNT;
    const uint32_t b0 = r0 + threadIdx.x * per, b1 = min(r1, b0 + per);
    for (uint32_t j = b0; j < b1; j += U) {
      float4 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = a.rec[min(j + u, b1 - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u < b1) f(r[u]);
    }
  } else {
    for (uint32_t j = r0 + threadIdx.x; j < r1; j += MERGE_TNT * U) {
      float4 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = a.rec[min(j + MERGE_TNT * u, r1 - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + MERGE_TNT * u < r1) f(r[u]);
    }
  }
}
template <bool RUNS>
__global__ __launch_bounds__(MERGE_TNT) void merge_tile_sum_kernel(MergeArgs a) {
  __shared__ uint32_t scnt[1024], sidx[1024];
  __shared__ double ssl[1024], ssi[1024];
  __shared__ unsigned long long smk[1024];
  extern __shared__ uint32_t sps[];
  const int tid = threadIdx.x, W = a.g.W, T = a.n_out * a.g.big;
  if (blockIdx.x >= a.pstart[T]) return;           // the grid is an upper bound of the part count
  for (int t = tid; t <= T; t += MERGE_TNT) sps[t] = a.pstart[t];
  for (int c = tid; c < W; c += MERGE_TNT) {
    scnt[c] = 0u;
    ssl[c] = 0.0;
    ssi[c] = 0.0;
    smk[c] = ~0ull;
    sidx[c] = ~0u;
  }
  __syncthreads();
  const int t = part_tile(sps, blockIdx.x, T);
  const uint32_t k = blockIdx.x - sps[t], np = sps[t + 1] - sps[t];
  const uint32_t tb = a.toff[t], te = a.toff[t + 1];
  const uint32_t r0 = tb + k * MERGE_TSEG, r1 = min(te, r0 + MERGE_TSEG);
  {
    int rc = -1;                                    // the run's cell and its partial sums
    uint32_t rn = 0u;
    double rl = 0.0, ri = 0.0;
    unsigned long long rm = ~0ull;
    auto flush = [&]() {
      if (rc < 0) return;
      atomicAdd(&scnt[rc], rn);
      atomicAdd(&ssl[rc], rl);
      atomicAdd(&ssi[rc], ri);
      atomicMin(&smk[rc], rm);
    };
    for_runs<RUNS>(a, r0, r1, [&](const float4 r) {
      unsigned long long cb;
      uint32_t w;
      rec_fields(r, cb, w);
      const int col = w & 1023u;
      if (col != rc) {
        flush();
        rc = col;
        rn = 0u;
        rl = 0.0;
        ri = 0.0;
        rm = ~0ull;
      }
      ++rn;
      rl += __longlong_as_double((long long)cb);
      ri += (double)r.z;
      rm = cb < rm ? cb : rm;
    });
    flush();
  }
  __syncthreads();
  const size_t cb0 = (size_t)t * W;                 // tile t = ol * big + row -> cells row-major per view
  if (np == 1u) {
    int rc = -1;
    uint32_t rs = ~0u;
    for_runs<RUNS>(a, r0, r1, [&](const float4 r) {
      unsigned long long cb;
      uint32_t w;
      rec_fields(r, cb, w);
      const int col = w & 1023u;
      if (col != rc) {
        if (rc >= 0 && rs != ~0u) atomicMin(&sidx[rc], rs);
        rc = col;
        rs = ~0u;
      }
      if (cb == smk[col]) rs = min(rs, w >> 10);
    });
    if (rc >= 0 && rs != ~0u) atomicMin(&sidx[rc], rs);
    __syncthreads();
    for (int c = tid; c < W; c += MERGE_TNT) {
      a.cnt[cb0 + c] = scnt[c];
      a.sumL[cb0 + c] = ssl[c];
      a.sumI[cb0 + c] = ssi[c];
      a.minkey[cb0 + c] = smk[c];
      a.minidx[cb0 + c] = sidx[c];
    }
    return;
  }
  for (int c = tid; c < W; c += MERGE_TNT) {
    if (scnt[c] == 0u) continue;
    atomicAdd(&a.cnt[cb0 + c], scnt[c]);
    atomicAdd(&a.sumL[cb0 + c], ssl[c]);
    atomicAdd(&a.sumI[cb0 + c], ssi[c]);
    atomicMin(&a.minkey[cb0 + c], smk[c]);
  }
}
// the nearest indices of the tiles of more than one part (the others were resolved by merge_tile_sum_kernel)
template <bool RUNS>
__global__ __launch_bounds__(MERGE_TNT) void merge_tile_minidx_kernel(MergeArgs a) {
  __shared__ uint32_t sidx[1024];
  extern __shared__ uint32_t sps[];
  const int tid = threadIdx.x, W = a.g.W, T = a.n_out * a.g.big;
  if (blockIdx.x >= a.pstart[T]) return;
  for (int t = tid; t <= T; t += MERGE_TNT) sps[t] = a.pstart[t];
  for (int c = tid; c < W; c += MERGE_TNT) sidx[c] = ~0u;
  __syncthreads();
  const int t = part_tile(sps, blockIdx.x, T);
  const uint32_t k = blockIdx.x - sps[t], np = sps[t + 1] - sps[t];
  if (np == 1u) return;
  const uint32_t r0 = a.toff[t] + k * MERGE_TSEG, r1 = min(a.toff[t + 1], r0 + MERGE_TSEG);
  const size_t cb0 = (size_t)t * W;
  int rc = -1;
  uint32_t rs = ~0u;
  unsigned long long mk = 0ull;
  for_runs<RUNS>(a, r0, r1, [&](const float4 r) {
    unsigned long long cb;
    uint32_t w;
    rec_fields(r, cb, w);
    const int col = w & 1023u;
    if (col != rc) {
      if (rc >= 0 && rs != ~0u) atomicMin(&sidx[rc], rs);
      rc = col;
      rs = ~0u;
      mk = a.minkey[cb0 + col];                     // one gather per run
    }
    if (cb == mk) rs = min(rs, w >> 10);
  });
  if (rc >= 0 && rs != ~0u) atomicMin(&sidx[rc], rs);
  __syncthreads();
  for (int c = tid; c < W; c += MERGE_TNT)
    if (sidx[c] != ~0u) atomicMin(&a.minidx[cb0 + c], sidx[c]);
}

// ---------------------------------------------------------------- K5: resolve cells -> new image, apply
// One pass per output pixel (the resolve and the correction were two launches): the cell the pixel
// reads (flip/roll for negative depth), the controlled average (KITTISampling.py:300-420), the new
// image, then -- unless tooHigh (KITTISampling.py:162) -- x += cc * -(x - new) on the unknown pixels
// of both channels.  The nearest point's intensity comes from the snapshot taken before any pixel is
// corrected; a pixel's own depth sign is read before the pass writes it.
// Trade-off of the fusion: with a multi-rank tooHigh (apply_wait) the whole pass, resolve included,
// now waits for the all_reduce(MAX) event, where the two-launch form ran the resolve beside it; the
// all_reduce of one word (<= ~20 us over xGMI) is issued right after the Langevin update and overlaps
// the five binning / segment launches before this one, so the wait is empty unless the collective is
// slower than that whole chain.
__global__ __launch_bounds__(256) void merge_resolve_apply_kernel(MergeArgs a) {
  const int H = a.g.H, W = a.g.W, HW = H * W;
  const int cells = a.g.big * W;
  const size_t n = (size_t)a.n_out * HW;
  const float mx = __uint_as_float(*a.absmax);
  const bool too_high = __fdiv_rn(__fmul_rn(mx, 6.0f), a.smod) > 50.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int ol = i / HW, p = i % HW;
    const int r = p / W, c = p % W;
    const int o = a.o_begin + ol;
    const int m0 = (o / a.aB) * a.aB;
    const size_t x0i = (size_t)o * 2 * HW + p;
    const float xd = a.x[x0i];
    const bool neg = xd < 0.f;
    const int brow = neg ? (H - 1 - r) : (r + a.g.big - H);
    const int bcol = neg ? ((c - W / 2) % W + W) % W : c;
    const size_t ci = (size_t)ol * cells + brow * W + bcol;
    const uint32_t nn = a.cnt[ci];
    double code = 0.0;
    float inten = 0.f;
    if (nn > 0) {
      const float scaling = (float)nn;   // float32(n + 1e-9) == n for n >= 1
      const double Abar = __ddiv_rn(a.sumL[ci], (double)scaling);
      const float Ibar = __fdiv_rn((float)a.sumI[ci], scaling);
      const bool controlled = a.variant == 0 || a.setting >= 7;
      if (controlled) {
        const double lmin = __longlong_as_double((long long)a.minkey[ci]);
        const uint32_t s = a.minidx[ci];
        const int vl = s / HW, ps = s % HW;
        const float Imin = a.isnap[(size_t)(m0 + vl) * HW + ps];
        const double sm = (double)a.smod;
        const double A = exp2(__dmul_rn(fabs(Abar), 6.0) / sm) - 1.0;
        const double M = exp2(__dmul_rn(fabs(lmin), 6.0) / sm) - 1.0;
        const double allow = (double)a.allowance;
        const bool cond = A > M + allow;
        inten = cond ? Imin : Ibar;
        const double D = cond ? M + allow / 5.0 : A;
        code = __dmul_rn(log2(D + 1.0) / 6.0, sm);
      } else {
        code = Abar;
        inten = Ibar;
      }
    }
    const float depth = (float)(neg ? -code : code);
    const bool m = nn > 0 && a.exist[p] && a.sky[(size_t)o * HW + p];
    a.newimg[((size_t)ol * 2 + 0) * HW + p] = depth;
    a.newimg[((size_t)ol * 2 + 1) * HW + p] = inten;
    if (too_high) continue;
    // KITTISampling.py:428-490: x += cc * -(maskImages * !mask * (x - new)).  Where the factor is 0 the
    // product is still NaN when x - new is not finite (a NaN intensity in the cell, an infinite x), and the
    // reference's x becomes NaN there; elsewhere it leaves x as it is.
    const float d0 = __fsub_rn(xd, depth);
    if (m && a.refmask[x0i] == 0) a.xout[x0i] = __fadd_rn(xd, __fmul_rn(a.cc, -d0));
    else if (!isfinite(d0)) a.xout[x0i] = __int_as_float(0x7fc00000);
    const float xi = a.xout[x0i + HW];
    const float d1 = __fsub_rn(xi, inten);
    if (m && a.refmask[x0i + HW] == 0) a.xout[x0i + HW] = __fadd_rn(xi, __fmul_rn(a.cc, -d1));
    else if (!isfinite(d1)) a.xout[x0i + HW] = __int_as_float(0x7fc00000);
  }
}

static int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 256 * 16); }

// pair chunks of the binning passes: ~1024 (4 per CU), at least 2048 pairs each
#ifndef SDP_MERGE_CHUNK_MAX   // A/B knob: most workgroups of the count / scatter passes
#define SDP_MERGE_CHUNK_MAX 1024
#endif
static int merge_chunks(size_t npair) {
  return (int)std::max<size_t>(1, std::min<size_t>(SDP_MERGE_CHUNK_MAX, (npair + 2047) / 2048));
}

size_t merge_ws_bytes(int n_src, int aB, int n_out, int H, int W) {
  const int big = (int)((25 * 2) * (long)H / 28);
  const size_t cells = (size_t)big * W;
  const size_t npair = (size_t)n_out * aB * H * W;
  const size_t T = (size_t)n_out * big, nt = T * merge_chunks(npair);
  size_t b = 0;
  auto add = [&](size_t x) { b += (x + 255) & ~size_t(255); };
  add((size_t)(W + H) * sizeof(double2));                    // trig
  add(cells * n_out * 4);                                    // cnt
  add(cells * n_out * 8);                                    // sumL
  add(cells * n_out * 8);                                    // sumI
  add(cells * n_out * 8);                                    // minkey
  add(cells * n_out * 4);                                    // minidx
  add(nt * 4);                                               // tcount
  add(((nt + 2047) / 2048 + 1) * 4);                         // bsum
  add(npair * 16);                                           // records
  add(npair * 4);                                            // pcell
  add(npair * 8);                                            // pcode
  add((size_t)n_out * 2 * H * W * 4);                        // newimg (internal)
  add((size_t)n_src * H * W * 4);                            // isnap
  add((T + 1) * 4);                                          // toff
  add((T + 1) * 4);                                          // pstart
  return b + 1024;
}

hipError_t consistency_merge(MergeArgs a, void* ws, size_t ws_bytes, float* new_out, hipStream_t st, const char** why,
                             hipEvent_t apply_wait) {
  const int H = a.g.H, W = a.g.W;
  const size_t cells = (size_t)a.g.big * W;
  if (ws_bytes < merge_ws_bytes(a.n_src, a.aB, a.n_out, H, W)) { *why = "merge: workspace too small"; return hipErrorInvalidValue; }
  if (a.n_src % a.aB || a.o_begin < 0 || a.o_begin + a.n_out > a.n_src) { *why = "merge: bad view ranges"; return hipErrorInvalidValue; }
  if (W % 2 || W > 1024) { *why = "merge: W must be even and <= 1024"; return hipErrorInvalidValue; }
    if ((size_t)a.aB * H * W > (1u << 22)) { *why = "merge: aB*H*W must be < 2^22 (record packing)"; return hipErrorInvalidValue; }
  const size_t npair = (size_t)a.n_out * a.aB * H * W, nout = (size_t)a.n_out * H * W, nw = (size_t)a.n_src * H * W;
  const int T = a.n_out * a.g.big;
  a.nchunk = merge_chunks(npair);
  const size_t nt = (size_t)T * a.nchunk;
  const int nb = (int)((nt + 2047) / 2048);
  if (nb > 8 * 1024) { *why = "merge: too many tiles x chunks"; return hipErrorInvalidValue; }
  char* p = reinterpret_cast<char*>(ws);
  auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) & ~size_t(255); return q; };
  a.trig = reinterpret_cast<double2*>(take((size_t)(W + H) * sizeof(double2)));
  a.cnt = reinterpret_cast<uint32_t*>(take(cells * a.n_out * 4));
  a.sumL = reinterpret_cast<double*>(take(cells * a.n_out * 8));
  a.sumI = reinterpret_cast<double*>(take(cells * a.n_out * 8));
  a.minkey = reinterpret_cast<unsigned long long*>(take(cells * a.n_out * 8));
  a.minidx = reinterpret_cast<uint32_t*>(take(cells * a.n_out * 4));
  a.tcount = reinterpret_cast<uint32_t*>(take(nt * 4));
  a.bsum = reinterpret_cast<uint32_t*>(take(((nt + 2047) / 2048 + 1) * 4));
  a.rec = reinterpret_cast<float4*>(take(npair * 16));
  a.pcell = reinterpret_cast<int32_t*>(take(npair * 4));
  a.pcode = reinterpret_cast<double*>(take(npair * 8));
  a.newimg = new_out ? new_out : reinterpret_cast<float*>(take((size_t)a.n_out * 2 * H * W * 4));
  a.isnap = reinterpret_cast<float*>(take(nw * 4));
  a.toff = reinterpret_cast<uint32_t*>(take(((size_t)T + 1) * 4));
  a.pstart = reinterpret_cast<uint32_t*>(take(((size_t)T + 1) * 4));
  const size_t per_chunk = ((size_t)a.aB * H * W + a.nchunk - 1) / a.nchunk;   // source points per chunk
  // dynamic LDS of each launch, checked against the per-workgroup limit BEFORE anything is enqueued:
  // count = the tile histogram [T]; scatter = the tile cursors [T] + the scanned block totals [nb + 1]
  // beside its 1 KB static scan array; tile passes = the part table [T + 1] beside 32 KB static
  const size_t lds = (size_t)T * 4;
  const size_t slds = lds + ((size_t)nb + 1) * 4;
  const size_t tlds = ((size_t)T + 1) * 4;
  constexpr size_t kDyn = 96 * 1024;   // the attribute set below (<= 160 KB per CU on gfx950)
  if (lds > kDyn) { *why = "merge: too many output views for the tile histogram"; return hipErrorInvalidValue; }
  if (slds + 1024 > kDyn) { *why = "merge: too many output views x chunks for the scatter's cursor + scan tables"; return hipErrorInvalidValue; }
  if (tlds + 33 * 1024 > kDyn) { *why = "merge: too many output views for the tile table"; return hipErrorInvalidValue; }
  hipError_t e;
  // the max-dynamic-LDS attribute acts on the current device: set once per device (thread-safe)
  {
    static std::mutex mu;
    static uint64_t done = 0;   // bit d: device d configured
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    if (dev >= 64 || !((done >> dev) & 1u)) {
      const void* fns[] = {(const void*)merge_bin_count_kernel, (const void*)merge_bin_scatter_kernel,
                           (const void*)merge_tile_sum_kernel<false>, (const void*)merge_tile_minidx_kernel<false>,
                           (const void*)merge_tile_sum_kernel<true>, (const void*)merge_tile_minidx_kernel<true>};
      for (const void* f : fns)
        if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDyn)) != hipSuccess) return e;
      if (dev < 64) done |= 1ull << dev;
    }
  }
  // seven dependent launches: prep (grid reset, intensity snapshot, trig table) -> count (+ world points) -> block scan ->
  // scatter (+ top scan, tile and part tables) -> tile sums (+ the nearest index of one-part tiles) ->
  // nearest index of the other tiles -> resolve + correction
  hipLaunchKernelGGL(merge_prep_kernel, dim3(std::min(grid_for(std::max(nw, (size_t)a.n_out * cells)), MERGE_PREP_WG)),
                     dim3(256), 0, st, a);
  hipLaunchKernelGGL(merge_bin_count_kernel, dim3(a.nchunk), dim3(256), lds, st, a, per_chunk);
  hipLaunchKernelGGL(merge_scan_block_kernel, dim3(nb), dim3(256), 0, st, a.tcount, nt, a.bsum);
  hipLaunchKernelGGL(merge_bin_scatter_kernel, dim3(a.nchunk), dim3(256), slds, st, a, per_chunk, nb);
  const int nparts = (int)(T + (npair + MERGE_TSEG - 1) / MERGE_TSEG);   // upper bound: records <= pairs
  if (a.aB >= 16) {
    hipLaunchKernelGGL(merge_tile_sum_kernel<true>, dim3(nparts), dim3(MERGE_TNT), tlds, st, a);
    hipLaunchKernelGGL(merge_tile_minidx_kernel<true>, dim3(nparts), dim3(MERGE_TNT), tlds, st, a);
  } else {
    hipLaunchKernelGGL(merge_tile_sum_kernel<false>, dim3(nparts), dim3(MERGE_TNT), tlds, st, a);
    hipLaunchKernelGGL(merge_tile_minidx_kernel<false>, dim3(nparts), dim3(MERGE_TNT), tlds, st, a);
  }
  if (apply_wait && (e = hipStreamWaitEvent(st, apply_wait, 0)) != hipSuccess) return e;   // tooHigh's global max
  hipLaunchKernelGGL(merge_resolve_apply_kernel, dim3(grid_for(nout)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace sdp
