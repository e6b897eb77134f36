// Merge launch arguments (see merge.hip).
#pragma once
#include "common.h"

namespace sdp {

struct MergeGeom {
  double hA, vA, hMin, bigMin, vMin;
  int H, W, big;
};

struct MergeArgs {
  const float* x;          // [n_src][2][HW]
  const double* toWorld;   // [n_src][16]  (POSES)
  const double* fromWorld; // [n_src][16]  (POSES)
  const float* origins;    // [aB][3]      (ORIGINS)
  const uint8_t* exist;    // [aB][HW]
  const uint8_t* sky;      // [n_src][HW]
  const int32_t* refmask;  // [n_src][2][HW]
  double2* trig;           // [W + H] (cos, sin) of the column azimuths, then of the row elevations
  float* isnap;            // [n_src][HW] the sources' intensity channel before the correction (resolve's
                           //   nearest-point intensity reads it while the fused pass corrects x in place)
  // per-cell results [n_out][cells] (cells = big x W), written once per cell by merge_tile
  uint32_t* cnt;
  double* sumL;
  double* sumI;
  unsigned long long* minkey;
  uint32_t* minidx;
  // binning of the (output view, source point) pairs by destination tile = (output view, big
  // row): per-chunk tile counts [T][nchunk] -> exclusive offsets (tile-major), and the records
  uint32_t* tcount;        // [T][nchunk], scanned in place
  uint32_t* bsum;          // scan block totals -> their exclusive scan (+ the grand total at [nb])
  uint32_t* toff;          // [T + 1] first record of every tile (+ the total): the segment passes' table
  uint32_t* pstart;        // [T + 1] first part of every tile (+ the part count): the tile passes' table
  float4* rec;             // [pairs]: (code as 2 floats' bits, intensity, s << 10 | column)
  int32_t* pcell;          // [pairs]: K1's projection of every pair (big-grid cell or -1) and its
  double* pcode;           //   depth code, so K3 scatters without projecting again (same bits)
  int nchunk;
  float* newimg;           // [n_out][2][HW]
  const uint32_t* absmax;  // max |x[:,0]| bits over all views
  float* xout;             // x_all (corrected in place for the output views)
  MergeGeom g;
  int n_src, aB, o_begin, n_out, variant, setting;
  float smod, allowance, cc, min_code;
};

size_t merge_ws_bytes(int n_src, int aB, int n_out, int H, int W);   // aB <= n_src
// apply_wait (may be null): the stream waits for it right before the correction pass, the one reader
// of a.absmax, so a cross-rank all_reduce(MAX) of that word can run beside the projection and binning
hipError_t consistency_merge(MergeArgs a, void* ws, size_t ws_bytes, float* new_out, hipStream_t st, const char** why,
                             hipEvent_t apply_wait = nullptr);

}  // namespace sdp
