#!/bin/bash
# TEST INFRASTRUCTURE: compile the reference's C++ grid subsampling from its own sources (read in
# place under /root/reference, nothing copied) into oracle/_ref/, with the driver above.  The
# reference's CPython wrappers use the numpy 1.x C API (NPY_IN_ARRAY), absent from this image's
# numpy 2.2, so the driver replaces only the wrapper; the algorithm files compile unchanged.
set -eu
REF=${REF:-/root/reference/LiDARGen/datasets/cpp_wrappers}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
[ -d "$REF" ] || { echo "reference sources absent: skipping oracle/_ref"; exit 0; }
mkdir -p "$OUT"
CXX="g++ -O2 -std=c++11 -fPIC -shared -D_GLIBCXX_USE_CXX11_ABI=0"   # the flags of the reference's setup.py
$CXX -I"$REF/cpp_subsampling" "$HERE/grid_ref/driver.cpp" "$REF/cpp_subsampling/grid_subsampling/grid_subsampling.cpp" \
  "$REF/cpp_utils/cloud/cloud.cpp" -o "$OUT/libgrid_ref.so"
$CXX -DREF_LIDAR -I"$REF/cpp_subsampling" "$HERE/grid_ref/driver.cpp" \
  "$REF/cpp_subsampling/grid_subsampling/grid_subsampling_lidar.cpp" "$REF/cpp_utils/cloud/cloud.cpp" \
  -o "$OUT/libgrid_ref_lidar.so"
echo "built $OUT/libgrid_ref.so $OUT/libgrid_ref_lidar.so"
