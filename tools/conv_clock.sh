#!/bin/bash
# In-network clock + MFMA-busy of the conv classes: two rocprofv3 --pmc passes (one counter group
# each, --kernel-trace only) over `bench.py --split 1` (one whole-batch launch per layer), reduced by
# tools/conv_clock.py into gpurun_out/conv_clock/<ROUND>_conv_clock.json (copied into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
O=gpurun_out/conv_clock
rm -rf $O; mkdir -p $O
BENCH="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/g -o run --output-format csv \
  -- python3 $BENCH > $O/g.log 2>&1 || { echo "pass g failed rc=$?"; tail -5 $O/g.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/m -o run --output-format csv \
  -- python3 $BENCH > $O/m.log 2>&1 || { echo "pass m failed rc=$?"; tail -5 $O/m.log; exit 1; }
python3 tools/conv_clock.py $O $ROUND
