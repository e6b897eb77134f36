#!/bin/bash
# Clock and MFMA-busy of the conv classes in the network, reduced by
# tools/conv_clock.py into gpurun_out/conv_clock/<ROUND>_conv_clock.json (copied into profiles/):
#  1. in-kernel clock (s_memtime / s_memrealtime, MI355X_MICROARCH.md 'DVFS give-back' item 6) of
#     isolated launches (tools/_cb/conv_bench_T, the SDP_TIMING build of the same conv sources) at
#     B=4 (the bench's launch) and B=32, each beside a GRBM_GUI_ACTIVE pass of the same command:
#     calibrates the GRBM clock (which reads high on dispatches < ~0.3 ms) against the in-kernel one;
#  2. two --pmc passes over `bench.py --split 1` (one whole-batch launch per layer), one counter
#     group each, --kernel-trace only: GRBM_GUI_ACTIVE + SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES +
#     GRBM_GUI_ACTIVE; at 4 views (the bench) and 16 views (0.65-0.8 ms launches: GRBM reads true).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
O=gpurun_out/conv_clock
rm -rf $O; mkdir -p $O
for B in 4 32; do
  for shape in "256 256 32 512" "128 128 64 1024"; do
    tag="cb_$(echo $shape | cut -d' ' -f1)_b$B"
    timeout -k 5 60 tools/_cb/conv_bench_T $shape $B 1 40 1 > $O/$tag.ik.log 2>&1 || { echo "$tag failed"; exit 1; }
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/$tag -o run \
      --output-format csv -- tools/_cb/conv_bench_T $shape $B 1 40 1 > $O/$tag.log 2>&1 || { echo "$tag pmc failed"; exit 1; }
  done
done
for V in 4 16; do
  BENCH="bench.py --steps 10 --warmup 3 --views $V --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/g_v$V -o run --output-format csv \
    -- python3 $BENCH > $O/g_v$V.log 2>&1 || { echo "pass g v$V failed rc=$?"; tail -5 $O/g_v$V.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/m_v$V -o run \
    --output-format csv -- python3 $BENCH > $O/m_v$V.log 2>&1 || { echo "pass m v$V failed rc=$?"; tail -5 $O/m_v$V.log; exit 1; }
done
python3 tools/conv_clock.py $O $ROUND
