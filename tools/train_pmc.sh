#!/bin/bash
# PMC passes over one DSM training step (bench.py --workload train), one counter group per pass;
# summary of the weight-gradient and data-gradient kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/trainpmc
mkdir -p $OUT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- \
    python bench.py --workload train --steps 1 --warmup 0 --views 4 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc: $grp"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU
GROUPS
python tools/pmc_kernels.py $OUT conv_wgrad_kernel > $OUT/summary.txt
python tools/pmc_kernels.py $OUT "conv_mfma_kernel<2, 1, 64, 3, false, false, false>" >> $OUT/summary.txt
head -80 $OUT/summary.txt
