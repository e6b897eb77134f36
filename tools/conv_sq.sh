#!/bin/bash
# SQ stall breakdown of isolated conv launches (tools/conv_bench knock-out builds): two --pmc passes
# per (binary, shape), one counter group each, --kernel-trace only; reduced by tools/conv_sq.py.
#   KOS: knock-out builds to profile (tools/conv_bench.sh); shapes 256->256 @32x512 and 128->128 @64x1024
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/conv_sq
rm -rf $O; mkdir -p $O
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
for ko in ${KOS:-0 31}; do
  while read -r shape; do
    [ -z "$shape" ] && continue
    tag="ko${ko}_$(echo $shape | cut -d' ' -f1)"
    for g in 1 2; do
      grp=G$g
      timeout -s KILL 60 rocprofv3 --kernel-trace --pmc ${!grp} -d $O/$tag/g$g -o run --output-format csv \
        -- tools/_cb/conv_bench_$ko $shape ${B:-4} 1 20 ${MODE:-1} > $O/$tag.g$g.log 2>&1 || { echo "$tag g$g failed rc=$?"; tail -3 $O/$tag.g$g.log; exit 1; }
    done
    echo "$tag: $(tail -1 $O/$tag.g1.log)"
  done <<EOF
256 256 32 512
128 128 64 1024
EOF
done
python3 tools/conv_sq.py $O
