#!/bin/bash
# HBM traffic of every kernel in one bench run, from the L2 memory-side request counters
# (MI355X_MICROARCH.md "HBM": FETCH_SIZE = TCC_EA0_RDREQ x 64 B reports half the bytes of a
# wide coalesced read on gfx950 -> x2; WRITE_SIZE is exact for 16-B stores).  Each counter
# group is its own --pmc pass with --kernel-trace only.  tools/pmc_traffic.py reduces the
# CSVs to bytes per launch per (kernel, grid) and writes profiles/<round>_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r01}
OUT=gpurun_out/traffic
mkdir -p $OUT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc: $grp"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done <<'GROUPS'
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
FETCH_SIZE
WRITE_SIZE
GROUPS
python tools/pmc_traffic.py $OUT $OUT/${ROUND}_traffic.json
