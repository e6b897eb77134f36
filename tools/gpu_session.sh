#!/bin/bash
# One GPU-box session: smoke -> GPU tests -> bench -> rocprofv3 kernel stats.
# Stops at the first step that ends in a fault/abort/timeout (exit >= 124); plain test
# failures (exit 1) let the measurement steps still run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a $OUT/session.log
  tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-all}
[[ $STEPS == *smoke* || $STEPS == all ]] && run smoke 400 python __graft_entry__.py smoke
[[ $STEPS == *tests* || $STEPS == all ]] && run pytest_gpu 900 python -m pytest tests -m gpu -q -rA
[[ $STEPS == *bench* || $STEPS == all ]] && run bench 600 python bench.py --steps 20 --warmup 3
[[ $STEPS == *prof* || $STEPS == all ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline
exit 0
