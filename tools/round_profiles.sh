#!/bin/bash
# Every measurement committed under profiles/ for a round, in one GPU session:
# smoke, GPU tests, the bench workloads, rocprofv3 kernel stats (line + train) and the PMC traffic
# of the dominant conv class.  Stops at the first step that faults or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-240
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then echo "STOP after $name"; exit $rc; fi
}
step smoke 300 python __graft_entry__.py smoke
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread
step traffic 300 bash tools/class_traffic.sh
cp gpurun_out/class_traffic/*_traffic.json profiles/ 2>/dev/null
step bench 600 python bench.py --steps 20 --warmup 3
step bench_views8 600 python bench.py --steps 10 --warmup 2 --views 8 --no-cpu-baseline --no-fp32-line
step bench_allforone 600 python bench.py --workload allforone --steps 10 --warmup 2
step bench_train 600 python bench.py --workload train --steps 10 --warmup 2
step rocprof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-line --split 1
step rocprof_train 600 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline
exit 0
