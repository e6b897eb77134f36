#!/bin/bash
# Every measurement committed under profiles/ for a round, in GPU sessions of <= 20 min:
#   PART=1: smoke, GPU tests, PMC traffic and in-network clock of the dominant classes;  PART=2: the bench workloads;
#   PART=3: rocprofv3 kernel stats (line + train); PART=all: the three in one call.  Stops at the first
#   step that faults or times out.
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
PART=${PART:-1}
if [ "$PART" = 1 ] || [ "$PART" = all ]; then
step smoke 300 python __graft_entry__.py smoke
step pytest_gpu 850 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread
step traffic 200 env ROUND=${ROUND:-r05} bash tools/class_traffic.sh
step clock 500 env ROUND=${ROUND:-r05} bash tools/conv_clock.sh
fi
if [ "$PART" = 2 ] || [ "$PART" = all ]; then
step bench 300 python bench.py --steps 20 --warmup 5
step bench_views8 200 python bench.py --steps 10 --warmup 2 --views 8 --no-cpu-baseline --no-fp32-line
step bench_mb32 200 python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line
step bench_allforone 300 python bench.py --workload allforone --steps 10 --warmup 2
step bench_train 300 python bench.py --workload train --steps 10 --warmup 2
step bench_project 200 python bench.py --workload project --steps 10 --warmup 2
fi
if [ "$PART" = 3 ] || [ "$PART" = all ]; then
step rocprof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0
step rocprof_train 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline
step rocprof_mb32 300 rocprofv3 --kernel-trace --stats -d $O/prof_mb32 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0
# the default two-stream step (--split 2): how much of each memory-bound kernel runs under a conv of the other stream
step rocprof_split2 300 rocprofv3 --kernel-trace -d $O/prof_split2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-line --sustained-s 0
step overlap 120 python3 tools/overlap.py $(find $O/prof_split2 -name "run_kernel_trace.csv" | head -1) $O/${ROUND:-r05}_overlap.json
fi
exit 0
