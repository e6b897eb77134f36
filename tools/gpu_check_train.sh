#!/bin/bash
# Training-path check on one box: GPU training parity, train + line benches, rocprofv3 kernel stats of the train step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ct_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/ct_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ct_train.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/ct_line.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ct_prof_train -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ct_rocprof_train.log 2>&1 || exit $?
grep -h -o '"value": [0-9.]*' gpurun_out/ct_train.log gpurun_out/ct_line.log
