#!/bin/bash
# Transposed 16x16 epilogue A/B on one box: the line and train benches with the HEAD conv kernels
# (A: tools/_var/head) and the working tree (B), plus the train bench with SDP_DGRAD16=1 (C).
set -u
mkdir -p gpurun_out
A="SDP_LIB=tools/_var/head/libsdp.so"
for r in 1 2; do
env $A timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/ab_A$r.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/ab_B$r.log 2>&1 || exit $?
done
env $A timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_trainA.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_trainB.log 2>&1 || exit $?
SDP_DGRAD16=1 timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_trainC.log 2>&1 || exit $?
python tools/ab_summary.py gpurun_out
grep -h '"value"' gpurun_out/ab_train*.log | cut -c1-200
