#!/bin/bash
# Pool-first ConvMeanPool 1x1 shortcut A/B: score-net parity of the tree (goldens at fp32x3 and fp32,
# batch/oracle, split, sampler) then the line bench with the previous commit's library (A) and the tree (B).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/pf_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for arm in A B; do
if [ $arm = A ]; then E="SDP_LIB=tools/_var/prev/libsdp.so"; else E="SDP_X=1"; fi
env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/pf_$arm$r.log 2>&1 || exit $?
echo "$arm $r: $(grep -o '"value": [0-9.]*' gpurun_out/pf_$arm$r.log | head -1) $(grep -h 'conv1x1\|avgpool2' gpurun_out/pf_$arm$r.log | tr -s ' ' | cut -c1-90 | tr '\n' '|')"
done
done
