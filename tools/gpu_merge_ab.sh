#!/bin/bash
# Merge projection-cache A/B: merge parity tests of the tree, then the line bench at 4 views and at
# a 32-view megabatch (one rank of config 4) with the previous commit's library (A) and the tree (B).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q --timeout 200 --timeout-method thread -k "merge or config4 or view or kitti or allforone or sampler" > gpurun_out/mg_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/mg_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for arm in A B; do
if [ $arm = A ]; then E="SDP_LIB=tools/_var/prev/libsdp.so"; else E="SDP_X=1"; fi
env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 0 > gpurun_out/mg_${arm}4_$r.log 2>&1 || exit $?
env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 0 --megabatch-views 32 > gpurun_out/mg_${arm}32_$r.log 2>&1 || exit $?
for v in 4 32; do
python - gpurun_out/mg_${arm}${v}_$r.log <<'PY'
import json, sys
f = sys.argv[1]
for l in open(f):
    if l.startswith("{"):
        j = json.loads(l)
        m = [e for e in j["roofline"]["memory_bound"] if e["kernel"].startswith("consistency")][0]
        print(f, j["value"], j["ms_per_step"], "merge_us", m["avg_launch_us"])
PY
done
done
done
