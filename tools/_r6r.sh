#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 200 python tools/grad_dump.py /tmp/gnew.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
SDP_LIB=tools/_var/prevh/libsdp.so timeout -k 10 200 python tools/grad_dump.py /tmp/gold.npz > $O/dump_old.log 2>&1 || { tail -5 $O/dump_old.log; exit 1; }
python3 - <<'PY'
import numpy as np
a, b = np.load("/tmp/gnew.npz"), np.load("/tmp/gold.npz")
diff = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("gradients compared:", len(a.files), "differing:", diff[:10])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -1 $O/train_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for arm in prev new; do
    if [ $arm = prev ]; then export SDP_LIB=tools/_var/prevh/libsdp.so; else unset SDP_LIB; fi
    timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > $O/${arm}_$r.log 2>&1 || { echo "$arm failed"; exit 1; }
    python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${arm}_$r.log ${arm}_$r
  done
done
unset SDP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); python3 tools/stats_top.py $f 11 40 | grep -i "begin_wgrad\|end_wgrad"
