#!/bin/bash
# bf16 tape: 16x16-tile 8-wave IO16 forward (w16 variant) -- training tests on the variant, train bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
SDP_LIB=tools/_var/w16/libsdp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread -k "bf16 or tape or loss_and_gradients" > $O/train_tests.log 2>&1
rc=$?; echo "train tests (w16) rc=$rc"; tail -1 $O/train_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for arm in base w16; do
    if [ $arm = w16 ]; then export SDP_LIB=tools/_var/w16/libsdp.so; else unset SDP_LIB; fi
    timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > $O/${arm}_$r.log 2>&1 || { echo "$arm failed"; tail -3 $O/${arm}_$r.log; exit 1; }
    python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${arm}_$r.log ${arm}_$r
  done
done
export SDP_LIB=tools/_var/w16/libsdp.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, collections, sys
f = glob.glob(sys.argv[1] + "/prof/**/run_kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "conv_mfma_kernel" in r["Kernel_Name"]:
        agg[(r["Kernel_Name"][:90], r["Grid_Size_X"], r["Grid_Size_Y"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"{sum(v) / len(v) / 1e3:8.1f} us n={len(v):4d} grid={k[1]}x{k[2]} {k[0]}")
PY
