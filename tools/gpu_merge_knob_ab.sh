#!/bin/bash
# Merge A/B: a knob variant (tools/_var/<name>, e.g. mrgu2 = SDP_MERGE_UNROLL=2) vs the tree:
# merge parity tests on each library, then one config-4 rank's step at a 32-view megabatch and the
# 4-view line step (merge_us = HIP events around the merge).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/merge_knob
mkdir -p $O
for v in tree mrgu2; do
  if [ $v = tree ]; then unset SDP_LIB; else export SDP_LIB=tools/_var/$v/libsdp.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_parity.py -k "merge or rank" -x -q \
    --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for v in tree mrgu2; do
    if [ $v = tree ]; then unset SDP_LIB; else export SDP_LIB=tools/_var/$v/libsdp.so; fi
    for mb in 32 4; do
      timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 0 \
        --megabatch-views $mb > $O/${v}_mb${mb}_$r.log 2>&1 || exit $?
      echo "$v mb$mb run $r: $(grep '^{' $O/${v}_mb${mb}_$r.log | python -c "
import json, sys
j = json.loads(sys.stdin.read()); m = [e for e in j['roofline']['memory_bound'] if e['kernel'].startswith('consistency')][0]
print(j['value'], j['ms_per_step'], 'merge_us', m['avg_launch_us'])")"
    done
  done
done
