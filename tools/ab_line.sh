#!/bin/bash
# In-network A/B of the line step on one box: arms "name|env|bench args", interleaved over rounds.
# usage: ARMS="base|SDP_LIB=tools/_var/base/libsdp.so|--merge-parts 1;new||--merge-parts 2" bash tools/ab_line.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
IFS=';' read -r -a ARMV <<< "$ARMS"
for round in ${ROUNDS:-1 2}; do
  for arm in "${ARMV[@]}"; do
    IFS='|' read -r name envs args <<< "$arm"
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 $args \
      > gpurun_out/ab/${name}_$round.log 2>&1 || { echo "arm $name failed rc=$?"; tail -5 gpurun_out/ab/${name}_$round.log; exit 1; }
    python3 - "$name" "$round" gpurun_out/ab/${name}_$round.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[3]) if x.startswith("{")][-1]
d = json.loads(l)
mb = {m["kernel"].split(" (")[0]: m["avg_launch_us"] for m in d["roofline"].get("memory_bound", [])}
print(f"{sys.argv[1]:>12} r{sys.argv[2]}: {d['value']:8.2f} img-steps/s  {d['ms_per_step']:7.3f} ms  sustained "
      f"{(d.get('sustained') or {}).get('value', 0):8.2f}  conv256 {d['roofline']['avg_launch_us']:.1f} us  merge "
      f"{mb.get('consistency_merge', 0):.1f} us", flush=True)
print("      " + "  ".join(f"{k[:22]} {v:.1f}" for k, v in mb.items() if k != "consistency_merge"), flush=True)
PY
  done
done
