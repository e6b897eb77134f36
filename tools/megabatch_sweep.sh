#!/bin/bash
# One rank's per-step cost of BASELINE config 4 emulated on one GPU: 4 own views merged against
# megabatches of 4..32 views (no all-gather).  Prints megabatch, image-steps/s, ms/step, conv ms,
# merge us (HIP events around sdp_consistency_merge) as JSON lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in 4 8 16 32; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 0 --megabatch-views $mb \
    > gpurun_out/mb_$mb.log 2>&1 || { tail -3 gpurun_out/mb_$mb.log; exit 1; }
  python - gpurun_out/mb_$mb.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        j = json.loads(l)
        m = [e for e in j["roofline"]["memory_bound"] if e["kernel"].startswith("consistency")][0]
        print(json.dumps({"megabatch_views": j["config"]["megabatch_views"], "value": j["value"],
                          "ms_per_step": j["ms_per_step"], "conv_ms_per_step": j["roofline"]["conv_ms_per_step"],
                          "merge_us": m["avg_launch_us"]}))
PY
done
