#!/bin/bash
# One rank's per-step cost of BASELINE config 4 emulated on one GPU: 4 own views merged against
# megabatches of 4..32 views (no all-gather).  Prints megabatch, image-steps/s, ms/step, conv ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in 4 8 16 32; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --megabatch-views $mb \
    > gpurun_out/mb_$mb.log 2>&1 || { tail -3 gpurun_out/mb_$mb.log; exit 1; }
  tail -1 gpurun_out/mb_$mb.log | python tools/json_fields.py config.megabatch_views value ms_per_step roofline.conv_ms_per_step
done
