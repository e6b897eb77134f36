#!/bin/bash
# Sustained-window A/Bs of the round-2 decisions made at <= 2 % margins: forward
# split ways (1 vs 2 streams) and non-temporal patch DMA (tools/_var/dmant: SDP_DMA_AUX=2) vs the
# cached DMA, each as >= 2 s warm + 3 s timed back-to-back steps (bench.py `sustained`), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sustained_ab
mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3"
for r in 1 2; do
  for v in split2 split1 dmant; do
    case $v in
      split2) timeout -k 10 120 python bench.py $A > $O/${v}_$r.log 2>&1 || exit $? ;;
      split1) timeout -k 10 120 python bench.py $A --split 1 > $O/${v}_$r.log 2>&1 || exit $? ;;
      dmant) SDP_LIB=tools/_var/dmant/libsdp.so timeout -k 10 120 python bench.py $A > $O/${v}_$r.log 2>&1 || exit $? ;;
    esac
    echo "$v run $r: $(grep '^{' $O/${v}_$r.log | python tools/json_fields.py value sustained.value sustained.dominant_conv.avg_launch_us)"
  done
done
