#!/bin/bash
# retry gpurun only while the pool reports no free box / busy slots (nothing charged)
OUT=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  if grep -q "nothing was charged\|no free box right now\|backing off" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then
    sleep 90; continue
  fi
  break
done
tail -20 $OUT
