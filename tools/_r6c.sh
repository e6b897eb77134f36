#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q --timeout 200 --timeout-method thread -k "merge or config4 or kitti or allforone" > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 $O/parity.log; [ $rc -ne 0 ] && exit $rc
A=""
for v in ${V32:-tile0 r16k r64k r16k1024 r2k}; do A="$A;$v|SDP_LIB=tools/_var/$v/libsdp.so|--megabatch-views 32 --sustained-s 0"; done
A="$A;r4k||--megabatch-views 32 --sustained-s 0"
for v in ${V4:-tile0 r16k}; do A="$A;${v}_4|SDP_LIB=tools/_var/$v/libsdp.so|--sustained-s 0"; done
A="$A;r4k_4||--sustained-s 0"
ARMS="${A#;}" bash tools/ab_line.sh | grep -v "^      "
