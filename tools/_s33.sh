set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s33
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q -rA --timeout 300 --timeout-method thread -k "merge or megabatch or rank_local or limit" -s > gpurun_out/s33/merge_parity.log 2>&1
echo "merge parity rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s33/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/s33/train.log 2>&1 || exit $?
