# round 6, GPU session 19: the coalesced episode-summary kernel with 16 chunks per thread in flight
# (RB = 16: 4096 envs in one batch) -- its GPU tests and device time behind a rollout step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s19_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u layered-safe-marl_amd/tools/summary_time.py > gpurun_out/r06_s19_summary_time.json 2>&1 || exit $?
echo done
