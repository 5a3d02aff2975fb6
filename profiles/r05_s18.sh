# round 5, GPU session 18: D-phase loops branch-free with batched LDS reads (parity subset + A/B configs 3, 2)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 900 python -u -m pytest $(cat profiles/r05_ab_tests.txt) -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s18_tests.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: > gpurun_out/r05_s18_ab_c3.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: > gpurun_out/r05_s18_ab_c2.txt 2>&1
echo rc=$?
