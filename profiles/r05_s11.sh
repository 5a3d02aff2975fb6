# round 5, GPU session 11: squared pair distances + checked reciprocal grid division: parity (all
# golden fixtures through the one-wave kernel, team kernels), A/B against the division and HEAD
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 900 python -u -m pytest $(cat profiles/r05_ab_tests.txt) "tests/test_gpu_parity.py::test_gpu_matches_reference_golden" \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle" "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env" \
   -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s11_tests.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: nomdiv:LSM_NO_MDIV=1 > gpurun_out/r05_s11_ab_c3.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 head:LSM_LIB=liblsm_rollout_head.so base: nomdiv:LSM_NO_MDIV=1 > gpurun_out/r05_s11_ab_c4.txt 2>&1
echo rc=$?
