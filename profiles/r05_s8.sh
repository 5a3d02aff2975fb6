# round 5, GPU session 8: QP in phase A (parity + A/B at configs 3 and 4), the summary kernel's own time
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_qpa.so timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[double_integrator-8-4]" \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[airtaxi-16-4]" \
   "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[5-t4]" "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[8-t4]" \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s8_tests_qpa.txt 2>&1 && \
timeout -k 10 120 python -u layered-safe-marl_amd/tools/summary_time.py > gpurun_out/r05_summary_time.json 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: qpa:LSM_LIB=liblsm_rollout_qpa.so > gpurun_out/r05_s8_ab_c3.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 base: qpa:LSM_LIB=liblsm_rollout_qpa.so > gpurun_out/r05_s8_ab_c4.txt 2>&1
echo rc=$?
