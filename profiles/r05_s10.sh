# round 5, GPU session 10: filter_prep on 8 lanes per ego (parity + A/B at config 3)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_oct.so timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[double_integrator-8-4]" \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s10_tests_oct.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: oct:LSM_LIB=liblsm_rollout_oct.so > gpurun_out/r05_s10_ab_c3.txt 2>&1
echo rc=$?
