# round 5, GPU session 5: RK45 shortcuts (exact) parity + A/B; workgroup start stagger A/B (config 3)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_rkb.so timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[double_integrator-8-4]" \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s5_tests_rkb.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: rkb:LSM_LIB=liblsm_rollout_rkb.so stag1:LSM_LIB=liblsm_rollout_stag1.so stag2:LSM_LIB=liblsm_rollout_stag2.so stag3:LSM_LIB=liblsm_rollout_stag3.so > gpurun_out/r05_s5_ab_c3.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 2 base: rkb:LSM_LIB=liblsm_rollout_rkb.so > gpurun_out/r05_s5_ab_c2.txt 2>&1
echo rc=$?
