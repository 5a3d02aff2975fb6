# round 5, GPU session 6: pow tables staged in LDS (exact) parity + A/B, the no-RK45 bound, stamps of the base
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_powlds.so timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[double_integrator-8-4]" \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s6_tests_powlds.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: powlds:LSM_LIB=liblsm_rollout_powlds.so nork:LSM_LIB=liblsm_rollout_nork.so > gpurun_out/r05_s6_ab_c3.txt 2>&1 && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 120 > ../gpurun_out/r05_v2_stamps_c3.txt 2>&1)
echo rc=$?
