# round 5, GPU session 3: A/B of the phase-A / magnetic-field changes (config 3 and 2) + parity of the combined variant
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_all.so timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s3_tests_all.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: dec:LSM_LIB=liblsm_rollout_dec.so gpre:LSM_LIB=liblsm_rollout_gpre.so all:LSM_LIB=liblsm_rollout_all.so > gpurun_out/r05_s3_ab_c3.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: all:LSM_LIB=liblsm_rollout_all.so > gpurun_out/r05_s3_ab_c2.txt 2>&1
echo rc=$?
