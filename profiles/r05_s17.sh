# round 5, GPU session 17: kernel-parameter scalar prefetch at entry (A/B configs 3, 2)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: kpre:LSM_LIB=liblsm_rollout_kpre.so > gpurun_out/r05_s17_ab_c3.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 base: kpre:LSM_LIB=liblsm_rollout_kpre.so > gpurun_out/r05_s17_ab_c2.txt 2>&1
echo rc=$?
