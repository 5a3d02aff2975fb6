# round 5, GPU session 37: action rows in LDS + one-group table loads (cur, build d6050b3a) vs the
# shipped build 2e6f0d8b (old): A/B at configs 3, 2 and 4
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 4 cur: old:LSM_LIB=liblsm_rollout_old.so > gpurun_out/r05_s37_ab_c3.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 cur: old:LSM_LIB=liblsm_rollout_old.so > gpurun_out/r05_s37_ab_c2.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 cur: old:LSM_LIB=liblsm_rollout_old.so > gpurun_out/r05_s37_ab_c4.txt 2>&1
echo rc=$?
