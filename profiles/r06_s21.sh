# round 6, GPU session 21: config 3 with each XCD taking one contiguous range of env groups (xremap:
# workgroup b -> group (b % 8) * (nb / 8) + b / 8) against round-robin groups (base)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 500 python -u $T/ab_bench.py --config 3 --reps 4 --steps 400 --warmup 50 --allow-old base: xremap:LSM_LIB=liblsm_rollout_xremap.so > gpurun_out/r06_s21_ab_c3.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
