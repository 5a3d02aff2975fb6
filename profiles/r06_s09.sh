# round 6, GPU session 9: config 4's occupancy slope -- the 2-wave-capped airtaxi team kernel at 2
# workgroups per CU (at22) and with 64 KB of extra LDS per workgroup, 1 per CU (pad1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 600 python -u $T/ab_bench.py --config 4 --reps 3 --steps 300 --warmup 30 --allow-old at22:LSM_LIB=liblsm_rollout_at22.so pad1:LSM_LIB=liblsm_rollout_pad1.so > gpurun_out/r06_s09_ab_c4_occupancy.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
