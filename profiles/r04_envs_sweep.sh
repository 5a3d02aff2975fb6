# config 3 per-step time vs envs per GPU (occupancy: 4 / 2 / 1 workgroups per CU), team stamps at 2048
set -o pipefail
mkdir -p gpurun_out
for n in 4096 2048 1024 3072; do
  timeout -k 10 200 python -u bench.py --config 3 --envs $n --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/r04_v3_envs_$n.json 2>&1 || exit 1
done
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 --envs 2048 > ../gpurun_out/r04_v3_stamps_team_2048.txt 2>&1)
echo rc=$?
