# config 4 (airtaxi N = 16): per-step time vs envs (1, 2, 4 rounds of resident workgroups), team stamps
set -o pipefail
mkdir -p gpurun_out
for n in 2048 4096 8192; do
  timeout -k 10 200 python -u bench.py --config 4 --envs $n --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r04_v3_c4_envs_$n.json 2>&1 || exit 1
done
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --config 4 --steps 60 > ../gpurun_out/r04_v3_stamps_team_c4.txt 2>&1)
echo rc=$?
