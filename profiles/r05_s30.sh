# round 5, GPU session 30: the driver's command with host waits spinning (LSM_HOST_SPIN=1:
# hipDeviceScheduleSpin) vs the default, alternating, three runs each
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s30_default_$k.json 2>&1 || exit 1
  LSM_HOST_SPIN=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s30_spin_$k.json 2>&1 || exit 1
done
echo rc=$?
