# round 5, GPU session 31: the driver's command with the window-opening fixes (garbage collection before
# the untimed steps; timing events created before the window) vs the old ordering, alternating, 3 each
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3; do
  LSM_BENCH_OLD_WINDOW=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s31_old_$k.json 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s31_new_$k.json 2>&1 || exit 1
done
echo rc=$?
