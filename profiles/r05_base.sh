# round 5, GPU session 1: HEAD baseline -- default bench (config 3), team stamps (config 3 and 2),
# and the rocprofv3 kernel trace of the driver's exact command (20 steps, warmup 5)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r05_base_bench_c3.json 2>&1 && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 120 > ../gpurun_out/r05_base_stamps_c3.txt 2>&1) && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --config 2 --steps 120 > ../gpurun_out/r05_base_stamps_c2.txt 2>&1) && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_drv -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT"/gpurun_out/r05_base_driver_bench.json 2>&1) && \
python layered-safe-marl_amd/tools/boundary_trace.py "$(find /tmp/r05_drv -name '*kernel_trace.csv' | head -n1)" > gpurun_out/r05_base_driver_window.txt && \
cp "$(find /tmp/r05_drv -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_base_driver_kernel_stats.csv
echo rc=$?
