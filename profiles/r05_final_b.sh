# round 5, final profiles B: config 5 (kernel trace, PMC traffic, SQ counters), then the driver's exact
# command under rocprofv3 (kernel trace -> window attribution)
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 5 > gpurun_out/r05_final_b_c5.log 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_fdrv -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT"/gpurun_out/r05_driver_bench_prof.json 2>&1) && \
python layered-safe-marl_amd/tools/boundary_trace.py "$(find /tmp/r05_fdrv -name '*kernel_trace.csv' | head -n1)" > gpurun_out/r05_driver_window.txt && \
cp "$(find /tmp/r05_fdrv -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_driver_kernel_stats.csv
echo rc=$?
