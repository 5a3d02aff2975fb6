# round 5, GPU session 28: the driver's 20-step window with the HIP runtime API trace next to the kernel
# trace (no counters): host calls vs kernel execution at the window's edges; and the plain driver command
# three times in a row (run-to-run spread of the wall-clock line)
set -o pipefail
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/r05_s28 -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT"/gpurun_out/r05_s28_bench_prof.json 2>&1) && \
cp "$(find /tmp/r05_s28 -name '*kernel_trace.csv' | head -n1)" gpurun_out/r05_s28_kernel_trace.csv && \
cp "$(find /tmp/r05_s28 -name '*hip_api_trace.csv' | head -n1)" gpurun_out/r05_s28_hip_api_trace.csv && \
for k in 1 2 3; do timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s28_driver_$k.json 2>&1 || exit 1; done
echo rc=$?
