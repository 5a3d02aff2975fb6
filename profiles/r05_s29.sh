# round 5, GPU session 29: the driver's command three times with the zero-op action fast path in
# step_async, then once more under the HIP runtime API trace (window attribution)
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3; do timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s29_driver_$k.json 2>&1 || exit 1; done && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/r05_s29 -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT"/gpurun_out/r05_s29_bench_prof.json 2>&1) && \
python layered-safe-marl_amd/tools/window_attrib.py "$(find /tmp/r05_s29 -name '*kernel_trace.csv' | head -n1)" "$(find /tmp/r05_s29 -name '*hip_api_trace.csv' | head -n1)" > gpurun_out/r05_s29_window_attrib.txt
echo rc=$?
