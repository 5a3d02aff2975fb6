# round 5, GPU session 39: process_adj with the one-workgroup offsets scan, coalesced loads + LDS tiles (new) vs hipcub's scan
# (old = the shipped library): edge tests, A/B of bench --edges, kernel trace of the new one
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export LSM_LIB_AB=1
timeout -k 10 400 python -u -m pytest tests/test_edges.py -m gpu -x -q --timeout 200 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/r05_s39_tests_edges.txt 2>&1 && \
for rep in 1 2; do
  for V in new old; do
    L=$R/layered-safe-marl_amd/csrc/liblsm_rollout.so; [ $V = old ] && L=$R/layered-safe-marl_amd/csrc/liblsm_rollout_old.so
    LSM_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges \
       > gpurun_out/r05_s39_edges_${V}_$rep.json 2>&1 || exit 3
    echo "$V $rep done"
  done
done && \
mkdir -p /tmp/et && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/et -o run --output-format csv \
   -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > $R/gpurun_out/r05_s39_edges_trace_bench.json 2>&1) && \
cp "$(find /tmp/et -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_s39_edges_kernel_stats.csv
echo rc=$?
