# round 6, GPU session 14: HBM traffic of process_adj's kernels on the final build (config 3): separate
# FETCH_SIZE / WRITE_SIZE passes on the edge kernels and the scan (bench --edges runs the count-pass and
# the one-pass call on the same adjacency; the one-pass call is offsets init + scan + emit)
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p /tmp/ep_$C
  echo "$(date +%T) pass $C"
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "edge_|offsets_init|scan" -d /tmp/ep_$C -o run --output-format csv \
     -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > $R/gpurun_out/r06_s14_edges_pmc_$C.log 2>&1) || exit 3
done
cd layered-safe-marl_amd
for K in edge_count_kernel edge_emit_kernel offsets_init_kernel init_lookback_scan_state scan_impl; do
  echo "== $K"; python -m lsm.pmc counters /tmp/ep_FETCH_SIZE /tmp/ep_WRITE_SIZE --kernel $K
done > $R/gpurun_out/r06_s14_edges_traffic.txt 2>&1
echo rc=$?
