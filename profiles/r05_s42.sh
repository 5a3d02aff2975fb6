# round 5, GPU session 42: HBM traffic of process_adj's count and emit kernels (config 3, shipped build):
# separate FETCH_SIZE / WRITE_SIZE passes on the edge kernels only -- do the emit pass's re-reads of the
# adjacency come from L2 / MALL?
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p /tmp/ep_$C
  echo "$(date +%T) pass $C"
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex edge_ -d /tmp/ep_$C -o run --output-format csv \
     -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > $R/gpurun_out/r05_s42_edges_pmc_$C.log 2>&1) || exit 3
done
cd layered-safe-marl_amd
for K in edge_count_kernel edge_emit_kernel; do
  echo "== $K"; python -m lsm.pmc counters /tmp/ep_FETCH_SIZE /tmp/ep_WRITE_SIZE --kernel $K
done > $R/gpurun_out/r05_s42_edges_traffic.txt 2>&1
echo rc=$?
