# round 5, GPU session 15 (second try: 4 counters; 8 incl. SQC_ hung past 180 s): instruction-cache and issue counters of the config-3 step kernel (PMC passes only)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
OUT=/tmp/prof_s15
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --config 3 --steps 200 --warmup 20 --no-cpu-baseline"
run() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 90 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT"/$BENCH > "$OUT/$name.log" 2>&1)
}
run ic --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES && \
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU && \
run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM && \
(cd layered-safe-marl_amd && python -m lsm.pmc counters $OUT/ic --kernel lsm::rollout > $ROOT/gpurun_out/r05_s15_icache.txt && \
 python -m lsm.pmc counters $OUT/sq1 $OUT/sq2 --kernel lsm::rollout > $ROOT/gpurun_out/r05_s15_sq.txt)
rc=$?
grep -v '^W20' $OUT/ic.log | tail -n 30 > gpurun_out/r05_s15_ic_log.txt
echo rc=$rc
