#!/bin/bash
# Profile collection for one round (run on the GPU box via gpurun, from the repo root):
#   bash profiles/collect.sh r01 3        (config 5: the workgroup kernel, rollout_block_kernel)
# 1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations);
# 2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction/stall counters) --
#    never combined with any trace domain;
# 3. reduce to profiles/<round>_config<c>_*.txt and profiles/pmc_traffic.json.
set -euo pipefail
ROUND=${1:-r01}
CFG=${2:-3}
ROOT=$(pwd)
OUT=${TMPDIR:-/tmp}/prof_${ROUND}_c${CFG}   # raw traces stay on the box (gpurun_out is capped at 64 MiB)
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --config $CFG --steps 200 --warmup 20 --no-cpu-baseline"
ENVS=$(python -c "import bench; print(bench.CONFIGS[$CFG]['envs'])")
# the step kernel of any variant (rollout_kernel / rollout_team_kernel / rollout_block_kernel);
# bench.py's line names the instantiation (lsm_kernel_name)
KERN="lsm::rollout"

run() {  # run <name> <rocprofv3 args...>
  local name=$1; shift
  echo "$(date +%T) config $CFG: $name ..."   # progress on stdout (a gpurun_out log): no silent minutes
  (cd /tmp && timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT"/$BENCH > "$OUT/$name.log" 2>&1)
  echo "$(date +%T) config $CFG: $name done"
}

run ktrace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM

cd "$ROOT/layered-safe-marl_amd"
python -m lsm.pmc stats "$OUT/ktrace" > "$ROOT/profiles/${ROUND}_config${CFG}_kernel_stats.txt"
python -m lsm.pmc launches "$OUT/ktrace" --kernel "$KERN" > "$ROOT/profiles/${ROUND}_config${CFG}_launches.json"
cp "$(find "$OUT/ktrace" -name '*kernel_stats.csv' | head -n1)" "$ROOT/profiles/${ROUND}_config${CFG}_kernel_stats.csv"
python -m lsm.pmc traffic "$OUT/fetch" "$OUT/write" --config "$CFG" --envs "$ENVS" --kernel "$KERN" --round "$ROUND" \
    --out "$ROOT/profiles/pmc_traffic.json" > "$ROOT/profiles/${ROUND}_config${CFG}_traffic.json"
python -m lsm.pmc counters "$OUT/sq1" "$OUT/sq2" --kernel "$KERN" > "$ROOT/profiles/${ROUND}_config${CFG}_sq_counters.txt"
cp "$ROOT/profiles/"${ROUND}_config${CFG}_* "$ROOT/profiles/pmc_traffic.json" "$ROOT/gpurun_out/"
echo done
