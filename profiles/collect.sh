#!/bin/bash
# Profile collection for one round (run on the GPU box via gpurun, from the repo root):
#   bash profiles/collect.sh r01 3        (config 5: the workgroup kernel, rollout_block_kernel)
# 1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations);
# 2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction/stall counters) --
#    never combined with any trace domain;
# 3. reduce to profiles/<round>_config<c>_*.txt and profiles/pmc_traffic.json.
set -uo pipefail
ROUND=${1:-r01}
CFG=${2:-3}
ROOT=$(pwd)
OUT=${TMPDIR:-/tmp}/prof_${ROUND}_c${CFG}   # raw traces stay on the box (gpurun_out is capped at 64 MiB)
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --config $CFG --steps 200 --warmup 20 --no-cpu-baseline"
# counter passes: counters on the step kernel only (the synthetic-action kernels are not sampled) and
# a shorter window -- per-dispatch counter collection made config 4's FETCH_SIZE pass exceed 100 s
PMCBENCH="bench.py --config $CFG --steps 60 --warmup 20 --no-cpu-baseline"
ENVS=$(python -c "import bench; print(bench.CONFIGS[$CFG]['envs'])")
# the step kernel of any variant (rollout_kernel / rollout_team_kernel / rollout_block_kernel);
# bench.py's line names the instantiation (lsm_kernel_name)
KERN="lsm::rollout"

# A pass that fails or times out ends the GPU work of this script (the remaining passes are skipped,
# what was collected is reduced, the exit status is nonzero). PMC passes get 150 s: a good one takes
# seconds, and a stuck one must end before the box's 180-s silence limit.
run() {  # run <name> <timeout s> <rocprofv3 args...>
  local name=$1; shift
  local limit=$1; shift
  echo "$(date +%T) config $CFG: $name ..."   # progress on stdout (a gpurun_out log): no silent minutes
  local rc=0
  local cmd=$BENCH
  case " $* " in *" --pmc "*) cmd=$PMCBENCH; set -- --kernel-include-regex rollout_ "$@";; esac
  (cd /tmp && timeout -k 10 "$limit" rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT"/$cmd > "$OUT/$name.log" 2>&1) || rc=$?
  echo "$(date +%T) config $CFG: $name done rc=$rc"
  (grep -v "^W20\|^E20\|amdgpu.ids" "$OUT/$name.log" | tail -n 4 | cut -c1-300) || true
  return $rc
}

ok=1
run ktrace 300 --kernel-trace --stats || ok=0
[ $ok = 1 ] && { run fetch 150 --pmc FETCH_SIZE || ok=0; }
[ $ok = 1 ] && { run write 150 --pmc WRITE_SIZE || ok=0; }
[ $ok = 1 ] && { run sq1 150 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || ok=0; }
[ $ok = 1 ] && { run sq2 150 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM || ok=0; }

cd "$ROOT/layered-safe-marl_amd"
if [ -d "$OUT/ktrace" ]; then
  python -m lsm.pmc stats "$OUT/ktrace" > "$ROOT/profiles/${ROUND}_config${CFG}_kernel_stats.txt"
  python -m lsm.pmc launches "$OUT/ktrace" --kernel "$KERN" > "$ROOT/profiles/${ROUND}_config${CFG}_launches.json"
  cp "$(find "$OUT/ktrace" -name '*kernel_stats.csv' | head -n1)" "$ROOT/profiles/${ROUND}_config${CFG}_kernel_stats.csv"
fi
if [ -d "$OUT/fetch" ] && [ -d "$OUT/write" ]; then
  python -m lsm.pmc traffic "$OUT/fetch" "$OUT/write" --config "$CFG" --envs "$ENVS" --kernel "$KERN" --round "$ROUND" \
      --out "$ROOT/profiles/pmc_traffic.json" > "$ROOT/profiles/${ROUND}_config${CFG}_traffic.json"
fi
if [ -d "$OUT/sq1" ] && [ -d "$OUT/sq2" ]; then
  python -m lsm.pmc counters "$OUT/sq1" "$OUT/sq2" --kernel "$KERN" > "$ROOT/profiles/${ROUND}_config${CFG}_sq_counters.txt"
fi
cp "$ROOT/profiles/"${ROUND}_config${CFG}_* "$ROOT/profiles/pmc_traffic.json" "$ROOT/gpurun_out/" 2>/dev/null
echo "done ok=$ok"
[ $ok = 1 ]
