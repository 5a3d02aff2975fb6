#!/bin/bash
# Reset-step cost, MT19937 replay vs Philox fast mode (run on the GPU box from the repo root):
#   bash profiles/reset_cost.sh r02 3
# rocprofv3 --kernel-trace of bench.py for each reset stream; lsm.pmc launches lists the slowest
# launches (the auto-reset steps) next to the median step.
set -euo pipefail
ROUND=${1:-r02}
CFG=${2:-3}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/reset_${ROUND}_c${CFG}
mkdir -p "$OUT"
export TMPDIR=/tmp
for RNG in mt19937 philox; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$RNG" -o run --output-format csv \
      -- python3 "$ROOT"/bench.py --config "$CFG" --steps 600 --warmup 20 --no-cpu-baseline --rng $RNG \
      > "$OUT/$RNG.log" 2>&1)
  (cd "$ROOT/layered-safe-marl_amd" && python -m lsm.pmc launches "$OUT/$RNG" --kernel "lsm::rollout") \
      > "$ROOT/gpurun_out/${ROUND}_config${CFG}_reset_${RNG}.json"
done
echo done
