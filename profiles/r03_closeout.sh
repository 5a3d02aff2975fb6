#!/bin/bash
# Round-3 close-out profiles (run on the GPU box from the repo root via gpurun):
#   bash profiles/r03_closeout.sh
# 1. the driver's 20-step command under rocprofv3 --kernel-trace, reduced by tools/boundary_trace.py;
# 2. reset-step cost A/B (product vs LSM_XP_SCEN_PERWAVE): kernel traces of a 600-step config-3 run,
#    lsm.pmc launches lists the slowest launches (the auto-reset steps);
# 3. profiles/collect.sh for config 2 (kernel stats, PMC traffic, SQ counters).
set -o pipefail
R=$(pwd) && export TMPDIR=/tmp && \
mkdir -p /tmp/bt && (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/bt -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03_v19_bt_bench.json 2> $R/gpurun_out/r03_v19_bt_bench.err) && \
python layered-safe-marl_amd/tools/boundary_trace.py $(find /tmp/bt -name "*kernel_trace.csv" | head -n1) --steps 20 > gpurun_out/r03_v19_config3_boundary_window.txt 2>&1 && \
cp $(find /tmp/bt -name "*kernel_stats.csv" | head -n1) gpurun_out/r03_v19_config3_boundary_kernel_stats.csv && \
for V in base scenwave; do L=$R/layered-safe-marl_amd/csrc/liblsm_rollout.so; [ $V = scenwave ] && L=$R/layered-safe-marl_amd/csrc/liblsm_rollout_scenwave.so; mkdir -p /tmp/rc_$V && (cd /tmp && LSM_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/rc_$V -o run --output-format csv -- python3 $R/bench.py --config 3 --steps 600 --warmup 20 --no-cpu-baseline > $R/gpurun_out/r03_v19_rc_$V.json 2>&1) && (cd $R/layered-safe-marl_amd && python -m lsm.pmc launches /tmp/rc_$V --kernel "lsm::rollout") > gpurun_out/r03_v19_reset_$V.json || exit 1; done && \
timeout -k 10 600 bash profiles/collect.sh r03 2 > gpurun_out/r03_collect_c2.log 2>&1
