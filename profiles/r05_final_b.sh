# round 5, final profiles B: the same for configs 4 and 5
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 4 > gpurun_out/r05_final_b_c4.log 2>&1 && \
bash profiles/collect.sh r05 5 > gpurun_out/r05_final_b_c5.log 2>&1
echo rc=$?
