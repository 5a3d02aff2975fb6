# round 5, final profiles of the shipped build: configs 3, 2, 4, 5 (kernel trace, PMC traffic, SQ counters)
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 3 > gpurun_out/r05_final_a_c3.log 2>&1 && \
bash profiles/collect.sh r05 2 > gpurun_out/r05_final_a_c2.log 2>&1 && \
bash profiles/collect.sh r05 4 > gpurun_out/r05_final_a_c4.log 2>&1 && \
bash profiles/collect.sh r05 5 > gpurun_out/r05_final_a_c5.log 2>&1
echo rc=$?
