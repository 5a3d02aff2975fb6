# round 6, GPU session 2: why session 1's edge_emit_kernel<4> (masks in registers, selected by
# branches) misplaced edges: per-graph counts / emits vs numpy and the oracle for this build (masks in
# registers, branch-free select), session 1's library (tools/liblsm_rollout_s01.so), the same branchy
# source built alone (tools/liblsm_edges_branchy.so) and round 5's edges code (tools/liblsm_edges_r05.so,
# git HEAD's lsm_edges.hip); plus the v_mov_b64 -> v_mov_b32 write-after-write microtest (the
# compiler emitted that pair in the failing kernel)
set -o pipefail
mkdir -p gpurun_out
T=layered-safe-marl_amd/tools
timeout -k 10 120 ./$T/movb64_hazard > gpurun_out/r06_s02_movb64.txt 2>&1
timeout -k 10 200 python -u $T/edges_check.py $T/liblsm_rollout_s01.so $T/liblsm_edges_branchy.so $T/liblsm_edges_r05.so > gpurun_out/r06_s02_edges_check.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_edges.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s02_tests_edges.txt 2>&1
echo rc=$?
