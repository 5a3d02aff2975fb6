# round 6, the final tree (summary kernel included): the whole GPU suite, smoke, and the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_tests_final.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke_final.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r06_bench_default_final.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
