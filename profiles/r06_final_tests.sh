# round 6, final build: the whole GPU suite (the driver's command) and smoke()
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
