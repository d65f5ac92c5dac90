# full GPU suite + smoke (the driver's round-end steps), logs under gpurun_out/
set -o pipefail
tag=${1:-all}
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/r04_${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r04_${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_${tag}_smoke.log 2>&1
