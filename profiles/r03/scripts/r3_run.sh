# round-3 GPU check: gpu tests (verbose log), smoke, bench (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:randomly > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/$T/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/$T/pytest_gpu.log | head -30; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo bench failed; tail gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json | head -c 1500
echo ALLDONE
