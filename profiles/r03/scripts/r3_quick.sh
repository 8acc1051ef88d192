# selected gpu tests (-k expression $2), smoke, bench (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$2" > gpurun_out/$T/pytest_sel.log 2>&1
rc=$?
tail -3 gpurun_out/$T/pytest_sel.log
if [ $rc -ne 0 ]; then grep -E "FAILED|^E " gpurun_out/$T/pytest_sel.log | head -30; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo bench failed; tail gpurun_out/$T/bench.err; exit 1; }
head -c 600 gpurun_out/$T/bench.json; echo
