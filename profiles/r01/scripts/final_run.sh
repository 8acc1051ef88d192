set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo bench failed; tail gpurun_out/final/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final/kt -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/final/kt_bench.log 2>&1 || { echo rocprof failed; tail gpurun_out/final/kt_bench.log; exit 1; }
find gpurun_out/final/kt -name "*stats*"
echo ALLDONE
