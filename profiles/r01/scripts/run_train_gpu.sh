set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/train
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/train/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/train/pytest.log; exit 1; }
tail -3 gpurun_out/train/pytest.log
timeout -k 10 300 python -u tools/bench_train.py --batch 16 --steps 5 --warmup 2 > gpurun_out/train/bench_e1.json 2> gpurun_out/train/bench_e1.err || { echo bench failed; tail -20 gpurun_out/train/bench_e1.err; exit 1; }
cat gpurun_out/train/bench_e1.json
