set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/traincl
timeout -k 10 300 python -u tools/bench_train.py --batch 16 --steps 10 --warmup 3 > gpurun_out/traincl/nchw.json 2> gpurun_out/traincl/nchw.err || { echo nchw failed; tail -20 gpurun_out/traincl/nchw.err; exit 1; }
timeout -k 10 300 python -u tools/bench_train.py --batch 16 --steps 10 --warmup 3 --channels-last > gpurun_out/traincl/nhwc.json 2> gpurun_out/traincl/nhwc.err || { echo nhwc failed; tail -20 gpurun_out/traincl/nhwc.err; exit 1; }
cat gpurun_out/traincl/nchw.json gpurun_out/traincl/nhwc.json
