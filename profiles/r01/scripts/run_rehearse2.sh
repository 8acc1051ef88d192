set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rehearse
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-dense --no-icp --dist-backend gloo > gpurun_out/rehearse/bench2.json 2> gpurun_out/rehearse/bench2.err || { echo bench2 failed; tail -30 gpurun_out/rehearse/bench2.err; exit 1; }
cat gpurun_out/rehearse/bench2.json | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 tools/bench_train.py --batch 8 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/rehearse/train2.json 2> gpurun_out/rehearse/train2.err || { echo train2 failed; tail -30 gpurun_out/rehearse/train2.err; exit 1; }
cat gpurun_out/rehearse/train2.json
