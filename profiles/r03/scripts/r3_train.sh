# config-4 training step, three runs of the same command, per-step EMD work
# logged (tools/bench_train.py) -- the step-time spread against the auction's
# iterations (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_train.py --steps 10 --warmup 3 > gpurun_out/$T/bench_train_$r.json 2> gpurun_out/$T/bench_train_$r.err || { echo train $r failed; tail gpurun_out/$T/bench_train_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/$T/bench_train_$r.json')); print($r, round(d['ms_per_step'],2), 'ms/step; loss path', round(d['loss_path_ms'],2), [(round(s['step_ms'],1), s['iterations_with_bidders'], round(s['emd_fwd_ms'],2)) for s in d['per_step']])"
done
