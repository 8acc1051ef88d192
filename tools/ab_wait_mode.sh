#!/bin/bash
# Host wait mode of the bench's timed region: the driver's command under the
# runtime's default (interrupt-driven) waits, with ROCclr's active-wait window,
# and with HSA signal polling.  Prints step, kernel and step - kernel (us).
# usage: bash tools/ab_wait_mode.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p "$O"
for r in 1 2; do
  for mode in default active poll; do
    case $mode in
      default) E="" ;;
      active) E="ROC_ACTIVE_WAIT_TIMEOUT=1000" ;;
      poll) E="HSA_ENABLE_INTERRUPT=0" ;;
    esac
    env $E timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_$mode$r.json" 2> "$O/bench_$mode$r.err" || exit 1
    python3 -c "
import json,sys; d=json.load(open('$O/bench_$mode$r.json')); r=d['roofline']
print('%-8s step %.3f us  kernel %.3f us  step-kernel %.3f us' % ('$mode', d['ms_per_step']*1e3, r['kernel_us'], d['ms_per_step']*1e3 - r['kernel_us']))" | tee -a "$O/wait_mode.txt"
  done
done
