#!/usr/bin/env bash
# rocprofv3 passes for the round's profiles (run ON the GPU box from the repo
# root, e.g. via gpurun).  Kernel trace + stats of the bench command, then one
# counter pass per group (FETCH_SIZE and WRITE_SIZE cannot share a pass on
# gfx950; counters never combined with trace domains).  Every GPU step has its
# own time limit and the chain stops at the first failure.
#   usage: tools/pmc_passes.sh OUTDIR
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
PROG="tools/profile_kernels.py"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o bench --output-format csv \
    -- python3 bench.py --steps 50 --warmup 10 --no-cpu > "$OUT/kt_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_eager" -o eager --output-format csv \
    -- python3 "$PROG" > "$OUT/kt_eager.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
    -- python3 "$PROG" > "$OUT/fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
    -- python3 "$PROG" > "$OUT/write.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/l2" -o l2 --output-format csv \
    -- python3 "$PROG" > "$OUT/l2.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/sq" -o sq --output-format csv \
    -- python3 "$PROG" > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/sq_emdtrain" -o sq --output-format csv \
    -- python3 "$PROG" emdtrain > "$OUT/sq_emdtrain.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/kt_emdtrain" -o kt --output-format csv \
    -- python3 "$PROG" emdtrain > "$OUT/kt_emdtrain.log" 2>&1
echo "pmc passes done"
