# EMD per-iteration diagnostics (config 3 and the training call) + fused Chamfer stamps
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/emd_diag.py --per-iter > gpurun_out/$T/emd_diag_c3.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_diag_c3.txt; exit 1; }
head -3 gpurun_out/$T/emd_diag_c3.txt
timeout -k 10 200 python -u tools/emd_diag.py --train > gpurun_out/$T/emd_diag_train.txt 2>&1 || { echo diag train failed; tail gpurun_out/$T/emd_diag_train.txt; exit 1; }
head -3 gpurun_out/$T/emd_diag_train.txt
timeout -k 10 200 python -u tools/stamp_filt.py fused 7 > gpurun_out/$T/stamps_fused.txt 2>&1 || { echo stamps failed; tail gpurun_out/$T/stamps_fused.txt; exit 1; }
cat gpurun_out/$T/stamps_fused.txt
echo DIAGDONE
