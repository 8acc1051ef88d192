# round-3 profiles of the final library (tag = $1): rocprofv3 kernel trace of
# the bench command + one counter pass per group (tools/pmc_passes.sh), and
# the EMD config-3 auction counter passes (tools/emd_pmc.sh)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
bash tools/pmc_passes.sh gpurun_out/$T/pmc > gpurun_out/$T/pmc_passes.log 2>&1 || { echo pmc failed; tail gpurun_out/$T/pmc_passes.log; exit 1; }
tail -1 gpurun_out/$T/pmc_passes.log
bash tools/emd_pmc.sh gpurun_out/$T/emd_pmc > gpurun_out/$T/emd_pmc.log 2>&1 || { echo emd pmc failed; tail gpurun_out/$T/emd_pmc.log; exit 1; }
tail -1 gpurun_out/$T/emd_pmc.log
find gpurun_out/$T -name "*stats.csv" | head
echo ALLDONE
