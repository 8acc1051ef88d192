# EMD config-3 per-iteration timers with the B1 sub-phase stamps (profiling build)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
PCM_HIP_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so timeout -k 10 200 python -u tools/emd_diag.py --per-iter > gpurun_out/$T/emd_stamps_c3.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_stamps_c3.txt; exit 1; }
grep -v "^    it" gpurun_out/$T/emd_stamps_c3.txt
timeout -k 10 200 python -u tools/emd_diag.py --per-iter > gpurun_out/$T/emd_c3.txt 2>&1 || { echo diag failed; exit 1; }
grep -v "^    it" gpurun_out/$T/emd_c3.txt
