# EMD A/B of the in-tree builds (base = previous source, v* variants, default)
# plus the config-3 sub-phase stamps of the profiling build when present (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
L=3d-pointcloudreconstruction_amd/lib
mkdir -p gpurun_out/$T
bash tools/ab_emd.sh > gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab.txt
if [ -f $L/libpcm_hip_stamps.so ]; then
  PCM_HIP_LIB=$PWD/$L/libpcm_hip_stamps.so timeout -k 10 200 python -u tools/emd_diag.py > gpurun_out/$T/emd_stamps_c3.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_stamps_c3.txt; exit 1; }
  grep -v "amdgpu.ids" gpurun_out/$T/emd_stamps_c3.txt
fi
for lib in $L/libpcm_hip_v*.so $L/libpcm_hip.so; do
  [ -f "$lib" ] || continue
  PCM_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/emd_diag.py > gpurun_out/$T/emd_c3_$(basename $lib .so).txt 2>&1 || { echo diag failed; exit 1; }
  grep -v "amdgpu.ids" gpurun_out/$T/emd_c3_$(basename $lib .so).txt
done
