# round-3 EMD iteration: GPU tests, same-box A/B of the builds, training diag
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_emd_gpu.py tests/test_train_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for v in 3d-pointcloudreconstruction_amd/lib/libpcm_hip_v*.so; do
  [ -f "$v" ] || continue
  PCM_HIP_LIB=$PWD/$v timeout -k 10 900 python -u -m pytest tests/test_emd_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_$(basename $v .so).log 2>&1 || { echo tests $v failed; grep -E "FAILED|^E " gpurun_out/$T/pytest_$(basename $v .so).log | head -20; exit 1; }
  echo "$(basename $v): $(tail -1 gpurun_out/$T/pytest_$(basename $v .so).log)"
done
bash tools/ab_emd.sh > gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab.txt
for lib in 3d-pointcloudreconstruction_amd/lib/libpcm_hip.so 3d-pointcloudreconstruction_amd/lib/libpcm_hip_v*.so; do
  [ -f "$lib" ] || continue
  b=$(basename $lib .so)
  PCM_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > gpurun_out/$T/emd_diag_train_$b.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_diag_train_$b.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/emd_diag_train_$b.txt
done
