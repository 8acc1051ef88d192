# round-3 iteration: Chamfer + EMD GPU tests, A/B of the builds, EMD training
# diag per build, Chamfer stamps
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_chamfer_gpu.py tests/test_emd_gpu.py tests/test_train_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/ab_chamfer.sh > gpurun_out/$T/ab_chamfer.txt 2>&1 || { echo abc failed; tail gpurun_out/$T/ab_chamfer.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab_chamfer.txt
bash tools/ab_emd.sh > gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab.txt
for lib in 3d-pointcloudreconstruction_amd/lib/libpcm_hip.so 3d-pointcloudreconstruction_amd/lib/libpcm_hip_v*.so; do
  [ -f "$lib" ] || continue
  b=$(basename $lib .so)
  PCM_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > gpurun_out/$T/emd_diag_train_$b.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_diag_train_$b.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/emd_diag_train_$b.txt
done
timeout -k 10 200 python -u tools/stamp_filt.py fused 7 > gpurun_out/$T/stamps_fused.txt 2>&1 || { echo stamps failed; tail gpurun_out/$T/stamps_fused.txt; exit 1; }
grep -E "fused variant|forward|wait|loads|grads|ties|scan|proof|rescan|stage" gpurun_out/$T/stamps_fused.txt
