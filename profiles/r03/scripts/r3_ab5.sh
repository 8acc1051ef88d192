# round-3 iteration: GPU tests (Chamfer + EMD), same-box A/B of the builds, stamps
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
L=$PWD/3d-pointcloudreconstruction_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_chamfer_gpu.py tests/test_emd_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/ab_chamfer.sh > gpurun_out/$T/ab_chamfer.txt 2>&1 || { echo abc failed; tail gpurun_out/$T/ab_chamfer.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab_chamfer.txt
bash tools/ab_emd.sh > gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab.txt
for v in stamps stamps_fma; do
  [ -f $L/libpcm_hip_$v.so ] || continue
  echo "== $v"
  PCM_STAMPS_LIB=$L/libpcm_hip_$v.so timeout -k 10 200 python -u tools/stamp_filt.py fused 7 > gpurun_out/$T/stamps_$v.txt 2>&1 || { echo stamps failed; tail gpurun_out/$T/stamps_$v.txt; exit 1; }
  grep -E "fused variant|forward|scan|proof|rescan" gpurun_out/$T/stamps_$v.txt
done
timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > gpurun_out/$T/emd_diag_train.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_diag_train.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/emd_diag_train.txt
