set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/emdtail
timeout -k 10 300 python -u -m pytest tests/test_emd_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/emdtail/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/emdtail/pytest.log; exit 1; }
tail -2 gpurun_out/emdtail/pytest.log
for t in 0 1 4 16; do
  lib=3d-pointcloudreconstruction_amd/lib/libpcm_hip_bs$t.so
  [ $t = 4 ] && lib=3d-pointcloudreconstruction_amd/lib/libpcm_hip.so
  echo "== block-scan max $t" >> gpurun_out/emdtail/tune.txt
  PCM_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/tune_emd_train.py >> gpurun_out/emdtail/tune.txt 2>&1 || { echo tune failed; tail gpurun_out/emdtail/tune.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/emdtail/tune.txt
