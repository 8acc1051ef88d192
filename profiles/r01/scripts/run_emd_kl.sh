set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/emdkl
L=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_kl64.so
PCM_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_emd_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/emdkl/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/emdkl/pytest.log; exit 1; }
tail -2 gpurun_out/emdkl/pytest.log
PCM_HIP_LIB=$L timeout -k 10 240 python -u tools/tune_emd_train.py > gpurun_out/emdkl/tune.txt 2>&1 || { echo tune failed; tail gpurun_out/emdkl/tune.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/emdkl/tune.txt
