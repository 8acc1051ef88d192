set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
L=$PWD/3d-pointcloudreconstruction_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_chamfer_grid_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_grid.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_grid.py > $O/ab_grid.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_chamfer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_chamfer.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_emd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_emd.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_chamfer.py > $O/ab_chamfer.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_chamfer.py >> $O/ab_chamfer.txt 2>&1 && \
for r in 1 2; do for lib in $L/libpcm_hip_base.so $L/libpcm_hip_v1slot.so $L/libpcm_hip.so; do
  PCM_HIP_LIB=$lib timeout -k 10 120 python -u tools/ab_emd.py >> $O/ab_emd.txt 2>&1 || exit 1
done; done && \
PCM_HIP_LIB=$L/libpcm_hip_stamps.so timeout -k 10 300 python -u tools/stamp_filt.py fused 7 11 12 > $O/stamps_fused.txt 2>&1
