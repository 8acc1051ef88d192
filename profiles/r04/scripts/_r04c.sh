set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
L=$PWD/3d-pointcloudreconstruction_amd/lib
timeout -k 10 120 ./tools/hybrid_probe > $O/hybrid_probe.txt 2>&1 && \
PCM_HIP_LIB=$L/libpcm_hip_stamps.so timeout -k 10 300 python -u tools/emd_diag.py --per-iter > $O/emd_diag_c3_stamps.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_emd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_emd.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_chamfer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "loss_grad" > $O/pytest_lossgrad.txt 2>&1 && \
for r in 1 2; do for lib in $L/libpcm_hip_base.so $L/libpcm_hip.so; do
  PCM_HIP_LIB=$lib timeout -k 10 120 python -u tools/ab_emd.py >> $O/ab_emd.txt 2>&1 || exit 1
done; done && \
PCM_HIP_LIB=$L/libpcm_hip_base.so timeout -k 10 300 python -u tools/ab_chamfer.py > $O/ab_chamfer_base.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_chamfer.py > $O/ab_chamfer.txt 2>&1
