set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
L=$PWD/3d-pointcloudreconstruction_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_chamfer_grid_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_grid.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_grid.py > $O/ab_grid.txt 2>&1 && \
PCM_HIP_LIB=$L/libpcm_hip.so timeout -k 10 120 python -u tools/ab_emd.py > $O/ab_emd.txt 2>&1 && \
PCM_HIP_LIB=$L/libpcm_hip_v1slot.so timeout -k 10 120 python -u tools/ab_emd.py >> $O/ab_emd.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o grid --output-format csv -- python3 tools/ab_grid.py > $O/kt.log 2>&1
