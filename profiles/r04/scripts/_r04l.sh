set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_chamfer_grid_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_grid.txt 2>&1 && \
timeout -k 10 300 python -u tools/grid_diag.py > $O/grid_diag.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_grid.py > $O/ab_grid.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04l/kt -o grid --output-format csv -- python3 tools/grid_diag.py > gpurun_out/r04l/kt.log 2>&1
