set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_chamfer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_chamfer.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_chamfer.py > $O/ab_chamfer.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_chamfer.py >> $O/ab_chamfer.txt 2>&1
