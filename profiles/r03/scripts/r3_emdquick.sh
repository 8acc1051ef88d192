# EMD iteration: GPU parity tests of the EMD paths, then the config-3 and
# training-call diagnostics of the in-tree build (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_emd_gpu.py tests/test_train_gpu.py tests/test_metrics_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -30; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 200 python -u tools/emd_diag.py > gpurun_out/$T/emd_c3.txt 2>&1 || { echo diag failed; tail gpurun_out/$T/emd_c3.txt; exit 1; }
grep -v "amdgpu.ids" gpurun_out/$T/emd_c3.txt
timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > gpurun_out/$T/emd_train.txt 2>&1 || { echo diag failed; exit 1; }
grep -v "amdgpu.ids" gpurun_out/$T/emd_train.txt
