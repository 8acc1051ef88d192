# round-3 Chamfer iteration: GPU tests, same-box A/B of the builds, stamps
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_chamfer_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/ab_chamfer.sh > gpurun_out/$T/ab_chamfer.txt 2>&1 || { echo abc failed; tail gpurun_out/$T/ab_chamfer.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab_chamfer.txt
timeout -k 10 200 python -u tools/stamp_filt.py fused 7 > gpurun_out/$T/stamps_fused.txt 2>&1 || { echo stamps failed; tail gpurun_out/$T/stamps_fused.txt; exit 1; }
grep -E "fused variant|forward|wait|loads|grads|ties|scan|proof|rescan" gpurun_out/$T/stamps_fused.txt
