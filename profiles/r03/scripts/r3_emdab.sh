# EMD-only A/B, four rounds (the training call varies +-2 % between calls)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_emd_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for r in 1 2; do
  bash tools/ab_emd.sh >> gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/$T/ab.txt
