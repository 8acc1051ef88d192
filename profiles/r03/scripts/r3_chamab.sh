# Chamfer iteration: GPU parity tests of the Chamfer paths (default build),
# same-box A/B of the one-launch step across builds, and each build's bench
# line without the CPU leg (tag = $1)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
L=3d-pointcloudreconstruction_amd/lib
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_chamfer_gpu.py tests/test_metrics_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo tests failed; grep -E "FAILED|^E " gpurun_out/$T/pytest.log | head -30; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/ab_chamfer.sh > gpurun_out/$T/ab_chamfer.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab_chamfer.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab_chamfer.txt
for lib in $L/libpcm_hip_v*.so $L/libpcm_hip.so; do
  b=$(basename $lib .so)
  PCM_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu > gpurun_out/$T/bench_$b.json 2> gpurun_out/$T/bench_$b.err || { echo bench failed; tail gpurun_out/$T/bench_$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/bench_$b.json')); print('$b', round(d['value']/1e12,3), 'e12 pairs/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_us'],2), 'fwd_loss', round(d['two_launch']['fwd_loss_us'],2), 'fp16 fwd', round(d['dense_fp16']['fwd_us'],1), 'emd c3', round(d['emd']['ms_per_forward']*1e3,1), 'train', round(d['emd_training_call']['ms_per_forward'],2))"
done
