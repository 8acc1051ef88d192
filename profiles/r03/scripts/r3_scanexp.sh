# scan-loop limiter experiment: stamps of the fused kernel with the scan's
# LDS reads removed / its arithmetic removed (timing-only builds)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out/$T
L=$PWD/3d-pointcloudreconstruction_amd/lib
for v in stamps stamps_nolds stamps_novalu; do
  echo "== $v"
  PCM_STAMPS_LIB=$L/libpcm_hip_$v.so timeout -k 10 200 python -u tools/stamp_filt.py fused 7 > gpurun_out/$T/stamps_$v.txt 2>&1 || { echo stamps failed; tail gpurun_out/$T/stamps_$v.txt; exit 1; }
  grep -E "fused variant|forward|wait|loads|grads|ties|scan|proof|rescan" gpurun_out/$T/stamps_$v.txt
done
