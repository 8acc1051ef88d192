# EMD seed workgroup-size A/B (lib/libpcm_hip_vs*.so against the default),
# then the seed kernel's own time per build from a rocprofv3 kernel trace
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}
L=$PWD/3d-pointcloudreconstruction_amd/lib
mkdir -p gpurun_out/$T
bash tools/ab_emd.sh > gpurun_out/$T/ab.txt 2>&1 || { echo ab failed; tail gpurun_out/$T/ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/ab.txt
for lib in $L/libpcm_hip_v*.so $L/libpcm_hip.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so)
  PCM_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt_$v -o run -- python3 tools/emd_once.py > gpurun_out/$T/kt_$v.log 2>&1 || { echo rocprof failed; tail gpurun_out/$T/kt_$v.log; exit 1; }
  f=$(find gpurun_out/$T/kt_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -o '"void (anonymous namespace)::emd_seed_kernel[^"]*",[0-9]*,[0-9]*,[0-9.]*' $f | awk -F, '{print "seed avg ns", $4}') $(grep -o '"void (anonymous namespace)::emd_auction_kernel[^"]*",[0-9]*,[0-9]*,[0-9.]*' $f | awk -F, '{print "auction avg ns", $4}')"
done
