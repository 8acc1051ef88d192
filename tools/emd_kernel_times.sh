# rocprofv3 kernel-trace stats of tools/emd_once.py (EMD config 3) for every
# in-tree EMD build (lib/libpcm_hip_base.so, lib/libpcm_hip_v*.so, the default)
L=$PWD/3d-pointcloudreconstruction_amd/lib
export TMPDIR=/tmp
for lib in $L/libpcm_hip_base.so $L/libpcm_hip_v*.so $L/libpcm_hip.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so)
  PCM_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$v -o run -- python3 tools/emd_once.py > gpurun_out/kt_$v.log 2>&1 || exit 1
done
