# one rocprofv3 counter pass over the EMD seed kernel (tools/emd_once.py,
# config 3) for the base and default builds
L=$PWD/3d-pointcloudreconstruction_amd/lib
export TMPDIR=/tmp
for lib in $L/libpcm_hip_base.so $L/libpcm_hip.so; do
  v=$(basename $lib .so)
  PCM_HIP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex emd_seed --output-format csv -d gpurun_out/pmc_$v -o run -- python3 tools/emd_once.py > gpurun_out/pmc_$v.log 2>&1 || exit 1
done
