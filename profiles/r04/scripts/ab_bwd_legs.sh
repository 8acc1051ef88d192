# same-box A/B of the backward-carrying bench legs for lib/libpcm_hip_base.so and the in-tree build
L=$PWD/3d-pointcloudreconstruction_amd/lib
mkdir -p gpurun_out/r04za
for r in 1 2; do
  for lib in $L/libpcm_hip_base.so $L/libpcm_hip.so; do
    PCM_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --no-emd --no-icp > gpurun_out/r04za/bench_$(basename $lib .so)_$r.json 2>> gpurun_out/r04za/err.log || exit 1
  done
done
