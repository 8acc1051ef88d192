L=$PWD/3d-pointcloudreconstruction_amd/lib
for r in 1 2; do
  PCM_HIP_LIB=$L/libpcm_hip_base.so timeout -k 10 120 python -u tools/ab_emd.py || exit 1
  PCM_HIP_LIB=$L/libpcm_hip.so timeout -k 10 120 python -u tools/ab_emd.py || exit 1
done
