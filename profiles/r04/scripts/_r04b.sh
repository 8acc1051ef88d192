set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 120 ./tools/dispatch_probe > $O/dispatch_probe.txt 2>&1 && \
PCM_HIP_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so timeout -k 10 300 python -u tools/stamp_filt.py fused 7 > $O/stamps_fused7.txt 2>&1 && \
timeout -k 10 300 python -u tools/emd_diag.py --hist --per-iter --by-nu > $O/emd_diag_c3.txt 2>&1 && \
timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > $O/emd_diag_train.txt 2>&1 || exit 1
L=$PWD/3d-pointcloudreconstruction_amd/lib
for r in 1 2; do for lib in $L/libpcm_hip.so $L/libpcm_hip_cw4.so $L/libpcm_hip_cw8.so; do
  PCM_HIP_LIB=$lib timeout -k 10 120 python -u tools/ab_emd.py >> $O/ab_chainw.txt 2>&1 || exit 1
done; done
