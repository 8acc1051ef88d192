set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python -u tools/seed_spread.py > $O/seed_spread.txt 2>&1
