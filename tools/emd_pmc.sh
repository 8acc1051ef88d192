#!/usr/bin/env bash
# instruction-cache and issue counters of the config-3 auction (masters only)
set -euo pipefail
OUT=${1:-gpurun_out/emd_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ \
    -d "$OUT/ic" -o ic --output-format csv -- python3 tools/emd_pmc_driver.py > "$OUT/ic.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_WAIT_ANY SQ_IFETCH -d "$OUT/sq" -o sq --output-format csv \
    -- python3 tools/emd_pmc_driver.py > "$OUT/sq.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU \
    SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d "$OUT/sq2" -o sq2 --output-format csv \
    -- python3 tools/emd_pmc_driver.py > "$OUT/sq2.log" 2>&1
echo done
