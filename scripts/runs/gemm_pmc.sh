#!/bin/bash
# rocprofv3 counter passes over the elimination GEMM (bench/gemm_probe.py), one pass per run.
#   bash scripts/runs/gemm_pmc.sh <tag> [probe args...]
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
tag=${1:-default}; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
timeout -k 10 120 python3 bench/gemm_probe.py "$@" > "$out/plain.json" 2>/dev/null || exit $?
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES ${MOPS:-SQ_INSTS_VALU_MFMA_MOPS_F64}" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
            "FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$out/p$i" -o run --output-format csv -- python3 bench/gemm_probe.py "$@" > "$out/p$i.log" 2>&1 || exit $?
done
echo done
