#!/bin/bash
# Stall / memory-path counters of the trailing-update GEMM against the vendor library at the
# solver's chunk shape.  One rocprofv3 --pmc pass per run, each within the
# per-block limits (<= 8 SQ, <= 4 TCC, <= 4 TCP, <= 2 GRBM); kernel trace not combined.
#   bash scripts/gemm_stall_pmc.sh [M N K]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
shape=${*:-32768 8192 512}
out=gpurun_out/stall
mkdir -p "$out"
passes=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
        "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
        "FETCH_SIZE TCP_TCR_TCP_STALL_CYCLES_sum")
for who in own vendor; do
  if [ $who = own ]; then cmd="python3 bench/gemm_probe.py $shape --variant glds --reps 10"
  else cmd="python3 bench/vendor_probe.py $shape --reps 10"; fi
  timeout -k 10 120 $cmd > "$out/$who.plain.json" 2>&1 || exit $?
  i=0
  for ctrs in "${passes[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$out/${who}_p$i" -o run --output-format csv -- $cmd > "$out/${who}_p$i.log" 2>&1 || exit $?
  done
done
python3 scripts/pmc_table.py "$out" > "$out/table.md"
cat "$out/table.md"
