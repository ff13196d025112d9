#!/bin/bash
# Round 6: stall / memory counters of the 128 x 128 trailing-update tile against the round-5 128 x 64
# tile at the solver's chunk shape (one rocprofv3 --pmc pass per counter group, per-block limits
# respected, no trace domains combined); table by scripts/pmc_table.py.  profiles/gemm_tile128_r6.md
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc128
mkdir -p "$out"
passes=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
        "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
        "FETCH_SIZE TCP_TCR_TCP_STALL_CYCLES_sum")
for t in 128 64; do
  cmd="python3 bench/gemm_probe.py 32768 8192 512 --ldc 32768 --variant glds --reps 10"
  GJ_GLDS_TILE=$t timeout -k 10 120 $cmd > "$out/t$t.plain.json" 2>&1 || exit $?
  tail -1 "$out/t$t.plain.json"
  i=0
  for ctrs in "${passes[@]}"; do
    i=$((i+1))
    GJ_GLDS_TILE=$t timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$out/t${t}_p$i" -o run --output-format csv -- $cmd > "$out/t${t}_p$i.log" 2>&1 || exit $?
  done
done
python3 scripts/pmc_table.py "$out" > "$out/table.md"
cat "$out/table.md"
