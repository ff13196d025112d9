#!/bin/bash
# Round 6: memory counters of the trailing-update GEMM (32768 x 8192 x 512, C ld 32768: the solver's
# chunk) with the C tile temporal (GJ_GLDS_CNT=0) and non-temporal (3).  One rocprofv3 --pmc pass
# per group (per-block limits respected, no trace domains); table by scripts/pmc_table.py.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmccnt
mkdir -p "$out"
passes=("GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAVE_CYCLES"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
        "FETCH_SIZE"
        "WRITE_SIZE TCC_EA0_WRREQ_sum")
for c in 0 3; do
  cmd="python3 bench/gemm_probe.py 32768 8192 512 --ldc 32768 --variant glds --reps 10"
  GJ_GLDS_CNT=$c timeout -k 10 120 $cmd > "$out/c$c.plain.json" 2>&1 || exit $?
  tail -1 "$out/c$c.plain.json"
  i=0
  for ctrs in "${passes[@]}"; do
    i=$((i+1))
    GJ_GLDS_CNT=$c timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$out/c${c}_p$i" -o run --output-format csv -- $cmd > "$out/c${c}_p$i.log" 2>&1 || exit $?
  done
done
python3 scripts/pmc_table.py "$out" > "$out/table.md"
cat "$out/table.md"
