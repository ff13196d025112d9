#!/bin/bash
# Round-5 evidence: (1) stall / MFMA-busy counters of the peeled 3-stage trailing-update GEMM vs the
# round-4 kernel vs hipBLASLt at 32768 x 8192 x 512 (one --pmc pass per run, per-block limits kept,
# no trace domains combined); (2) N = 32768 kernel trace.  The RCCL footprint and the deeper-pipeline
# A/B run in scripts/runs/r5_next.sh.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc5
mkdir -p "$out"
passes=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
        "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
        "FETCH_SIZE TCP_TCR_TCP_STALL_CYCLES_sum")
for who in r5 r4 vendor; do
  case $who in
    r5) cmd="python3 bench/gemm_probe.py 32768 8192 512 --ldc 32768 --variant glds --reps 10"; envs="" ;;
    r4) cmd="python3 bench/gemm_probe.py 32768 8192 512 --ldc 32768 --variant glds --reps 10"; envs="GJ_GLDS_PEEL=0 GJ_GLDS_BUILD=2.3" ;;
    vendor) cmd="python3 bench/vendor_probe.py 32768 8192 512 --reps 10"; envs="" ;;
  esac
  env $envs timeout -k 10 120 $cmd > "$out/$who.plain.json" 2>&1 || exit $?
  echo "$who $(tail -1 $out/$who.plain.json | cut -c1-220)"
  i=0
  for ctrs in "${passes[@]}"; do
    i=$((i+1))
    env $envs timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$out/${who}_p$i" -o run --output-format csv -- $cmd > "$out/${who}_p$i.log" 2>&1 || exit $?
  done
done
python3 scripts/pmc_table.py "$out" > "$out/table.md"
cat "$out/table.md"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof32k -o run -- python3 bench.py --steps 2 --warmup 1 --no-residual > $out/prof32k.log 2>&1
echo "trace rc=$?"
