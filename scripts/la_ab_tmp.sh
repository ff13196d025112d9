set -o pipefail
bash scripts/ab.sh -r 2 -t 200 -v "late:" -v "early:GJ_EARLY=1" -- python bench/bench_emulate.py --ranks 8 4 --size 16384 --reps 2 --bw 50 --bcast direct && \
bash scripts/ab.sh -r 2 -t 200 -v "late:" -v "early:GJ_EARLY=1" -- python bench.py --size 8192 --steps 5 --warmup 2 --no-residual && \
for d in 3 4; do bash scripts/ab.sh -r 2 -t 200 -v "late-d$d:" -v "early-d$d:GJ_EARLY=1" -- python bench.py --size 8192 --depth $d --steps 5 --warmup 2 --no-residual || exit 1; done && \
bash scripts/ab.sh -r 2 -t 200 -v "late:" -v "early:GJ_EARLY=1" -- python bench.py --size 16384 --steps 3 --warmup 1 --no-residual && \
bash scripts/ab.sh -r 1 -t 200 -v "late:" -v "early:GJ_EARLY=1" -- python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct && \
bash scripts/ab.sh -r 1 -t 200 -v "late:" -v "early:GJ_EARLY=1" -- python bench.py --steps 3 --warmup 1 --no-residual
