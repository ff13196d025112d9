set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu 2>&1 | tail -3 && \
GJ_LA_UPDATE=side timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu 2>&1 | tail -3 && \
bash scripts/ab.sh -r 2 -t 200 -v "main:" -v "side:GJ_LA_UPDATE=side" -- python bench/bench_emulate.py --ranks 8 4 --size 16384 --reps 2 --bw 50 --bcast direct && \
bash scripts/ab.sh -r 2 -t 200 -v "main:" -v "side:GJ_LA_UPDATE=side" -- python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct && \
bash scripts/ab.sh -r 2 -t 200 -v "main:" -v "side:GJ_LA_UPDATE=side" -- python bench.py --size 8192 --steps 5 --warmup 2 --no-residual && \
bash scripts/ab.sh -r 2 -t 200 -v "main:" -v "side:GJ_LA_UPDATE=side" -- python bench.py --size 16384 --steps 3 --warmup 1 --no-residual && \
bash scripts/ab.sh -r 1 -t 200 -v "main:" -v "side:GJ_LA_UPDATE=side" -- python bench.py --steps 3 --warmup 1 --no-residual
