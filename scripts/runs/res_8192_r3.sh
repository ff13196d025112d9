#!/bin/bash
# N = 8192 after the K = 256 LDS-DMA switch: CU reservation 32 (default) / 64, depth 2 / 3
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/ab.sh -r 2 -t 200 -v "r32:" -v "r64:GJ_RESERVE_CUS=64" -- python bench.py --size 8192 --steps 5 --warmup 2 --no-residual && \
bash scripts/ab.sh -r 1 -t 200 -v "r32d3:" -v "r64d3:GJ_RESERVE_CUS=64" -- python bench.py --size 8192 --depth 3 --steps 5 --warmup 2 --no-residual && \
bash scripts/ab.sh -r 1 -t 200 -v "r32:" -v "r64:GJ_RESERVE_CUS=64" -- python bench.py --size 16384 --steps 3 --warmup 1 --no-residual
