#!/bin/bash
# Block size m below 128 with the matrix-core inverse (m = 64: 5-wave workgroups) at the BASELINE sizes.
set -o pipefail
cd "$(dirname "$0")/../.."
b() { echo "== $*"; timeout -k 10 200 python bench.py "$@" || exit $?; }
b --size 8192 --steps 5 --warmup 2
b --size 8192 --block 64 --depth 4 --steps 5 --warmup 2
b --size 8192 --block 64 --depth 8 --steps 5 --warmup 2
b --size 8192 --block 96 --depth 4 --steps 5 --warmup 2
b --size 16384 --steps 3 --warmup 1
b --size 16384 --block 64 --depth 8 --steps 3 --warmup 1
b --size 16384 --block 64 --depth 4 --steps 3 --warmup 1
b --steps 3 --warmup 1
b --block 64 --depth 8 --steps 3 --warmup 1
b --block 96 --depth 4 --steps 3 --warmup 1
b --block 64 --depth 4 --steps 3 --warmup 1
