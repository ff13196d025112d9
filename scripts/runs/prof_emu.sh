cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/prof_emu8_16k
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 > $out/emu.log 2>&1
rc=$?; echo rc=$rc; tail -3 $out/emu.log; ls $out
