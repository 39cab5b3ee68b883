set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/sweep.py --size 8448 --width 65536 --gens 512 --depths 16 --rpw 0 --handoffs 1,2 --streams 1 > $O/shape8448.jsonl 2> $O/s.err || exit 4
timeout -k 10 300 python3 tools/sweep.py --size 16896 --width 65536 --gens 512 --depths 16 --rpw 0 --handoffs 1,2 --streams 2 >> $O/shape8448.jsonl 2>> $O/s.err || exit 5
timeout -k 10 300 python3 tools/sweep.py --size 16896 --width 65536 --gens 512 --depths 16 --rpw 0 --handoffs 1,2 --streams 1 >> $O/shape8448.jsonl 2>> $O/s.err || exit 6
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --size 4096 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_4096_traced.json 2> $O/prof_c2.err || exit 7
