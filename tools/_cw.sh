set -o pipefail
O=gpurun_out/cw; mkdir -p $O
timeout -k 10 300 python -u bench.py --rule conway --no-cpu-baseline --steps 2 > $O/bench_conway.json 2> $O/err || { tail $O/err; exit 9; }
cut -c1-300 $O/bench_conway.json
timeout -k 10 300 python -u tools/ab_skew.py --shapes 65536,8448 --rhos auto --handoffs 0 --gens 256 --rounds 3 --rule conway > $O/ab.jsonl 2>> $O/err || { tail $O/err; exit 9; }
cat $O/ab.jsonl
