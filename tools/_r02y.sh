set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 500 python3 tools/sweep.py --size 8448 --width 65536 --gens 480 --depths 8,12,16 --rpw 0 --handoffs 1,2 --lanes 0,32 --streams 1 --rounds 3 > $O/k8448.jsonl 2> $O/s.err || exit 4
timeout -k 10 300 python3 tools/sweep.py --size 8448 --width 65536 --gens 480 --depths 12 --rpw 30,34,38,42,46,58 --handoffs 2 --streams 1 --rounds 3 >> $O/k8448.jsonl 2>> $O/s.err || exit 5
