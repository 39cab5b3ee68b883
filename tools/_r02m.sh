set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 400 python3 tools/sweep.py --size 8448 --width 65536 --gens 512 --depths 16 --rpw 74,110,142,206,270,398 --handoffs 2 --streams 1 > $O/rpw8448.jsonl 2> $O/s.err || exit 4
timeout -k 10 400 python3 tools/sweep.py --size 8448 --width 65536 --gens 512 --depths 16 --rpw 71,100,140,200,280,420 --handoffs 1 --streams 1 >> $O/rpw8448.jsonl 2>> $O/s.err || exit 5
timeout -k 10 400 python3 tools/sweep.py --size 16640 --width 65536 --gens 512 --depths 16 --rpw 142,206,270,398 --handoffs 2 --streams 1 >> $O/rpw8448.jsonl 2>> $O/s.err || exit 6
