set -o pipefail
bash tools/gpu_profile_r02.sh r02c || exit $?
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python3 tools/sweep.py --size 4096 --gens 1000 --depths 4,6,8,12,16 --rpw 0,2,4,6,10 --handoffs 1 > $O/c2_sweep.jsonl 2> $O/c2.err || exit 5
timeout -k 10 120 python3 tools/sweep.py --size 4096 --gens 1000 --depths 8,12,16 --rpw 0 --handoffs 2 >> $O/c2_sweep.jsonl 2>> $O/c2.err || exit 6
timeout -k 10 300 python3 tools/ab_handoff.py --shapes 32768 --width 262144 --handoffs 0 --gens 256 --rounds 3 > $O/c5.jsonl 2> $O/c5.err || exit 7
timeout -k 10 300 python3 tools/ab_handoff.py --shapes 262144c --width 262144 --handoffs 0 --gens 256 --rounds 3 >> $O/c5.jsonl 2>> $O/c5.err || exit 8
cat $O/c5.jsonl
