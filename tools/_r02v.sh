set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
bash tools/gpu_round.sh r02v || exit $?
timeout -k 10 300 python3 tools/ab_handoff.py --rounds 3 > $O/ab.jsonl 2> $O/ab.err || exit 5
bash tools/gpu_profile_r02.sh r02v
