set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transport.py tests/test_gpu_multirank.py -k "gol_mpi or concurrent" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 3; }
tail -1 $O/t.log
timeout -k 10 300 python3 tools/ab_handoff.py --rounds 3 > $O/ab.jsonl 2> $O/ab.err || exit 5
bash tools/gpu_profile_r02.sh r02u
