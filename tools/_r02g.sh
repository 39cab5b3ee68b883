set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/res_tests.log 2>&1 || { tail -30 $O/res_tests.log; exit 3; }
tail -3 $O/res_tests.log
timeout -k 10 300 python3 tools/sweep.py --size 4096 --gens 1000 --depths 0,4,8,12,16 --rpw 0,2,3,4,6,8 --resident 2 > $O/c2_res_sweep.jsonl 2> $O/c2r.err || exit 5
timeout -k 10 200 python3 tools/sweep.py --size 4096 --gens 1000 --depths 0 --rpw 0 --resident 0,1 >> $O/c2_res_sweep.jsonl 2>> $O/c2r.err || exit 6
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "c2" > $O/c2_tests.log 2>&1 || { tail -30 $O/c2_tests.log; exit 7; }
tail -3 $O/c2_tests.log
