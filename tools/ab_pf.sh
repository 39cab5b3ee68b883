# Dev A/B (via gpurun) of two K=16-only builds: tools/build_alt.sh pf4; tools/build_alt.sh pf8 -DGOL_PF_NP2=8 -DGOL_DEV_FLIP_PAD=1
mkdir -p gpurun_out
for round in 1 2; do
for n in pf4 pf8; do
  GOL_LIB=tools/libgol_$n.so timeout -k 10 120 python -u tools/sweep.py --size 8448 --width 65536 --gens 480 --depths 16 --planes 2 --rpw 0,72 --rounds 3 | sed "s/^/$n 8448 /" >> gpurun_out/ab_pf.txt || exit 1
  GOL_LIB=tools/libgol_$n.so timeout -k 10 120 python -u tools/sweep.py --size 65536 --gens 480 --depths 16 --planes 2 --rounds 3 | sed "s/^/$n 65536 /" >> gpurun_out/ab_pf.txt || exit 1
done
done
