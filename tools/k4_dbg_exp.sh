# K4 at Wn 8 (LLaMA-2-7B, 224 modules): H2 deferred-merge variants, and without W traffic
set -o pipefail
B="timeout -k 10 200 python tools/delta_bench.py --layers 32 --wn 8 --pol 3 --reps 3"
for d in 2 3 0; do echo "defer $d"; HDP_K4_DEFER=$d $B || exit 1; done
echo h2-now; HDP_K4_DBG_NOW=1 $B || exit 1
