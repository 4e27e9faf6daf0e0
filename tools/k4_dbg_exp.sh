# K4 x3w at Wn 8: real kernel vs measurement-only variants (no W traffic; no W and no LDS reads)
set -o pipefail
B="timeout -k 10 200 python tools/delta_bench.py --layers 32 --wn 8 --pol 3 --reps 3"
echo base; $B || exit 1
echo now; HDP_K4_DBG_NOW=1 $B || exit 1
echo nolds; HDP_K4_DBG_NOLDS=1 $B || exit 1
