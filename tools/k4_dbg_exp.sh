# K4 x3w at Wn 8: real kernel vs measurement-only variants (each drops one more part)
set -o pipefail
B="timeout -k 10 200 python tools/delta_bench.py --layers 32 --wn 8 --pol 3 --reps 3"
echo base; $B || exit 1
echo nolds; HDP_K4_DBG_NOLDS=1 $B || exit 1
echo nosync; HDP_K4_DBG_NOSYNC=1 $B || exit 1
echo pure; HDP_K4_DBG_PURE=1 $B || exit 1
