"""One rank of bench.py on the CPU harness -- TEST INFRASTRUCTURE ONLY.

`python bench.py --gpus N` without WORLD_SIZE starts its N ranks as a torch.distributed.run child
(bench.self_launch).  tests/test_bench_dist.py points that child at this file
(HDP_BENCH_RANK_SCRIPT) so the self-launched ranks run bench.main with the test op set injected
(gloo, CPU tensors) -- the launch, rendezvous and JSON relay are bench.py's own.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "hd-pissa_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

torch.set_num_threads(1)

from cpu_ops import CpuOps  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    bench.main(sys.argv[1:], host_ops=CpuOps())
