"""bench.py's multi-rank orchestration, executed (world size 2 and 4, gloo, CPU).

The driver runs ``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` on an
8-GPU node; that path (env rendezvous, process group, the module-sharded SVD init through the
communicator, HDPissaStep's all-gather exchange, the barrier-bracketed timed region, the MAX / SUM
reductions of time and tokens, rank 0's JSON line) is run here end to end on CPU: each rank calls
``bench.main`` with the environment torch.distributed.run would set and the test op set injected
(the bench's CPU harness platform: gloo, CPU tensors, no kernel timing).  Checked: the JSON line's
contract fields, tokens summed over ranks, and every rank holding bitwise-identical merged weights.
"""
import json
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, wn, port, exchange, outdir):
    for p in (HERE, ROOT, os.path.join(ROOT, "hd-pissa_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(wn), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from cpu_ops import CpuOps
    import bench
    out = open(os.path.join(outdir, f"rank{rank}.out"), "w")
    sys.stdout = out
    try:
        res, layers = bench.main(["--gpus", str(wn), "--steps", "2", "--warmup", "1", "--workload", "tiny-test",
                                  "--micro", "2", "--batch", "2", "--seq", "48", "--exchange", exchange,
                                  "--no-cpu-baseline", "--no-ref-torch"], host_ops=CpuOps(), return_state=True)
        # every rank applied the same aggregated update: bitwise-identical W_res (gather: same
        # gathered deltas, same rank order; all-reduce: one summed buffer)
        for L in layers:
            w = L.W_res.float().clone()
            ws = [torch.zeros_like(w) for _ in range(wn)]
            dist.all_gather(ws, w)
            assert all(torch.equal(ws[0], x) for x in ws), L.name
        json.dump({"rows": res["config"]["rows_per_micro_mean"], "steps": res["steps"]},
                  open(os.path.join(outdir, f"rank{rank}.json"), "w"))
    finally:
        sys.stdout = sys.__stdout__
        out.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("wn,exchange", [(2, "gather"), (2, "allreduce"), (4, "gather")])
def test_bench_multirank_cpu(tmp_path, wn, exchange):
    mp.spawn(_worker, args=(wn, _port(), exchange, str(tmp_path)), nprocs=wn, join=True)
    lines = [l for l in open(tmp_path / "rank0.out") if l.startswith("{")]
    assert len(lines) == 1, "rank 0 prints exactly one JSON line"
    for r in range(1, wn):
        assert not [l for l in open(tmp_path / f"rank{r}.out") if l.startswith("{")], "only rank 0 prints"
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == wn and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 2 * 2 * wn and d["config"]["exchange"] == exchange
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # tokens are summed over ranks: value * time = every rank's non-padding tokens of the timed steps
    sys.path.insert(0, ROOT)
    import bench
    tokens = 0
    for r in range(wn):
        mb = bench.synthetic_micro_batches((1 + 2) * 2, 2, 48, 42 + r)[1 * 2:]
        tokens += sum(n for n, _ in mb)
    assert abs(d["value"] * d["ms_per_step"] * 2 / 1e3 - tokens) / tokens < 1e-3
