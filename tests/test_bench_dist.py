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


def _worker(rank, wn, port, exchange, outdir, workload="tiny-test"):
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
        res, layers = bench.main(["--gpus", str(wn), "--steps", "2", "--warmup", "1", "--workload", workload,
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


def _check_line(d, wn, exchange):
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


@pytest.mark.parametrize("wn,exchange,workload", [(2, "gather", "tiny-test"), (2, "allreduce", "tiny-test"),
                                                  (4, "gather", "tiny-test"), (8, "gather", "tiny-test"),
                                                  (2, "allreduce", "tiny-test-bf16"),
                                                  (4, "allreduce", "tiny-test-bf16")])
def test_bench_multirank_cpu(tmp_path, wn, exchange, workload):
    """The driver's torchrun form: every rank calls bench.main with the env torch.distributed.run sets.
    World 8 gather (the scaling node's width) and the bf16 model's rank-ordered all-reduce leg
    (all-to-all of the float32 terms, bf16 fold in rank order, all-gather) included."""
    mp.spawn(_worker, args=(wn, _port(), exchange, str(tmp_path), workload), nprocs=wn, join=True)
    lines = [l for l in open(tmp_path / "rank0.out") if l.startswith("{")]
    assert len(lines) == 1, "rank 0 prints exactly one JSON line"
    for r in range(1, wn):
        assert not [l for l in open(tmp_path / f"rank{r}.out") if l.startswith("{")], "only rank 0 prints"
    d = json.loads(lines[0])
    _check_line(d, wn, exchange)
    if workload.endswith("bf16"):
        assert d["dtype"].startswith("bf16")


def test_bench_self_launch_cpu(tmp_path):
    """`python bench.py --gpus 2 ...` from a bare shell (no WORLD_SIZE): bench.py starts its two ranks
    itself (a torch.distributed.run child) and rank 0's JSON line comes back on the parent's stdout.
    The children run tests/bench_cpu_rank.py (HDP_BENCH_RANK_SCRIPT): bench.main with the CPU op set."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                                "MASTER_PORT", "HDP_BENCH_SELF_LAUNCHED")}
    env["HDP_BENCH_RANK_SCRIPT"] = os.path.join(HERE, "bench_cpu_rank.py")
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--workload", "tiny-test", "--micro", "2", "--batch", "2", "--seq", "48",
                        "--no-cpu-baseline", "--no-ref-torch"], env=env, capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    _check_line(json.loads(lines[0]), 2, "gather")


def test_bench_rejects_mismatched_world(monkeypatch):
    """A launcher that sets WORLD_SIZE different from --gpus is an error (no silent re-launch)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main(["--gpus", "4"])
