"""bench.py's launch contract on CPU (gloo): ``--gpus 2`` without torchrun starts the two ranks itself (torchrun
as a child process) and prints ONE JSON line with the real world size and the communication fields; under
torchrun the same command runs as before; the N = 1 and N = 2 lines carry the same keys."""
import json
import os
import subprocess

import pytest
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--model", "tiny_llama", "--seq", "64", "--mbs", "2", "--accum", "2", "--steps", "2",
        "--warmup", "1", "--bucket-mb", "1", "--gemm-tuning", "off"]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    return env


def _port() -> str:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return str(s.getsockname()[1])


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _run(cmd, timeout=300):
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return _json_lines(p.stdout)


def test_bench_self_launches_ranks_without_torchrun():
    lines = _run([sys.executable, "bench.py", "--gpus", "2"] + ARGS)
    assert len(lines) == 1, lines
    r = lines[0]
    assert r["n_gpus"] == 2 and r["rccl_world"] == 2 and r["backend"] == "gloo"
    assert r["config"]["parallelism"] == "dp2-zero1"
    assert r["config"]["global_batch"] == 2 * 2 * 2
    assert r["grad_comm_bytes_per_step"] > 0 and r["param_gather_bytes_per_step"] > 0
    assert r["steps"] == 2 and r["warmup"] == 1

    one = _run([sys.executable, "bench.py", "--gpus", "1"] + ARGS)
    assert len(one) == 1
    assert one[0]["n_gpus"] == 1 and one[0]["rccl_world"] == 1 and one[0]["grad_comm_bytes_per_step"] == 0
    assert set(one[0]) == set(r) and set(one[0]["config"]) == set(r["config"])


def test_bench_under_torchrun_unchanged():
    lines = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", _port(), "bench.py", "--gpus", "2"] + ARGS)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["rccl_world"] == 2


def test_bench_refuses_mismatched_world():
    env = _env()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", _port(), "bench.py", "--gpus", "4"] + ARGS,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert not _json_lines(p.stdout)


def test_one_rank_collective_selftest_runs_the_dp_path():
    """KOP_RCCL_SELFTEST=1 under torchrun: a one-rank job builds its process group (gloo here, RCCL on a GPU box) and
    every data-parallel collective runs: ZeRO-1 reduce-scatter + all-gather bytes are counted, exposed time is
    measured, and the step matches the plain one-rank job's loss."""
    env = _env()
    env["KOP_RCCL_SELFTEST"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", _port(), "bench.py", "--gpus", "1"] + ARGS
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 1 and r["rccl_world"] == 1 and r["backend"] == "gloo"
    assert r["config"]["parallelism"] == "dp1-zero1"
    assert r["grad_comm_bytes_per_step"] > 0 and r["param_gather_bytes_per_step"] > 0
    plain = _run([sys.executable, "bench.py", "--gpus", "1"] + ARGS)[0]
    assert abs(plain["last_loss"] - r["last_loss"]) < 1e-3, (plain["last_loss"], r["last_loss"])


def _reference_params(mbs, seq, accum, world, steps, grad_dtype):
    """One process on the same global batch: every rank's synthetic stream, ranks in order, accumulated."""
    import torch

    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    torch.set_num_threads(2)
    tc = TrainConfig(model="tiny_llama", micro_batch=mbs, seq_len=seq, grad_accum=accum * world, dp_mode="allreduce",
                     bucket_mb=1, warmup_steps=10, total_steps=1000, grad_dtype=grad_dtype)
    tr = Trainer(tc, DistInfo())
    init = torch.cat([p.detach().reshape(-1).float() for _, p in tr.store.named_params()])
    streams = [SyntheticTokens(tr.cfg.vocab_size, mbs, seq, "cpu", seed=tc.seed, rank=r) for r in range(world)]
    for _ in range(steps):
        tr.train_step([b for s in streams for b in s.batches(accum)])
    return init, torch.cat([p.detach().reshape(-1).float() for _, p in tr.store.named_params()])


@pytest.mark.parametrize("dp,grad_dtype,tol", [("zero1", "fp32", 1e-3), ("allreduce", "fp32", 1e-3),
                                               ("zero1", "bf16", 0.1)])
def test_bench_world8_matches_one_process(dp, grad_dtype, tol, tmp_path):
    """``bench.py --gpus 8 --device cpu`` self-launches 8 gloo ranks (world-8 bucket padding,
    in-place reduce-scatter piece aliasing, ZeRO-1 all-gather, accumulation 2); the final parameters equal one
    process on the same global batch, and the JSON names the world and the runtime environment. fp32 gradient
    buffers are the exact check (measured < 1e-5 relative to the update); with bf16 buffers Adam's per-element
    normalisation at the default eps turns bf16 reduction-order noise into ~6 % of the update (a dropped or
    doubled bucket is O(1))."""
    import torch

    dump = tmp_path / "p8.pt"
    env = _env()
    env.update(KOP_BENCH_DUMP_PARAMS=str(dump), OMP_NUM_THREADS="1", NCCL_DEBUG="WARN")
    args = ["--device", "cpu", "--model", "tiny_llama", "--seq", "32", "--mbs", "1", "--accum", "2", "--steps", "1",
            "--warmup", "1", "--bucket-mb", "1", "--gemm-tuning", "off", "--dp", dp, "--grad-dtype", grad_dtype]
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "8"] + args, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    (r,) = _json_lines(p.stdout)
    assert r["n_gpus"] == 8 and r["rccl_world"] == 8 and r["backend"] == "gloo"
    assert r["config"]["parallelism"] == ("dp8-zero1" if dp == "zero1" else "dp8")
    assert r["config"]["global_batch"] == 1 * 2 * 8
    assert r["runtime"]["torch"] and r["runtime"]["env"]["NCCL_DEBUG"] == "WARN"
    assert r["cpu_affinity_rank0"] is None  # CPU ranks are not pinned
    got = torch.load(dump, weights_only=True)
    init, want = _reference_params(1, 32, 2, 8, 2, grad_dtype)
    rel = ((got - want).norm() / (want - init).norm()).item()
    assert rel < tol, rel


def test_cpulist_parsing():
    from kubeoperator_amd.parallel.dist import parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


# --- the first 8-GPU run must be attributable -------------------------------------------------
# an MI355X node as sysfs shows it: GPUs 0-3 on NUMA node 0 (CPUs 0-63), GPUs 4-7 on node 1 (CPUs 64-127)
_NODE = {i: list(range(0, 64)) if i < 4 else list(range(64, 128)) for i in range(8)}


def test_rank_cpu_plan_splits_each_numa_node_and_records_why():
    from kubeoperator_amd.parallel.dist import plan_rank_cpus

    allowed = set(range(128))
    plans = [plan_rank_cpus(r, _NODE, allowed) for r in range(8)]
    assert [p[0][0] for p in plans] == [0, 16, 32, 48, 64, 80, 96, 112]
    assert all(len(p[0]) == 16 and p[1].startswith("numa share") for p in plans)
    # a cgroup that grants 16 CPUs of node 0 only (the gpurun box's share): node-0 ranks keep their shares within it,
    # node-1 ranks cannot get a NUMA-local CPU and split the allowed set evenly -- with the reason recorded
    allowed = set(range(0, 16))
    p0 = plan_rank_cpus(0, _NODE, allowed)
    assert p0 == (list(range(0, 16)), "numa share 1/4")
    p1 = plan_rank_cpus(1, _NODE, allowed)
    assert p1[0] == list(range(0, 16)) and p1[1].startswith("numa share not allowed")
    p5 = plan_rank_cpus(5, _NODE, allowed)
    assert p5 == ([10, 11], "no numa-local cpu allowed: even split of the allowed cpus")
    assert all(plan_rank_cpus(r, _NODE, allowed)[0] for r in range(8))  # never an empty CPU set


def test_rank_threads_never_oversubscribe(monkeypatch):
    from kubeoperator_amd.parallel.dist import rank_threads

    assert rank_threads(16, 128, 8) == 16  # pinned: the CPUs it is pinned to
    assert rank_threads(0, 16, 8) == 2  # unpinned: an even share of the allowed CPUs, not OMP's 16 each
    assert rank_threads(None, 4, 8) == 1

    # the self-launch hands each child rank an even share of this process's CPUs unless the operator set a count
    # (each rank re-sizes its pool in bind_rank_cpus anyway)
    import bench

    seen = {}
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.update(env=env) or 0)
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench._self_launch(8) == 0
    assert seen["env"]["OMP_NUM_THREADS"] == "2"
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench._self_launch(8) == 0
    assert seen["env"]["OMP_NUM_THREADS"] == "3"


def test_bucket_timeline_summary_is_the_median_over_steps():
    from kubeoperator_amd.parallel.ddp import summarize_rows

    rows = [{"n_buckets": 3, "first_ready_ms": -40.0 - i, "last_ready_ms": -1.0, "first_done_ms": -30.0,
             "last_done_ms": 2.0 + i, "in_flight_ms": 42.0} for i in range(3)]
    s = summarize_rows(rows)
    assert s == {"n_buckets": 3, "first_ready_ms": -41.0, "last_ready_ms": -1.0, "first_done_ms": -30.0,
                 "last_done_ms": 3.0, "in_flight_ms": 42.0, "steps": 3}
    assert summarize_rows([]) is None


def test_bucket_timeline_is_passive_and_uses_rccl_durations():
    """The timeline records compute-stream ready events and RCCL's own per-collective durations (Work._get_duration,
    TORCH_NCCL_ENABLE_TIMING=1): collective i runs from max(ready_i, done_{i-1}) for its duration. No stream of
    its own (ddp.DataParallel has no timeline stream any more)."""
    from kubeoperator_amd.parallel import ddp

    class Ev:
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

    class Work:
        def __init__(self, d):
            self.d = d

        def _get_duration(self):
            if self.d is None:
                raise RuntimeError("timing not enabled")
            return self.d

    # backward ends at t = 10; buckets ready at 2, 5, 9; collectives of 4, 1, 3 ms
    step = {"bwd_end": Ev(10.0), "buckets": [(0, Ev(2.0), Work(4.0)), (1, Ev(5.0), Work(1.0)), (2, Ev(9.0), Work(3.0))]}
    s = ddp.timeline_summary([step, step, step])
    assert s["n_buckets"] == 3 and s["steps"] == 3
    assert s["first_ready_ms"] == -8.0 and s["last_ready_ms"] == -1.0
    # done: 2+4 = 6, max(5, 6)+1 = 7, max(9, 7)+3 = 12 -> relative to 10: -4, -3, +2
    assert s["first_done_ms"] == -4.0 and s["last_done_ms"] == 2.0 and s["comm_ms"] == 8.0
    assert s["in_flight_ms"] == 10.0 and s["max_collective_ms"] == 4.0
    # without RCCL timing: ready times only
    step2 = {"bwd_end": Ev(10.0), "buckets": [(0, Ev(2.0), Work(None))]}
    s2 = ddp.timeline_summary([step2])
    assert "last_done_ms" not in s2 and s2["last_ready_ms"] == -8.0
    import inspect

    assert "Stream(" not in inspect.getsource(ddp)


def test_stream_inventory_against_hw_queues(monkeypatch):
    import bench

    class T:
        class opt:
            overlap = True

        class store:
            wgrad_stream = True

    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    inv = bench.stream_inventory(T, rccl=True)
    assert inv == {"in_use": ["compute", "optimizer", "wgrad", "rccl"], "hw_queues": 4, "fits": True}
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    assert bench.stream_inventory(T, rccl=True)["fits"] is False


def test_deferred_weight_gradient_refused_while_collectives_live():
    """_sink(defer=True) marks a parameter ready before its deferred gradient launch; that is only sound
    while readiness launches no bucket collective. The flat store refuses a deferral on a micro-batch whose backward
    reduces (dp.sync on, collectives on) instead of relying on the trainer's defer_ok wiring."""
    import pytest

    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    tr = Trainer(TrainConfig(model="tiny_llama", micro_batch=1, seq_len=32), DistInfo())
    tr.dp.sync = False
    tr.store.defer(lambda: None)
    tr.store.run_deferred()
    tr.dp.force = True  # as the one-rank RCCL self-test: buckets go through collectives
    tr.dp.sync = True
    with pytest.raises(RuntimeError, match="collectives are live"):
        tr.store.defer(lambda: None)
