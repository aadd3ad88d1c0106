"""bench.py's launch contract on CPU (gloo): ``--gpus 2`` without torchrun starts the two ranks itself (torchrun
as a child process) and prints ONE JSON line with the real world size and the communication fields; under
torchrun the same command runs as before; the N = 1 and N = 2 lines carry the same keys."""
import json
import os
import subprocess
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
