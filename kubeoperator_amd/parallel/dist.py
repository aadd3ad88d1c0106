"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl" on ROCm)
for GPU ranks, gloo for CPU ranks (tests). Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
environment (torchrun contract); a single process without those variables runs as world size 1 with no
process group at all.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    # a sub-group view (the data-parallel ranks of a tensor-parallel job, parallel.tensor): rank / world are
    # within ``group``, ``src`` is the global rank of the group's rank 0, ``global_rank`` this process's rank in the whole job
    group: object = None
    src: int = 0
    global_rank: int = -1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def rccl_selftest() -> bool:
    """``KOP_RCCL_SELFTEST=1`` under torchrun: even a one-rank job builds its process group and runs every
    data-parallel collective (the gradient reduce-scatter / all-reduce, the ZeRO-1 all-gathers, the grad-norm
    all-reduce, barriers) through the backend -- the RCCL code path of the multi-GPU bench, executed on a one-GPU
    box. A one-rank collective moves no bytes over xGMI but goes through RCCL's launch, stream and in-place
    argument handling exactly as at world size 8."""
    return os.environ.get("KOP_RCCL_SELFTEST") == "1" and "MASTER_ADDR" in os.environ


def collectives_on(info: "DistInfo") -> bool:
    """Whether this job runs its collectives: more than one rank, or the one-rank RCCL self-test."""
    return info.world > 1 or (info.backend not in ("none", "") and rccl_selftest())


def init_distributed(device: str = "auto", timeout_s: int = 1800) -> DistInfo:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    # rehearsal knobs (tests): several ranks on one GPU need gloo (RCCL refuses two ranks on one device)
    dev_index = int(os.environ.get("KOP_DEVICE_INDEX", local))
    if use_gpu:
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
    backend = "none"
    if (world > 1 or rccl_selftest()) and not dist.is_initialized():
        backend = os.environ.get("KOP_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        init = os.environ.get("KOP_DIST_INIT")  # e.g. file:///tmp/x (tests: no TCP port race)
        if init:
            kw["init_method"] = init
        elif os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
            # Under torchrun the agent hosts the store and keeps it across elastic restarts (static
            # rendezvous), while env:// adds no per-attempt prefix: a restarted attempt would read the crashed
            # attempt's process-group keys (gloo peer addresses / the RCCL unique id) and connect to dead ranks.
            # One prefix per restart keeps every attempt's rendezvous keys apart.
            store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, is_master=False,
                                  timeout=datetime.timedelta(seconds=timeout_s))
            kw["store"] = dist.PrefixStore(f"kop/attempt_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}", store)
        if use_gpu and backend == "nccl":
            kw["device_id"] = dev
            # gradient reduce-scatters overlap the backward GEMMs: a high-priority RCCL stream lets each bucket's
            # collective start as soon as its producer finishes instead of queueing behind the compute kernels
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    return DistInfo(rank, dev_index if use_gpu else local, world, backend, dev)


def parse_cpulist(text: str) -> list[int]:
    """``0-3,8,10-11`` (sysfs ``local_cpulist``) -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def _gpu_pci_dir(index: int) -> str:
    p = torch.cuda.get_device_properties(index)
    return f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def _read(path: str) -> str:
    with open(path) as f:
        return f.read().strip()


def plan_rank_cpus(local_rank: int, gpu_cpus: dict[int, list[int]], allowed: set[int]) -> tuple[list[int], str]:
    """Which CPUs local rank ``local_rank`` should run on, and why (pure: ``bind_rank_cpus`` and the tests use it).

    ``gpu_cpus``: local rank -> its GPU's NUMA-local CPUs (sysfs ``local_cpulist``); ``allowed``: the CPUs this
    process may use (cgroup / ``sched_getaffinity``). The ranks whose GPUs share one NUMA CPU list split it evenly
    (in local-rank order); the rank takes its share intersected with ``allowed``. When that is empty (a cgroup that
    leaves this NUMA node's share out) it falls back to every allowed CPU of its NUMA node, then to the allowed CPUs
    split evenly over all local ranks -- never to nothing, and the reason says which."""
    cpus = gpu_cpus[local_rank]
    peers = sorted(r for r, c in gpu_cpus.items() if c == cpus)
    k, n = peers.index(local_rank), len(peers)
    share = cpus[k * len(cpus) // n:(k + 1) * len(cpus) // n]
    want = [c for c in share if c in allowed]
    if want:
        return want, f"numa share {k + 1}/{n}"
    want = [c for c in cpus if c in allowed]
    if want:
        return want, "numa share not allowed: all allowed cpus of the numa node"
    al = sorted(allowed)
    ranks = sorted(gpu_cpus)
    k, n = ranks.index(local_rank), len(ranks)
    want = al[k * len(al) // n:(k + 1) * len(al) // n] or al
    return want, "no numa-local cpu allowed: even split of the allowed cpus"


def rank_threads(ncpus_bound: int | None, nallowed: int, local_world: int) -> int:
    """Intra-op threads per rank: the CPUs the rank is bound to, else an even share of the allowed ones (never the
    box's whole count per rank: 8 ranks x OMP_NUM_THREADS=16 on a 16-CPU share oversubscribes 8x)."""
    if ncpus_bound:
        return max(1, ncpus_bound)
    return max(1, nallowed // max(1, local_world))


def _fmt_cpus(want: list[int]) -> str:
    return f"{want[0]}-{want[-1]}" if want == list(range(want[0], want[-1] + 1)) else ",".join(map(str, want))


def bind_rank_cpus(info: DistInfo) -> dict | None:
    """Pin this rank to the CPUs next to its GPU (``plan_rank_cpus``) and size torch's intra-op thread pool to them
    (``rank_threads``). Multi-rank GPU jobs only (the one-GPU headline runs unpinned); ``KOP_CPU_AFFINITY=0`` turns
    the pinning off (and with OMP_NUM_THREADS set, leaves the pool alone); ``KOP_RANK_THREADS`` forces the count. Returns what was done and why, for the bench JSON:
    {"rank", "gpu", "numa_node", "cpus", "ncpus", "allowed", "threads", "reason"} (None: one rank / CPU)."""
    if info.device.type != "cuda" or info.world <= 1:
        return None
    allowed = os.sched_getaffinity(0)
    nloc = int(os.environ.get("LOCAL_WORLD_SIZE", torch.cuda.device_count()))
    rec = {"rank": info.rank, "gpu": info.local_rank, "numa_node": None, "cpus": None, "ncpus": 0,
           "allowed": len(allowed), "threads": None, "reason": ""}
    if os.environ.get("KOP_CPU_AFFINITY", "1") == "0":
        rec["reason"] = "KOP_CPU_AFFINITY=0: unpinned"
    else:
        try:
            ndev = min(nloc, torch.cuda.device_count())
            gpu_cpus = {i: parse_cpulist(_read(_gpu_pci_dir(i) + "/local_cpulist")) for i in range(ndev)}
            rec["numa_node"] = int(_read(_gpu_pci_dir(info.local_rank) + "/numa_node"))
            want, rec["reason"] = plan_rank_cpus(info.local_rank, gpu_cpus, allowed)
            os.sched_setaffinity(0, want)
            rec["cpus"], rec["ncpus"] = _fmt_cpus(want), len(want)
        except (OSError, ValueError, RuntimeError, KeyError) as e:
            rec["reason"] = f"unpinned: {type(e).__name__}: {e}"[:160]
    forced = os.environ.get("KOP_RANK_THREADS")
    if forced:  # the operator's choice
        rec["threads"] = max(1, int(forced))
    elif os.environ.get("KOP_CPU_AFFINITY", "1") == "0" and os.environ.get("OMP_NUM_THREADS"):
        rec["threads"] = torch.get_num_threads()  # unpinned: the pool stays as OMP_NUM_THREADS made it
        return rec
    else:
        rec["threads"] = rank_threads(rec["ncpus"], len(allowed), nloc)
    torch.set_num_threads(rec["threads"])
    os.environ["OMP_NUM_THREADS"] = str(rec["threads"])  # for anything this rank starts later
    return rec


def runtime_env() -> dict:
    """Versions and communication environment of this process, for interpreting multi-GPU results."""
    rccl = None
    try:
        v = torch.cuda.nccl.version()
        rccl = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- no RCCL in a CPU-only build
        pass
    keep = ("NCCL_", "RCCL_", "HSA_", "TORCH_NCCL_", "HIP_", "ROCR_", "GPU_MAX_HW_QUEUES", "OMP_NUM_THREADS")
    return {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None), "rccl": rccl,
            "env": {k: os.environ[k] for k in sorted(os.environ) if k.startswith(keep)}}


def barrier(info: DistInfo) -> None:
    if collectives_on(info):
        if info.backend == "nccl":
            dist.barrier(group=info.group, device_ids=[info.local_rank])
        else:
            dist.barrier(group=info.group)


def all_reduce_max(x: float, info: DistInfo) -> float:
    if not collectives_on(info):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=info.group)
    return float(t.item())


def all_reduce_sum(x: float, info: DistInfo) -> float:
    if not collectives_on(info):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, group=info.group)
    return float(t.item())


def gather_objects(obj, info: DistInfo) -> list | None:
    """Every rank's ``obj`` on every rank (None without collectives)."""
    if not collectives_on(info):
        return None
    out = [None] * dist.get_world_size(info.group)
    dist.all_gather_object(out, obj, group=info.group)
    return out


def shutdown(info: DistInfo) -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
