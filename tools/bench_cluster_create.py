"""Cluster-create time (BASELINE metric "cluster-create min") of the 1-master / 1-worker plan.

Runs the real install operation (same steps and playbooks as a bare-metal install: config, prepare,
master, worker, addon) through the control plane against the simulated host farm, and reports
``DeployExecution.timedelta`` in minutes -- the quantity the reference records per run
(kubeops_api/signal_handlers.py:54-70). With ``--latency`` each remote command also costs that many seconds,
to model SSH round trips; with the default 0 the number is pure control-plane plumbing (engine, store,
job runtime), which is what BASELINE.md config #1 asks for on CPU. A real-hardware number needs
``DEFAULT_TRANSPORT: ssh`` and reachable nodes.

Usage: python tools/bench_cluster_create.py [--latency 0.0] [--gpu-workers 1] [--repeat 3]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one_run(latency: float, gpu_workers: int, template: str) -> dict:
    os.environ.setdefault("KOP_PBKDF2_ITERS", "1000")
    from kubeoperator_amd.control.conf import Config, set_config
    from kubeoperator_amd.control.domain import clusters, context, deploy, hosts
    from kubeoperator_amd.control.engine.simfarm import SimFarm
    from kubeoperator_amd.control.store import db

    cfg = Config(path=None)
    cfg["DATA_DIR"] = tempfile.mkdtemp(prefix="kop-bench-")
    set_config(cfg)
    db.reset_for_tests(cfg.db_url)
    db.init_db()
    masters = 3 if template == "multiple-master" else 1
    gpu_ips = {f"10.0.1.{i + 1}" for i in range(gpu_workers)}
    farm = SimFarm(gpu_hosts=gpu_ips, latency_s=latency)
    context.set_transport_factory(lambda: farm)
    clusters.create_cluster({"name": "bench", "template": template, "network_plugin": "flannel",
                             "persistent_storage": "local-volume"})
    for i in range(masters):
        hosts.create_host({"name": f"m{i + 1}", "ip": f"10.0.0.{i + 1}", "password": "pw"})
        clusters.add_node("bench", {"name": f"m{i + 1}", "host": f"m{i + 1}", "roles": ["master"]})
    for i in range(gpu_workers):
        hosts.create_host({"name": f"gpu{i + 1}", "ip": f"10.0.1.{i + 1}", "password": "pw"})
        clusters.add_node("bench", {"name": f"gpu{i + 1}", "host": f"gpu{i + 1}", "roles": ["worker"]})
    e = deploy.create("bench", "install", run="inline")
    return {"state": e["state"], "seconds": e["timedelta"], "commands": len(farm.log),
            "steps": {s["name"]: s.get("seconds") for s in e["steps"]}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--latency", type=float, default=0.0, help="seconds per remote command (SSH round trip model)")
    ap.add_argument("--gpu-workers", type=int, default=1)
    ap.add_argument("--template", default="single-master", choices=["single-master", "multiple-master"])
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    runs = [one_run(a.latency, a.gpu_workers, a.template) for _ in range(a.repeat)]
    ok = all(r["state"] == "SUCCESS" for r in runs)
    secs = [r["seconds"] for r in runs]
    print(json.dumps({
        "metric": "cluster-create min", "value": round(statistics.median(secs) / 60.0, 4), "unit": "min",
        "higher_is_better": False, "state": "SUCCESS" if ok else "FAILURE", "transport": "simulated host farm",
        "latency_per_command_s": a.latency, "remote_commands": runs[-1]["commands"],
        "config": {"plan": a.template, "gpu_workers": a.gpu_workers, "gpus_per_worker": 8, "network": "flannel"},
        "seconds_per_run": [round(s, 3) for s in secs], "steps_seconds": runs[-1]["steps"],
    }))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
