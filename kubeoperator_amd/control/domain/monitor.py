"""Cluster observability read path: Kubernetes API, Prometheus (incl. AMD GPU metrics), Loki, events,
health, availability history, compliance grade, system-log search.

Reference: kubeops_api/cluster_monitor.py:26-632 (ClusterMonitor; set_cluster_data :157-192 -> Redis blob;
list_events :355-400 -> ES + Warning messages; sync_node_time :600-632), prometheus_client.py:9-149,
apps_client.py (Host-header vhost to the first master), cluster_health_utils.py, models/health/*,
grade.py (KubeGrade), log/es.py.

MI355X-first differences: node resource data adds GPU count / utilisation / HBM use / power from the
AMD device-metrics-exporter (``gpu_gfx_activity``, ``gpu_used_vram``, ``gpu_power_usage`` series); the
per-cluster data blob, events and system logs are JSON/JSONL files under ``DATA_DIR`` (no Redis / ES);
node clock skew is compared in seconds (the reference compares against 300000, i.e. ~3.5 days).
"""
from __future__ import annotations

import datetime as dt
import glob
import json
import logging
import os
import re
import time

import httpx
from sqlalchemy import select

from ..conf import get_config
from ..store import models as M
from ..store.db import session_scope
from . import clusters, context

log = logging.getLogger("kubeoperator.monitor")


# ------------------------------------------------------------------------------------------- clients
class K8sClient:
    def __init__(self, server: str, token: str, verify=False, timeout=15):
        self.server, self.token, self.verify, self.timeout = server.rstrip("/"), token, verify, timeout

    def get(self, path: str, params: dict | None = None) -> dict:
        r = httpx.get(self.server + path, params=params, headers={"Authorization": f"Bearer {self.token}"},
                      verify=self.verify, timeout=self.timeout)
        r.raise_for_status()
        return r.json()


class PrometheusClient:
    def __init__(self, base: str, host_header: str | None = None, timeout=15):
        self.base, self.host, self.timeout = base.rstrip("/"), host_header, timeout

    def query(self, promql: str) -> list:
        r = httpx.get(f"{self.base}/api/v1/query", params={"query": promql},
                      headers={"Host": self.host} if self.host else None, timeout=self.timeout)
        r.raise_for_status()
        return r.json().get("data", {}).get("result", [])

    def scalar(self, promql: str, default=0.0) -> float:
        res = self.query(promql)
        try:
            return float(res[0]["value"][1])
        except (IndexError, KeyError, ValueError, TypeError):
            return default


_client_override = {}


def set_clients(cluster_name: str, k8s=None, prom=None, loki=None) -> None:
    """Inject API clients (tests, or a controller that reaches the cluster through a tunnel)."""
    _client_override[cluster_name] = {"k8s": k8s, "prom": prom, "loki": loki}


def _clients(c: M.Cluster):
    ov = _client_override.get(c.name)
    if ov:
        return ov["k8s"], ov["prom"], ov.get("loki")
    master_ip = _master_ip(c)
    token = (c.configs or {}).get("_k8s_token") or clusters.cluster_token(c.name)
    if token and not (c.configs or {}).get("_k8s_token"):
        clusters.set_config(c.name, "_k8s_token", token)
    domain = (c.configs or {}).get("APP_DOMAIN", "")
    k8s = K8sClient(f"https://{master_ip}:6443", token)
    prom = PrometheusClient(f"http://{master_ip}", host_header=f"prometheus.{domain}")
    loki = PrometheusClient(f"http://{master_ip}", host_header=f"loki.{domain}")
    return k8s, prom, loki


def _master_ip(c: M.Cluster) -> str:
    inv = context.project_inventory(c.project_id)
    ms = inv.group_hosts("master")
    return inv.host_vars(ms[0]).get("ansible_host") if ms else "127.0.0.1"


# ------------------------------------------------------------------------------------------- cluster data
def _data_dir(kind: str) -> str:
    d = os.path.join(get_config().data_dir, kind)
    os.makedirs(d, exist_ok=True)
    return d


def node_resources(prom: PrometheusClient, node_ip: str) -> dict:
    inst = f'instance=~"{re.escape(node_ip)}.*"'
    out = {
        "cpu_usage": prom.scalar(f'1 - avg(rate(node_cpu_seconds_total{{mode="idle",{inst}}}[5m]))'),
        "mem_usage": prom.scalar(f'1 - node_memory_MemAvailable_bytes{{{inst}}} / node_memory_MemTotal_bytes{{{inst}}}'),
        "cpu_total": prom.scalar(f'count(node_cpu_seconds_total{{mode="idle",{inst}}})'),
        "mem_total": prom.scalar(f'node_memory_MemTotal_bytes{{{inst}}}'),
    }
    # AMD device-metrics-exporter series (per GPU); averaged / summed per node
    out["gpu_count"] = prom.scalar(f'count(gpu_gfx_activity{{hostname=~".*",{inst}}})')
    out["gpu_util"] = prom.scalar(f'avg(gpu_gfx_activity{{{inst}}})') / 100.0
    out["gpu_vram_used_gb"] = prom.scalar(f'sum(gpu_used_vram{{{inst}}})') / 1024.0
    out["gpu_power_w"] = prom.scalar(f'sum(gpu_power_usage{{{inst}}})')
    return out


def set_cluster_data(cluster_name: str) -> dict:
    """Collect the dashboard blob for one cluster (reference ClusterMonitor.set_cluster_data)."""
    c = clusters.get_cluster(cluster_name)
    k8s, prom, _ = _clients(c)
    nodes = k8s.get("/api/v1/nodes").get("items", [])
    pods = k8s.get("/api/v1/pods").get("items", [])
    nss = k8s.get("/api/v1/namespaces").get("items", [])
    deps = k8s.get("/apis/apps/v1/deployments").get("items", [])
    data = {"name": c.name, "date": M.now().isoformat(), "nodes": [], "pods": [], "namespaces": [], "deployments": [],
            "restart_pods": [], "error_pods": [], "warn_containers": [], "cpu_usage": 0, "mem_usage": 0,
            "gpu_total": 0, "gpu_allocatable": 0}
    for n in nodes:
        addr = next((a["address"] for a in n["status"].get("addresses", []) if a["type"] == "InternalIP"), "")
        alloc = n["status"].get("allocatable", {})
        res = {}
        try:
            res = node_resources(prom, addr) if prom is not None else {}
        except httpx.HTTPError:
            res = {}
        gpus = int(alloc.get("amd.com/gpu", 0) or 0)
        data["gpu_allocatable"] += gpus
        data["gpu_total"] += int(n["status"].get("capacity", {}).get("amd.com/gpu", 0) or 0)
        ready = next((cd["status"] for cd in n["status"].get("conditions", []) if cd["type"] == "Ready"), "Unknown")
        data["nodes"].append({"name": n["metadata"]["name"], "ip": addr, "ready": ready, "amd_gpu": gpus, **res})
    for p in pods:
        st = p.get("status", {})
        restarts = sum(cs.get("restartCount", 0) for cs in st.get("containerStatuses", []) or [])
        item = {"name": p["metadata"]["name"], "namespace": p["metadata"]["namespace"], "status": st.get("phase"),
                "restart_count": restarts, "host_ip": st.get("hostIP")}
        data["pods"].append(item)
        if restarts > 0:
            data["restart_pods"].append(item)
        if st.get("phase") not in ("Running", "Succeeded"):
            data["error_pods"].append(item)
    data["namespaces"] = [{"name": n["metadata"]["name"], "status": n["status"].get("phase")} for n in nss]
    data["deployments"] = [{"name": d["metadata"]["name"], "namespace": d["metadata"]["namespace"],
                            "ready_replicas": d.get("status", {}).get("readyReplicas", 0),
                            "replicas": d.get("spec", {}).get("replicas", 0)} for d in deps]
    if data["nodes"]:
        data["cpu_usage"] = sum(n.get("cpu_usage", 0) for n in data["nodes"]) / len(data["nodes"])
        data["mem_usage"] = sum(n.get("mem_usage", 0) for n in data["nodes"]) / len(data["nodes"])
    for n in data["nodes"]:
        for k, lim in (("cpu_usage", 0.8), ("mem_usage", 0.8)):
            if n.get(k, 0) > lim:
                _warn(c, f"node {n['name']} {k} {n[k]:.0%} > {lim:.0%}")
    with open(os.path.join(_data_dir("cluster_data"), f"{c.name}.json"), "w") as f:
        json.dump(data, f)
    return data


def get_cluster_data(cluster_name: str) -> dict | None:
    p = os.path.join(_data_dir("cluster_data"), f"{cluster_name}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def delete_cluster_data(cluster_name: str) -> None:
    p = os.path.join(_data_dir("cluster_data"), f"{cluster_name}.json")
    if os.path.exists(p):
        os.remove(p)


def _warn(c: M.Cluster, text: str) -> None:
    from . import messages

    messages.insert_message({"title": "Cluster alert", "level": "WARNING", "type": "CLUSTER",
                             "content": {"resource_name": c.name, "resource_type": "CLUSTER", "detail": text}})


# ------------------------------------------------------------------------------------------- events
def save_events(cluster_name: str) -> int:
    """k8s events -> ``events/<cluster>-YYYY.M.jsonl``; Warning events -> message center."""
    c = clusters.get_cluster(cluster_name)
    k8s, _, _ = _clients(c)
    items = k8s.get("/api/v1/events").get("items", [])
    path = os.path.join(_data_dir("events"), f"{c.name}-{dt.date.today():%Y.%-m}.jsonl")
    seen = set()
    if os.path.exists(path):
        with open(path) as f:
            seen = {json.loads(l).get("uid") for l in f if l.strip()}
    n = 0
    with open(path, "a") as f:
        for e in items:
            uid = e["metadata"].get("uid")
            if uid in seen:
                continue
            doc = {"uid": uid, "cluster_name": c.name, "type": e.get("type"), "reason": e.get("reason"),
                   "message": e.get("message"), "namespace": e["metadata"].get("namespace"),
                   "kind": e.get("involvedObject", {}).get("kind"), "name": e.get("involvedObject", {}).get("name"),
                   "last_timestamp": e.get("lastTimestamp") or e.get("eventTime"), "count": e.get("count", 1)}
            f.write(json.dumps(doc) + "\n")
            n += 1
            if e.get("type") == "Warning":
                _warn(c, f"{doc['kind']}/{doc['name']}: {doc['reason']}: {doc['message']}")
    return n


def search_events(cluster_name: str, limit: int = 100, offset: int = 0, type_: str | None = None,
                  keywords: str | None = None) -> dict:
    docs = []
    for p in sorted(glob.glob(os.path.join(_data_dir("events"), f"{cluster_name}-*.jsonl")), reverse=True):
        with open(p) as f:
            for line in f:
                d = json.loads(line)
                if type_ and d.get("type") != type_:
                    continue
                if keywords and keywords.lower() not in json.dumps(d).lower():
                    continue
                docs.append(d)
    docs.sort(key=lambda d: d.get("last_timestamp") or "", reverse=True)
    return {"total": len(docs), "items": docs[offset:offset + limit]}


# ------------------------------------------------------------------------------------------- health
GPU_TEMP_LIMIT_C = 105.0  # MI355X junction temperature above which the node is flagged


def gpu_condition(node: dict, prom) -> dict:
    """``AMDGPUHealthy`` node condition (new: the reference only counts GPUs). Unhealthy when the device
    plugin advertises fewer ``amd.com/gpu`` than the node has, or the device-metrics exporter reports
    uncorrectable ECC errors, an unhealthy device (``gpu_health`` 0) or a junction temperature over the limit."""
    st = node.get("status", {})
    cap = int(st.get("capacity", {}).get("amd.com/gpu", 0) or 0)
    alloc = int(st.get("allocatable", {}).get("amd.com/gpu", 0) or 0)
    problems = []
    if cap and alloc < cap:
        problems.append(f"{cap - alloc} of {cap} GPUs not allocatable")
    if prom is not None and cap:
        ip = next((a["address"] for a in st.get("addresses", []) if a.get("type") == "InternalIP"), "")
        inst = f'instance=~"{ip}:.*"'
        try:
            ecc = prom.scalar(f"sum(gpu_ecc_uncorrect_total{{{inst}}})", 0.0)
            unhealthy = prom.scalar(f"count(gpu_health{{{inst}}} == 0)", 0.0)
            temp = prom.scalar(f"max(gpu_junction_temperature{{{inst}}})", 0.0)
        except httpx.HTTPError:
            ecc = unhealthy = temp = 0.0
        if ecc > 0:
            problems.append(f"{int(ecc)} uncorrectable ECC errors")
        if unhealthy > 0:
            problems.append(f"{int(unhealthy)} GPUs report unhealthy")
        if temp > GPU_TEMP_LIMIT_C:
            problems.append(f"junction temperature {temp:.0f} C > {GPU_TEMP_LIMIT_C:.0f} C")
    return {"type": "AMDGPUHealthy", "status": "False" if problems else "True",
            "message": "; ".join(problems) or f"{alloc} GPUs healthy", "reason": "GPUFault" if problems else "",
            "lastTransitionTime": None}


def node_health(cluster_name: str) -> list[dict]:
    """Node conditions + nodeInfo from the k8s API into the node rows (reference node_health.py:10-56),
    plus an ``AMDGPUHealthy`` condition on GPU nodes."""
    c = clusters.get_cluster(cluster_name)
    k8s, prom, _ = _clients(c)
    out = []
    nodes = {n["metadata"]["name"]: n for n in k8s.get("/api/v1/nodes").get("items", [])}
    with session_scope() as s:
        for row in s.scalars(select(M.InvHost).where(M.InvHost.project_id == c.project_id, M.InvHost.name != "localhost")):
            n = nodes.get(row.name) or nodes.get(row.name.split(".")[0])
            if n is None:
                row.conditions = [{"type": "Ready", "status": "Unknown", "message": "node not registered in k8s"}]
            else:
                row.conditions = [{k: cd.get(k) for k in ("type", "status", "message", "reason", "lastTransitionTime")}
                                  for cd in n["status"].get("conditions", [])]
                if n["status"].get("capacity", {}).get("amd.com/gpu"):
                    row.conditions = row.conditions + [gpu_condition(n, prom)]
                row.info = n["status"].get("nodeInfo", {}) | {"allocatable": n["status"].get("allocatable", {})}
            out.append({"name": row.name, "conditions": row.conditions})
    return out


def cluster_health(cluster_name: str) -> dict:
    """Component / namespace / node health summary (reference cluster/<name>/health endpoints)."""
    c = clusters.get_cluster(cluster_name)
    k8s, prom, _ = _clients(c)
    comps = []
    try:
        for cs in k8s.get("/api/v1/componentstatuses").get("items", []):
            cond = (cs.get("conditions") or [{}])[0]
            comps.append({"name": cs["metadata"]["name"], "status": cond.get("status"), "message": cond.get("message")})
    except httpx.HTTPError:
        pass
    for name, path in (("apiserver", "/livez"), ("etcd", "/livez/etcd")):
        try:
            k8s.get(path)
            comps.append({"name": name, "status": "True", "message": "ok"})
        except Exception as e:  # noqa: BLE001
            comps.append({"name": name, "status": "False", "message": str(e)[:200]})
    rate = 100.0
    if prom is not None:
        try:
            rate = 100.0 * prom.scalar("sum(up) / count(up)", 1.0)
        except httpx.HTTPError:
            pass
    return {"components": comps, "available_rate": rate}


def record_availability(cluster_name: str, rate: float, date_type: str = "HOUR") -> None:
    c = clusters.get_cluster(cluster_name)
    with session_scope() as s:
        s.add(M.ClusterHealthHistory(cluster_id=c.id, available_rate=rate, date_type=date_type,
                                     month=f"{dt.date.today():%Y-%m}"))


def availability_history(cluster_id: str, date_type: str = "HOUR") -> list[dict]:
    with session_scope() as s:
        rows = s.scalars(select(M.ClusterHealthHistory).where(M.ClusterHealthHistory.cluster_id == cluster_id,
                                                              M.ClusterHealthHistory.date_type == date_type)
                         .order_by(M.ClusterHealthHistory.date_created))
        return [r.to_dict() for r in rows]


def roll_up_day(cluster_id: str) -> float | None:
    """Daily availability = mean of the day's hourly samples (guards the empty day the reference divides by)."""
    today = dt.date.today()
    hours = [h for h in availability_history(cluster_id, "HOUR") if h["date_created"][:10] == str(today)]
    if not hours:
        return None
    rate = sum(h["available_rate"] for h in hours) / len(hours)
    with session_scope() as s:
        s.add(M.ClusterHealthHistory(cluster_id=cluster_id, available_rate=rate, date_type="DAY",
                                     month=f"{today:%Y-%m}"))
    return rate


def node_time_skew(cluster_name: str, max_skew_s: float = 300.0) -> dict:
    """Compare every node's clock with the controller (seconds; reference compared against 300000)."""
    c = clusters.get_cluster(cluster_name)
    res = clusters.run_adhoc(c, "cluster_nodes", "shell", {"_raw_params": "date +%s"})
    now = time.time()
    out = {}
    for host, tasks in res["raw"]["ok"].items():
        r = next(iter(tasks.values()))
        try:
            skew = float(r.get("stdout", "0").strip()) - now
        except ValueError:
            continue
        out[host] = {"skew_s": skew, "ok": abs(skew) <= max_skew_s}
    return out


# ------------------------------------------------------------------------------------------- grade
GRADE_CHECKS = (
    ("cpuRequestsMissing", "warning", lambda ct, pod: not (ct.get("resources", {}).get("requests", {}) or {}).get("cpu")),
    ("memoryLimitsMissing", "warning", lambda ct, pod: not (ct.get("resources", {}).get("limits", {}) or {}).get("memory")),
    ("livenessProbeMissing", "warning", lambda ct, pod: not ct.get("livenessProbe")),
    ("readinessProbeMissing", "warning", lambda ct, pod: not ct.get("readinessProbe")),
    ("tagNotSpecified", "danger", lambda ct, pod: ":" not in ct.get("image", "") or ct.get("image", "").endswith(":latest")),
    ("runAsPrivileged", "danger", lambda ct, pod: (ct.get("securityContext") or {}).get("privileged", False)),
    ("hostNetworkSet", "warning", lambda ct, pod: pod.get("hostNetwork", False)),
    ("gpuLimitMissing", "warning", lambda ct, pod: "amd.com/gpu" in (ct.get("resources", {}).get("requests", {}) or {})
     and "amd.com/gpu" not in (ct.get("resources", {}).get("limits", {}) or {})),
)


def grade(cluster_name: str) -> dict:
    """Best-practice audit of workload specs (replaces the external KubeGrade/validator, cached 60 s)."""
    cache = os.path.join(_data_dir("grade"), f"{cluster_name}.json")
    if os.path.exists(cache) and time.time() - os.path.getmtime(cache) < 60:
        with open(cache) as f:
            return json.load(f)
    c = clusters.get_cluster(cluster_name)
    k8s, _, _ = _clients(c)
    results, totals = [], {"success": 0, "warning": 0, "danger": 0}
    for d in k8s.get("/apis/apps/v1/deployments").get("items", []) + k8s.get("/apis/apps/v1/daemonsets").get("items", []):
        spec = d["spec"]["template"]["spec"]
        for ct in spec.get("containers", []):
            msgs = []
            for name, sev, fn in GRADE_CHECKS:
                bad = fn(ct, spec)
                msgs.append({"id": name, "type": sev if bad else "success", "success": not bad})
                totals[sev if bad else "success"] += 1
            results.append({"namespace": d["metadata"]["namespace"], "name": d["metadata"]["name"],
                            "kind": d.get("kind", "Deployment"), "container": ct["name"], "results": msgs})
    n = sum(totals.values()) or 1
    score = round(100.0 * (totals["success"] + 0.5 * totals["warning"]) / n)
    out = {"score": score, "totals": totals, "results": results}
    with open(cache, "w") as f:
        json.dump(out, f)
    return out


# ------------------------------------------------------------------------------------------- system logs
class JsonlLogHandler(logging.Handler):
    """Monthly JSONL system-log index (replaces the ES CMRESHandler, settings.py:228-276)."""

    def emit(self, record):
        try:
            doc = {"@timestamp": dt.datetime.utcfromtimestamp(record.created).isoformat() + "Z",
                   "levelname": record.levelname, "name": record.name, "msg": record.getMessage()}
            p = os.path.join(_data_dir("logs"), f"kubeoperator-{dt.date.today():%Y.%m}.jsonl")
            with open(p, "a") as f:
                f.write(json.dumps(doc) + "\n")
        except Exception:  # noqa: BLE001
            self.handleError(record)


def search_system_log(level: str | None = None, keywords: str | None = None, days: int = 7, limit: int = 50,
                      offset: int = 0) -> dict:
    """Reference log/es.py search_log: level, keywords, last N days, paging (newest first)."""
    since = dt.datetime.utcnow() - dt.timedelta(days=days)
    docs = []
    for p in sorted(glob.glob(os.path.join(_data_dir("logs"), "kubeoperator-*.jsonl")), reverse=True):
        with open(p) as f:
            for line in f:
                d = json.loads(line)
                if level and d.get("levelname") != level.upper():
                    continue
                if keywords and keywords.lower() not in d.get("msg", "").lower():
                    continue
                if d["@timestamp"][:19] < since.isoformat()[:19]:
                    continue
                docs.append(d)
    docs.sort(key=lambda d: d["@timestamp"], reverse=True)
    return {"total": len(docs), "items": docs[offset:offset + limit]}
