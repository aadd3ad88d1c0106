"""Background jobs run by the job runtime / scheduler (reference kubeops_api/tasks.py:28-89,
users/tasks.py, ansible_api/tasks.py run_im_adhoc)."""
from __future__ import annotations

from sqlalchemy import select

from ..runtime import jobs
from ..store import models as M
from ..store.db import session_scope
from . import backup, clusters, deploy, hosts, monitor, users


def _running_clusters() -> list[str]:
    with session_scope() as s:
        return [c.name for c in s.scalars(select(M.Cluster).where(M.Cluster.status.in_(("RUNNING", "WARNING"))))]


@jobs.task("cluster_backup_all")
def cluster_backup_all(job_id, logger):
    """Daily strategy backups + retention (reference cluster_backup_utils.cluster_backup)."""
    done = []
    for name, storage_id, save_num in backup.due_strategies():
        try:
            e = deploy.create(name, "backup", {"backupStorageId": storage_id}, run="inline")
            done.append((name, e["id"]))
            backup.apply_retention(clusters.get_cluster(name).id, save_num)
        except Exception as ex:  # noqa: BLE001
            logger.info(f"backup of {name} failed: {ex}")
    return {"backups": done}


@jobs.task("save_cluster_data")
def save_cluster_data(job_id, logger):
    out = {}
    for name in _running_clusters():
        try:
            monitor.set_cluster_data(name)
            h = monitor.cluster_health(name)
            monitor.record_availability(name, h["available_rate"])
            out[name] = "ok"
        except Exception as ex:  # noqa: BLE001
            out[name] = f"error: {ex}"
    return out


@jobs.task("save_cluster_events")
def save_cluster_events(job_id, logger):
    return {n: _safe(monitor.save_events, n) for n in _running_clusters()}


@jobs.task("host_health_check")
def host_health_check(job_id, logger):
    return hosts.host_health_check()


@jobs.task("node_health_check")
def node_health_check(job_id, logger):
    return {n: _safe(monitor.node_health, n) for n in _running_clusters()}


@jobs.task("save_loki_data")
def save_loki_data(job_id, logger):
    out = {}
    for n in _running_clusters():
        c = clusters.get_cluster(n)
        try:
            _, _, loki = monitor._clients(c)
            out[n] = loki.scalar('sum(count_over_time({level="error"}[1h]))') if loki else 0
        except Exception as ex:  # noqa: BLE001
            out[n] = f"error: {ex}"
    return out


@jobs.task("sync_ldap_users")
def sync_ldap(job_id, logger):
    return {"created": users.sync_ldap_users()}


@jobs.task("sync_host_info")
def sync_host_info(job_id, logger, host_id):
    return hosts.gather_info(host_id)


@jobs.task("run_adhoc")
def run_adhoc(job_id, logger, cluster, pattern, module, args=None):
    c = clusters.get_cluster(cluster)
    return clusters.run_adhoc(c, pattern, module, args or {}, logger=logger)["summary"]


def _safe(fn, *a):
    try:
        return fn(*a)
    except Exception as ex:  # noqa: BLE001
        return f"error: {ex}"
