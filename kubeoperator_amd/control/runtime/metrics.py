"""Prometheus metrics of the control plane, served on ``GET /metrics`` (the reference
only records per-execution timedelta; here executions, steps and jobs are histograms/counters and the
cluster / host / GPU inventory is exported as gauges computed at scrape time from the store)."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest
from prometheus_client.core import GaugeMetricFamily

REGISTRY = CollectorRegistry(auto_describe=True)
_DURATION_BUCKETS = (1, 5, 15, 30, 60, 120, 300, 600, 1200, 1800, 3600, 7200, 14400, float("inf"))

EXECUTION_SECONDS = Histogram("kubeoperator_execution_seconds", "Wall time of cluster operations",
                              ["operation", "state"], buckets=_DURATION_BUCKETS, registry=REGISTRY)
STEP_SECONDS = Histogram("kubeoperator_step_seconds", "Wall time of execution steps (playbooks)",
                         ["operation", "step", "status"], buckets=_DURATION_BUCKETS, registry=REGISTRY)
JOBS_TOTAL = Counter("kubeoperator_jobs_total", "Background jobs finished", ["name", "state"], registry=REGISTRY)
TASK_SECONDS = Histogram("kubeoperator_task_seconds", "Wall time of one playbook task on one host",
                         ["module", "status"], buckets=(0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120, 300, 600,
                                                        float("inf")), registry=REGISTRY)
TASKS_TOTAL = Counter("kubeoperator_playbook_tasks_total", "Playbook task results per host",
                      ["status"], registry=REGISTRY)


class _InventoryCollector:
    """Cluster counts by status, hosts by status, registered AMD GPUs (read from the store per scrape)."""

    def collect(self):
        from sqlalchemy import func, select

        from ..store import models as M
        from ..store.db import session_scope

        clusters = GaugeMetricFamily("kubeoperator_clusters", "Clusters by status", labels=["status"])
        hosts = GaugeMetricFamily("kubeoperator_hosts", "Registered hosts by status", labels=["status"])
        gpus = GaugeMetricFamily("kubeoperator_gpus", "AMD Instinct GPUs on registered hosts", labels=["model"])
        try:
            with session_scope() as s:
                for status, n in s.execute(select(M.Cluster.status, func.count()).group_by(M.Cluster.status)):
                    clusters.add_metric([status], n)
                by_model: dict[str, int] = {}
                for status, gl in s.execute(select(M.Host.status, M.Host.gpus)):
                    for g in gl or []:
                        by_model[g.get("name", "unknown")] = by_model.get(g.get("name", "unknown"), 0) + 1
                for status, n in s.execute(select(M.Host.status, func.count()).group_by(M.Host.status)):
                    hosts.add_metric([status], n)
                for model, n in by_model.items():
                    gpus.add_metric([model], n)
        except Exception:  # noqa: BLE001 - a scrape must not fail because the store is busy
            pass
        yield clusters
        yield hosts
        yield gpus


REGISTRY.register(_InventoryCollector())


def exposition() -> bytes:
    return generate_latest(REGISTRY)
