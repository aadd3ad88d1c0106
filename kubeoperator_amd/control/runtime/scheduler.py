"""Periodic-job scheduler (replaces celery beat + django-celery-beat's DatabaseScheduler).

Schedules live in the ``periodic_tasks`` table (interval seconds or a 5-field crontab "m h dom mon dow"
with ``*``, ``*/n``, lists and ranges); a scheduler thread submits due jobs to the job queue.
Default schedule = the reference's beat table (kubeops_api/tasks.py:40-89): cluster backup daily at
01:00, cluster data every 5 min, events every 5 min, host health every 5 min, node health every 5 min,
Loki error counts hourly; plus the LDAP user sync (users/tasks.py).
"""
from __future__ import annotations

import datetime as dt
import logging
import threading

from sqlalchemy import select

from ..store import models as M
from ..store.db import session_scope
from . import jobs

log = logging.getLogger("kubeoperator.scheduler")

DEFAULT_SCHEDULE = [
    ("cluster-backup-daily", "cluster_backup_all", "0 1 * * *", 0),
    ("save-cluster-data", "save_cluster_data", "", 300),
    ("save-cluster-events", "save_cluster_events", "", 300),
    ("host-health-check", "host_health_check", "", 300),
    ("node-health-check", "node_health_check", "", 300),
    ("loki-error-counts", "save_loki_data", "0 * * * *", 0),
    ("ldap-user-sync", "sync_ldap_users", "0 2 * * *", 0),
]


def _field_match(spec: str, value: int) -> bool:
    for part in spec.split(","):
        if part == "*":
            return True
        step = 1
        if "/" in part:
            part, s = part.split("/")
            step = int(s)
            if part == "*":
                if value % step == 0:
                    return True
                continue
        if "-" in part:
            a, b = map(int, part.split("-"))
            if a <= value <= b and (value - a) % step == 0:
                return True
        elif part and int(part) == value:
            return True
    return False


def cron_match(expr: str, t: dt.datetime) -> bool:
    m, h, dom, mon, dow = expr.split()
    return (_field_match(m, t.minute) and _field_match(h, t.hour) and _field_match(dom, t.day)
            and _field_match(mon, t.month) and _field_match(dow, (t.weekday() + 1) % 7))


def seed_defaults() -> None:
    with session_scope() as s:
        for name, task, cron, interval in DEFAULT_SCHEDULE:
            if s.scalar(select(M.PeriodicTask).where(M.PeriodicTask.name == name)) is None:
                s.add(M.PeriodicTask(name=name, task=task, crontab=cron, interval_s=interval))


def register(name: str, task: str, crontab: str = "", interval_s: int = 0, args: dict | None = None,
             enabled: bool = True) -> None:
    """Create or update a schedule (reference create_or_update_periodic_task, celery_api/utils.py:59-133)."""
    with session_scope() as s:
        pt = s.scalar(select(M.PeriodicTask).where(M.PeriodicTask.name == name))
        if pt is None:
            pt = M.PeriodicTask(name=name, task=task)
            s.add(pt)
        pt.task, pt.crontab, pt.interval_s, pt.args, pt.enabled = task, crontab, interval_s, args or {}, enabled


def due(now: dt.datetime | None = None) -> list[tuple[str, str, dict]]:
    """Schedules due at ``now`` (minute resolution for crontab); marks them as run."""
    now = now or M.now()
    out = []
    with session_scope() as s:
        for pt in s.scalars(select(M.PeriodicTask).where(M.PeriodicTask.enabled.is_(True))):
            last = pt.last_run
            if pt.interval_s:
                ok = last is None or (now - last).total_seconds() >= pt.interval_s
            elif pt.crontab:
                ok = cron_match(pt.crontab, now) and (last is None or last.replace(second=0, microsecond=0)
                                                      < now.replace(second=0, microsecond=0))
            else:
                ok = False
            if ok:
                pt.last_run = now
                out.append((pt.name, pt.task, dict(pt.args or {})))
    return out


class Scheduler:
    def __init__(self, tick_s: float = 20.0):
        self.tick_s = tick_s
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def tick(self, now=None) -> list[str]:
        fired = []
        for name, task, args in due(now):
            if task in jobs.registered_tasks():
                jobs.submit(task, args)
                fired.append(name)
            else:
                log.debug("schedule %s: task %s not registered", name, task)
        return fired

    def start(self):
        seed_defaults()
        self._t = threading.Thread(target=self._loop, name="kop-scheduler", daemon=True)
        self._t.start()
        return self

    def _loop(self):
        while not self._stop.wait(self.tick_s):
            try:
                self.tick()
            except Exception:  # noqa: BLE001
                log.exception("scheduler tick failed")

    def stop(self):
        self._stop.set()
