"""Durable job runtime: queue in the store, worker threads, per-job log files, crash recovery.

Replaces Celery worker + Redis broker + result backend (reference core/kubeops.py:143-194,
celery_api/*). A job row is claimed atomically (``UPDATE ... WHERE state='PENDING'``), so any number of
worker processes can share one store; ``WORKER_CONCURRENCY`` threads per process (reference: prefork
``-c 4``). Each job's log goes to ``<DATA_DIR>/celery/<id[0]>/<id[1]>/<id>.log`` -- the reference's path
convention (celery_api/utils.py:212-217) -- which the log API / websocket tail.

Recovery: a job left STARTED by a DEAD worker is marked FAILURE, together with the execution of the same id,
instead of the reference's "mark the previous STARTED execution FAILURE when a new one starts"
(kubeops_api/api.py:244-248). Every runner -- pool workers and inline runs (CLI, ``run_inline``) alike -- owns a
heartbeat row; a worker counts as dead when its row is missing, its pid is gone on this host, or it has not
beaten for ``3 x heartbeat_s``. A live worker's jobs are never touched, so a second worker process starting on
the same store cannot unlock a cluster whose operation is still running.

Task monitor (the reference runs Celery Flower, core/kubeops.py:197-213, proxied at /flower/): every worker
process keeps a heartbeat row (jobs running, jobs processed, last seen); ``stats`` aggregates the job table per
task name; a PENDING job can be revoked (REVOKED: never claimed) and a finished one retried as a new job.
"""
from __future__ import annotations

import logging
import os
import socket
import threading
import time
import traceback
import uuid

from sqlalchemy import delete, select, update

from ..store import models as M
from ..store.db import session_scope

log = logging.getLogger("kubeoperator.runtime")

_TASKS: dict[str, callable] = {}


def task(name: str):
    """Register a job function ``fn(job_id, logger, **args) -> dict``."""
    def deco(fn):
        _TASKS[name] = fn
        fn.task_name = name
        return fn
    return deco


def registered_tasks() -> list[str]:
    return sorted(_TASKS)


def log_path(job_id: str) -> str:
    from ..conf import get_config

    d = os.path.join(get_config().data_dir, "celery", job_id[0], job_id[1])
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"{job_id}.log")


class JobLogger:
    """Line logger bound to one job's log file (also the engine's display callback)."""

    def __init__(self, path: str):
        self.path = path
        self._f = open(path, "a", buffering=1)
        self._lock = threading.Lock()

    def __call__(self, msg: str) -> None:
        self.write(msg)

    def write(self, msg: str) -> None:
        with self._lock:
            self._f.write(msg if msg.endswith("\n") else msg + "\n")
            self._f.flush()

    def info(self, msg: str) -> None:
        self.write(f"{time.strftime('%Y-%m-%d %H:%M:%S')} {msg}")

    def close(self):
        with self._lock:
            self._f.close()


def tail(path: str, offset: int = 0, limit: int = 4096) -> tuple[str, int]:
    """Read up to ``limit`` bytes of a log from ``offset`` (reference LogTailApi / ws.py: 4 KiB chunks)."""
    if not os.path.exists(path):
        return "", offset
    with open(path, "rb") as f:
        f.seek(offset)
        data = f.read(limit)
    return data.decode(errors="replace"), offset + len(data)


def add_job(s, name: str, args: dict | None = None, job_id: str | None = None, inline: bool = False) -> M.Job:
    """Add a job row inside the caller's transaction ``s`` (so e.g. an execution and its job commit together).
    ``inline=True``: the row is born STARTED and owned by a fresh inline worker with its own heartbeat row, so no
    pool worker can claim it between insert and run; run it with ``run_claimed``."""
    if name not in _TASKS:
        raise KeyError(f"unknown task {name!r}")
    jid = job_id or str(uuid.uuid4())
    if inline:
        t = M.now()
        wname = f"inline:{socket.gethostname()}:{os.getpid()}:{uuid.uuid4().hex[:8]}"
        s.add(M.WorkerHeartbeat(name=wname, hostname=socket.gethostname(), pid=os.getpid(), concurrency=1,
                                started=t, last_seen=t, active=[jid], processed=0, stopped=False))
        job = M.Job(id=jid, name=name, args=args or {}, state="STARTED", worker=wname, date_start=t, attempts=1,
                    log_path=log_path(jid))
    else:
        job = M.Job(id=jid, name=name, args=args or {}, state="PENDING", log_path=log_path(jid))
    s.add(job)
    return job


def wake() -> None:
    """Tell this process's idle workers that a job was queued (other processes find it on their next poll)."""
    _wake.set()


def submit(name: str, args: dict | None = None, job_id: str | None = None) -> str:
    with session_scope() as s:
        jid = add_job(s, name, args, job_id).id
    wake()
    return jid


def get(job_id: str) -> M.Job | None:
    with session_scope() as s:
        return s.get(M.Job, job_id)


def revoke(job_id: str) -> tuple[bool, str]:
    """PENDING -> REVOKED (a worker never claims it): (True, "REVOKED"). Any other state -- a running job cannot
    be stopped from outside its thread -- is left alone: (False, state)."""
    with session_scope() as s:
        n = s.execute(update(M.Job).where(M.Job.id == job_id, M.Job.state == "PENDING")
                      .values(state="REVOKED", date_end=M.now(), result={"error": "revoked"})).rowcount
        j = s.get(M.Job, job_id)
        if j is None:
            raise KeyError(job_id)
        return (True, "REVOKED") if n else (False, j.state)


def retry(job_id: str) -> str:
    """Submit a finished (FAILURE / REVOKED / SUCCESS) job again with the same task and arguments."""
    j = get(job_id)
    if j is None:
        raise KeyError(job_id)
    if j.state in ("PENDING", "STARTED"):
        raise ValueError(f"job {job_id} is {j.state}")
    return submit(j.name, dict(j.args or {}))


def stats(since: "dt.datetime | None" = None) -> list[dict]:
    """Per task name: job counts by state and run-time statistics of the finished ones."""
    import collections

    agg: dict = collections.defaultdict(lambda: {"states": collections.Counter(), "runtimes": []})
    with session_scope() as s:
        q = select(M.Job.name, M.Job.state, M.Job.date_start, M.Job.date_end)
        if since is not None:
            q = q.where(M.Job.date_created >= since)
        for name, state, t0, t1 in s.execute(q):
            a = agg[name]
            a["states"][state] += 1
            if t0 is not None and t1 is not None:
                a["runtimes"].append((t1 - t0).total_seconds())
    out = []
    for name, a in sorted(agg.items()):
        rt = sorted(a["runtimes"])
        out.append({"task": name, "total": sum(a["states"].values()), **{k.lower(): v for k, v in a["states"].items()},
                    "runtime_avg_s": round(sum(rt) / len(rt), 3) if rt else None,
                    "runtime_p50_s": round(rt[len(rt) // 2], 3) if rt else None,
                    "runtime_max_s": round(rt[-1], 3) if rt else None})
    return out


def workers(online_after_s: float = 30.0) -> list[dict]:
    now = M.now()
    with session_scope() as s:
        rows = list(s.scalars(select(M.WorkerHeartbeat).order_by(M.WorkerHeartbeat.name)))
        return [{"name": w.name, "hostname": w.hostname, "pid": w.pid, "concurrency": w.concurrency,
                 "started": w.started, "last_seen": w.last_seen, "active": list(w.active or []),
                 "processed": w.processed,
                 "online": (not w.stopped and w.last_seen is not None
                            and (now - w.last_seen).total_seconds() < online_after_s)} for w in rows]


def _claim(worker: str) -> M.Job | None:
    with session_scope() as s:
        for j in s.scalars(select(M.Job).where(M.Job.state == "PENDING").order_by(M.Job.date_created).limit(8)):
            n = s.execute(update(M.Job).where(M.Job.id == j.id, M.Job.state == "PENDING")
                          .values(state="STARTED", worker=worker, date_start=M.now(), attempts=j.attempts + 1)).rowcount
            if n == 1:
                s.flush()
                return s.get(M.Job, j.id)
    return None


def run_job(job: M.Job) -> dict:
    fn = _TASKS[job.name]
    lg = JobLogger(job.log_path or log_path(job.id))
    lg.info(f"Start task: {job.name} {job.id}")
    state, result = "SUCCESS", {}
    try:
        out = fn(job.id, lg, **(job.args or {}))
        result = out if isinstance(out, dict) else {"result": out}
    except Exception as e:  # noqa: BLE001 - a job failure is data, not a crash
        state = "FAILURE"
        result = {"error": f"{type(e).__name__}: {e}"}
        lg.write(traceback.format_exc())
    lg.info(f"Task finish: {state}")
    lg.close()
    with session_scope() as s:
        s.execute(update(M.Job).where(M.Job.id == job.id).values(state=state, result=result, date_end=M.now()))
    from . import metrics

    metrics.JOBS_TOTAL.labels(job.name, state).inc()
    return {"state": state, "result": result}


def run_inline(name: str, args: dict | None = None, job_id: str | None = None) -> dict:
    """Execute a new job in the calling thread (tests, CLI, single-process mode)."""
    with session_scope() as s:
        job = add_job(s, name, args, job_id, inline=True)
    return {"id": job.id, **run_claimed(job)}


INLINE_HEARTBEAT_S = 5.0


def claim_pending(jid: str) -> M.Job:
    """Claim one PENDING job for the calling thread (an inline worker with a heartbeat row, as ``add_job``'s
    ``inline``); raises if a pool worker took it first. Run it with ``run_claimed``."""
    name = f"inline:{socket.gethostname()}:{os.getpid()}:{uuid.uuid4().hex[:8]}"
    with session_scope() as s:
        n = s.execute(update(M.Job).where(M.Job.id == jid, M.Job.state == "PENDING")
                      .values(state="STARTED", worker=name, date_start=M.now(), attempts=M.Job.attempts + 1)).rowcount
        if n != 1:
            raise RuntimeError(f"job {jid} is not PENDING")
        s.add(M.WorkerHeartbeat(name=name, hostname=socket.gethostname(), pid=os.getpid(), concurrency=1,
                                started=M.now(), last_seen=M.now(), active=[jid], processed=0, stopped=False))
        s.flush()
        return s.get(M.Job, jid)


def run_claimed(job: M.Job, heartbeat_s: float = INLINE_HEARTBEAT_S) -> dict:
    """``run_job`` for an inline-owned job (``add_job(inline=True)`` / ``claim_pending``): a daemon thread beats the inline
    worker's row every ``heartbeat_s`` until the job ends; the row is then deleted (it existed only to prove the run
    alive, and the task monitor lists worker processes, not finished inline runs)."""
    stop = threading.Event()

    def beat():
        with session_scope() as s:
            s.execute(update(M.WorkerHeartbeat).where(M.WorkerHeartbeat.name == job.worker)
                      .values(last_seen=M.now()))

    def loop():
        while not stop.wait(heartbeat_s):
            try:
                beat()
            except Exception:  # noqa: BLE001 - a missed heartbeat is not fatal
                log.exception("inline heartbeat failed")

    t = threading.Thread(target=loop, name="kop-inline-heartbeat", daemon=True)
    t.start()
    try:
        return run_job(job)
    finally:
        stop.set()
        t.join(heartbeat_s + 1.0)
        try:
            with session_scope() as s:
                s.execute(delete(M.WorkerHeartbeat).where(M.WorkerHeartbeat.name == job.worker))
        except Exception:  # noqa: BLE001
            log.exception("retiring the inline worker row failed")


def _pid_alive(pid: int) -> bool:
    if pid <= 0:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def worker_dead(w: M.WorkerHeartbeat | None, now, stale_s: float) -> bool:
    """The liveness rule orphan recovery applies to a job's worker row."""
    if w is None:
        return True
    if w.hostname == socket.gethostname() and not _pid_alive(int(w.pid or 0)):
        return True
    return w.last_seen is None or (now - w.last_seen).total_seconds() > stale_s


def recover_orphans(heartbeat_s: float = 5.0) -> int:
    """Mark jobs left STARTED by a dead worker (see ``worker_dead``; stale after ``3 x heartbeat_s``) as
    FAILURE, each together with its execution (same id). Jobs of live workers -- other pool processes, inline
    runs -- are left alone. Returns how many jobs were failed."""
    now = M.now()
    n = 0
    with session_scope() as s:
        rows = list(s.execute(select(M.Job.id, M.Job.worker).where(M.Job.state == "STARTED")))
        beats = {w.name: w for w in s.scalars(select(M.WorkerHeartbeat).where(
            M.WorkerHeartbeat.name.in_({wk for _, wk in rows})))} if rows else {}
        for jid, wk in rows:
            if not worker_dead(beats.get(wk), now, 3.0 * heartbeat_s):
                continue
            err = {"error": f"worker died ({wk or 'unknown'})"}
            k = s.execute(update(M.Job).where(M.Job.id == jid, M.Job.state == "STARTED", M.Job.worker == wk)
                          .values(state="FAILURE", result=err, date_end=now)).rowcount
            if k:
                n += k
                s.execute(update(M.Execution).where(M.Execution.id == jid,
                                                    M.Execution.state.in_(("PENDING", "STARTED")))
                          .values(state="FAILURE", date_end=now, result_summary=err))
    return n


_wake = threading.Event()


class WorkerPool:
    def __init__(self, concurrency: int | None = None, poll_s: float = 1.0, heartbeat_s: float = 5.0):
        from ..conf import get_config

        self.concurrency = concurrency or int(get_config()["WORKER_CONCURRENCY"])
        self.poll_s = poll_s
        self.heartbeat_s = heartbeat_s
        self.name = f"{socket.gethostname()}:{os.getpid()}:{id(self) & 0xffff:04x}"
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._active: set = set()
        self._processed = 0
        self._lock = threading.Lock()

    def start(self, recover: bool = True):
        self._recover = recover
        if recover:
            self._recover_orphans()
        with session_scope() as s:
            s.merge(M.WorkerHeartbeat(name=self.name, hostname=socket.gethostname(), pid=os.getpid(),
                                      concurrency=self.concurrency, started=M.now(), last_seen=M.now(), active=[],
                                      processed=0, stopped=False))
        for i in range(self.concurrency):
            t = threading.Thread(target=self._loop, name=f"kop-worker-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        hb = threading.Thread(target=self._heartbeat_loop, name="kop-worker-heartbeat", daemon=True)
        hb.start()
        self._threads.append(hb)
        return self

    def _beat(self, stopped: bool = False) -> None:
        with self._lock:
            active, processed = sorted(self._active), self._processed
        with session_scope() as s:
            s.execute(update(M.WorkerHeartbeat).where(M.WorkerHeartbeat.name == self.name)
                      .values(last_seen=M.now(), active=active, processed=processed, stopped=stopped))

    def _safe_beat(self) -> None:
        """A heartbeat inside the job loop: a store error (e.g. SQLite 'database is locked') is logged and never
        stops the claimed job or kills the worker thread (the periodic loop beats again shortly)."""
        try:
            self._beat()
        except Exception:  # noqa: BLE001
            log.exception("worker heartbeat failed")

    def _recover_orphans(self) -> None:
        n = recover_orphans(self.heartbeat_s)
        if n:
            log.warning("recovered %d orphaned jobs", n)

    def _heartbeat_loop(self):
        beats = 0
        while not self._stop.wait(self.heartbeat_s):
            try:
                self._beat()
                beats += 1
                if self._recover and beats % 6 == 0:  # a worker that dies later is noticed without a restart
                    self._recover_orphans()
            except Exception:  # noqa: BLE001 - a missed heartbeat is not fatal
                log.exception("worker heartbeat failed")

    def _loop(self):
        while not self._stop.is_set():
            job = _claim(self.name)
            if job is None:
                _wake.wait(self.poll_s)
                _wake.clear()
                continue
            with self._lock:
                self._active.add(job.id)
            self._safe_beat()
            try:
                run_job(job)
            finally:
                with self._lock:
                    self._active.discard(job.id)
                    self._processed += 1
                self._safe_beat()

    def stop(self, timeout: float = 5.0):
        self._stop.set()
        _wake.set()
        for t in self._threads:
            t.join(timeout)
        with self._lock:
            busy = bool(self._active)
        try:
            # A job still running in a (daemon) worker thread: the row is not marked stopped.
            self._beat(stopped=not busy)
        except Exception:  # noqa: BLE001
            pass
