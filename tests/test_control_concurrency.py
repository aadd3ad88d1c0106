"""Control-plane concurrency across PROCESSES: the one-active-execution-per-cluster lock, IP
allocation and orphan recovery, each raced by spawned processes sharing one file-backed SQLite store -- the
deployment shape of an API server, a worker pool and a CLI on one host.

Reference behaviour being replaced: kubeops_api/api.py:244-248 (an unlocked "mark the previous STARTED execution
FAILURE" check), cloud_provider/models.py:140-144 (an unlocked read-modify-write of the zone's used IPs)."""
import multiprocessing as mp
import os
import threading
import time

import pytest
from sqlalchemy import select, update

from kubeoperator_amd.control.domain import cloud, clusters, deploy
from kubeoperator_amd.control.runtime import jobs
from kubeoperator_amd.control.store import models as M
from kubeoperator_amd.control.store.db import session_scope

CTX = mp.get_context("spawn")


def _child_store(data_dir: str):
    """A child process attaches to the parent's store through the production path (WAL, busy timeout)."""
    os.environ["KOP_PBKDF2_ITERS"] = "1000"
    from kubeoperator_amd.control.conf import Config, set_config
    from kubeoperator_amd.control.store import db

    cfg = Config(path=None)
    cfg["DATA_DIR"] = data_dir
    set_config(cfg)
    db.configure(cfg.db_url)


def _race_create(data_dir, rank, rounds, barrier, q):
    _child_store(data_dir)
    wins = []
    for r in range(rounds):
        barrier.wait()
        try:
            deploy.create("demo", "gpu-validate", run="queue")  # no worker runs: the job stays PENDING
            wins.append(r)
        except clusters.Conflict:
            pass
        barrier.wait()
        if rank == 0:  # finish this round's winner so the next round starts with a free cluster
            with session_scope() as s:
                s.execute(update(M.Execution).where(M.Execution.state == "PENDING").values(state="SUCCESS"))
                s.execute(update(M.Job).where(M.Job.state == "PENDING").values(state="SUCCESS"))
        barrier.wait()
    q.put((rank, wins))


def test_deploy_create_race_one_winner_per_round(control):
    clusters.create_cluster({"name": "demo", "template": "single-master"})
    rounds, nproc = 50, 2
    barrier, q = CTX.Barrier(nproc), CTX.Queue()
    ps = [CTX.Process(target=_race_create, args=(str(control.tmp / "data"), i, rounds, barrier, q))
          for i in range(nproc)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    per_round = [sum(r in got[i] for i in got) for r in range(rounds)]
    assert per_round == [1] * rounds, per_round
    with session_scope() as s:
        n = len(list(s.scalars(select(M.Execution).where(M.Execution.kind == "deploy"))))
    assert n == rounds


def test_partial_unique_index_rejects_second_active_execution(control):
    """The database itself refuses a second PENDING/STARTED deploy execution of one cluster, whatever code path
    inserts it; finished ones do not count."""
    from sqlalchemy.exc import IntegrityError

    c = clusters.create_cluster({"name": "demo", "template": "single-master"})
    pid = clusters.get_cluster(c["name"]).project_id
    with session_scope() as s:
        s.add(M.Execution(kind="deploy", project_id=pid, operation="install", state="SUCCESS"))
        s.add(M.Execution(kind="deploy", project_id=pid, operation="install", state="STARTED"))
        s.add(M.Execution(kind="playbook", project_id=pid, operation="x", state="STARTED"))
    with pytest.raises(IntegrityError):
        with session_scope() as s:
            s.add(M.Execution(kind="deploy", project_id=pid, operation="upgrade", state="PENDING"))


def _alloc(data_dir, zone_id, n, barrier, q):
    _child_store(data_dir)
    barrier.wait()
    q.put([cloud.allocate_ip(zone_id) for _ in range(n)])


def test_allocate_ip_two_processes_no_duplicates(control):
    with session_scope() as s:
        r = M.Region(name="r1", cloud_region="dc1", vars={"provider": "fake"})
        s.add(r)
        s.flush()
        z = M.Zone(name="z1", region_id=r.id, cloud_zone="a",
                   vars={"ip_start": "10.9.0.1", "ip_end": "10.9.0.200", "net_mask": "255.255.255.0"})
        s.add(z)
        s.flush()
        zid = z.id
    barrier, q = CTX.Barrier(2), CTX.Queue()
    ps = [CTX.Process(target=_alloc, args=(str(control.tmp / "data"), zid, 50, barrier, q)) for _ in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120) + q.get(timeout=120)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    assert len(got) == 100 and len(set(got)) == 100
    with session_scope() as s:
        used = s.get(M.Zone, zid).ip_used
    assert sorted(used) == sorted(got)


_release = threading.Event()


@jobs.task("test_blocking_job")
def _blocking_job(job_id, logger, **_):
    assert _release.wait(60)
    return {"ok": True}


def _start_second_pool(data_dir, q):
    _child_store(data_dir)
    pool = jobs.WorkerPool(concurrency=1, poll_s=0.05, heartbeat_s=1.0).start(recover=True)
    n = jobs.recover_orphans(1.0)
    pool.stop()
    q.put(n)


def test_second_worker_pool_leaves_live_job_alone(control):
    """A second worker process starting on the same store must not fail a job a live worker is running (nor
    free its cluster); the job ends SUCCESS."""
    _release.clear()
    pool = jobs.WorkerPool(concurrency=1, poll_s=0.05, heartbeat_s=0.2).start()
    try:
        jid = jobs.submit("test_blocking_job")
        t0 = time.time()
        while jobs.get(jid).state != "STARTED":
            assert time.time() - t0 < 30
            time.sleep(0.02)
        q = CTX.Queue()
        p = CTX.Process(target=_start_second_pool, args=(str(control.tmp / "data"), q))
        p.start()
        assert q.get(timeout=120) == 0
        p.join(30)
        assert p.exitcode == 0
        assert jobs.get(jid).state == "STARTED"
        _release.set()
        while jobs.get(jid).state == "STARTED":
            assert time.time() - t0 < 60
            time.sleep(0.02)
        assert jobs.get(jid).state == "SUCCESS"
    finally:
        _release.set()
        pool.stop()


def test_inline_run_is_not_an_orphan(control):
    """An inline run (CLI / run_inline) owns a heartbeat row: recovery started meanwhile leaves it alone."""
    _release.clear()
    out = {}
    t = threading.Thread(target=lambda: out.update(jobs.run_inline("test_blocking_job")))
    t.start()
    t0 = time.time()
    while True:
        with session_scope() as s:
            j = s.scalar(select(M.Job).where(M.Job.name == "test_blocking_job"))
        if j is not None and j.state == "STARTED":
            break
        assert time.time() - t0 < 30
        time.sleep(0.02)
    assert j.worker.startswith("inline:")
    assert jobs.recover_orphans(heartbeat_s=5.0) == 0
    _release.set()
    t.join(30)
    assert out["state"] == "SUCCESS"
    with session_scope() as s:  # the inline runner's liveness row is retired with its run
        assert s.get(M.WorkerHeartbeat, j.worker) is None


def test_dead_worker_jobs_and_executions_are_recovered(control):
    """Jobs of a worker whose pid is gone, or whose heartbeat is stale on another host, fail together with their
    execution; a job of a fresh worker does not."""
    import datetime as dt
    import subprocess
    import sys

    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    clusters.create_cluster({"name": "demo", "template": "single-master"})
    clusters.create_cluster({"name": "demo2", "template": "single-master"})
    e1 = deploy.create("demo", "gpu-validate", run="none")
    e2 = deploy.create("demo2", "gpu-validate", run="none")
    host = __import__("socket").gethostname()
    old = M.now() - dt.timedelta(seconds=120)
    with session_scope() as s:
        s.add(M.WorkerHeartbeat(name="w-dead", hostname=host, pid=dead.pid, last_seen=M.now()))
        s.add(M.WorkerHeartbeat(name="w-stale", hostname="elsewhere", pid=1, last_seen=old))
        s.add(M.WorkerHeartbeat(name="w-live", hostname="elsewhere", pid=1, last_seen=M.now()))
        s.add(M.Job(id=e1["id"], name="start_deploy_execution", state="STARTED", worker="w-dead"))
        s.add(M.Job(id=e2["id"], name="start_deploy_execution", state="STARTED", worker="w-stale"))
        s.add(M.Job(id="live-job", name="start_deploy_execution", state="STARTED", worker="w-live"))
        s.execute(update(M.Execution).where(M.Execution.id.in_((e1["id"], e2["id"]))).values(state="STARTED"))
    assert jobs.recover_orphans(heartbeat_s=5.0) == 2
    for eid in (e1["id"], e2["id"]):
        assert jobs.get(eid).state == "FAILURE"
        assert deploy.get(eid)["state"] == "FAILURE"
    assert jobs.get("live-job").state == "STARTED"
    deploy.create("demo", "gpu-validate", run="none")  # the cluster is free again


def test_index_added_to_an_older_store_retires_duplicate_active_executions(tmp_path, monkeypatch):
    """A store created before the one-active-execution index (several PENDING deploy executions of one cluster, as the
    old unlocked check allowed) still starts: the newest stays active, the others are marked FAILURE, the index is
    created and enforced from then on."""
    import sqlite3

    from sqlalchemy.exc import IntegrityError

    from kubeoperator_amd.control.conf import Config, set_config
    from kubeoperator_amd.control.store import db

    monkeypatch.setenv("KOP_PBKDF2_ITERS", "1000")
    cfg = Config(path=None)
    cfg["DATA_DIR"] = str(tmp_path / "data")
    set_config(cfg)
    db.configure(cfg.db_url)
    db.init_db()
    c = clusters.create_cluster({"name": "old", "template": "single-master"})
    pid = clusters.get_cluster(c["name"]).project_id
    path = cfg.db_url.split("///", 1)[1]
    con = sqlite3.connect(path)
    con.execute("DROP INDEX uq_one_active_deploy_per_project")
    for i, t in enumerate(("2020-01-01 00:00:00", "2020-01-02 00:00:00", "2020-01-03 00:00:00")):
        con.execute("INSERT INTO executions (id, kind, project_id, operation, params, steps, current_step, state, num, "
                    "timedelta, result_summary, result_raw, created_by, date_created) VALUES "
                    "(?, 'deploy', ?, 'install', '{}', '[]', 0, 'PENDING', 1, 0, '{}', '{}', '', ?)", (f"e{i}", pid, t))
    con.commit()
    con.close()
    db.configure(cfg.db_url)
    db.init_db()
    with session_scope() as s:
        states = {e.id: e.state for e in s.scalars(select(M.Execution).where(M.Execution.project_id == pid))}
    assert states == {"e0": "FAILURE", "e1": "FAILURE", "e2": "PENDING"}
    with pytest.raises(IntegrityError):
        with session_scope() as s:
            s.add(M.Execution(kind="deploy", project_id=pid, operation="upgrade", state="STARTED"))
