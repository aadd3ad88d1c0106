"""Engine / session management and first-run seeding of the control-plane store.

SQLite in WAL mode (concurrent readers with one writer, busy timeout 30 s) replaces the reference's MySQL;
any SQLAlchemy URL can be configured with ``DB_URL``. ``init_db`` creates the schema, records the schema
version and seeds what the reference seeds in migrations: the ``admin`` superuser
(users/migrations/0001_create_user.py:13), the default item "KubeOperator"
(kubeops_api/migrations/0058_auto_20200210_0618.py:11-17), the ``local_hostname`` setting
(kubeops_api/migrations/0005...py:15) and the cloud-provider templates.
"""
from __future__ import annotations

import contextlib
import threading

from sqlalchemy import create_engine, event, select
from sqlalchemy.orm import Session, sessionmaker

from . import models as M
from .crypto import hash_password

SCHEMA_VERSION = 1

_lock = threading.Lock()
_engine = None
_Session = None


def _sqlite_pragmas(dbapi_conn, _rec):
    cur = dbapi_conn.cursor()
    cur.execute("PRAGMA journal_mode=WAL")
    cur.execute("PRAGMA synchronous=NORMAL")
    cur.execute("PRAGMA foreign_keys=ON")
    cur.execute("PRAGMA busy_timeout=30000")
    cur.close()


def configure(url: str):
    global _engine, _Session
    with _lock:
        kw = {}
        if url.startswith("sqlite"):
            kw["connect_args"] = {"check_same_thread": False, "timeout": 30}
        eng = create_engine(url, future=True, **kw)
        if url.startswith("sqlite"):
            event.listen(eng, "connect", _sqlite_pragmas)
        _engine = eng
        _Session = sessionmaker(bind=eng, expire_on_commit=False, future=True)
        return eng


def engine():
    if _engine is None:
        from ..conf import get_config

        configure(get_config().db_url)
    return _engine


def session() -> Session:
    engine()
    return _Session()


@contextlib.contextmanager
def session_scope():
    s = session()
    try:
        yield s
        s.commit()
    except Exception:
        s.rollback()
        raise
    finally:
        s.close()


_write_lock = threading.RLock()


@contextlib.contextmanager
def write_scope():
    """A session whose transaction takes the store's write lock before its first read, for read-check-write
    sequences that must be atomic across threads AND processes (one active execution per cluster, IP
    allocation). SQLite: ``BEGIN IMMEDIATE`` -- the write lock up front, so a second writer (another thread or
    another process on the same file) waits in ``busy_timeout`` instead of interleaving its check with ours.
    Other databases: the caller's ``with_for_update`` row locks do the same job. A process-local lock also
    serialises threads that share one connection (the in-memory test store's single pooled connection, where
    a nested ``BEGIN`` is not allowed). Replaces the reference's unlocked check-then-insert
    (kubeops_api/api.py:244-248, cloud_provider/models.py:140-144)."""
    with _write_lock:
        s = session()
        try:
            conn = s.connection()
            if conn.dialect.name == "sqlite":
                dbapi = conn.connection.dbapi_connection
                if not dbapi.in_transaction:
                    conn.exec_driver_sql("BEGIN IMMEDIATE")
            yield s
            s.commit()
        except Exception:
            s.rollback()
            raise
        finally:
            s.close()


def _retire_duplicate_active_executions() -> int:
    """Before the one-active-execution index is added to an older store: a cluster holding several PENDING / STARTED
    deploy executions (possible before the lock was atomic) keeps its newest, the others are marked FAILURE."""
    n = 0
    with session_scope() as s:
        rows = list(s.scalars(select(M.Execution).where(M.Execution.kind == "deploy",
                                                        M.Execution.state.in_(("PENDING", "STARTED")))
                              .order_by(M.Execution.project_id, M.Execution.date_created.desc())))
        seen = set()
        for e in rows:
            if e.project_id in seen:
                e.state, e.date_end = "FAILURE", M.now()
                e.result_summary = {"error": "superseded: a newer operation was active when the store was upgraded"}
                n += 1
            seen.add(e.project_id)
    return n


def ensure_indexes() -> None:
    """Create indexes added after a store's tables were first created (``create_all`` skips existing tables)."""
    from sqlalchemy import inspect as sa_inspect

    eng = engine()
    insp = sa_inspect(eng)
    for t in M.Base.metadata.sorted_tables:
        existing = {ix["name"] for ix in insp.get_indexes(t.name)} if insp.has_table(t.name) else set()
        for ix in t.indexes:
            if ix.name in existing:
                continue
            if ix.name == "uq_one_active_deploy_per_project":
                _retire_duplicate_active_executions()
            ix.create(eng, checkfirst=True)


def init_db(admin_password: str | None = None) -> None:
    from ..conf import get_config

    eng = engine()
    M.Base.metadata.create_all(eng)
    ensure_indexes()
    cfg = get_config()
    with session_scope() as s:
        if s.get(M.SchemaVersion, SCHEMA_VERSION) is None:
            s.add(M.SchemaVersion(version=SCHEMA_VERSION))
        if s.scalar(select(M.User).where(M.User.username == "admin")) is None:
            s.add(M.User(username="admin", email="admin@kubeoperator.local", is_superuser=True,
                         password_hash=hash_password(admin_password or cfg["ADMIN_PASSWORD"])))
        if s.scalar(select(M.Item).where(M.Item.name == "KubeOperator")) is None:
            s.add(M.Item(name="KubeOperator", description="default item"))
        if s.scalar(select(M.Setting).where(M.Setting.key == "local_hostname")) is None:
            s.add(M.Setting(tab="system", key="local_hostname", value="127.0.0.1"))
        for name, meta in _cloud_templates().items():
            if s.scalar(select(M.CloudProviderTemplate).where(M.CloudProviderTemplate.name == name)) is None:
                s.add(M.CloudProviderTemplate(name=name, meta=meta))


def _cloud_templates() -> dict:
    import os

    import yaml

    from ..conf import RESOURCE_DIR

    out = {}
    root = os.path.join(RESOURCE_DIR, "clouds")
    if os.path.isdir(root):
        for name in sorted(os.listdir(root)):
            p = os.path.join(root, name, "meta.yml")
            if os.path.isfile(p):
                with open(p) as f:
                    out[name] = yaml.safe_load(f) or {}
    return out


def reset_for_tests(url: str = "sqlite://") -> None:
    """Fresh in-memory (or given) database; used by the test-suite."""
    from sqlalchemy.pool import StaticPool

    global _engine, _Session
    with _lock:
        kw = {"connect_args": {"check_same_thread": False}}
        if url == "sqlite://":
            kw["poolclass"] = StaticPool
        eng = create_engine(url, future=True, **kw)
        event.listen(eng, "connect", lambda c, r: c.execute("PRAGMA foreign_keys=ON"))
        _engine = eng
        _Session = sessionmaker(bind=eng, expire_on_commit=False, future=True)
