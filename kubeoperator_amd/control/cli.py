"""``kubeopsctl`` -- service launcher and command-line client of the control plane.

Service management (reference ``core/kubeops.py`` start/stop/status/restart of web / celery / beat / flower
with pidfiles, and the host-side ``kubeopsctl.sh``):

    kubeopsctl init                          # create the store, seed admin / item / settings
    kubeopsctl start [all|web|worker|beat] [-d]
    kubeopsctl stop|status|restart [all|web|worker|beat]
    kubeopsctl install [--start] | uninstall [--purge] | upgrade     # the operator itself (5/6/7_*.sh)
    kubeopsctl reload [SVC] | down [SVC] | tail [SVC] [-n N] [-f]    # (re)start, stop + clean, follow logs
    kubeopsctl python [-c CODE] | db [-c SQL]                         # shell with the store loaded / SQL shell
    kubeopsctl exec SVC [-- CMD]                                      # a shell in the service's environment

Cluster operations (the UI's flows, usable headless; ``--server URL`` talks to a running control plane over
the REST API, otherwise the store is used in-process and operations run inline with their log on stdout):

    kubeopsctl host add NAME IP [--password P | --credential C] | host list | host import FILE | host gpu-check NAME
    kubeopsctl cluster create -f plan.yml        # cluster-plan YAML (name/template/package/network/storage/nodes)
    kubeopsctl cluster install|uninstall NAME [--resume]
    kubeopsctl cluster scale NAME --num N        # AUTOMATIC (IaaS) clusters
    kubeopsctl cluster add-worker NAME --host H | remove-worker NAME --node N
    kubeopsctl cluster upgrade NAME --package P
    kubeopsctl cluster backup NAME --storage S | restore NAME --backup ID
    kubeopsctl cluster gpu-validate NAME | list | show NAME | kubeconfig NAME | delete NAME
    kubeopsctl exec list NAME | exec log ID
    kubeopsctl app deploy NAME --chart nginx|pytorch-rocm-train [--release R] [--namespace N] [--set k=v ...]
                   [--wait-job]                  # Helm release; a training run reports its tokens/s
    kubeopsctl app list NAME | app remove NAME --release R [--namespace N]
    kubeopsctl package list
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

import yaml

SERVICES = ("web", "worker", "beat", "repo")  # repo: per-package file repository + OCI registry


# ------------------------------------------------------------------------------------------------ bootstrap
def _bootstrap(config: str | None = None):
    from .conf import Config, set_config
    from .store import db

    if config:
        os.environ["KUBEOPERATOR_CONFIG"] = config
        set_config(Config(path=config))
    from .conf import get_config

    db.configure(get_config().db_url)
    db.init_db()
    from .domain import deploy, storage, tasks  # noqa: F401  (registers jobs)
    return get_config()


def _pid_dir(cfg) -> str:
    d = os.path.join(cfg.data_dir, "tmp")
    os.makedirs(d, exist_ok=True)
    return d


def _pidfile(cfg, svc: str) -> str:
    return os.path.join(_pid_dir(cfg), f"{svc}.pid")


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def _read_pid(cfg, svc) -> int | None:
    try:
        with open(_pidfile(cfg, svc)) as f:
            pid = int(f.read().strip())
        return pid if _alive(pid) else None
    except (OSError, ValueError):
        return None


def _expand(which: str) -> list[str]:
    return list(SERVICES) if which in ("all", "", None) else [which]


def run_services(cfg, services: list[str]) -> int:
    """Foreground: web server + worker pool + scheduler in this process (threads), until SIGTERM/SIGINT."""
    import logging

    from .domain.monitor import JsonlLogHandler
    from .runtime import jobs, scheduler

    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    logging.getLogger().addHandler(JsonlLogHandler())
    for svc in services:
        with open(_pidfile(cfg, svc), "w") as f:
            f.write(str(os.getpid()))
    pool = sched = None
    if "worker" in services:
        pool = jobs.WorkerPool().start()
    if "beat" in services:
        sched = scheduler.Scheduler().start()
    repo_stop = threading.Event()
    if "repo" in services:  # reference: one Nexus container per package (package_manage.py:31-45)
        from .domain import packages

        host = str(cfg["HTTP_BIND_HOST"] or "0.0.0.0")
        packages.serve_all(host)

        def rescan():  # packages dropped into PACKAGE_DIR later are served without a restart
            while not repo_stop.wait(60):
                try:
                    packages.serve_all(host)
                except Exception:  # noqa: BLE001 -- a bad package must not stop the loop
                    logging.getLogger("kubeops.packages").exception("package rescan failed")

        threading.Thread(target=rescan, name="pkg-rescan", daemon=True).start()
    try:
        if "web" in services:
            from .api import create_app
            from .api.server import run

            run(create_app(), str(cfg["HTTP_BIND_HOST"] or "0.0.0.0"), int(cfg["HTTP_LISTEN_PORT"]))
        else:
            stop = []
            signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
            while not stop:
                time.sleep(0.5)
    except KeyboardInterrupt:
        pass
    finally:
        repo_stop.set()
        if "repo" in services:
            from .domain import packages

            packages.stop_servers()
        if pool:
            pool.stop()
        if sched:
            sched.stop()
        for svc in services:
            try:
                os.remove(_pidfile(cfg, svc))
            except OSError:
                pass
    return 0


def cmd_start(a, cfg) -> int:
    svcs = _expand(a.service)
    running = [s for s in svcs if _read_pid(cfg, s)]
    if running:
        print(f"already running: {', '.join(running)}")
        return 1
    if not a.daemon:
        return run_services(cfg, svcs)
    logf = open(os.path.join(_pid_dir(cfg), "kubeops.log"), "a")
    env = dict(os.environ)
    if a.config:
        env["KUBEOPERATOR_CONFIG"] = a.config
    p = subprocess.Popen([sys.executable, "-m", "kubeoperator_amd.control.cli", "start", a.service or "all"],
                         stdout=logf, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    for _ in range(50):
        if all(_read_pid(cfg, s) for s in svcs) or p.poll() is not None:
            break
        time.sleep(0.1)
    ok = p.poll() is None
    print(f"{'started' if ok else 'failed to start'}: {', '.join(svcs)} (pid {p.pid})")
    return 0 if ok else 1


def cmd_stop(a, cfg) -> int:
    pids = {s: _read_pid(cfg, s) for s in _expand(a.service)}
    for pid in {p for p in pids.values() if p}:
        os.kill(pid, signal.SIGTERM)
    for _ in range(100):
        if not any(_read_pid(cfg, s) for s in pids):
            break
        time.sleep(0.1)
    for s, pid in pids.items():
        print(f"{s}: {'stopped' if pid else 'not running'}")
    return 0


def cmd_status(a, cfg) -> int:
    rc = 0
    for s in _expand(a.service):
        pid = _read_pid(cfg, s)
        print(f"{s}: {'running (pid %d)' % pid if pid else 'stopped'}")
        rc |= 0 if pid else 3
    return rc


# ------------------------------------------------------------------------- operator lifecycle (kubeopsctl.sh)
_UNIT = """[Unit]
Description=KubeOperator-AMD control plane (API, workers, scheduler)
After=network-online.target

[Service]
Type=simple
Environment=KUBEOPERATOR_CONFIG={config}
ExecStart={python} -m kubeoperator_amd.control.cli start all
ExecReload={python} -m kubeoperator_amd.control.cli reload
Restart=on-failure
WorkingDirectory={data}

[Install]
WantedBy=multi-user.target
"""


def _unit_path(cfg) -> str:
    return os.path.join(cfg.data_dir, "kubeops.service")


def _config_path(a, cfg) -> str:
    return a.config or os.environ.get("KUBEOPERATOR_CONFIG") or os.path.join(cfg.data_dir, "config.yml")


def cmd_install(a, cfg) -> int:
    """Reference scripts/5_install.sh: prepare the data directory, store, default config and service unit
    (systemd runs ``kubeopsctl start all``; ``scripts/install.sh`` adds the environment checks and the compose
    mode). ``--start`` starts the services in the background right away."""
    os.makedirs(cfg.data_dir, exist_ok=True)
    conf = _config_path(a, cfg)
    if not os.path.exists(conf):
        with open(conf, "w") as f:
            yaml.safe_dump({"DATA_DIR": cfg.data_dir, "HTTP_LISTEN_PORT": int(cfg["HTTP_LISTEN_PORT"]),
                            "DEFAULT_TRANSPORT": cfg["DEFAULT_TRANSPORT"]}, f)
        os.chmod(conf, 0o600)
    with open(_unit_path(cfg), "w") as f:
        f.write(_UNIT.format(config=conf, python=sys.executable, data=cfg.data_dir))
    print(f"data dir:  {cfg.data_dir}\nconfig:    {conf}\nstore:     {cfg.db_url}\n"
          f"unit file: {_unit_path(cfg)}  (install with: cp {_unit_path(cfg)} /etc/systemd/system/ && "
          f"systemctl enable --now kubeops)")
    if a.start:
        a.service, a.daemon = "all", True
        return cmd_start(a, cfg)
    return 0


def cmd_uninstall(a, cfg) -> int:
    """Reference scripts/6_uninstall.sh: stop every service, remove the unit; ``--purge`` also deletes the data
    directory (store, logs, execution logs, backups kept locally)."""
    a.service = "all"
    cmd_stop(a, cfg)
    try:
        os.remove(_unit_path(cfg))
    except OSError:
        pass
    if a.purge:
        import shutil

        from .store import db
        db.engine().dispose()
        d = cfg.data_dir  # (the property creates the directory on access)
        shutil.rmtree(d, ignore_errors=True)
        print(f"removed {d}")
    return 0


def cmd_upgrade(a, cfg) -> int:
    """Reference scripts/7_upgrade.sh: stop, back up the store, migrate the schema, restart what was running."""
    from .store import db

    was = [s for s in SERVICES if _read_pid(cfg, s)]
    if was:
        a.service = "all"
        cmd_stop(a, cfg)
    url = cfg.db_url
    if url.startswith("sqlite:///"):
        import sqlite3

        path = url[len("sqlite:///"):]
        if os.path.exists(path):
            bak = f"{path}.{time.strftime('%Y%m%d%H%M%S')}.bak"
            src, dst = sqlite3.connect(path), sqlite3.connect(bak)
            with dst:
                src.backup(dst)
            src.close()
            dst.close()
            print(f"store backed up to {bak}")
    db.init_db()
    print(f"schema at version {db.SCHEMA_VERSION}")
    if was:
        a.service, a.daemon = "all", True
        return cmd_start(a, cfg)
    return 0


def cmd_reload(a, cfg) -> int:
    """Restart (or start) the given services in the background (reference ``reload``: up -d + restart)."""
    cmd_stop(a, cfg)
    a.daemon = True
    return cmd_start(a, cfg)


def cmd_down(a, cfg) -> int:
    """Stop the services and clear their runtime state (pidfiles, SSH control sockets)."""
    cmd_stop(a, cfg)
    for name in os.listdir(_pid_dir(cfg)):
        if name.endswith(".pid") and (a.service in ("all", None) or name == f"{a.service}.pid"):
            os.remove(os.path.join(_pid_dir(cfg), name))
    return 0


def _log_files(cfg, svc) -> list[str]:
    files = [os.path.join(_pid_dir(cfg), "kubeops.log")]
    logdir = os.path.join(cfg.data_dir, "logs")
    if os.path.isdir(logdir):
        files += sorted(os.path.join(logdir, f) for f in os.listdir(logdir) if f.endswith(".jsonl"))[-1:]
    return [f for f in files if os.path.exists(f)]


def cmd_tail(a, cfg, out=None) -> int:
    """Last N lines of the service log (``-f`` follows it). With a service name, only its lines."""
    out = out or sys.stdout
    files = _log_files(cfg, a.service)
    if not files:
        print("no logs yet", file=out)
        return 1
    path = files[0]
    want = None if a.service in ("all", None) else a.service

    def keep(line):
        return want is None or want in line or (want == "web" and "api" in line) or \
            (want == "worker" and "jobs" in line) or (want == "beat" and "scheduler" in line)

    with open(path, errors="replace") as f:
        lines = [ln for ln in f.readlines() if keep(ln)]
        for ln in lines[-a.lines:]:
            out.write(ln)
        out.flush()
        while a.follow:
            ln = f.readline()
            if not ln:
                time.sleep(0.3)
                continue
            if keep(ln):
                out.write(ln)
                out.flush()
    return 0


def cmd_python(a, cfg) -> int:
    """Interactive Python with the store configured (reference ``python manage.py shell``)."""
    from .domain import clusters, deploy, hosts  # noqa: F401
    from .store import models as M  # noqa: F401
    from .store.db import session_scope  # noqa: F401
    ns = {k: v for k, v in locals().items() if k not in ("a",)}
    if a.code:
        exec(compile(a.code, "<kubeopsctl python -c>", "exec"), ns)
        return 0
    import code

    code.interact(banner="KubeOperator-AMD shell: clusters, deploy, hosts, M (models), session_scope", local=ns)
    return 0


def cmd_db(a, cfg, out=None) -> int:
    """SQL against the store (reference ``manage.py dbshell``): ``-c SQL`` runs one statement, otherwise a
    read-eval-print loop (``.tables`` lists the tables)."""
    from sqlalchemy import inspect, text

    from .store import db
    out = out or sys.stdout

    def run(sql):
        sql = sql.strip().rstrip(";")
        if not sql:
            return
        if sql == ".tables":
            print("  ".join(sorted(inspect(db.engine()).get_table_names())), file=out)
            return
        with db.engine().begin() as c:
            res = c.execute(text(sql))
            if res.returns_rows:
                cols = list(res.keys())
                print("|".join(cols), file=out)
                for row in res:
                    print("|".join("" if v is None else str(v) for v in row), file=out)
            else:
                print(f"{res.rowcount} row(s)", file=out)

    if a.code:
        run(a.code)
        return 0
    while True:
        try:
            line = input("kubeops-db> ")
        except EOFError:
            return 0
        if line.strip() in (".quit", ".exit", "\\q"):
            return 0
        try:
            run(line)
        except Exception as e:  # noqa: BLE001 -- a REPL reports and continues
            print(f"error: {e}", file=out)


def cmd_exec_service(a, cfg) -> int:
    """A shell (or ``CMD``) in the environment the services run with (reference ``exec`` into a container)."""
    env = dict(os.environ, KUBEOPERATOR_CONFIG=_config_path(a, cfg), KUBEOPERATOR_SERVICE=a.action)
    argv = a.rest[1:] if a.rest and a.rest[0] == "--" else (a.rest or [os.environ.get("SHELL", "/bin/bash")])
    return subprocess.call(argv, env=env, cwd=cfg.data_dir)


# ------------------------------------------------------------------------------------------------ backends
class Local:
    """In-process: domain calls against the local store; operations run inline (log to stdout)."""

    def __init__(self):
        from .domain import clusters, deploy, hosts, packages
        self.clusters, self.deploy, self.hosts, self.packages = clusters, deploy, hosts, packages

    def add_host(self, d):
        return self.hosts.create_host(d)

    def list_hosts(self):
        from sqlalchemy import select

        from .store import models as M
        from .store.db import session_scope
        with session_scope() as s:
            ids = [h.id for h in s.scalars(select(M.Host))]
        return [self.hosts.host_dict(i) for i in ids]

    def import_hosts(self, path):
        with open(path, "rb") as f:
            return self.hosts.import_hosts(os.path.basename(path), f.read())

    def gpu_check(self, name):
        from sqlalchemy import select

        from .store import models as M
        from .store.db import session_scope

        with session_scope() as s:
            h = s.scalar(select(M.Host).where(M.Host.name == name))
            if h is None:
                raise SystemExit(f"no host {name}")
            hid = h.id
        return self.hosts.check_gpu_node(hid)

    def create_cluster(self, plan_doc):
        for h in plan_doc.get("hosts") or []:
            try:
                self.hosts.create_host(h)
            except Exception as e:  # noqa: BLE001
                print(f"host {h.get('name')}: {e}", file=sys.stderr)
        out = self.clusters.create_cluster(plan_doc)
        for n in plan_doc.get("nodes") or []:
            self.clusters.add_node(plan_doc["name"], n)
        return self.clusters.cluster_dict(self.clusters.get_cluster(out["id"]))

    def list_apps(self, name):
        return self.clusters.list_apps(name)

    def operate(self, name, op, params):
        from .runtime import jobs

        e = self.deploy.create(name, op, params, user="kubeopsctl", run="claim")
        path = jobs.log_path(e["id"])
        import threading

        done = threading.Event()

        def follow():
            off = 0
            while not done.is_set() or off < os.path.getsize(path):
                data, off = jobs.tail(path, off, 1 << 16)
                if data:
                    sys.stdout.write(data.replace("\r\n", "\n"))
                    sys.stdout.flush()
                else:
                    time.sleep(0.2)

        open(path, "a").close()
        t = threading.Thread(target=follow, daemon=True)
        t.start()
        jobs.run_claimed(jobs.get(e["id"]))
        done.set()
        t.join(5)
        return self.deploy.get(e["id"])

    def list_clusters(self):
        from sqlalchemy import select

        from .store import models as M
        from .store.db import session_scope
        with session_scope() as s:
            rows = list(s.scalars(select(M.Cluster)))
        return [self.clusters.cluster_dict(c) for c in rows]

    def show(self, name):
        return self.clusters.cluster_dict(self.clusters.get_cluster(name))

    def kubeconfig(self, name):
        return self.clusters.fetch_kubeconfig(name)

    def delete(self, name):
        self.clusters.delete_cluster(name, force=True)

    def executions(self, name):
        from sqlalchemy import select

        from .store import models as M
        from .store.db import session_scope
        c = self.clusters.get_cluster(name)
        with session_scope() as s:
            return [e.to_dict(exclude=("result_raw",)) for e in s.scalars(
                select(M.Execution).where(M.Execution.project_id == c.project_id, M.Execution.kind == "deploy")
                .order_by(M.Execution.date_created.desc()))]

    def exec_log(self, eid):
        from .runtime import jobs
        return jobs.tail(jobs.log_path(eid), 0, 1 << 24)[0]

    def trace(self, name, eid, view):
        return self.deploy.get_trace(eid, view)

    def list_packages(self):
        return self.packages.sync_packages()


class Remote:
    """REST client of a running control plane (``JWT`` auth)."""

    def __init__(self, server, user, password):
        import httpx

        self.http = httpx.Client(base_url=server.rstrip("/") + "/api/v1", timeout=60)
        r = self.http.post("/token/auth/", json={"username": user, "password": password})
        r.raise_for_status()
        self.http.headers["Authorization"] = "JWT " + r.json()["token"]

    def _j(self, r):
        if r.status_code >= 400:
            raise SystemExit(f"error {r.status_code}: {r.text}")
        return r.json() if r.content else None

    def add_host(self, d):
        return self._j(self.http.post("/host/", json=d))

    def list_hosts(self):
        return self._j(self.http.get("/host/"))

    def import_hosts(self, path):
        with open(path, "rb") as f:
            return self._j(self.http.post("/host/import/", params={"filename": os.path.basename(path)},
                                          content=f.read()))

    def gpu_check(self, name):
        hs = [h for h in self.list_hosts() if h["name"] == name]
        if not hs:
            raise SystemExit(f"no host {name}")
        return self._j(self.http.post(f"/host/{hs[0]['id']}/gpu-check/"))

    def create_cluster(self, plan_doc):
        for h in plan_doc.get("hosts") or []:
            self.http.post("/host/", json=h)
        return self._j(self.http.post("/clusters/", json=plan_doc))

    def list_apps(self, name):
        return self._j(self.http.get(f"/clusters/{name}/apps/"))

    def operate(self, name, op, params):
        e = self._j(self.http.post(f"/clusters/{name}/executions/", json={"operation": op, "params": params}))
        mark = 0
        while True:
            lg = self._j(self.http.get(f"/tasks/{e['id']}/log/", params={"mark": mark}))
            if lg["data"]:
                sys.stdout.write(lg["data"].replace("\r\n", "\n"))
                sys.stdout.flush()
            mark = lg["mark"]
            if lg["end"]:
                break
            time.sleep(1)
        return self._j(self.http.get(f"/clusters/{name}/executions/{e['id']}/"))

    def list_clusters(self):
        return self._j(self.http.get("/clusters/"))

    def show(self, name):
        return self._j(self.http.get(f"/clusters/{name}/"))

    def kubeconfig(self, name):
        r = self.http.get(f"/cluster/{name}/download/")
        r.raise_for_status()
        return r.text

    def delete(self, name):
        self._j(self.http.delete(f"/clusters/{name}/"))

    def executions(self, name):
        return self._j(self.http.get(f"/clusters/{name}/executions/"))

    def exec_log(self, eid):
        return self._j(self.http.get(f"/tasks/{eid}/log/"))["data"]

    def trace(self, name, eid, view):
        return self._j(self.http.get(f"/clusters/{name}/executions/{eid}/trace/", params={"view": view}))

    def list_packages(self):
        return self._j(self.http.get("/packages/"))


def _backend(a):
    server = a.server or os.environ.get("KUBEOPERATOR_SERVER")
    if server:
        return Remote(server, a.user, a.password or os.environ.get("KUBEOPERATOR_PASSWORD", "kubeoperator@admin123"))
    return Local()


def _table(rows, cols):
    if not rows:
        print("(none)")
        return
    w = {c: max(len(c), *(len(str(r.get(c, ""))) for r in rows)) for c in cols}
    print("  ".join(c.upper().ljust(w[c]) for c in cols))
    for r in rows:
        print("  ".join(str(r.get(c, "")).ljust(w[c]) for c in cols))


def _finish(e) -> int:
    print(f"\n{e['operation']}: {e['state']} in {e.get('timedelta') or 0:.1f}s "
          f"[{' -> '.join(s['name'] + ':' + s['status'] for s in e.get('steps') or [])}]")
    return 0 if e["state"] == "SUCCESS" else 1


def cmd_cluster(a, cfg) -> int:
    b = _backend(a)
    if a.action == "create":
        with open(a.file) as f:
            doc = yaml.safe_load(f)
        out = b.create_cluster(doc)
        print(f"cluster {out['name']} created ({out['template']}, {out['node_size']} nodes)")
        if a.install:
            return _finish(b.operate(out["name"], "install", {}))
        return 0
    if a.action == "list":
        _table(b.list_clusters(), ["name", "status", "template", "package", "node_size", "gpu_num", "deploy_type"])
        return 0
    if a.action == "show":
        print(json.dumps(b.show(a.name), indent=2, default=str))
        return 0
    if a.action == "kubeconfig":
        sys.stdout.write(b.kubeconfig(a.name))
        return 0
    if a.action == "delete":
        b.delete(a.name)
        print(f"cluster {a.name} deleted")
        return 0
    if a.action == "trace":
        return _trace(b, a)
    params = {}
    op = a.action
    if op == "install" and a.resume:
        params["resume"] = True
    elif op == "scale":
        params["num"] = a.num
    elif op == "add-worker":
        params["host"] = a.host
    elif op == "remove-worker":
        params["node"] = a.node
    elif op == "upgrade":
        params["package"] = a.package
    elif op == "backup":
        params["backupStorageId"] = a.storage
    elif op == "restore":
        params["clusterBackupId"] = a.backup
    return _finish(b.operate(a.name, op, params))


def _trace(b, a) -> int:
    """Where an execution's time went (default: the cluster's latest): per step the slowest tasks; ``-o`` writes
    the Chrome trace-event JSON (Perfetto / chrome://tracing)."""
    eid = a.execution
    if not eid:
        ex = b.executions(a.name)
        if not ex:
            print(f"cluster {a.name} has no executions", file=sys.stderr)
            return 1
        eid = ex[0]["id"]
    if a.output:
        with open(a.output, "w") as f:
            json.dump(b.trace(a.name, eid, "chrome"), f)
        print(f"trace of {eid} written to {a.output}")
        return 0
    sm = b.trace(a.name, eid, "summary")
    print(f"execution {eid}: {sm['total_seconds']:.1f}s")
    for st in sm["steps"]:
        busy = ", ".join(f"{h} {t:.1f}s" for h, t in sorted(st["hosts"].items()))
        print(f"\n{st['step']}: {st['seconds']:.1f}s, {st['task_count']} tasks ({st['status']}); host busy: {busy}")
        _table([{"task": t["task"][:70], "seconds": f"{t['seconds']:.2f}", "hosts": t["hosts"],
                 "slowest": f"{t['slowest_host']} {t['slowest_host_seconds']:.2f}s" if t["slowest_host"] else ""}
                for t in st["tasks"]], ["task", "seconds", "hosts", "slowest"])
    return 0


def _set_values(pairs) -> dict:
    """``--set a.b=1`` (helm style, dotted keys, YAML-typed values) -> nested dict."""
    out: dict = {}
    for kv in pairs or []:
        k, _, v = kv.partition("=")
        cur = out
        parts = k.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = yaml.safe_load(v) if v != "" else ""
    return out


def cmd_app(a, cfg) -> int:
    b = _backend(a)
    if a.action == "list":
        rows = [dict(r, result=(f"{r['training']['tokens_per_s']:.0f} tok/s" if r.get("training") else ""))
                for r in b.list_apps(a.name)]
        _table(rows, ["namespace", "release", "chart", "date", "result"])
        return 0
    params = {"chart": a.chart, "namespace": a.namespace}
    if a.release:
        params["release"] = a.release
    if a.action == "deploy":
        params.update(values=_set_values(a.set), wait_job=a.wait_job)
        res = b.operate(a.name, "app-deploy", params)
        run = (res.get("result_summary") or {}).get("training")
        if run:
            print(json.dumps({"training": run}))
        return _finish(res)
    return _finish(b.operate(a.name, "app-remove", params))


def cmd_host(a, cfg) -> int:
    b = _backend(a)
    if a.action == "add":
        d = {"name": a.name, "ip": a.ip, "port": a.port, "username": a.username}
        if a.password:
            d["password"] = a.password
        if a.credential:
            d["credential"] = a.credential
        h = b.add_host(d)
        print(f"host {h['name']} {h['status']} cpu={h.get('cpu_core')} mem={h.get('memory')}MiB gpus={h.get('gpu_num')}"
              f" {h.get('gpu_info') or ''}")
        return 0
    if a.action == "import":
        print(json.dumps(b.import_hosts(a.file), indent=2))
        return 0
    if a.action == "gpu-check":  # read-only kfd / rocminfo / amd-smi tasks of the GPU roles on that host
        r = b.gpu_check(a.name)
        ok = r["summary"]["success"]
        print(f"{a.name}: {'ok' if ok else 'FAILED'} kfd GPUs={r['kfd_gpus']} rocminfo GPU agents={r['rocminfo_gpus']}")
        if not ok:
            print(json.dumps(r["summary"]["dark"], indent=2))
        return 0 if ok else 1
    _table(b.list_hosts(), ["name", "ip", "status", "os", "cpu_core", "memory", "gpu_num", "gpu_info"])
    return 0


def cmd_exec(a, cfg) -> int:
    b = _backend(a)
    if a.action == "list":
        _table(b.executions(a.target), ["id", "operation", "state", "timedelta", "date_created"])
    else:
        sys.stdout.write(b.exec_log(a.target).replace("\r\n", "\n"))
    return 0


def cmd_package(a, cfg) -> int:
    rows = [dict(p, version=p["meta"].get("version", ""), kube=p["meta"].get("vars", {}).get("kube_version", ""),
                 rocm=p["meta"].get("vars", {}).get("rocm_version", "")) for p in _backend(a).list_packages()]
    _table(rows, ["name", "version", "kube", "rocm", "path"])
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kubeopsctl", description="KubeOperator-AMD control plane")
    ap.add_argument("--config", default=os.environ.get("KUBEOPERATOR_CONFIG"))
    ap.add_argument("--server", default=None, help="REST endpoint of a running control plane")
    ap.add_argument("--user", default=os.environ.get("KUBEOPERATOR_USER", "admin"))
    ap.add_argument("--password", default=None)
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("init")
    sub.add_parser("version")
    for name in ("start", "stop", "status", "restart", "reload", "down", "tail"):
        p = sub.add_parser(name)
        p.add_argument("service", nargs="?", default="all", choices=["all", *SERVICES])
        if name in ("start", "restart"):
            p.add_argument("-d", "--daemon", action="store_true")
        if name == "tail":
            p.add_argument("-n", "--lines", type=int, default=100)
            p.add_argument("-f", "--follow", action="store_true")
    sub.add_parser("install").add_argument("--start", action="store_true")
    sub.add_parser("uninstall").add_argument("--purge", action="store_true")
    sub.add_parser("upgrade")
    sub.add_parser("python").add_argument("-c", dest="code")
    sub.add_parser("db").add_argument("-c", dest="code")
    c = sub.add_parser("cluster")
    c.add_argument("action", choices=["create", "list", "show", "kubeconfig", "delete", "install", "uninstall",
                                      "scale", "add-worker", "remove-worker", "upgrade", "backup", "restore",
                                      "gpu-validate", "bigip-config", "trace"])
    c.add_argument("name", nargs="?")
    c.add_argument("-f", "--file")
    c.add_argument("--install", action="store_true", help="with create: install right away")
    c.add_argument("--resume", action="store_true")
    c.add_argument("--num", type=int, default=0)
    c.add_argument("--host")
    c.add_argument("--node")
    c.add_argument("--package")
    c.add_argument("--storage")
    c.add_argument("--backup")
    c.add_argument("--execution", help="with trace: execution id (default: the latest)")
    c.add_argument("-o", "--output", help="with trace: write the Chrome trace-event JSON here")
    h = sub.add_parser("host")
    h.add_argument("action", choices=["add", "list", "import", "gpu-check"])
    h.add_argument("name", nargs="?")
    h.add_argument("ip", nargs="?")
    h.add_argument("--port", type=int, default=22)
    h.add_argument("--username", default="root")
    h.add_argument("--password")
    h.add_argument("--credential")
    h.add_argument("--file")
    e = sub.add_parser("exec")
    e.add_argument("action", choices=["list", "log", *SERVICES])
    e.add_argument("target", nargs="?")
    e.add_argument("rest", nargs=argparse.REMAINDER)
    sub.add_parser("package").add_argument("action", nargs="?", default="list", choices=["list"])
    ap_ = sub.add_parser("app")
    ap_.add_argument("action", choices=["deploy", "list", "remove"])
    ap_.add_argument("name", help="cluster")
    ap_.add_argument("--chart", default="nginx")
    ap_.add_argument("--release")
    ap_.add_argument("--namespace", default="default")
    ap_.add_argument("--set", action="append", help="value override k=v (dotted keys)")
    ap_.add_argument("--wait-job", action="store_true", help="wait for the release's Job and collect its result")
    a = ap.parse_args(argv)

    if a.cmd == "version":
        from .. import __version__
        print(__version__)
        return 0
    cfg = _bootstrap(a.config)
    if a.cmd == "init":
        print(f"store ready at {cfg.db_url}")
        return 0
    if a.cmd == "start":
        return cmd_start(a, cfg)
    if a.cmd == "stop":
        return cmd_stop(a, cfg)
    if a.cmd == "status":
        return cmd_status(a, cfg)
    if a.cmd == "restart":
        cmd_stop(a, cfg)
        return cmd_start(a, cfg)
    simple = {"install": cmd_install, "uninstall": cmd_uninstall, "upgrade": cmd_upgrade, "reload": cmd_reload,
              "down": cmd_down, "tail": cmd_tail, "python": cmd_python, "db": cmd_db}
    if a.cmd in simple:
        return simple[a.cmd](a, cfg)
    if a.cmd == "exec" and a.action in SERVICES:
        if a.target:
            a.rest = [a.target, *a.rest]
        return cmd_exec_service(a, cfg)
    if a.cmd == "host" and a.action == "import":
        a.file = a.file or a.name
    return {"cluster": cmd_cluster, "host": cmd_host, "exec": cmd_exec, "package": cmd_package,
            "app": cmd_app}[a.cmd](a, cfg)


if __name__ == "__main__":
    sys.exit(main())
