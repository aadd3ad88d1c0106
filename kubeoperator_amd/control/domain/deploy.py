"""DeployExecution: the cluster lifecycle state machine (reference kubeops_api/models/deploy.py:25-337).

Operations (same names and params as the reference API): ``install``, ``uninstall``, ``bigip-config``,
``upgrade`` {package}, ``scale`` {num}, ``add-worker`` {host}, ``remove-worker`` {node},
``backup`` {backupStorageId}, ``restore`` {clusterBackupId}, plus ``gpu-validate`` (run the rocminfo
validation pod on every GPU worker), ``app-deploy`` {chart, release, namespace, values, wait_job} and
``app-remove`` {release, namespace}: Helm releases of the bundled charts (nginx, the PyTorch-ROCm training
chart) recorded on the cluster; a training release run with ``wait_job`` gets its last logged step
(tokens/s, step time, loss) attached to the execution result.

Per operation: cluster status while running -> after (INSTALLING -> RUNNING/ERROR, DELETING -> READY,
UPGRADING, SCALING, BACKUP, RESTORING -> RUNNING); ``ignore_errors`` operations (scale / add / remove /
bigip) do not put the cluster in ERROR and return it to RUNNING; step list from the plan with
pending/running/success/error bookkeeping persisted on every transition (read by the progress
websocket); first failing playbook stops the run; a message is sent to the message center.

Added by design: one active execution per cluster (409 Conflict instead of silently marking the previous
one FAILURE), ``params.resume`` re-runs an install from its first unfinished step (kubeasz tasks are
idempotent), and ``timedelta`` is recorded in float seconds -- the cluster-create metric. Every execution
also leaves a span trace (step -> playbook -> play -> task -> host, ``engine/trace.py``) under
``DATA_DIR/traces``: where the minutes of a cluster-create went.
"""
from __future__ import annotations

import json
import logging
import os
import re
import time

from sqlalchemy import select
from sqlalchemy.exc import IntegrityError

from ..engine.trace import Tracer, chrome_trace
from ..engine.trace import summary as trace_summary
from ..runtime import jobs, metrics
from ..store import models as M
from ..store.db import session_scope, write_scope
from . import clusters, plan

log = logging.getLogger("kubeoperator.deploy")

OPERATIONS = ("install", "uninstall", "bigip-config", "upgrade", "scale", "add-worker", "remove-worker", "backup",
              "restore", "gpu-validate", "app-deploy", "app-remove")
_DNS1123 = re.compile(r"^[a-z0-9]([-a-z0-9]{0,51}[a-z0-9])?$")
_CHART = re.compile(r"^[A-Za-z0-9][A-Za-z0-9._-]*(/[A-Za-z0-9][A-Za-z0-9._-]*)?$")
IGNORE_ERRORS = {"bigip-config", "scale", "add-worker", "remove-worker"}
RETURN_RUNNING = {"scale", "add-worker", "remove-worker"}
RUNNING_STATUS = {"install": "INSTALLING", "uninstall": "DELETING", "upgrade": "UPGRADING", "scale": "SCALING",
                  "add-worker": "SCALING", "remove-worker": "SCALING", "restore": "RESTORING", "backup": "BACKUP"}
OPERATION_NAME = {"install": "Cluster install", "uninstall": "Cluster uninstall", "upgrade": "Cluster upgrade",
                  "scale": "Cluster scale", "add-worker": "Cluster scale", "remove-worker": "Cluster scale",
                  "restore": "Cluster restore", "backup": "Cluster backup", "bigip-config": "F5 BIG-IP config",
                  "gpu-validate": "GPU validation", "app-deploy": "Application deploy",
                  "app-remove": "Application remove"}


def create(cluster_name: str, operation: str, params: dict | None = None, user: str = "",
           run: str = "queue") -> dict:
    """Create a DeployExecution and start it. ``run``: ``queue`` (a worker runs it), ``inline`` (run it here and
    return when done), ``claim`` (its job is created STARTED and owned by the caller, which runs it with
    ``jobs.run_claimed(jobs.get(id))``), ``none`` (no job; such an execution does not lock the cluster)."""
    if operation not in OPERATIONS:
        raise ValueError(f"unknown operation {operation!r}; one of {OPERATIONS}")
    c = clusters.get_cluster(cluster_name)
    params = dict(params or {})
    if operation in ("app-deploy", "app-remove"):
        _check_app_params(operation, params)
    if c.deploy_type == "AUTOMATIC" and operation in ("install", "scale"):
        from . import cloud

        need = len(clusters.list_nodes(cluster_name)) if operation == "install" else int(params.get("num", 0))
        cloud.check_capacity(c, need)
    steps = [dict(st, status="pending") for st in plan.operation_steps(operation)]
    # Check-and-insert under the store's write lock (BEGIN IMMEDIATE on SQLite), backed by the partial unique
    # index uq_one_active_deploy_per_project: two creators -- API threads, the scheduled backup's worker thread,
    # a CLI process on the same store -- can never both pass the busy check.
    try:
        with write_scope() as s:
            busy = s.scalar(select(M.Execution).where(M.Execution.project_id == c.project_id,
                                                      M.Execution.kind == "deploy",
                                                      M.Execution.state.in_(("PENDING", "STARTED")))
                            .with_for_update())
            if busy is not None and _stale(s, busy):
                busy.state, busy.date_end = "FAILURE", M.now()
                busy.result_summary = {"error": "abandoned: no job was ever run for this execution"}
                s.flush()
                busy = None
            if busy is not None:
                raise clusters.Conflict(f"cluster {cluster_name} is busy with {busy.operation} ({busy.id})")
            e = M.Execution(kind="deploy", project_id=c.project_id, operation=operation, params=params, steps=steps,
                            state="PENDING", created_by=user)
            s.add(e)
            s.flush()
            eid = e.id
            # The execution's job commits in the same transaction: there is no window in which a concurrent
            # creator sees a job-less execution and takes it for abandoned (``_stale``).
            job = None if run == "none" else jobs.add_job(s, "start_deploy_execution", {"execution_id": eid},
                                                          job_id=eid, inline=run in ("inline", "claim"))
    except IntegrityError as err:
        raise clusters.Conflict(f"cluster {cluster_name} is busy with another operation") from err
    if run == "queue":
        jobs.wake()
    elif run == "inline":
        jobs.run_claimed(job)
    return get(eid)


def _stale(s, e: M.Execution) -> bool:
    """A PENDING/STARTED execution whose job is missing or finished (e.g. a client died between creating the
    execution and queueing it) must not lock the cluster forever."""
    j = s.get(M.Job, e.id)
    return j is None or j.state in ("SUCCESS", "FAILURE", "REVOKED")


def get(execution_id: str) -> dict:
    with session_scope() as s:
        e = s.get(M.Execution, execution_id)
        if e is None:
            raise clusters.NotFound(f"execution {execution_id} not found")
        d = e.to_dict()
    d["progress_ws_url"] = f"/ws/progress/{execution_id}/"
    d["log_ws_url"] = f"/ws/tasks/{execution_id}/log/"
    return d


def to_json(execution_id: str) -> dict:
    """What the progress websocket pushes (reference DeployExecution.to_json)."""
    d = get(execution_id)
    return {"id": d["id"], "steps": d["steps"], "operation": d["operation"], "state": d["state"],
            "current_step": d["current_step"],
            "timedelta": d["timedelta"]}


class _Exec:
    def __init__(self, eid: str, logger):
        self.id = eid
        self.log = logger or (lambda m: None)
        with session_scope() as s:
            e = s.get(M.Execution, eid)
            self.operation, self.params, self.steps = e.operation, dict(e.params or {}), list(e.steps or [])
            self.project_id = e.project_id
        with session_scope() as s:
            c = s.scalar(select(M.Cluster).where(M.Cluster.project_id == self.project_id))
            self.cluster_name = c.name
        self.tracer = Tracer(on_host_span=_observe_host_span)
        self._step_spans: dict[str, int] = {}

    @property
    def cluster(self) -> M.Cluster:
        return clusters.get_cluster(self.cluster_name)

    def save(self, **fields):
        with session_scope() as s:
            e = s.get(M.Execution, self.id)
            e.steps = [dict(x) for x in self.steps]
            for k, v in fields.items():
                setattr(e, k, v)

    def set_steps(self, operation: str, drop=()):
        self.steps = [dict(st, status="pending") for st in plan.operation_steps(operation) if st["name"] not in drop]
        self.save()

    def update_step(self, name: str, status: str):
        """Step status + timing: ``start`` / ``end`` epoch seconds and ``seconds`` (exported as metrics)."""
        now = time.time()
        for i, st in enumerate(self.steps):
            if st["name"] == name:
                st["status"] = status
                if status == "running":
                    st["start"] = now
                    self._step_spans[name] = self.tracer.begin(name, "step", playbook=st.get("playbook"))
                elif status in ("success", "error") and "start" in st:
                    st["end"] = now
                    st["seconds"] = round(now - st["start"], 3)
                    metrics.STEP_SECONDS.labels(self.operation, name, status).observe(st["seconds"])
                    sid = self._step_spans.pop(name, None)
                    if sid is not None:
                        self.tracer.end(sid, status)
                self.save(current_step=i)

    def run_playbooks(self, ev: dict) -> dict:
        result = {"raw": {}, "summary": {"success": True}}
        skip = set(self.params.get("_skip_steps", []))
        for st in self.steps:
            pb = st.get("playbook")
            if not pb:
                continue
            if st["name"] in skip:
                self.update_step(st["name"], "success")
                continue
            self.update_step(st["name"], "running")
            self.log(f"===== step {st['name']}: playbook {plan.playbook_alias(pb)} =====")
            r = clusters.run_playbook(self.cluster, pb, ev, logger=self.log, tracer=self.tracer)
            result["summary"].update(r["summary"])
            result["raw"] = r["raw"]
            if not r["summary"].get("success", False):
                self.update_step(st["name"], "error")
                result["summary"]["success"] = False
                return result
            self.update_step(st["name"], "success")
        return result


def start(execution_id: str, logger=None) -> dict:
    ex = _Exec(execution_id, logger)
    t0 = M.now()
    ex.save(state="STARTED", date_start=t0)
    c = ex.cluster
    ev = clusters.extra_vars(c)
    op = ex.operation
    result = {"raw": {}, "summary": {"success": False}}
    ignore = op in IGNORE_ERRORS
    try:
        if op in RUNNING_STATUS:
            clusters.change_status(c.id, RUNNING_STATUS[op])
        result = _dispatch(ex, c, ev)
        ok = result.get("summary", {}).get("success", False)
        after = {"uninstall": "READY"}.get(op, "RUNNING")
        if ok or ignore:
            if op not in ("bigip-config", "gpu-validate") or c.status in RUNNING_STATUS.values():
                clusters.change_status(c.id, after)
        else:
            clusters.change_status(c.id, "ERROR")
    except Exception as e:  # noqa: BLE001 - recorded on the execution and the cluster
        log.exception("execution %s failed", execution_id)
        ex.log(f"ERROR: {type(e).__name__}: {e}")
        for st in ex.steps:
            if st.get("status") == "running":
                st["status"] = "error"
        clusters.change_status(c.id, "ERROR")
        result = {"raw": {}, "summary": {"success": False, "error": f"{type(e).__name__}: {e}"}}
    ok = bool(result.get("summary", {}).get("success", False))
    t1 = M.now()
    ex.save(state="SUCCESS" if ok else "FAILURE", date_end=t1, timedelta=(t1 - t0).total_seconds(),
            result_summary=clusters._jsonable(result.get("summary", {})),
            result_raw=clusters._jsonable({k: v for k, v in (result.get("raw") or {}).items() if k != "ok"}))
    metrics.EXECUTION_SECONDS.labels(op, "SUCCESS" if ok else "FAILURE").observe((t1 - t0).total_seconds())
    for name, sid in list(ex._step_spans.items()):  # steps an exception left running
        ex.tracer.end(sid, "error")
    _save_trace(execution_id, ex.tracer)
    _notify(c, op, ok)
    return {"success": ok, "timedelta": (t1 - t0).total_seconds()}


def _observe_host_span(sp) -> None:
    metrics.TASK_SECONDS.labels(sp.attrs.get("module", ""), sp.status).observe(sp.seconds)


def _trace_path(execution_id: str) -> str:
    from ..conf import get_config

    return os.path.join(get_config().data_dir, "traces", f"{execution_id}.json")


def _save_trace(execution_id: str, tracer: Tracer) -> None:
    """Spans of the execution (step -> playbook -> play -> task -> host) next to its log."""
    p = _trace_path(execution_id)
    try:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"execution_id": execution_id, "spans": tracer.to_list()}, f, default=str)
        os.replace(tmp, p)
    except OSError:
        log.exception("could not write the trace of execution %s", execution_id)


def get_trace(execution_id: str, view: str = "chrome") -> dict:
    """``chrome``: trace-event JSON (Perfetto / chrome://tracing); ``summary``: per step the slowest tasks and
    per-host busy time; ``spans``: the raw span list."""
    get(execution_id)  # 404 for unknown executions
    p = _trace_path(execution_id)
    if not os.path.exists(p):
        raise clusters.NotFound(f"execution {execution_id} has no trace (still running or never started)")
    with open(p) as f:
        spans = json.load(f)["spans"]
    if view == "spans":
        return {"execution_id": execution_id, "spans": spans}
    if view == "summary":
        return {"execution_id": execution_id, **trace_summary(spans)}
    return chrome_trace(spans, process=f"execution {execution_id}")


def _dispatch(ex: _Exec, c: M.Cluster, ev: dict) -> dict:
    op = ex.operation
    if op == "install":
        drop = () if c.deploy_type == "AUTOMATIC" else ("create-resource",)
        ex.set_steps("install", drop)
        if ex.params.get("resume"):
            ex.params["_skip_steps"] = _resume_skips(ex)
        if c.deploy_type == "AUTOMATIC":
            from . import cloud

            ex.update_step("create-resource", "running")
            cloud.create_resources(c.name, logger=ex.log)
            ex.update_step("create-resource", "success")
            ev.update(clusters.get_cluster(c.name).configs)
        return ex.run_playbooks(ev)
    if op == "uninstall":
        ex.set_steps("uninstall")
        if c.deploy_type == "AUTOMATIC":
            from . import cloud

            ex.update_step("uninstall", "running")
            cloud.destroy_resources(c.name, logger=ex.log)
            ex.update_step("uninstall", "success")
            return {"raw": {}, "summary": {"success": True}}
        return ex.run_playbooks(ev)
    if op == "bigip-config":
        ex.set_steps("bigip-config")
        return ex.run_playbooks(ev)
    if op == "upgrade":
        from . import packages

        name = ex.params.get("package")
        meta = packages.get_package(name)["meta"]
        ev.update(meta.get("vars", {}))
        ex.set_steps("upgrade")
        res = ex.run_playbooks(ev)
        if res["summary"].get("success"):
            packages.upgrade_cluster_package(c.name, name)
        return res
    if op == "scale":
        ex.set_steps("scale", () if c.deploy_type == "AUTOMATIC" else ("create-resource",))
        if c.deploy_type == "AUTOMATIC":
            from . import cloud

            ex.update_step("create-resource", "running")
            cloud.scale_to(c.name, int(ex.params.get("num", 0)), logger=ex.log)
            ex.update_step("create-resource", "success")
        res = ex.run_playbooks(ev)
        clusters.exit_new_node(c.name)
        return res
    if op == "add-worker":
        ex.set_steps("add-worker")
        hosts = ex.params.get("host") or ex.params.get("hosts")
        for h in hosts if isinstance(hosts, list) else [hosts]:
            clusters.add_worker(c.name, h)
        res = ex.run_playbooks(ev)
        clusters.exit_new_node(c.name)
        return res
    if op == "remove-worker":
        ex.set_steps("remove-worker")
        node = ex.params.get("node")
        clusters.set_node_groups(c.name, node, ["new_node", "worker"])
        res = ex.run_playbooks(ev)
        if res["summary"].get("success"):
            clusters.remove_node_record(c.name, node)
        else:
            clusters.exit_new_node(c.name)
        return res
    if op == "backup":
        from . import backup

        ex.set_steps("backup")
        res = ex.run_playbooks(ev)
        if res["summary"].get("success"):
            backup.upload_backup(c.name, ex.params.get("backupStorageId"), logger=ex.log)
        return res
    if op == "restore":
        from . import backup

        ex.set_steps("restore")
        backup.download_backup(c.name, ex.params.get("clusterBackupId"), logger=ex.log)
        return ex.run_playbooks(ev)
    if op == "gpu-validate":
        ex.set_steps("gpu-validate")
        return ex.run_playbooks(ev)
    if op in ("app-deploy", "app-remove"):
        p = ex.params
        chart = p.get("chart", "nginx")
        from ..engine.templating import mark_unsafe

        # the values are user data written to a file: never evaluated as templates
        ev.update(app_chart=chart, app_release=p.get("release") or chart.split("/")[-1],
                  app_namespace=p.get("namespace", "default"), app_values=mark_unsafe(p.get("values") or {}),
                  app_wait_job=bool(p.get("wait_job", False)))
        if p.get("timeout"):
            ev["app_timeout"] = str(p["timeout"])
        ex.set_steps(op)
        res = ex.run_playbooks(ev)
        if res["summary"].get("success"):
            run = _training_result(res.get("raw") or {}) if op == "app-deploy" else None
            if run:
                res["summary"]["training"] = run
            clusters.record_app(c.name, op, {"release": ev["app_release"], "chart": chart,
                                             "namespace": ev["app_namespace"], "values": p.get("values") or {},
                                             "execution_id": ex.id, **({"training": run} if run else {})})
        return res
    raise ValueError(op)


def _check_app_params(op: str, p: dict) -> None:
    """Release / namespace / chart end up in helm command lines: accept Kubernetes names only."""
    chart = p.get("chart", "nginx")
    release = p.get("release") or str(chart).split("/")[-1]
    for what, v, rx in (("release", release, _DNS1123), ("namespace", p.get("namespace", "default"), _DNS1123),
                        ("chart", chart, _CHART)):
        if not isinstance(v, str) or not rx.match(v):
            raise ValueError(f"invalid {what} {v!r}")
    if not isinstance(p.get("values", {}) or {}, dict):
        raise ValueError("values must be a mapping")
    if p.get("timeout") is not None and not re.match(r"^\d+[smh]?$", str(p["timeout"])):
        raise ValueError(f"invalid timeout {p['timeout']!r}")


def _training_result(raw: dict) -> dict | None:
    """Last JSON step record (tokens_per_s, step_s, loss, ...) in the collected Job log, if any."""
    for host_tasks in (raw.get("ok") or {}).values():
        for name, r in host_tasks.items():
            if "collect the Job log" not in name or not isinstance(r, dict):
                continue
            last = None
            for line in str(r.get("stdout", "")).splitlines():
                line = line.strip()
                if line.startswith("{") and "tokens_per_s" in line:
                    try:
                        last = json.loads(line)
                    except ValueError:
                        continue
            if last is not None:
                return last
    return None


def _resume_skips(ex: _Exec) -> list[str]:
    with session_scope() as s:
        prev = s.scalar(select(M.Execution).where(M.Execution.project_id == ex.project_id,
                                                  M.Execution.kind == "deploy", M.Execution.operation == ex.operation,
                                                  M.Execution.id != ex.id, M.Execution.state == "FAILURE")
                        .order_by(M.Execution.date_created.desc()).limit(1))
        if prev is None:
            return []
        return [st["name"] for st in prev.steps or [] if st.get("status") == "success"]


def _notify(c: M.Cluster, op: str, ok: bool) -> None:
    from . import messages

    try:
        messages.insert_message({
            "title": OPERATION_NAME.get(op, op), "level": "INFO" if ok else "WARNING", "type": "CLUSTER",
            "item_id": _item_of(c.id),
            "content": {"resource": "cluster", "resource_name": c.name, "resource_type": "CLUSTER",
                        "detail": {"message": f"{OPERATION_NAME.get(op, op)} {'succeeded' if ok else 'failed'}"},
                        "status": clusters.get_cluster(c.name).status}})
    except Exception:  # noqa: BLE001 - notification failure never fails the execution
        log.exception("message insert failed")


def _item_of(cluster_id: str):
    with session_scope() as s:
        r = s.scalar(select(M.ItemResource).where(M.ItemResource.resource_id == cluster_id,
                                                  M.ItemResource.resource_type == "CLUSTER"))
        return r.item_id if r else None


@jobs.task("start_deploy_execution")
def _job_start_deploy(job_id, logger, execution_id):
    return start(execution_id, logger=logger)
