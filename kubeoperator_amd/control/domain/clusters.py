"""Cluster model operations (reference kubeops_api/models/cluster.py:30-432, node.py, role.py).

A cluster is a project whose inventory groups come from the plan (``roles`` + the template's roles), whose
playbooks are the plan's playbooks, and whose ``configs`` are the merged network / storage / package /
template / plan variables (``on_cluster_create`` :416-426). Nodes are inventory hosts bound to registered
hosts; a node whose host carries AMD Instinct GPUs gets ``has_gpu`` / ``gpu_vendor`` / ``gpu_num`` /
``gpu_arch`` host vars and joins the ``gpu_nodes`` group, which the worker play uses to install the
amdgpu / ROCm stack and the addon play to label nodes for the device plugin.
"""
from __future__ import annotations

import os

from sqlalchemy import delete, func, select

from ..engine import ResultCallback, Runner
from ..store import models as M
from ..store.db import session_scope
from . import context, plan

STATUS = ("READY", "RUNNING", "ERROR", "WARNING", "INSTALLING", "DELETING", "UPGRADING", "RESTORING", "BACKUP",
          "SCALING")


class NotFound(Exception):
    pass


class Conflict(Exception):
    pass


def get_cluster(name_or_id: str) -> M.Cluster:
    with session_scope() as s:
        c = s.scalar(select(M.Cluster).where((M.Cluster.name == name_or_id) | (M.Cluster.id == name_or_id)))
        if c is None:
            raise NotFound(f"cluster {name_or_id} not found")
        return c


def cluster_dict(c: M.Cluster) -> dict:
    d = c.to_dict()
    with session_scope() as s:
        nodes = list(s.scalars(select(M.InvHost).where(M.InvHost.project_id == c.project_id,
                                                      M.InvHost.name != "localhost")))
        d["node_size"] = len(nodes)
        d["gpu_num"] = sum(int((n.vars or {}).get("gpu_num", 0)) for n in nodes)
        item = s.scalar(select(M.Item).join(M.ItemResource, M.ItemResource.item_id == M.Item.id)
                        .where(M.ItemResource.resource_id == c.id, M.ItemResource.resource_type == "CLUSTER"))
        d["item_name"] = item.name if item else ""
        last = s.scalar(select(M.Execution).where(M.Execution.project_id == c.project_id)
                        .order_by(M.Execution.date_created.desc()).limit(1))
        d["current_execution"] = last.to_dict() if last else None
    d["apps"] = [dict(a, url=f"http://{a['url_key']}.{c.configs.get('APP_DOMAIN', '')}")
                 for a in plan.load_plan().get("apps", [])]
    return d


def create_cluster(data: dict, created_by: str = "") -> dict:
    name = data["name"]
    if not name or not all(ch.isalnum() or ch == "-" for ch in name):
        raise ValueError("cluster name must be alphanumeric / '-'")
    tmpl = plan.template(data.get("template") or "single-master")
    with session_scope() as s:
        if s.scalar(select(M.Project).where(M.Project.name == name)) is not None:
            raise Conflict(f"cluster {name} already exists")
        proj = M.Project(name=name, kind="cluster", created_by=created_by, comment=data.get("comment", ""))
        s.add(proj)
        s.flush()
        c = M.Cluster(project_id=proj.id, name=name, package=data.get("package", ""),
                      persistent_storage=data.get("persistent_storage", ""),
                      network_plugin=data.get("network_plugin", "flannel"), template=tmpl["name"],
                      plan_id=data.get("plan"), worker_size=int(data.get("worker_size", 3)),
                      deploy_type=data.get("deploy_type", "MANUAL"), configs=dict(data.get("configs") or {}),
                      cluster_doamin_suffix=data.get("cluster_doamin_suffix", data.get("cluster_domain_suffix", "")),
                      comment=data.get("comment", ""))
        s.add(c)
        s.flush()
        cid, pid = c.id, proj.id
    _create_roles(pid, tmpl)
    _create_playbooks(pid)
    _create_localhost(pid)
    _set_configs(cid, tmpl)
    if data.get("item_name"):
        with session_scope() as s:
            item = s.scalar(select(M.Item).where(M.Item.name == data["item_name"]))
            if item is not None:
                s.add(M.ItemResource(item_id=item.id, resource_id=cid, resource_type="CLUSTER"))
    return cluster_dict(get_cluster(cid))


def _create_roles(project_id: str, tmpl: dict) -> None:
    """Plan role groups + template roles + new_node/lb/daemon (reference create_roles :247-277)."""
    p = plan.load_plan()
    with session_scope() as s:
        def upsert(name, children=(), vars=None, meta=None):
            g = s.scalar(select(M.InvGroup).where(M.InvGroup.project_id == project_id, M.InvGroup.name == name))
            if g is None:
                g = M.InvGroup(project_id=project_id, name=name, children=[], vars={}, meta={})
                s.add(g)
            g.children = list(dict.fromkeys(list(g.children or []) + list(children or [])))
            if vars:
                g.vars = {**(g.vars or {}), **vars}
            if meta:
                g.meta = {**(g.meta or {}), **meta}
            s.flush()

        for base in ("master", "worker", "new_node", "lb", "daemon", "gpu_nodes"):
            upsert(base)
        for r in p["roles"]:
            upsert(r["name"], r.get("children", []), None, r.get("meta"))
        for r in tmpl["roles"]:
            upsert(r["name"], r.get("children", []), r.get("vars") or {}, r.get("meta"))
        for name, gvars in (tmpl.get("private_vars") and {"all": tmpl["private_vars"]} or {}).items():
            upsert(name, (), gvars)


def _create_playbooks(project_id: str) -> None:
    with session_scope() as s:
        for pb in plan.load_plan()["playbooks"]:
            s.add(M.Playbook(project_id=project_id, name=pb["name"], alias=pb["alias"], type="local",
                             url=f"file://{plan.PLAYBOOK_DIR}"))


def _create_localhost(project_id: str) -> None:
    with session_scope() as s:
        s.add(M.InvHost(project_id=project_id, name="localhost", ip="127.0.0.1",
                        vars={"ansible_connection": "local", "ansible_python_interpreter": "/usr/bin/python3"},
                        groups=[]))


def _set_configs(cluster_id: str, tmpl: dict) -> None:
    """network / storage / package / template / plan variables -> cluster.configs."""
    with session_scope() as s:
        c = s.get(M.Cluster, cluster_id)
        cfg = {}
        net = plan.network(c.network_plugin)
        cfg.update(net.get("vars", {}))
        for item in net.get("configs", []):
            cfg.setdefault(item["name"], item.get("value"))
        st = plan.storage(c.persistent_storage) if c.persistent_storage else None
        if st:
            cfg.update(st.get("vars", {}))
        cfg.update(tmpl.get("private_vars", {}))
        cfg.update(_package_vars(c.package))
        if c.plan_id:
            p = s.get(M.Plan, c.plan_id)
            if p is not None:
                cfg.update(p.vars or {})
        for pc in plan.load_plan().get("public_config", []):
            if pc["name"] == "APP_DOMAIN":
                dflt = str(pc.get("default", "")).replace("$cluster_name", c.name).replace(
                    "$domain_suffix", "." + c.cluster_doamin_suffix if c.cluster_doamin_suffix else "")
                cfg.setdefault("APP_DOMAIN", dflt)
            else:
                cfg.setdefault(pc["name"], pc.get("default"))
        cfg.update(c.configs or {})  # user-supplied values win
        c.configs = cfg


def _package_vars(name: str) -> dict:
    if not name:
        return dict(plan.builtin_package_meta().get("vars", {}))
    for p in plan.scan_packages():
        if p["name"] == name:
            return dict(p["meta"].get("vars", {}))
    with session_scope() as s:
        row = s.scalar(select(M.Package).where(M.Package.name == name))
        if row is not None:
            return dict((row.meta or {}).get("vars", {}))
    if name in ("mi355x-k8s", ""):
        return dict(plan.builtin_package_meta().get("vars", {}))
    raise NotFound(f"package {name} not found")


def set_config(cluster_name: str, key: str, value) -> None:
    with session_scope() as s:
        c = s.scalar(select(M.Cluster).where(M.Cluster.name == cluster_name).with_for_update())
        c.configs = {**(c.configs or {}), key: value}


def record_app(cluster_name: str, op: str, rel: dict) -> None:
    """Keep the cluster's Helm releases (``configs["app_releases"]``, keyed by namespace/release)."""
    key = f"{rel['namespace']}/{rel['release']}"
    with session_scope() as s:
        c = s.scalar(select(M.Cluster).where(M.Cluster.name == cluster_name).with_for_update())
        apps = dict((c.configs or {}).get("app_releases") or {})
        if op == "app-remove":
            apps.pop(key, None)
        else:
            apps[key] = dict(rel, date=M.now().isoformat())
        c.configs = {**(c.configs or {}), "app_releases": apps}


def list_apps(cluster_name: str) -> list[dict]:
    return sorted((get_cluster(cluster_name).configs or {}).get("app_releases", {}).values(),
                  key=lambda a: (a["namespace"], a["release"]))


def del_config(cluster_name: str, key: str) -> None:
    # (the reference edits a non-existent ``self.vars`` here, cluster.py:296-300)
    with session_scope() as s:
        c = s.scalar(select(M.Cluster).where(M.Cluster.name == cluster_name))
        cfg = dict(c.configs or {})
        cfg.pop(key, None)
        c.configs = cfg


def change_status(cluster_id: str, status: str) -> None:
    assert status in STATUS, status
    with session_scope() as s:
        s.get(M.Cluster, cluster_id).status = status


def delete_cluster(name: str, force: bool = False) -> None:
    c = get_cluster(name)
    if c.status not in ("READY", "ERROR") and not force:
        raise Conflict(f"cluster {name} is {c.status}; uninstall it first")
    with session_scope() as s:
        s.execute(delete(M.ItemResource).where(M.ItemResource.resource_id == c.id))
        s.delete(s.get(M.Project, c.project_id))


# --------------------------------------------------------------------------------------------- nodes
def list_nodes(cluster_name: str) -> list[dict]:
    c = get_cluster(cluster_name)
    with session_scope() as s:
        rows = s.scalars(select(M.InvHost).where(M.InvHost.project_id == c.project_id, M.InvHost.name != "localhost"))
        return [n.to_dict(exclude=("password", "private_key")) | {"roles": n.groups} for n in rows]


def add_node(cluster_name: str, data: dict) -> dict:
    """Bind a registered host as a node with roles (reference Node.save -> on_node_save, node.py:40-50)."""
    c = get_cluster(cluster_name)
    with session_scope() as s:
        h = s.scalar(select(M.Host).where((M.Host.name == data["host"]) | (M.Host.id == data["host"])))
        if h is None:
            raise NotFound(f"host {data['host']} not registered")
        if h.node_id:
            raise Conflict(f"host {h.name} already belongs to a cluster")
        user, pw, key = h.username, h.password, h.private_key
        if h.credential_id:
            cr = s.get(M.Credential, h.credential_id)
            if cr is not None:
                user, pw, key = cr.username, cr.password, cr.private_key
        groups = list(data.get("roles") or [])
        vars = dict(data.get("vars") or {})
        if h.gpus:
            vars.update(has_gpu=True, gpu_vendor=h.gpu_vendor or "amd", gpu_num=len(h.gpus),
                        gpu_arch=(h.gpus[0].get("arch") or ""), gpu_model=h.gpus[0].get("name", ""))
            if "gpu_nodes" not in groups and ("worker" in groups or "new_node" in groups):
                groups.append("gpu_nodes")
        n = M.InvHost(project_id=c.project_id, name=data["name"], ip=h.ip, port=h.port, username=user, password=pw,
                      private_key=key, vars=vars, groups=groups, host_id=h.id)
        s.add(n)
        s.flush()
        h.node_id = n.id
        return n.to_dict(exclude=("password", "private_key"))


def remove_node_record(cluster_name: str, node_name: str) -> None:
    c = get_cluster(cluster_name)
    with session_scope() as s:
        n = s.scalar(select(M.InvHost).where(M.InvHost.project_id == c.project_id, M.InvHost.name == node_name))
        if n is None:
            raise NotFound(f"node {node_name} not found")
        if n.host_id:
            h = s.get(M.Host, n.host_id)
            if h is not None:
                h.node_id = None
        s.delete(n)


def add_worker(cluster_name: str, host_name: str) -> str:
    """Day-2 add-worker: ``worker<N+1>.<cluster>.<suffix>`` in groups worker,new_node (cluster.py:326-334)."""
    c = get_cluster(cluster_name)
    with session_scope() as s:
        n = s.scalar(select(func.count()).select_from(M.InvHost).where(M.InvHost.project_id == c.project_id,
                                                                      M.InvHost.groups.like('%"worker"%')))
    suffix = f".{c.cluster_doamin_suffix}" if c.cluster_doamin_suffix else ""
    name = f"worker{(n or 0) + 1}.{c.name}{suffix}"
    add_node(cluster_name, {"name": name, "host": host_name, "roles": ["worker", "new_node"]})
    return name


def set_node_groups(cluster_name: str, node_name: str, groups: list[str]) -> None:
    c = get_cluster(cluster_name)
    with session_scope() as s:
        n = s.scalar(select(M.InvHost).where(M.InvHost.project_id == c.project_id, M.InvHost.name == node_name))
        n.groups = list(dict.fromkeys(groups + (["gpu_nodes"] if "gpu_nodes" in (n.groups or []) else [])))


def exit_new_node(cluster_name: str) -> None:
    c = get_cluster(cluster_name)
    with session_scope() as s:
        for n in s.scalars(select(M.InvHost).where(M.InvHost.project_id == c.project_id)):
            if "new_node" in (n.groups or []):
                n.groups = [g for g in n.groups if g != "new_node"]


# --------------------------------------------------------------------------------------------- execution
def _storage_vars(c: M.Cluster) -> dict:
    """Variables of the storage back-end the cluster uses: the NFS server named by ``configs["nfs_storage"]``
    (its address / export path), or the external Ceph cluster bound to it (monitors, fsid, pool, key; the key
    stays encrypted at rest and is decrypted here, for the run only)."""
    out: dict = {}
    cfg = c.configs or {}
    with session_scope() as s:
        if cfg.get("nfs_storage"):
            n = s.scalar(select(M.NfsStorage).where(M.NfsStorage.name == cfg["nfs_storage"]))
            if n is None:
                raise NotFound(f"nfs storage {cfg['nfs_storage']} not found")
            v = n.vars or {}
            out.update({k: v[k] for k in ("storage_nfs_server", "storage_nfs_server_path") if k in v})
        b = s.scalar(select(M.ClusterCephStorage).where(M.ClusterCephStorage.cluster_id == c.id))
        if b is not None:
            v = dict(s.get(M.CephStorage, b.storage_id).vars or {})
            if v.get("ceph_key"):
                try:
                    v["ceph_key"] = context.dec(v["ceph_key"])
                except Exception:
                    pass  # stored in clear by an older record
            out.update(v)
    return out


def _cloud_vars(c: M.Cluster) -> dict:
    """AUTOMATIC clusters: the plan's region / zone variables (vCenter or OpenStack endpoint and credentials,
    datastores / volume types) for the vSphere and Cinder storage roles -- resolved per run, never copied into
    the stored cluster configs."""
    if not c.plan_id:
        return {}
    from . import cloud

    return cloud.mixed_vars(c.plan_id)


def extra_vars(c: M.Cluster) -> dict:
    """{cluster_name, cluster_domain} + settings + cloud / storage back-end vars + cluster configs
    (deploy.py:41-47)."""
    ev = {"cluster_name": c.name, "cluster_domain": c.cluster_doamin_suffix}
    ev.update(context.get_settings())
    ev.update(_cloud_vars(c))
    ev.update(_storage_vars(c))
    ev.update(c.configs or {})
    ev.setdefault("base_dir", "/etc/kubeoperator")
    from ..conf import get_config

    ev["controller_fetch_dir"] = os.path.join(get_config().data_dir, "fetch", c.name)
    return ev


def run_playbook(c: M.Cluster, playbook: str, variables: dict, logger=None, forks: int | None = None,
                 tracer=None) -> dict:
    from ..conf import get_config

    path = os.path.join(plan.PLAYBOOK_DIR, plan.playbook_alias(playbook))
    inv = context.project_inventory(c.project_id)
    cb = ResultCallback(display=logger)
    runner = Runner(inv, context.transport(), forks=forks or int(get_config()["ANSIBLE_FORKS"]), extra_vars=variables,
                    callback=cb, roles_path=[os.path.join(plan.PLAYBOOK_DIR, "roles")],
                    controller_dir=os.path.join(get_config().data_dir, "fetch", c.name), tracer=tracer)
    t0 = M.now()
    res = runner.run_playbook(path)
    with session_scope() as s:
        s.add(M.Execution(kind="playbook", project_id=c.project_id, operation=playbook,
                          state="SUCCESS" if res["summary"]["success"] else "FAILURE", date_start=t0,
                          date_end=M.now(), timedelta=(M.now() - t0).total_seconds(),
                          result_summary=_jsonable(res["summary"]), result_raw={}))
    return res


def run_adhoc(c: M.Cluster, pattern: str, module: str, args: dict, logger=None) -> dict:
    inv = context.project_inventory(c.project_id)
    r = Runner(inv, context.transport(), forks=5, callback=ResultCallback(display=logger))
    return r.run_adhoc(pattern, module, args)


def _jsonable(x):
    import json

    return json.loads(json.dumps(x, default=str))


def first_master(c: M.Cluster) -> str | None:
    inv = context.project_inventory(c.project_id)
    ms = inv.group_hosts("master")
    return ms[0] if ms else None


def fetch_kubeconfig(cluster_name: str) -> str:
    """Admin kubeconfig from the first master (reference adhoc.fetch_cluster_config, /root/.kube/config)."""
    c = get_cluster(cluster_name)
    m = first_master(c)
    if m is None:
        raise NotFound("cluster has no master")
    res = run_adhoc(c, m, "shell", {"_raw_params": "cat /etc/kubernetes/admin.conf 2>/dev/null || cat /root/.kube/config"})
    out = res["raw"]["ok"].get(m, {})
    if not out:
        raise RuntimeError(f"could not read kubeconfig from {m}")
    return next(iter(out.values())).get("stdout", "")


def cluster_token(cluster_name: str) -> str:
    """Bearer token of the kubeoperator-admin service account (replaces the tiller-secret scrape)."""
    c = get_cluster(cluster_name)
    m = first_master(c)
    cmd = ("kubectl -n kube-system get sa kubeoperator-admin >/dev/null 2>&1 || "
           "(kubectl -n kube-system create sa kubeoperator-admin && kubectl create clusterrolebinding "
           "kubeoperator-admin --clusterrole=cluster-admin --serviceaccount=kube-system:kubeoperator-admin); "
           "kubectl -n kube-system create token kubeoperator-admin --duration=87600h")
    res = run_adhoc(c, m, "shell", {"_raw_params": cmd})
    out = res["raw"]["ok"].get(m, {})
    return next(iter(out.values())).get("stdout", "").strip().splitlines()[-1] if out else ""
