"""Storage back-ends offered to clusters: NFS servers deployed by the engine, external Ceph configs.

Reference: storage/models.py:20-102 (NfsStorage is its own Ansible project running ``nfs.yml``; CephStorage
rows; ClusterCephStorage binding), storage/signal_handlers.py. Cluster-side provisioners (nfs client
provisioner, rook-ceph, external ceph RBD, local volumes, vSphere, Cinder) are installed by the addon
play from the cluster's ``persistent_storage`` choice.
"""
from __future__ import annotations

import os
import threading

from sqlalchemy import select

from ..engine import Inventory, ResultCallback, Runner
from ..runtime import jobs
from ..store import models as M
from ..store.db import session_scope
from . import context, plan


def create_nfs(data: dict, run: str = "queue") -> dict:
    """Register an NFS server; ``vars.storage_nfs_server`` etc.; deploys it unless ``vars.external``."""
    with session_scope() as s:
        if s.scalar(select(M.NfsStorage).where(M.NfsStorage.name == data["name"])) is not None:
            raise ValueError(f"nfs {data['name']} exists")
        proj = M.Project(name=f"nfs-{data['name']}", kind="nfs")
        s.add(proj)
        s.flush()
        n = M.NfsStorage(project_id=proj.id, name=data["name"], vars=dict(data.get("vars") or {}),
                         status="CREATING" if not (data.get("vars") or {}).get("external") else "RUNNING")
        s.add(n)
        s.flush()
        nid = n.id
    if not (data.get("vars") or {}).get("external"):
        if run == "queue":
            jobs.submit("deploy_nfs", {"nfs_id": nid})
        elif run == "inline":
            jobs.run_inline("deploy_nfs", {"nfs_id": nid})
    with session_scope() as s:
        return s.get(M.NfsStorage, nid).to_dict()


@jobs.task("deploy_nfs")
def deploy_nfs(job_id, logger, nfs_id):
    with session_scope() as s:
        n = s.get(M.NfsStorage, nfs_id)
        v = dict(n.vars or {})
    inv = Inventory()
    hv = {"ansible_host": v.get("storage_nfs_server"), "ansible_port": int(v.get("port", 22)),
          "ansible_user": v.get("username", "root")}
    if v.get("password"):
        hv["ansible_ssh_pass"] = context.dec(v["password"])
    inv.add_host("nfs-server", hv, ["nfs"])
    r = Runner(inv, context.transport(), callback=ResultCallback(display=logger), extra_vars=v,
               roles_path=[os.path.join(plan.PLAYBOOK_DIR, "roles")])
    res = r.run_playbook(os.path.join(plan.PLAYBOOK_DIR, "nfs.yml"))
    with session_scope() as s:
        s.get(M.NfsStorage, nfs_id).status = "RUNNING" if res["summary"]["success"] else "ERROR"
    return {"success": res["summary"]["success"]}


def list_nfs() -> list[dict]:
    with session_scope() as s:
        return [n.to_dict() for n in s.scalars(select(M.NfsStorage))]


def delete_nfs(name: str) -> None:
    with session_scope() as s:
        n = s.scalar(select(M.NfsStorage).where(M.NfsStorage.name == name))
        if n is not None:
            if n.project_id:
                s.delete(s.get(M.Project, n.project_id))
            s.delete(n)


def create_ceph(data: dict) -> dict:
    """External Ceph cluster (fsid ``ceph_cluster_id``, ``ceph_monitors``, ``ceph_pool``, ``ceph_user``, ``ceph_key``);
    the key is stored encrypted (store/crypto) and decrypted only into a deploy run's variables."""
    v = dict(data.get("vars") or {})
    if v.get("ceph_key"):
        v["ceph_key"] = context.enc(v["ceph_key"])
    with session_scope() as s:
        c = M.CephStorage(name=data["name"], vars=v)
        s.add(c)
        s.flush()
        return c.to_dict()


def list_ceph() -> list[dict]:
    with session_scope() as s:
        return [c.to_dict() for c in s.scalars(select(M.CephStorage))]


def delete_ceph(name: str) -> None:
    with session_scope() as s:
        c = s.scalar(select(M.CephStorage).where(M.CephStorage.name == name))
        if c is not None:
            s.delete(c)


def bind_ceph(cluster_id: str, ceph_name: str) -> None:
    with session_scope() as s:
        c = s.scalar(select(M.CephStorage).where(M.CephStorage.name == ceph_name))
        s.add(M.ClusterCephStorage(cluster_id=cluster_id, storage_id=c.id))


_lock = threading.Lock()
