"""Offline packages (reference kubeops_api/models/package.py:16-63, package_manage.py:10-69).

A package directory ``<PACKAGE_DIR>/<name>/`` holds ``meta.yml`` and the repository content (apt/yum
repo, OCI images, kube/ROCm binaries). The reference starts one Nexus container per package through the
Docker socket; here the control plane serves each package's ``repo/`` tree itself over HTTP (a
``ThreadingHTTPServer`` per package on its ``repo_port``) and expects an OCI registry (the package's
``registry/`` content, e.g. a ``distribution`` binary) on ``registry_port`` -- no Docker daemon on the
controller is required.
"""
from __future__ import annotations

import functools
import http.server
import os
import threading

from sqlalchemy import select

from ..store import models as M
from ..store.db import session_scope
from . import plan
from .clusters import NotFound, get_cluster


def sync_packages() -> list[dict]:
    """Re-scan the package directory into the store (called by every package list, like api.py:130-135)."""
    found = plan.scan_packages()
    names = {p["name"] for p in found}
    for p in plan.builtin_packages():
        if p["name"] not in names:
            found.append({**p, "path": "builtin"})
    with session_scope() as s:
        for p in found:
            row = s.scalar(select(M.Package).where(M.Package.name == p["name"]))
            if row is None:
                s.add(M.Package(name=p["name"], meta=p["meta"], path=p["path"]))
            else:
                row.meta, row.path = p["meta"], p["path"]
        return [r.to_dict() for r in s.scalars(select(M.Package).order_by(M.Package.name))]


def get_package(name: str) -> dict:
    for p in sync_packages():
        if p["name"] == name:
            return p
    raise NotFound(f"package {name} not found")


def upgrade_cluster_package(cluster_name: str, package: str) -> None:
    """After a successful upgrade: record the new package and merge its vars (Cluster.upgrade_package)."""
    meta = get_package(package)["meta"]
    c = get_cluster(cluster_name)
    with session_scope() as s:
        row = s.get(M.Cluster, c.id)
        row.upgrade_from = row.package
        row.package = package
        row.configs = {**(row.configs or {}), **(meta.get("vars") or {})}


_servers: dict[str, http.server.ThreadingHTTPServer] = {}


def serve_package(name: str, host: str = "0.0.0.0") -> int:
    """Serve ``<package>/repo`` over HTTP on the package's repo_port; returns the port."""
    p = get_package(name)
    port = int((p["meta"].get("vars") or {}).get("repo_port", 8081))
    root = os.path.join(p["path"], "repo")
    if name in _servers or not os.path.isdir(root):
        return port
    handler = functools.partial(http.server.SimpleHTTPRequestHandler, directory=root)
    srv = http.server.ThreadingHTTPServer((host, port), handler)
    threading.Thread(target=srv.serve_forever, name=f"pkg-{name}", daemon=True).start()
    _servers[name] = srv
    return port


def stop_servers() -> None:
    for srv in _servers.values():
        srv.shutdown()
    _servers.clear()
