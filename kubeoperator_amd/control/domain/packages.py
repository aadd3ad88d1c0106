"""Offline packages (reference kubeops_api/models/package.py:16-63, package_manage.py:10-69).

A package directory ``<PACKAGE_DIR>/<name>/`` holds ``meta.yml``, ``repo/`` (apt / yum trees, charts,
kube / ROCm binaries, manifests) and ``registry/`` (an OCI image layout with every image the roles pull).
The reference starts one Nexus container per package through the Docker socket; here the ``repo`` service
(``kubeopsctl start repo``, part of ``all``) serves each package itself: the file repository on
``repo_port`` and a read-only OCI distribution registry on ``registry_port`` (``repo_server.py``). Ports are
checked across packages and a clashing package is refused, never half-served.
"""
from __future__ import annotations

import logging
import os
import threading

from sqlalchemy import select

from ..store import models as M
from ..store.db import session_scope
from . import plan
from .clusters import NotFound, get_cluster

log = logging.getLogger("kubeops.packages")


def sync_packages(_start: bool = True) -> list[dict]:
    """Re-scan the package directory into the store (called by every package list, like api.py:130-135).
    Rows carry the ports, a port-``conflict`` message and which endpoints are ``serving``; with the repo
    service on in this process, newly found packages are served here too (as Package.lookup does)."""
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
        rows = _with_status([r.to_dict() for r in s.scalars(select(M.Package).order_by(M.Package.name))])
    if _start and _serving["on"]:
        for r in rows:
            if r["path"] != "builtin" and not r["conflict"] and r["name"] not in _servers:
                try:
                    serve_package(r["name"])
                except (OSError, ValueError) as e:
                    log.error("package %s not served: %s", r["name"], e)
        rows = _with_status(rows)
    return rows


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


_servers: dict[str, dict] = {}  # package -> {"repo": RepoServer | None, "registry": RegistryServer | None}
_serve_lock = threading.RLock()
_serving = {"on": False, "host": "0.0.0.0"}  # set by serve_all(): later syncs also start new packages


def _ports(meta: dict) -> dict:
    v = meta.get("vars") or {}
    return {"repo_port": int(v.get("repo_port", 8081)), "registry_port": int(v.get("registry_port", 8082))}


def port_conflicts(pkgs: list[dict]) -> dict[str, str]:
    """Packages whose repo / registry port is already claimed by another package (first by name wins), or
    whose two ports are equal. A package in this map is never served: two Nexus-style endpoints cannot share a
    port (reference package_manage.py:31-45 maps each package's container to its own ports)."""
    claimed: dict[int, str] = {}
    bad: dict[str, str] = {}
    # packages with content first (by name), then the built-in metas: a built-in (nothing to serve) never takes a
    # port away from a package dropped into PACKAGE_DIR
    for p in sorted(pkgs, key=lambda x: (x.get("path") == "builtin", x["name"])):
        ports = _ports(p.get("meta") or {})
        if ports["repo_port"] == ports["registry_port"]:
            bad[p["name"]] = f"repo_port and registry_port are both {ports['repo_port']}"
            continue
        clash = [(k, ports[k], claimed[ports[k]]) for k in ports if ports[k] in claimed]
        if clash:
            k, port, other = clash[0]
            bad[p["name"]] = f"{k} {port} is already claimed by package {other}"
            continue
        for port in ports.values():
            claimed[port] = p["name"]
    return bad


def _with_status(rows: list[dict]) -> list[dict]:
    bad = port_conflicts(rows)
    for r in rows:
        r.update(_ports(r.get("meta") or {}))
        r["conflict"] = bad.get(r["name"], "")
        srv = _servers.get(r["name"]) or {}
        r["serving"] = {k: bool(srv.get(k)) for k in ("repo", "registry")}
    return rows


def serve_package(name: str, host: str | None = None) -> dict:
    """Start the package's endpoints: ``<package>/repo`` over HTTP on ``repo_port`` and the OCI registry over
    ``<package>/registry`` on ``registry_port`` (domain/repo_server.py). Idempotent; refuses a package whose
    ports clash with another package. Returns {"repo": port | None, "registry": port | None}."""
    from .repo_server import RegistryServer, RepoServer

    rows = sync_packages(_start=False)
    p = next((r for r in rows if r["name"] == name), None)
    if p is None:
        raise NotFound(f"package {name} not found")
    if p["conflict"]:
        raise ValueError(f"package {name} not served: {p['conflict']}")
    host = host or _serving["host"]
    with _serve_lock:
        cur = _servers.setdefault(name, {"repo": None, "registry": None})
        repo_dir, reg_dir = os.path.join(p["path"], "repo"), os.path.join(p["path"], "registry")
        if cur["repo"] is None and os.path.isdir(repo_dir):
            cur["repo"] = RepoServer(repo_dir, host, p["repo_port"], name)
            log.info("package %s: repository on :%d (%s)", name, cur["repo"].port, repo_dir)
        if cur["registry"] is None and os.path.isfile(os.path.join(reg_dir, "index.json")):
            cur["registry"] = RegistryServer(reg_dir, host, p["registry_port"], name)
            log.info("package %s: OCI registry on :%d (%d repositories)", name, cur["registry"].port,
                     len(cur["registry"].layout.tags))
        return {k: (srv.port if srv else None) for k, srv in cur.items()}


def serve_all(host: str = "0.0.0.0") -> dict:
    """Serve every package with content (the ``repo`` service; reference Package.lookup starts a container per
    package at scan time, models/package.py:41-62). Clashing packages are logged and skipped."""
    _serving.update(on=True, host=host)
    out = {}
    for p in sync_packages(_start=False):
        if p["path"] == "builtin":
            continue
        if p["conflict"]:
            log.error("package %s not served: %s", p["name"], p["conflict"])
            out[p["name"]] = {"error": p["conflict"]}
            continue
        try:
            out[p["name"]] = serve_package(p["name"], host)
        except OSError as e:  # port in use by something else
            log.error("package %s not served: %s", p["name"], e)
            out[p["name"]] = {"error": str(e)}
    return out


def stop_servers() -> None:
    with _serve_lock:
        for srv in _servers.values():
            for x in srv.values():
                if x is not None:
                    x.stop()
        _servers.clear()
        _serving["on"] = False
