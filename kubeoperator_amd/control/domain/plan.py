"""Cluster plan (reference core/resource/cluster/config.yml, read by models/cluster.py) and offline package
metadata (reference models/package.py:16-63, package_manage.py).

The plan defines which playbook each operation step runs, the role groups a cluster inventory gets, the
network / storage choices with their variables, and the deployment templates (node counts + hardware
requirements). A package is a directory ``<PACKAGE_DIR>/<name>/meta.yml`` with ``version``, ``resource``,
``vars`` (must include ``repo_port`` and ``registry_port``; every image/version/binary variable the roles
consume) and optional ``templates``.
"""
from __future__ import annotations

import copy
import functools
import os

import yaml

from ..conf import RESOURCE_DIR, get_config

PLAN_PATH = os.path.join(RESOURCE_DIR, "cluster", "config.yml")
PLAYBOOK_DIR = os.path.join(RESOURCE_DIR, "kubeasz")


@functools.lru_cache(maxsize=4)
def load_plan(path: str = PLAN_PATH) -> dict:
    with open(path) as f:
        return yaml.safe_load(f)


def plan() -> dict:
    return copy.deepcopy(load_plan())


def playbook_alias(name: str) -> str:
    for pb in load_plan()["playbooks"]:
        if pb["name"] == name:
            return pb["alias"]
    raise KeyError(f"no playbook {name!r} in plan")


def operation_steps(operation: str) -> list[dict]:
    """Step list of an operation; backup/restore map to cluster-backup/cluster-restore (deploy.py:235-250)."""
    op = {"backup": "cluster-backup", "restore": "cluster-restore"}.get(operation, operation)
    for o in load_plan()["operations"]:
        if o["name"] == op:
            return [dict(s) for s in o["steps"]]
    raise KeyError(f"no operation {operation!r} in plan")


def template(name: str) -> dict:
    for t in load_plan()["templates"]:
        if t["name"] == name or t.get("deploy_type") == name:
            return copy.deepcopy(t)
    raise KeyError(f"no template {name!r} in plan")


def network(name: str) -> dict:
    for n in load_plan()["networks"]:
        if n["name"] == name:
            return copy.deepcopy(n)
    raise KeyError(f"no network plugin {name!r} in plan")


def storage(name: str) -> dict | None:
    for s in load_plan()["storages"]:
        if s["name"] == name:
            return copy.deepcopy(s)
    return None


def check_requirements(tmpl: dict, role: str, host: dict) -> list[str]:
    """Device checks of the create wizard (reference ui device-check.service.ts): [] when the host fits."""
    errs = []
    for r in tmpl["roles"]:
        if r["name"] != role:
            continue
        req = (r.get("meta") or {}).get("requires") or {}
        for d in req.get("device_require", []):
            have = host.get("cpu_core", 0) if d["name"] == "cpu_core" else host.get("memory", 0) / 1024.0
            if have < d["minimal"]:
                errs.append(f"{d['verbose']}: {have:g} < minimal {d['minimal']}")
        allow = (r.get("meta") or {}).get("allow_os") or []
        if allow and host.get("os"):
            ok = any(host["os"].lower().startswith(a["name"].lower()) and
                     any(str(host.get("os_version", "")).startswith(v) for v in a["version"]) for a in allow)
            if not ok:
                errs.append(f"OS {host.get('os')} {host.get('os_version')} not in {[a['name'] for a in allow]}")
    return errs


def check_node_counts(tmpl: dict, counts: dict) -> list[str]:
    errs = []
    for r in tmpl["roles"]:
        req = ((r.get("meta") or {}).get("requires") or {}).get("nodes_require")
        if not req:
            continue
        op, n = req
        have = counts.get(r["name"], 0)
        if (op == "=" and have != n) or (op == ">" and have < n) or (op == ">=" and have < n):
            errs.append(f"role {r['name']}: needs {op} {n} nodes, got {have}")
    return errs


# --------------------------------------------------------------------------------------------- packages
def package_dir() -> str:
    return get_config().package_dir


def scan_packages(root: str | None = None) -> list[dict]:
    """Every ``<PACKAGE_DIR>/<name>/meta.yml`` (re-scanned on each list, as api.py:130-135 does)."""
    out = []
    root = root or package_dir()
    for name in sorted(os.listdir(root)) if os.path.isdir(root) else []:
        p = os.path.join(root, name, "meta.yml")
        if os.path.isfile(p):
            with open(p) as f:
                meta = yaml.safe_load(f) or {}
            out.append({"name": name, "meta": meta, "path": os.path.join(root, name)})
    return out


def builtin_packages() -> list[dict]:
    """Package metadata shipped with the control plane (usable without repository content: the nodes then
    pull from the upstream mirrors named in the meta)."""
    return scan_packages(os.path.join(RESOURCE_DIR, "packages"))


def builtin_package_meta() -> dict:
    """Default MI355X package (ROCm + Kubernetes versions) shipped with the control plane."""
    with open(os.path.join(RESOURCE_DIR, "packages", "mi355x-k8s", "meta.yml")) as f:
        return yaml.safe_load(f)
