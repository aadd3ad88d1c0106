"""Shared services of the domain layer: transport provider, secret helpers, settings, inventory building.

There is no thread-local "current project" (reference ansible_api/ctx.py:12-34): every query names its
project explicitly, so concurrent executions of different clusters cannot see each other's rows.
"""
from __future__ import annotations

import threading

from sqlalchemy import select

from ..conf import get_config
from ..engine import Inventory, Transport, make_transport
from ..store import models as M
from ..store.crypto import decrypt, encrypt
from ..store.db import session_scope

_factory_lock = threading.Lock()
_transport_factory = None


def set_transport_factory(fn) -> None:
    """Override how the engine reaches hosts (tests install a FakeTransport farm here)."""
    global _transport_factory
    with _factory_lock:
        _transport_factory = fn


def transport() -> Transport:
    with _factory_lock:
        fn = _transport_factory
    if fn is not None:
        return fn()
    cfg = get_config()
    kind = cfg["DEFAULT_TRANSPORT"]
    if kind == "ssh":  # host keys pinned per host under DATA_DIR (survive restarts of the control plane)
        import os

        return make_transport(kind, known_hosts_dir=os.path.join(cfg["DATA_DIR"], "ssh", "known_hosts"))
    return make_transport(kind)


def enc(value: str) -> str:
    return encrypt(value or "", get_config().secret_key())


def dec(value: str) -> str:
    return decrypt(value or "", get_config().secret_key())


def get_settings(tab: str | None = None) -> dict:
    """Flat key -> value map (reference Setting.get_settings, models/setting.py:16-44)."""
    with session_scope() as s:
        q = select(M.Setting)
        if tab:
            q = q.where(M.Setting.tab == tab)
        return {r.key: r.value for r in s.scalars(q)}


def set_settings(values: dict, tab: str = "system") -> None:
    with session_scope() as s:
        for k, v in values.items():
            row = s.scalar(select(M.Setting).where(M.Setting.tab == tab, M.Setting.key == k))
            if row is None:
                s.add(M.Setting(tab=tab, key=k, value="" if v is None else str(v)))
            else:
                row.value = "" if v is None else str(v)


def project_inventory(project_id: str) -> Inventory:
    """Inventory of a project from the store (reference LocalModelInventory, ansible_api/inventory.py)."""
    inv = Inventory()
    with session_scope() as s:
        groups = list(s.scalars(select(M.InvGroup).where(M.InvGroup.project_id == project_id)))
        hosts = list(s.scalars(select(M.InvHost).where(M.InvHost.project_id == project_id)))
        for g in groups:
            inv.add_group(g.name, dict(g.vars or {}))
        for g in groups:
            inv.add_group(g.name, None, list(g.children or []))
        for h in hosts:
            hv = dict(h.vars or {})
            if h.ip:
                hv.setdefault("ansible_host", h.ip)
            hv.setdefault("ansible_port", h.port)
            hv.setdefault("ansible_user", h.username)
            if h.password:
                hv.setdefault("ansible_ssh_pass", dec(h.password))
            if h.private_key:
                hv.setdefault("ansible_ssh_private_key_file", dec(h.private_key))
            inv.add_host(h.name, hv, list(h.groups or []))
    return inv
