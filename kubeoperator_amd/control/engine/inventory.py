"""In-memory inventory: hosts, groups (vars + children), host patterns, per-host variable resolution.

Replaces the reference's BaseInventory / LocalModelInventory over the Ansible API
(ansible_api/ansible/inventory.py:13-126, ansible_api/inventory.py:225-310). Same semantics the kubeasz
roles rely on: ``groups[...]`` (transitive through children), ``group_names``, ``hostvars``,
``inventory_hostname``, ``ansible_host``; variable precedence all-group < parent group < child group <
host vars; patterns ``all``, ``g1:g2`` (union), ``g1:&g2`` (intersection), ``g1:!g2`` (difference),
exact host names, and ``*`` globs.
"""
from __future__ import annotations

import copy
import fnmatch
import re
from dataclasses import dataclass, field

import yaml


@dataclass
class InvHostSpec:
    name: str
    vars: dict = field(default_factory=dict)

    @property
    def address(self) -> str:
        return str(self.vars.get("ansible_host") or self.vars.get("ansible_ssh_host") or self.name)


@dataclass
class InvGroupSpec:
    name: str
    hosts: list = field(default_factory=list)
    children: list = field(default_factory=list)
    vars: dict = field(default_factory=dict)


class Inventory:
    def __init__(self):
        self.hosts: dict[str, InvHostSpec] = {}
        self.groups: dict[str, InvGroupSpec] = {"all": InvGroupSpec("all"), "ungrouped": InvGroupSpec("ungrouped")}

    # construction ---------------------------------------------------------------------------------
    def add_host(self, name: str, vars: dict | None = None, groups=()):
        h = self.hosts.get(name)
        if h is None:
            h = self.hosts[name] = InvHostSpec(name, dict(vars or {}))
        else:
            h.vars.update(vars or {})
        for g in groups:
            grp = self.add_group(g)
            if name not in grp.hosts:
                grp.hosts.append(name)
        return h

    def add_group(self, name: str, vars: dict | None = None, children=()):
        g = self.groups.get(name)
        if g is None:
            g = self.groups[name] = InvGroupSpec(name)
        if vars:
            g.vars.update(vars)
        for c in children:
            self.add_group(c)
            if c not in g.children:
                g.children.append(c)
        return g

    @classmethod
    def from_dict(cls, data: dict) -> "Inventory":
        """``{"hosts": [{"name", "vars"|flat fields}], "groups": [{"name", "hosts", "children", "vars"}]}``
        (the reference's ``inventory_data`` shape) or the Ansible YAML shape ``{"all": {"children": ...}}``."""
        inv = cls()
        if "all" in data and isinstance(data["all"], dict):
            inv._load_yaml_group("all", data["all"])
            return inv
        for h in data.get("hosts", []):
            hv = dict(h.get("vars", {}))
            for k in ("ip", "port", "username", "password", "private_key"):
                if h.get(k) not in (None, ""):
                    hv[{"ip": "ansible_host", "port": "ansible_port", "username": "ansible_user",
                        "password": "ansible_ssh_pass", "private_key": "ansible_ssh_private_key_file"}[k]] = h[k]
            inv.add_host(h["name"], hv, h.get("groups", []))
        for g in data.get("groups", []):
            grp = inv.add_group(g["name"], g.get("vars"), g.get("children", []))
            for hn in g.get("hosts", []):
                inv.add_host(hn)
                if hn not in grp.hosts:
                    grp.hosts.append(hn)
        return inv

    def _load_yaml_group(self, name, body):
        body = body or {}
        g = self.add_group(name, body.get("vars"))
        for hn, hv in (body.get("hosts") or {}).items():
            self.add_host(hn, hv or {})
            if hn not in g.hosts:
                g.hosts.append(hn)
        for cn, cb in (body.get("children") or {}).items():
            self._load_yaml_group(cn, cb)
            if cn not in g.children:
                g.children.append(cn)

    # queries ---------------------------------------------------------------------------------------
    def group_hosts(self, name: str, _seen=None) -> list[str]:
        if name == "all":
            return list(self.hosts)
        g = self.groups.get(name)
        if g is None:
            return []
        _seen = _seen or set()
        if name in _seen:
            return []
        _seen.add(name)
        out = list(g.hosts)
        for c in g.children:
            for h in self.group_hosts(c, _seen):
                if h not in out:
                    out.append(h)
        return out

    def groups_dict(self) -> dict:
        d = {n: self.group_hosts(n) for n in self.groups}
        ung = [h for h in self.hosts if not any(h in g.hosts for n, g in self.groups.items() if n not in ("all", "ungrouped"))]
        d["ungrouped"] = ung
        return d

    def host_groups(self, host: str) -> list[str]:
        return sorted(n for n in self.groups if n not in ("all",) and host in self.group_hosts(n))

    def _group_depth(self, name, memo):
        if name in memo:
            return memo[name]
        memo[name] = 0
        parents = [n for n, g in self.groups.items() if name in g.children]
        d = 1 + max((self._group_depth(p, memo) for p in parents), default=0)
        memo[name] = d
        return d

    def host_vars(self, host: str) -> dict:
        """Merged variables: all < groups by depth (parents before children) < host."""
        memo = {}
        out = copy.deepcopy(self.groups["all"].vars)
        gs = sorted(self.host_groups(host), key=lambda n: (self._group_depth(n, memo), n))
        for g in gs:
            out.update(copy.deepcopy(self.groups[g].vars))
        h = self.hosts.get(host)
        if h is not None:
            out.update(copy.deepcopy(h.vars))
        out.setdefault("ansible_host", h.address if h else host)
        out["inventory_hostname"] = host
        out["inventory_hostname_short"] = host.split(".")[0]
        out["group_names"] = [g for g in gs if g != "ungrouped"]
        return out

    def match(self, pattern) -> list[str]:
        """Resolve an Ansible host pattern to host names (inventory order)."""
        if isinstance(pattern, list):
            pattern = ":".join(pattern)
        pattern = str(pattern).strip()
        if pattern in ("", "all", "*"):
            return list(self.hosts)
        result: list[str] = []
        for raw in [p for p in re.split(r"[:,](?![^\[]*\])", pattern) if p]:
            op = ""
            if raw[0] in "&!":
                op, raw = raw[0], raw[1:]
            sel = self._atom(raw)
            if op == "&":
                result = [h for h in result if h in sel]
            elif op == "!":
                result = [h for h in result if h not in sel]
            else:
                result += [h for h in sel if h not in result]
        order = list(self.hosts)
        return sorted(result, key=lambda h: order.index(h) if h in order else 1 << 30)

    def _atom(self, a: str) -> list[str]:
        m = re.match(r"^(.+)\[(-?\d*)(?::(-?\d*))?\]$", a)
        if m:  # group[i] / group[i:j] subscripts (e.g. kube-master[0])
            hosts = self._atom(m.group(1))
            i = int(m.group(2)) if m.group(2) not in ("", None) else None
            if m.group(3) is None and ":" not in a:
                return hosts[i:i + 1] if i is not None and -len(hosts) <= i < len(hosts) else []
            j = int(m.group(3)) if m.group(3) not in ("", None) else None
            return hosts[i:j]
        if a in self.groups:
            return self.group_hosts(a)
        if a in self.hosts:
            return [a]
        if any(c in a for c in "*?["):
            out = [h for h in self.hosts if fnmatch.fnmatch(h, a)]
            for gname in self.groups:
                if fnmatch.fnmatch(gname, a):
                    out += [h for h in self.group_hosts(gname) if h not in out]
            return out
        return []

    # rendering ----------------------------------------------------------------------------------------
    def to_dict(self) -> dict:
        """Ansible YAML inventory structure (what `ansible-inventory --list -y` would show)."""
        def group_body(name):
            g = self.groups[name]
            body = {}
            if g.hosts:
                body["hosts"] = {h: dict(self.hosts[h].vars) for h in g.hosts}
            if g.vars:
                body["vars"] = dict(g.vars)
            if g.children:
                body["children"] = {c: group_body(c) for c in g.children}
            return body

        top_children = [n for n in self.groups if n not in ("all", "ungrouped")
                        and not any(n in g.children for g in self.groups.values())]
        all_body = {"children": {n: group_body(n) for n in top_children}}
        if self.groups["all"].vars:
            all_body["vars"] = dict(self.groups["all"].vars)
        loose = [h for h in self.hosts if not any(h in self.group_hosts(n) for n in top_children)]
        if loose:
            all_body["hosts"] = {h: dict(self.hosts[h].vars) for h in loose}
        return {"all": all_body}

    def to_yaml(self) -> str:
        return yaml.safe_dump(self.to_dict(), sort_keys=False, default_flow_style=False)
