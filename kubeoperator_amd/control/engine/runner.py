"""Playbook / ad-hoc execution engine (replaces the Ansible 2.6 Python API of the reference:
ansible_api/ansible/runner.py:84-258, callback.py:10-133).

Executes playbooks written in Ansible's YAML language over an :class:`Inventory` through a
:class:`Transport`, with the constructs the provisioning roles use:

plays: ``hosts`` patterns, ``vars``, ``vars_files``, ``roles`` (with role ``vars`` / ``when`` / ``tags``),
``pre_tasks`` / ``tasks`` / ``post_tasks`` / ``handlers``, ``serial`` (rolling batches, int or %),
``gather_facts``, ``any_errors_fatal``, ``become``, ``environment``, ``import_playbook``;
tasks: module calls (free-form or dict args), ``name``, ``when``, ``loop`` / ``with_items`` / ``with_list``
/ ``with_dict`` / ``with_sequence`` + ``loop_control``, ``register``, ``until`` / ``retries`` / ``delay``,
``ignore_errors``, ``failed_when``, ``changed_when``, ``delegate_to``, ``run_once``, ``notify`` + handlers
(+ ``meta: flush_handlers``), ``tags`` / skip-tags, ``vars``, ``environment``, ``block`` / ``rescue`` /
``always``, ``include_tasks`` / ``import_tasks`` / ``include_role`` / ``import_role``, ``no_log``.
Roles: ``tasks/ handlers/ defaults/ vars/ templates/ files/ meta(dependencies)``.

Strategy "linear" like Ansible: each task runs on all live hosts of the batch in parallel (``forks``
threads, default 5 as in the reference) before the next task starts; a failed or unreachable host leaves
the play. Results are collected in the reference's shape: ``raw = {ok, failed, unreachable, skipped}``
and ``summary = {contacted, dark, success}`` per host per task.
"""
from __future__ import annotations

import copy
import re
import datetime
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import yaml

from .inventory import Inventory
from .modules import MODULES, ModuleContext, ModuleError
from .templating import LazyVars, TemplateError, evaluate, render
from .transport import FakeTransport, HostConn, Transport, Unreachable

TASK_KEYWORDS = {
    "name", "when", "loop", "with_items", "with_list", "with_dict", "with_sequence", "with_nested", "loop_control", "register",
    "until", "retries", "delay", "ignore_errors", "failed_when", "changed_when", "delegate_to", "run_once",
    "notify", "tags", "vars", "environment", "become", "become_user", "no_log", "args", "block", "rescue",
    "always", "include_tasks", "import_tasks", "include_role", "import_role", "listen", "check_mode",
    "connection", "local_action", "any_errors_fatal", "timeout", "async", "poll", "_role", "_when_extra",
    "_tags_extra", "_role_vars", "_role_defaults", "_role_path", "ignore_unreachable", "debugger", "throttle",
}


class PlaybookError(Exception):
    pass


# ---------------------------------------------------------------------------------------------- callback
class ResultCallback:
    """Collects results (reference callback.py:10-133 shape) and writes an Ansible-like display log."""

    def __init__(self, display=None):
        self._display = display
        self.results_raw = {"ok": {}, "failed": {}, "unreachable": {}, "skipped": {}}
        self.results_summary = {"contacted": {}, "dark": {}, "success": True}
        self.stats = {}
        self._lock = threading.Lock()

    @property
    def results(self):
        return {"raw": self.results_raw, "summary": self.results_summary}

    def display(self, msg: str) -> None:
        if self._display is not None:
            self._display(msg)

    def _detail(self, res: dict) -> dict:
        if res.get("rc") is not None:
            cmd = res.get("cmd")
            return {"cmd": " ".join(cmd) if isinstance(cmd, list) else str(cmd), "stderr": res.get("stderr"),
                    "stdout": res.get("stdout"), "rc": res.get("rc"), "delta": res.get("delta"),
                    "msg": res.get("msg", "")}
        return {"changed": res.get("changed", False), "msg": res.get("msg", "")}

    def _stat(self, host, key):
        s = self.stats.setdefault(host, {"ok": 0, "changed": 0, "failed": 0, "unreachable": 0, "skipped": 0,
                                         "ignored": 0})
        s[key] += 1

    def gather(self, kind: str, host: str, task: str, res: dict, ignore=False):
        with self._lock:
            if kind == "failed" and ignore:
                self._stat(host, "ignored")
                self.results_summary["contacted"].setdefault(host, {})[task] = self._detail(res)
                return
            self.results_raw[kind].setdefault(host, {})[task] = res
            if kind in ("ok", "skipped"):
                self.results_summary["contacted"].setdefault(host, {})[task] = self._detail(res)
            else:
                self.results_summary["dark"].setdefault(host, {})[task] = self._detail(res)
                self.results_summary["success"] = False
            self._stat(host, kind)
            if kind == "ok" and res.get("changed"):
                self._stat(host, "changed")

    def rescue(self, host: str, tasks: set) -> None:
        with self._lock:
            for tn in tasks:
                res = self.results_raw["failed"].get(host, {}).pop(tn, None)
                if res is not None:
                    self.results_raw["ok"].setdefault(host, {})[tn] = {**res, "rescued": True}
                d = self.results_summary["dark"].get(host, {}).pop(tn, None)
                if d is not None:
                    self.results_summary["contacted"].setdefault(host, {})[tn] = {**d, "rescued": True}
                s = self.stats.get(host)
                if s:
                    s["failed"] -= 1
                    s["rescued"] = s.get("rescued", 0) + 1
            for k in ("failed", "unreachable"):
                self.results_raw[k] = {h: v for h, v in self.results_raw[k].items() if v}
            self.results_summary["dark"] = {h: v for h, v in self.results_summary["dark"].items() if v}
            self.results_summary["success"] = not (self.results_raw["failed"] or self.results_raw["unreachable"])

    def on_playbook_start(self, name):
        self.display(f"{datetime.datetime.now():%Y-%m-%d %H:%M:%S} Start task: {name}\r\n")

    def on_play_start(self, name):
        self.display(f"\r\nPLAY [{name}] {'*' * max(3, 70 - len(str(name)))}\r\n")

    def on_task_start(self, name):
        self.display(f"\r\nTASK [{name}] {'*' * max(3, 70 - len(str(name)))}\r\n")

    def on_result(self, status, host, res, item=None):
        label = f"{host}" + (f"] => (item={item}" if item is not None else "")
        line = f"{status}: [{label}]"
        if status in ("fatal", "failed") and res:
            line += " => " + yaml.safe_dump(self._detail(res), default_flow_style=True, width=200).strip()
        self.display(line + "\r\n")

    def on_playbook_end(self, name):
        self.display("\r\nPLAY RECAP " + "*" * 60 + "\r\n")
        for h, s in self.stats.items():
            self.display(f"{h:<30}: ok={s['ok']} changed={s['changed']} unreachable={s['unreachable']} "
                         f"failed={s['failed']} skipped={s['skipped']} ignored={s['ignored']}\r\n")
        self.display(f"{datetime.datetime.now():%Y-%m-%d %H:%M:%S} Task finish\r\n")


# ---------------------------------------------------------------------------------------------- loader
@dataclass
class Role:
    name: str
    path: str
    defaults: dict = field(default_factory=dict)
    vars: dict = field(default_factory=dict)
    tasks: list = field(default_factory=list)
    handlers: list = field(default_factory=list)


def _load_yaml(path: str):
    with open(path) as f:
        return yaml.safe_load(f)


class Loader:
    def __init__(self, roles_path: list[str]):
        self.roles_path = roles_path
        self._cache: dict[str, Role] = {}

    def find_role(self, name: str, base_dir: str) -> str:
        for root in [os.path.join(base_dir, "roles"), *self.roles_path]:
            p = os.path.join(root, name)
            if os.path.isdir(p):
                return p
        raise PlaybookError(f"role {name!r} not found in {[os.path.join(base_dir, 'roles'), *self.roles_path]}")

    def load_role(self, name: str, base_dir: str) -> Role:
        path = self.find_role(name, base_dir)
        if path in self._cache:
            return self._cache[path]
        r = Role(name, path)
        for sub, attr in (("defaults", "defaults"), ("vars", "vars")):
            p = os.path.join(path, sub, "main.yml")
            if os.path.exists(p):
                setattr(r, attr, _load_yaml(p) or {})
        for sub, attr in (("tasks", "tasks"), ("handlers", "handlers")):
            p = os.path.join(path, sub, "main.yml")
            if os.path.exists(p):
                setattr(r, attr, self.expand_tasks(_load_yaml(p) or [], os.path.join(path, sub), r))
        self._cache[path] = r
        return r

    def expand_tasks(self, tasks: list, base_dir: str, role: Role | None) -> list:
        """Resolve static imports (import_tasks) recursively; tag tasks with their role."""
        out = []
        for t in tasks or []:
            if not isinstance(t, dict):
                raise PlaybookError(f"task must be a mapping, got {t!r}")
            t = dict(t)
            if role is not None:
                t.setdefault("_role", role.name)
                t.setdefault("_role_path", role.path)
            if "import_tasks" in t:
                sub = os.path.join(base_dir, str(t["import_tasks"]))
                inner = self.expand_tasks(_load_yaml(sub) or [], os.path.dirname(sub), role)
                for it in inner:
                    _inherit(it, t)
                out.extend(inner)
                continue
            for key in ("block", "rescue", "always"):
                if key in t:
                    t[key] = self.expand_tasks(t[key], base_dir, role)
            if "include_tasks" in t:
                t["_include_base"] = base_dir
            out.append(t)
        return out


def _inherit(child: dict, parent: dict):
    if parent.get("when") is not None:
        w = child.get("_when_extra", [])
        child["_when_extra"] = w + (parent["when"] if isinstance(parent["when"], list) else [parent["when"]])
    if parent.get("tags"):
        tg = parent["tags"] if isinstance(parent["tags"], list) else [parent["tags"]]
        child["_tags_extra"] = child.get("_tags_extra", []) + tg
    if parent.get("vars"):
        child["vars"] = {**parent["vars"], **child.get("vars", {})}
    for k in ("become", "environment", "delegate_to", "run_once", "ignore_errors"):
        if k in parent and k not in child:
            child[k] = parent[k]


# ---------------------------------------------------------------------------------------------- runner
@dataclass
class HostState:
    facts: dict = field(default_factory=dict)
    failed: bool = False
    unreachable: bool = False
    notified: set = field(default_factory=set)


# connection secrets stay with the transport: templates (and so anything an API user can put in a cluster
# config or execution parameter) never see them -- the roles do not need them (they connect through the
# engine, which reads them from the inventory directly, ``Runner._conn``)
SECRET_VARS = ("ansible_ssh_pass", "ansible_password", "ansible_become_pass", "ansible_become_password",
               "ansible_ssh_private_key_file")


def _without_secrets(v: dict) -> dict:
    for k in SECRET_VARS:
        v.pop(k, None)
    return v


class _HostVars(dict):
    def __init__(self, runner: "Runner"):
        super().__init__()
        self._r = runner

    def __getitem__(self, host):
        # inventory + facts + extra vars (as Ansible's HostVars); templated values render on lookup
        return LazyVars(_without_secrets({**self._r.base_vars(host), **self._r.extra_vars}))

    def __contains__(self, host):
        return host in self._r.inventory.hosts

    def keys(self):
        return self._r.inventory.hosts.keys()

    def get(self, host, default=None):
        return self[host] if host in self else default


class Runner:
    def __init__(self, inventory: Inventory, transport: Transport, forks: int = 5, extra_vars: dict | None = None,
                 callback: ResultCallback | None = None, roles_path: list[str] | None = None,
                 check: bool = False, tags: list | None = None, skip_tags: list | None = None,
                 controller_dir: str | None = None, default_user: str = "root", tracer=None):
        self.inventory = inventory
        self.transport = transport
        self.forks = max(1, forks)
        self.extra_vars = dict(extra_vars or {})
        self.cb = callback or ResultCallback()
        self.tracer = tracer
        self.loader = Loader(roles_path or [])
        self.check = check
        self.tags = set(tags or [])
        self.skip_tags = set(skip_tags or [])
        self.state: dict[str, HostState] = {h: HostState() for h in inventory.hosts}
        self.controller_dir = controller_dir or os.getcwd()
        self.default_user = default_user
        self._play_vars: dict = {}
        self._play_hosts: list = []
        self._stop = threading.Event()

    # ------------------------------------------------------------------------------------ variables
    def base_vars(self, host: str) -> dict:
        v = self.inventory.host_vars(host)
        st = self.state.setdefault(host, HostState())
        v.update(st.facts)
        return v

    def task_vars(self, host: str, task: dict, item=None, loop_var="item") -> dict:
        v = {}
        v.update(task.get("_role_defaults", {}))
        v.update(_without_secrets(self.base_vars(host)))
        v.update(self._play_vars)
        v.update(task.get("_role_vars", {}))
        v.update(task.get("vars", {}) or {})
        v.update(self.state[host].facts)  # set_fact / register beat play and role vars (as in Ansible)
        v.update(self.extra_vars)
        v["hostvars"] = _HostVars(self)
        v["groups"] = self.inventory.groups_dict()
        v["play_hosts"] = v["ansible_play_hosts"] = list(self._play_hosts)
        v["ansible_play_batch"] = list(self._batch)
        v["role_path"] = task.get("_role_path", "")
        v["omit"] = "__omit_place_holder__"
        if item is not None or loop_var != "item":
            v[loop_var] = item
        return v

    def _conn(self, host: str, variables: dict) -> HostConn:
        hv = self.base_vars(host)
        return HostConn(
            name=host, address=str(hv.get("ansible_host", host)), port=int(hv.get("ansible_port", 22) or 22),
            user=str(hv.get("ansible_user") or hv.get("ansible_ssh_user") or self.default_user),
            password=str(hv.get("ansible_ssh_pass") or hv.get("ansible_password") or ""),
            private_key=str(hv.get("ansible_ssh_private_key_file") or ""),
            become=bool(variables.get("ansible_become", False)), extra={"connection": hv.get("ansible_connection")})

    # ------------------------------------------------------------------------------------ playbooks
    def _span(self, name, kind, **attrs):
        return self.tracer.begin(name, kind, **attrs) if self.tracer is not None else None

    def _span_end(self, sid, status="ok", **attrs):
        if sid is not None:
            self.tracer.end(sid, status, **attrs)

    def run_playbook(self, path: str) -> dict:
        name = os.path.basename(path)
        self.cb.on_playbook_start(name)
        sid = self._span(name, "playbook")
        try:
            self._run_playbook_file(path)
        finally:
            self.cb.on_playbook_end(name)
            self._span_end(sid, "ok" if self.cb.results_summary.get("success", True) else "failed")
        return self.cb.results

    def _run_playbook_file(self, path: str):
        plays = _load_yaml(path) or []
        base = os.path.dirname(os.path.abspath(path))
        for play in plays:
            if self._stop.is_set():
                break
            if "import_playbook" in play:
                self._run_playbook_file(os.path.join(base, str(play["import_playbook"])))
                continue
            self.run_play(play, base)

    def run_play(self, play: dict, base_dir: str) -> None:
        sid = self._span(play.get("name", play.get("hosts", "all")), "play")
        try:
            self._run_play(play, base_dir)
        finally:
            self._span_end(sid)

    def _run_play(self, play: dict, base_dir: str) -> None:
        pattern = render(play.get("hosts", "all"), self.extra_vars)
        hosts = [h for h in self.inventory.match(pattern) if not self.state[h].failed and not self.state[h].unreachable]
        pname = play.get("name", pattern)
        self.cb.on_play_start(pname)
        if not hosts:
            self.cb.display("skipping: no hosts matched\r\n")
            return
        pvars = dict(play.get("vars", {}) or {})
        for vf in play.get("vars_files", []) or []:
            p = os.path.join(base_dir, render(vf, {**pvars, **self.extra_vars}))
            pvars.update(_load_yaml(p) or {})
        play_env = play.get("environment")
        play_become = play.get("become")
        tasks: list = []

        def decorate(ts, role: Role | None = None, role_entry: dict | None = None):
            out = []
            for t in ts:
                t = copy.deepcopy(t)
                if role is not None:
                    t["_role_defaults"] = role.defaults
                    t["_role_vars"] = {**role.vars, **((role_entry or {}).get("vars") or {})}
                    if role_entry:
                        _inherit(t, {k: v for k, v in role_entry.items() if k in ("when", "tags", "become")})
                if play_env is not None and "environment" not in t:
                    t["environment"] = play_env
                if play_become is not None and "become" not in t:
                    t["become"] = play_become
                out.append(t)
            return out

        tasks += decorate(self.loader.expand_tasks(play.get("pre_tasks", []), base_dir, None))
        handlers = decorate(self.loader.expand_tasks(play.get("handlers", []), base_dir, None))
        for entry in play.get("roles", []) or []:
            entry = {"role": entry} if isinstance(entry, str) else dict(entry)
            rname = render(entry.get("role") or entry.get("name"), {**pvars, **self.extra_vars})
            role = self.loader.load_role(rname, base_dir)
            for dep in self._role_deps(role, base_dir):
                tasks += decorate(dep.tasks, dep)
                handlers += decorate(dep.handlers, dep)
            tasks += decorate(role.tasks, role, entry)
            handlers += decorate(role.handlers, role, entry)
        tasks += decorate(self.loader.expand_tasks(play.get("tasks", []), base_dir, None))
        tasks += decorate(self.loader.expand_tasks(play.get("post_tasks", []), base_dir, None))

        serial = play.get("serial")
        batches = [hosts]
        if serial:
            s = str(serial)
            n = max(1, int(len(hosts) * float(s[:-1]) / 100)) if s.endswith("%") else int(s)
            batches = [hosts[i:i + n] for i in range(0, len(hosts), n)]
        self._play_vars = pvars
        self._play_hosts = hosts
        for batch in batches:
            self._batch = batch
            if play.get("gather_facts", True) not in (False, "no", "false"):
                self._run_task({"name": "Gathering Facts", "setup": {}}, batch, base_dir, [])
            self._run_tasks(tasks, batch, base_dir, handlers)
            self._flush_handlers(batch, handlers, base_dir)
            if play.get("any_errors_fatal") and any(self.state[h].failed or self.state[h].unreachable for h in batch):
                self._stop.set()
                break
            if all(self.state[h].failed or self.state[h].unreachable for h in batch):
                break  # Ansible aborts the remaining batches when a whole batch failed

    def _role_deps(self, role: Role, base_dir: str) -> list[Role]:
        p = os.path.join(role.path, "meta", "main.yml")
        if not os.path.exists(p):
            return []
        meta = _load_yaml(p) or {}
        out = []
        for d in meta.get("dependencies", []) or []:
            dn = d if isinstance(d, str) else (d.get("role") or d.get("name"))
            dr = self.loader.load_role(dn, base_dir)
            out += self._role_deps(dr, base_dir) + [dr]
        return out

    # ------------------------------------------------------------------------------------ tasks
    def _live(self, hosts):
        return [h for h in hosts if not self.state[h].failed and not self.state[h].unreachable]

    def _run_tasks(self, tasks, hosts, base_dir, handlers):
        for t in tasks:
            if self._stop.is_set():
                return
            live = self._live(hosts)
            if not live:
                return
            if t.get("meta") == "flush_handlers":
                self._flush_handlers(live, handlers, base_dir)
                continue
            if "block" in t:
                self._run_block(t, live, base_dir, handlers)
                continue
            if "include_tasks" in t or "include_role" in t or "import_role" in t:
                self._run_include(t, live, base_dir, handlers)
                continue
            self._run_task(t, live, base_dir, handlers)

    def _run_block(self, t, hosts, base_dir, handlers):
        def sub(ts):
            out = []
            for x in ts:
                x = dict(x)
                _inherit(x, t)
                for k in ("_role", "_role_path", "_role_vars", "_role_defaults", "environment", "become"):
                    if k in t and k not in x:
                        x[k] = t[k]
                out.append(x)
            return out

        before = {h: self.state[h].failed for h in hosts}
        seen = {h: set(self.cb.results_raw["failed"].get(h, {})) for h in hosts}
        self._run_tasks(sub(t["block"]), hosts, base_dir, handlers)
        failed_now = [h for h in hosts if self.state[h].failed and not before[h]]
        if failed_now and t.get("rescue"):
            for h in failed_now:
                self.state[h].failed = False
            self._run_tasks(sub(t["rescue"]), failed_now, base_dir, handlers)
            for h in failed_now:
                if not self.state[h].failed:  # rescued: the block's failures do not fail the run
                    self.cb.rescue(h, set(self.cb.results_raw["failed"].get(h, {})) - seen[h])
        if t.get("always"):
            self._run_tasks(sub(t["always"]), hosts, base_dir, handlers)

    def _run_include(self, t, hosts, base_dir, handlers):
        for h in hosts:
            v = self.task_vars(h, t)
            if not self._when(t, v):
                continue
            if "include_tasks" in t:
                base = t.get("_include_base", base_dir)
                path = os.path.join(base, str(render(t["include_tasks"], v)))
                role = Role(t.get("_role", ""), t.get("_role_path", "")) if t.get("_role") else None
                inner = self.loader.expand_tasks(_load_yaml(path) or [], os.path.dirname(path), role)
            else:
                spec = t.get("include_role") or t.get("import_role")
                rn = render(spec["name"] if isinstance(spec, dict) else spec, v)
                role = self.loader.load_role(rn, base_dir)
                tasks = role.tasks
                tf = render(spec.get("tasks_from"), v) if isinstance(spec, dict) and spec.get("tasks_from") else None
                if tf:  # one task file of the role, with the role's defaults / vars (Ansible tasks_from)
                    tp = os.path.join(role.path, "tasks", tf if str(tf).endswith((".yml", ".yaml")) else f"{tf}.yml")
                    tasks = self.loader.expand_tasks(_load_yaml(tp) or [], os.path.dirname(tp), role)
                inner = []
                for x in tasks:
                    x = copy.deepcopy(x)
                    x["_role_defaults"] = role.defaults
                    x["_role_vars"] = role.vars
                    inner.append(x)
                handlers = handlers + role.handlers
            for x in inner:
                _inherit(x, {k: t[k] for k in ("tags", "vars", "become", "environment") if k in t})
                for k in ("_role_vars", "_role_defaults"):
                    if k in t and k not in x:
                        x[k] = t[k]
            self._run_tasks(inner, [h], base_dir, handlers)

    def _tags_ok(self, t) -> bool:
        tg = t.get("tags", []) or []
        tg = (tg if isinstance(tg, list) else [tg]) + t.get("_tags_extra", [])
        tg = set(map(str, tg))
        if "always" in tg:
            return not (self.skip_tags & {"always"})
        if self.tags and not (self.tags & tg or "all" in self.tags):
            return False
        return not (self.skip_tags & tg)

    def _when(self, t, v) -> bool:
        conds = list(t.get("_when_extra", []))
        w = t.get("when")
        if w is not None:
            conds += w if isinstance(w, list) else [w]
        return all(evaluate(c, v) for c in conds)

    def _module_of(self, t) -> tuple[str, dict]:
        if "local_action" in t:
            la = t["local_action"]
            if isinstance(la, str):
                mod, _, rest = la.partition(" ")
                return mod, {"_raw_params": rest, "_local": True}
            la = dict(la)
            return la.pop("module"), {**la, "_local": True}
        for k, val in t.items():
            if k in TASK_KEYWORDS or k.startswith("_"):
                continue
            mod = k.split(".")[-1]  # ansible.builtin.shell -> shell
            if isinstance(val, dict):
                args = dict(val)
            elif val is None:
                args = {}
            else:
                args = _parse_free_form(mod, str(val))
            if isinstance(t.get("args"), dict):
                args.update(t["args"])
            return mod, args
        raise PlaybookError(f"no module in task {t.get('name', t)}")

    def _run_task(self, t, hosts, base_dir, handlers=None):
        if not self._tags_ok(t) and t.get("name") != "Gathering Facts":
            return
        mod, raw_args = self._module_of(t)
        name = t.get("name") or f"{mod} {raw_args.get('_raw_params', '')}".strip()
        if t.get("_role"):
            name = f"{t['_role']} : {name}"
        self.cb.on_task_start(name)
        tsid = self._span(name, "task", module=mod)
        try:
            self._run_task_on(t, hosts, mod, raw_args, name, base_dir, handlers, tsid)
        finally:
            self._span_end(tsid)

    def _run_task_on(self, t, hosts, mod, raw_args, name, base_dir, handlers, tsid):
        if mod not in MODULES:
            for h in hosts:
                res = {"failed": True, "msg": f"module {mod!r} is not supported by the engine"}
                self.cb.gather("failed", h, name, res)
                self.state[h].failed = True
            return
        targets = hosts[:1] if t.get("run_once") else hosts
        results: dict[str, dict] = {}

        def one(h):
            hsid = self.tracer.begin(name, "host", host=h, parent=tsid, module=mod) if self.tracer is not None else None
            try:
                results[h] = self._execute_on(h, t, mod, raw_args, name, base_dir)
            except Unreachable as e:
                results[h] = {"unreachable": True, "msg": str(e), "changed": False}
            except (TemplateError, ModuleError, PlaybookError, KeyError, ValueError, IOError) as e:
                results[h] = {"failed": True, "msg": f"{type(e).__name__}: {e}", "changed": False}
            finally:
                if hsid is not None:
                    r = results.get(h) or {}
                    st = ("unreachable" if r.get("unreachable") else "failed" if r.get("failed") else
                          "skipped" if r.get("skipped") else "changed" if r.get("changed") else "ok")
                    extra = {"rc": r["rc"]} if isinstance(r.get("rc"), int) else {}
                    self.tracer.end(hsid, st, **extra)

        if len(targets) == 1 or self.forks == 1:
            for h in targets:
                one(h)
        else:
            with ThreadPoolExecutor(max_workers=min(self.forks, len(targets))) as ex:
                list(ex.map(one, targets))
        if t.get("run_once") and targets:
            for h in hosts[1:]:
                results[h] = results[targets[0]]
                if t.get("register"):
                    self.state[h].facts[t["register"]] = self.state[targets[0]].facts.get(t["register"])
        for h in hosts:
            res = results.get(h, {"skipped": True})
            self._account(h, name, res, t, handlers)

    def _account(self, h, name, res, t, handlers):
        ignore = _truthy(t.get("ignore_errors", False))
        if res.get("unreachable"):
            if t.get("ignore_unreachable"):
                self.cb.gather("skipped", h, name, res)
                return
            self.state[h].unreachable = True
            self.cb.gather("unreachable", h, name, res)
            self.cb.on_result("fatal", h, res)
        elif res.get("failed"):
            self.cb.gather("failed", h, name, res, ignore=ignore)
            self.cb.on_result("fatal" if not ignore else "failed (ignored)", h, res)
            if not ignore:
                self.state[h].failed = True
        elif res.get("skipped"):
            self.cb.gather("skipped", h, name, res)
            self.cb.on_result("skipping", h, res)
        else:
            self.cb.gather("ok", h, name, res)
            self.cb.on_result("changed" if res.get("changed") else "ok", h, res)
            if res.get("changed") and t.get("notify"):
                n = t["notify"]
                self.state[h].notified.update(n if isinstance(n, list) else [n])

    def _execute_on(self, h, t, mod, raw_args, name, base_dir) -> dict:
        lc = t.get("loop_control", {}) or {}
        loop_var = lc.get("loop_var", "item")
        v0 = self.task_vars(h, t)
        # conditions inherited from a role / import / block do not depend on the loop item: a task skipped by
        # them never templates its loop (which may name a variable only its skipped siblings register)
        if t.get("_when_extra") and not all(evaluate(c, v0) for c in t["_when_extra"]):
            return {"skipped": True, "changed": False, "msg": "Conditional result was False"}
        items = self._loop_items(t, v0)
        if items is None:
            if not self._when(t, v0):
                return {"skipped": True, "changed": False, "msg": "Conditional result was False"}
            res = self._execute_once(h, t, mod, raw_args, v0, base_dir)
        else:
            outs = []
            for it in items:
                v = self.task_vars(h, t, it, loop_var)
                if not self._when(t, v):
                    outs.append({"skipped": True, "changed": False, loop_var: it})
                    continue
                r = self._execute_once(h, t, mod, raw_args, v, base_dir)
                r[loop_var] = it
                outs.append(r)
                if r.get("failed") and not _truthy(t.get("ignore_errors", False)):
                    break
            res = {"results": outs, "changed": any(o.get("changed") for o in outs),
                   "failed": any(o.get("failed") for o in outs),
                   "skipped": bool(outs) and all(o.get("skipped") for o in outs),
                   "msg": "All items completed" if outs else "No items in the list"}
            if not outs:
                res["skipped"] = True
            if t.get("register"):
                self.state[h].facts[t["register"]] = res
        return res

    def _loop_items(self, t, v):
        for key in ("loop", "with_items", "with_list"):
            if key in t:
                items = render(t[key], v)
                if isinstance(items, str):
                    items = [items]
                if key == "with_items":
                    flat = []
                    for x in items or []:
                        flat.extend(x if isinstance(x, list) else [x])
                    items = flat
                return list(items or [])
        if "with_nested" in t:  # cartesian product of the listed lists
            import itertools

            lists = [x if isinstance(x, list) else [x] for x in (render(t["with_nested"], v) or [])]
            return [list(p) for p in itertools.product(*lists)] if lists else []
        if "with_dict" in t:
            d = render(t["with_dict"], v) or {}
            return [{"key": k, "value": val} for k, val in d.items()]
        if "with_sequence" in t:
            spec = render(t["with_sequence"], v)
            kv = dict(p.split("=") for p in str(spec).split()) if "=" in str(spec) else {"end": spec}
            start, end, stride = int(kv.get("start", 1)), int(kv.get("end", kv.get("count", 0))), int(kv.get("stride", 1))
            fmt = kv.get("format", "%d")
            return [fmt % i for i in range(start, end + 1, stride)]
        return None

    def _execute_once(self, h, t, mod, raw_args, v, base_dir) -> dict:
        args = render(raw_args, v)
        args = {k: val for k, val in args.items() if val != "__omit_place_holder__"}
        local = args.pop("_local", False)
        exec_host = h
        if t.get("delegate_to"):
            exec_host = str(render(t["delegate_to"], v))
        if local or exec_host in ("localhost", "127.0.0.1"):
            conn = HostConn(name="localhost", address="127.0.0.1", user=self.default_user)
            transport = self.transport if isinstance(self.transport, FakeTransport) else _local_transport()
        else:
            if exec_host not in self.inventory.hosts:
                self.inventory.add_host(exec_host)
                self.state.setdefault(exec_host, HostState())
            conn = self._conn(exec_host, v)
            transport = self.transport
            if self.base_vars(exec_host).get("ansible_connection") == "local" and not isinstance(transport, FakeTransport):
                transport = _local_transport()
        if _truthy(t.get("become", v.get("ansible_become", False))):
            conn.become = True
        env = render(t.get("environment") or {}, v)
        search = []
        if t.get("_role_path"):
            search.append(t["_role_path"])
        search.append(base_dir)
        ctx = ModuleContext(transport, conn, h, v, search, {}, self.check or _truthy(t.get("check_mode", False)),
                            env if isinstance(env, dict) else {}, self.controller_dir)
        retries = int(render(t.get("retries", 3), v)) if "until" in t else 1
        delay = float(render(t.get("delay", 5), v)) if "until" in t else 0
        attempt = 0
        while True:
            attempt += 1
            res = MODULES[mod](ctx, args)
            res.setdefault("changed", False)
            res.setdefault("failed", False)
            if ctx.facts_out:
                self.state[h].facts.update(ctx.facts_out)
                ctx.facts_out = {}
            vv = dict(v)
            if t.get("register"):
                vv[t["register"]] = res
            if "changed_when" in t:
                res["changed"] = evaluate(t["changed_when"], vv)
            if "failed_when" in t:
                res["failed"] = evaluate(t["failed_when"], vv)
            if t.get("register"):
                self.state[h].facts[t["register"]] = res
                vv[t["register"]] = res
            if "until" not in t:
                break
            ok = evaluate(t["until"], vv)
            if ok:
                # as Ansible: the until condition ends the retries; the result still fails if the module failed
                # (a non-zero rc) and no failed_when overrides that -- a met condition never hides a failing command
                break
            if attempt >= max(1, retries):
                res["failed"] = True
                res["msg"] = res.get("msg") or f"until condition not met after {attempt} attempts"
                break
            if not isinstance(self.transport, FakeTransport):
                time.sleep(delay)
        res["attempts"] = attempt
        if t.get("no_log"):
            res = {k: ("********" if k in ("stdout", "stderr", "cmd", "stdout_lines") else val) for k, val in res.items()}
        return res

    def _flush_handlers(self, hosts, handlers, base_dir):
        for hd in handlers:
            names = {hd.get("name")} | set((hd.get("listen") if isinstance(hd.get("listen"), list)
                                           else [hd.get("listen")]) if hd.get("listen") else [])
            hs = [h for h in self._live(hosts) if self.state[h].notified & names]
            if hs:
                self._run_task(hd, hs, base_dir)
        for h in hosts:
            self.state[h].notified.clear()

    # ------------------------------------------------------------------------------------ ad-hoc
    def run_adhoc(self, pattern: str, module: str, args=None, name: str | None = None) -> dict:
        """Single module on matching hosts (reference AdHocRunner.run, ansible/runner.py:169-215)."""
        hosts = self.inventory.match(pattern)
        t = {"name": name or f"{module}", module: args if args is not None else {}}
        self._play_vars, self._play_hosts, self._batch = {}, hosts, hosts
        self.cb.on_playbook_start(t["name"])
        self._run_task(t, hosts, self.controller_dir)
        self.cb.on_playbook_end(t["name"])
        return self.cb.results


def _truthy(v) -> bool:
    return str(v).strip().lower() in ("1", "yes", "true", "on", "y")


_LOCAL = None


def _local_transport():
    global _LOCAL
    if _LOCAL is None:
        from .transport import LocalTransport

        _LOCAL = LocalTransport()
    return _LOCAL


def _split_top_level(s: str) -> list[str]:
    """Split on whitespace outside quotes and outside Jinja ``{{ }}`` / ``{% %}``."""
    out, cur, depth, quote = [], [], 0, ""
    i = 0
    while i < len(s):
        ch = s[i]
        two = s[i:i + 2]
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = ""
        elif two in ("{{", "{%"):
            depth += 1
            cur.append(two)
            i += 2
            continue
        elif two in ("}}", "%}") and depth:
            depth -= 1
            cur.append(two)
            i += 2
            continue
        elif ch in "'\"" and depth == 0:
            quote = ch
            cur.append(ch)
        elif ch.isspace() and depth == 0:
            if cur:
                out.append("".join(cur))
                cur = []
        else:
            cur.append(ch)
        i += 1
    if cur:
        out.append("".join(cur))
    return out


def _parse_free_form(mod: str, s: str) -> dict:
    """``shell: echo hi`` -> {_raw_params}; ``copy: src=a dest=b`` -> {src, dest}."""
    if mod in ("shell", "command", "raw", "script", "include_vars", "meta"):
        # command modules accept trailing k=v options like chdir= / creates=
        args = {}
        toks = s.split(" ")
        keep = []
        for tok in toks:
            k, eq, val = tok.partition("=")
            if eq and k in ("chdir", "creates", "removes", "executable", "warn"):
                args[k] = val
            else:
                keep.append(tok)
        args["_raw_params"] = " ".join(keep)
        return args
    parts = _split_top_level(s)
    if parts and all(re.match(r"^[A-Za-z_][\w\-]*=", p) for p in parts):
        out = {}
        for p in parts:
            k, v = p.split("=", 1)
            if len(v) >= 2 and v[0] == v[-1] and v[0] in "'\"":
                v = v[1:-1]
            out[k] = v
        return out
    if mod == "debug":
        return {"msg": s}
    return {"_raw_params": s}
