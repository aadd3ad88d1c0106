"""Task modules of the execution engine (the subset of Ansible modules the provisioning roles use).

Every module runs on the controller and acts on the target through a :class:`Transport` (shell command,
file put / get), returning an Ansible-shaped result dict: ``changed``, ``failed``, ``msg``, and for command
modules ``rc``, ``stdout``, ``stderr``, ``stdout_lines``, ``cmd``, ``delta`` (the fields the reference's
callback keeps, ansible_api/ansible/callback.py:60-80). File-editing modules (lineinfile, replace,
blockinfile, sysctl) read the file, edit it on the controller, and write it back only when it changed, so
re-runs are idempotent and report ``changed: false``.
"""
from __future__ import annotations

import base64
import json
import os
import re
import shlex
import time
from dataclasses import dataclass, field

from . import filecheck
from .templating import render_text
from .transport import CmdResult, FakeTransport, HostConn, Transport


class ModuleError(Exception):
    pass


@dataclass
class ModuleContext:
    transport: Transport
    conn: HostConn
    host: str
    variables: dict
    search_paths: list = field(default_factory=list)  # role dirs + playbook dir, most specific first
    facts_out: dict = field(default_factory=dict)  # set_fact / setup results to merge into host facts
    check_mode: bool = False
    env: dict = field(default_factory=dict)
    controller_dir: str = ""  # where fetch writes

    def run(self, cmd: str, timeout: float = 3600, stdin: str | None = None) -> CmdResult:
        return self.transport.run(self.conn, cmd, timeout=timeout, env=self.env or None, stdin=stdin)

    def find(self, name: str, kind: str) -> str:
        """Locate a role/playbook file (``files`` / ``templates``) on the controller."""
        if os.path.isabs(name) and os.path.exists(name):
            return name
        for base in self.search_paths:
            for cand in (os.path.join(base, kind, name), os.path.join(base, name)):
                if os.path.exists(cand):
                    return cand
        raise ModuleError(f"could not find {kind} file {name!r} in {self.search_paths}")


def _cmd_result(r: CmdResult, cmd: str, changed=True) -> dict:
    return {"changed": changed, "failed": r.rc != 0, "rc": r.rc, "stdout": r.stdout.rstrip("\n"),
            "stderr": r.stderr.rstrip("\n"), "stdout_lines": r.stdout.splitlines(),
            "stderr_lines": r.stderr.splitlines(), "cmd": cmd, "delta": f"{r.delta:.3f}",
            "msg": "" if r.rc == 0 else "non-zero return code"}


# ------------------------------------------------------------------------------------------- commands
def m_command(ctx: ModuleContext, a: dict) -> dict:
    cmd = a.get("_raw_params") or a.get("cmd") or ""
    if isinstance(a.get("argv"), list):
        cmd = " ".join(shlex.quote(str(x)) for x in a["argv"])
    creates, removes = a.get("creates"), a.get("removes")
    if creates and ctx.run(f"test -e {shlex.quote(str(creates))}").rc == 0:
        return {"changed": False, "rc": 0, "stdout": f"skipped, since {creates} exists", "stdout_lines": [],
                "stderr": "", "cmd": cmd}
    if removes and ctx.run(f"test -e {shlex.quote(str(removes))}").rc != 0:
        return {"changed": False, "rc": 0, "stdout": f"skipped, since {removes} does not exist",
                "stdout_lines": [], "stderr": "", "cmd": cmd}
    if a.get("chdir"):
        cmd = f"cd {shlex.quote(str(a['chdir']))} && {cmd}"
    if ctx.check_mode:
        return {"changed": True, "rc": 0, "stdout": "", "stdout_lines": [], "stderr": "", "cmd": cmd}
    return _cmd_result(ctx.run(cmd, stdin=a.get("stdin")), cmd)


def m_pause(ctx, a):
    secs = float(a.get("seconds", 0)) + 60 * float(a.get("minutes", 0))
    if not isinstance(ctx.transport, FakeTransport):
        time.sleep(secs)
    return {"changed": False, "msg": f"paused {secs}s"}


# ------------------------------------------------------------------------------------------- files
def _chmod_chown(ctx, path: str, a: dict) -> None:
    q = shlex.quote(path)
    if a.get("mode") is not None:
        mode = a["mode"]
        mode = format(mode, "o") if isinstance(mode, int) else str(mode)
        ctx.run(f"chmod {mode} {q}")
    if a.get("owner") or a.get("group"):
        ctx.run(f"chown {a.get('owner', '')}{':' + a['group'] if a.get('group') else ''} {q}")


def _read_remote(ctx, path: str) -> bytes | None:
    try:
        return ctx.transport.get(ctx.conn, path)
    except (IOError, OSError):
        return None


def _write_if_changed(ctx, path: str, data: bytes, a: dict, backup=False) -> bool:
    old = _read_remote(ctx, path)
    if old == data:
        _chmod_chown(ctx, path, a)
        return False
    if ctx.check_mode:
        return True
    if backup and old is not None:
        ctx.transport.put(ctx.conn, old, path + time.strftime(".%Y%m%d%H%M%S.bak"))
    ctx.transport.put(ctx.conn, data, path)
    _chmod_chown(ctx, path, a)
    return True


def m_copy(ctx: ModuleContext, a: dict) -> dict:
    dest = str(a["dest"])
    if "content" in a:
        data = a["content"] if isinstance(a["content"], bytes) else str(a["content"]).encode()
        if dest.endswith("/"):
            raise ModuleError("copy with content needs a file dest")
        _check_rendered(dest, data, a)
        return {"changed": _write_if_changed(ctx, dest, data, a, a.get("backup", False)), "dest": dest}
    src = str(a["src"])
    if a.get("remote_src"):
        r = ctx.run(f"cp -a {shlex.quote(src)} {shlex.quote(dest)}")
        return _cmd_result(r, "cp", changed=True)
    local = ctx.find(src, "files")
    changed = False
    if os.path.isdir(local):
        base = dest if src.endswith("/") else os.path.join(dest, os.path.basename(local.rstrip("/")))
        for root, _dirs, files in os.walk(local):
            for fn in files:
                lp = os.path.join(root, fn)
                rp = os.path.join(base, os.path.relpath(lp, local))
                with open(lp, "rb") as f:
                    changed |= _write_if_changed(ctx, rp, f.read(), a)
        return {"changed": changed, "dest": base}
    if dest.endswith("/"):
        dest = os.path.join(dest, os.path.basename(local))
    with open(local, "rb") as f:
        data = f.read()
    return {"changed": _write_if_changed(ctx, dest, data, a, a.get("backup", False)), "dest": dest}


def m_template(ctx: ModuleContext, a: dict) -> dict:
    local = ctx.find(str(a["src"]), "templates")
    with open(local) as f:
        text = render_text(f.read(), ctx.variables)
    dest = str(a["dest"])
    if dest.endswith("/"):
        dest = os.path.join(dest, os.path.basename(local)[:-3] if local.endswith(".j2") else os.path.basename(local))
    _check_rendered(dest, text.encode(), a)
    return {"changed": _write_if_changed(ctx, dest, text.encode(), a, a.get("backup", False)), "dest": dest}


def _check_rendered(dest: str, data: bytes, a: dict) -> None:
    """Parse a rendered file by type before it leaves the control node (engine/filecheck.py)."""
    if a.get("validate", True) is False:
        return
    try:
        filecheck.check(dest, data)
    except filecheck.FileCheckError as e:
        raise ModuleError(f"rendered file does not parse: {e}") from None


def m_file(ctx: ModuleContext, a: dict) -> dict:
    path = str(a.get("path") or a.get("dest") or a.get("name"))
    state = a.get("state", "file")
    q = shlex.quote(path)
    if state == "absent":
        exists = ctx.run(f"test -e {q} -o -L {q}").rc == 0
        if exists and not ctx.check_mode:
            ctx.run(f"rm -rf {q}")
        return {"changed": exists, "path": path}
    if state == "directory":
        exists = ctx.run(f"test -d {q}").rc == 0
        if not exists and not ctx.check_mode:
            r = ctx.run(f"mkdir -p {q}")
            if r.rc != 0:
                return _cmd_result(r, "mkdir")
        if a.get("recurse") and a.get("mode") is not None:
            m = a["mode"]
            ctx.run(f"chmod -R {format(m, 'o') if isinstance(m, int) else m} {q}")
        else:
            _chmod_chown(ctx, path, a)
        return {"changed": not exists, "path": path}
    if state == "touch":
        ctx.run(f"mkdir -p $(dirname {q}) && touch {q}")
        _chmod_chown(ctx, path, a)
        return {"changed": True, "path": path}
    if state in ("link", "hard"):
        src = shlex.quote(str(a["src"]))
        cur = ctx.run(f"readlink {q}").stdout.strip()
        if cur == str(a["src"]):
            return {"changed": False, "path": path}
        ctx.run(f"ln -{'s' if state == 'link' else ''}fn {src} {q}")
        return {"changed": True, "path": path}
    # state == file: must exist
    if ctx.run(f"test -e {q}").rc != 0:
        return {"changed": False, "failed": True, "msg": f"file {path} is absent, cannot continue"}
    _chmod_chown(ctx, path, a)
    return {"changed": False, "path": path}


def m_lineinfile(ctx: ModuleContext, a: dict) -> dict:
    path = str(a.get("path") or a.get("dest") or a.get("name"))
    old = _read_remote(ctx, path)
    if old is None:
        if not a.get("create", False) and a.get("state", "present") == "present":
            return {"failed": True, "changed": False, "msg": f"Destination {path} does not exist !", "rc": 257}
        old = b""
    lines = old.decode(errors="replace").splitlines()
    state = a.get("state", "present")
    rx = re.compile(a["regexp"]) if a.get("regexp") else None
    line = str(a.get("line", ""))
    new = list(lines)
    if state == "absent":
        new = [l for l in lines if not ((rx and rx.search(l)) or (not rx and l == line))]
    else:
        idx = [i for i, l in enumerate(lines) if (rx and rx.search(l)) or l == line]
        if idx:
            i = idx[-1]
            if a.get("backrefs") and rx:
                new[i] = rx.sub(line, lines[i])
            else:
                new[i] = line
        elif not a.get("backrefs"):
            ia, ib = a.get("insertafter"), a.get("insertbefore")
            if ib == "BOF":
                new.insert(0, line)
            elif ib:
                pos = [i for i, l in enumerate(lines) if re.search(ib, l)]
                new.insert(pos[-1] if pos else len(new), line)
            elif ia and ia != "EOF":
                pos = [i for i, l in enumerate(lines) if re.search(ia, l)]
                new.insert(pos[-1] + 1 if pos else len(new), line)
            else:
                new.append(line)
    data = ("\n".join(new) + ("\n" if new else "")).encode()
    if data == old:
        return {"changed": False, "msg": ""}
    return {"changed": _write_if_changed(ctx, path, data, a, a.get("backup", False)), "msg": "line changed"}


def m_replace(ctx: ModuleContext, a: dict) -> dict:
    path = str(a.get("path") or a.get("dest"))
    old = _read_remote(ctx, path)
    if old is None:
        return {"failed": True, "changed": False, "msg": f"Path {path} does not exist !"}
    text = old.decode(errors="replace")
    new = re.sub(a["regexp"], a.get("replace", ""), text, flags=re.M)
    if new == text:
        return {"changed": False, "msg": ""}
    return {"changed": _write_if_changed(ctx, path, new.encode(), a, a.get("backup", False)), "msg": "replaced"}


def m_blockinfile(ctx: ModuleContext, a: dict) -> dict:
    path = str(a.get("path") or a.get("dest"))
    marker = a.get("marker", "# {mark} KUBEOPERATOR MANAGED BLOCK")
    begin, end = marker.replace("{mark}", "BEGIN"), marker.replace("{mark}", "END")
    old = (_read_remote(ctx, path) or b"").decode(errors="replace")
    block = str(a.get("block", "")).rstrip("\n")
    pat = re.compile(re.escape(begin) + r".*?" + re.escape(end) + r"\n?", re.S)
    body = f"{begin}\n{block}\n{end}\n" if a.get("state", "present") == "present" else ""
    new = pat.sub(body, old) if pat.search(old) else (old + ("" if old.endswith("\n") or not old else "\n") + body)
    if new == old:
        return {"changed": False}
    return {"changed": _write_if_changed(ctx, path, new.encode(), a)}


def m_stat(ctx: ModuleContext, a: dict) -> dict:
    q = shlex.quote(str(a["path"]))
    r = ctx.run(f"stat -c '%F|%s|%a|%U|%Y' {q} 2>/dev/null")
    if r.rc != 0 or not r.stdout.strip():
        return {"changed": False, "stat": {"exists": False}}
    kind, size, mode, owner, mtime = (r.stdout.strip().split("|") + ["", "", "", "", ""])[:5]
    return {"changed": False, "stat": {"exists": True, "isdir": "directory" in kind, "isreg": "regular" in kind,
                                       "islnk": "link" in kind, "size": int(size or 0), "mode": "0" + mode,
                                       "pw_name": owner, "mtime": float(mtime or 0), "path": a["path"]}}


def m_slurp(ctx, a):
    data = ctx.transport.get(ctx.conn, str(a["src"]))
    return {"changed": False, "content": base64.b64encode(data).decode(), "encoding": "base64"}


def m_fetch(ctx: ModuleContext, a: dict) -> dict:
    src = str(a["src"])
    data = ctx.transport.get(ctx.conn, src)
    dest = str(a["dest"])
    if a.get("flat"):
        out = dest if not dest.endswith("/") else os.path.join(dest, os.path.basename(src))
    else:
        out = os.path.join(dest, ctx.host, src.lstrip("/"))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "wb") as f:
        f.write(data)
    return {"changed": True, "dest": out, "size": len(data)}


def m_unarchive(ctx: ModuleContext, a: dict) -> dict:
    dest = str(a["dest"])
    src = str(a["src"])
    if a.get("remote_src") or a.get("copy") is False:
        remote = src
    else:
        local = ctx.find(src, "files")
        remote = f"/tmp/.kop-{os.path.basename(local)}"
        with open(local, "rb") as f:
            ctx.transport.put(ctx.conn, f.read(), remote)
    creates = a.get("creates")
    if creates and ctx.run(f"test -e {shlex.quote(str(creates))}").rc == 0:
        return {"changed": False}
    extra = " ".join(a.get("extra_opts", []) or [])
    cmd = (f"mkdir -p {shlex.quote(dest)} && " +
           (f"unzip -o {shlex.quote(remote)} -d {shlex.quote(dest)}" if remote.endswith(".zip")
            else f"tar -xf {shlex.quote(remote)} -C {shlex.quote(dest)} {extra}"))
    return _cmd_result(ctx.run(cmd), cmd)


def m_get_url(ctx: ModuleContext, a: dict) -> dict:
    dest, url = str(a["dest"]), str(a["url"])
    if not a.get("force") and ctx.run(f"test -s {shlex.quote(dest)}").rc == 0 and not dest.endswith("/"):
        return {"changed": False, "dest": dest}
    cmd = f"curl -fsSL --retry 3 {'-k ' if not a.get('validate_certs', True) else ''}-o {shlex.quote(dest)} {shlex.quote(url)}"
    res = _cmd_result(ctx.run(cmd), cmd)
    if res["rc"] == 0 and a.get("mode") is not None:
        _chmod_chown(ctx, dest, a)
    return res


def m_synchronize(ctx, a):
    return m_copy(ctx, {"src": a["src"], "dest": a["dest"], "mode": a.get("mode")})


# ------------------------------------------------------------------------------------------- system
def m_service(ctx: ModuleContext, a: dict) -> dict:
    name = str(a["name"])
    cmds = []
    if a.get("daemon_reload") or a.get("daemon-reload"):
        cmds.append("systemctl daemon-reload")
    en = a.get("enabled")
    if en is not None:
        cmds.append(f"systemctl {'enable' if _truthy(en) else 'disable'} {shlex.quote(name)}")
    st = a.get("state")
    if st:
        verb = {"started": "start", "stopped": "stop", "restarted": "restart", "reloaded": "reload"}[st]
        if st == "started" and ctx.run(f"systemctl is-active --quiet {shlex.quote(name)}").rc == 0 and not cmds:
            return {"changed": False, "name": name, "state": st}
        cmds.append(f"systemctl {verb} {shlex.quote(name)}")
    if not cmds:
        return {"changed": False, "name": name}
    cmd = " && ".join(cmds)
    return {**_cmd_result(ctx.run(cmd), cmd), "name": name}


def _truthy(v):
    return str(v).lower() in ("1", "yes", "true", "on")


def m_package(ctx: ModuleContext, a: dict) -> dict:
    names = a.get("name") or a.get("pkg") or []
    if isinstance(names, str):
        names = [n.strip() for n in names.split(",") if n.strip()]
    state = a.get("state", "present")
    pk = " ".join(shlex.quote(str(n)) for n in names)
    if not pk:
        return {"changed": False}
    if state in ("absent", "removed"):
        cmd = (f"if command -v apt-get >/dev/null; then DEBIAN_FRONTEND=noninteractive apt-get remove -y {pk}; "
               f"elif command -v dnf >/dev/null; then dnf remove -y {pk}; else yum remove -y {pk}; fi")
    else:
        upd = "apt-get update -qq; " if a.get("update_cache") else ""
        opt = " ".join(a.get("install_options", []) or [])
        cmd = (f"if command -v apt-get >/dev/null; then {upd}DEBIAN_FRONTEND=noninteractive apt-get install -y "
               f"--no-install-recommends {opt} {pk}; elif command -v dnf >/dev/null; then dnf install -y {opt} {pk}; "
               f"else yum install -y {opt} {pk}; fi")
    return _cmd_result(ctx.run(cmd, timeout=7200), cmd)


def m_modprobe(ctx, a):
    name = shlex.quote(str(a["name"]))
    cmd = f"modprobe -r {name}" if a.get("state") == "absent" else f"modprobe {name} {a.get('params', '')}"
    return _cmd_result(ctx.run(cmd), cmd)


def m_sysctl(ctx: ModuleContext, a: dict) -> dict:
    name, value = str(a["name"]), str(a.get("value", ""))
    f = str(a.get("sysctl_file", "/etc/sysctl.d/99-kubeoperator.conf"))
    changed = m_lineinfile(ctx, {"path": f, "regexp": r"^\s*" + re.escape(name) + r"\s*=", "line": f"{name} = {value}",
                                 "create": True, "state": a.get("state", "present")})["changed"]
    if a.get("reload", True) and a.get("state", "present") == "present":
        ctx.run(f"sysctl -w {shlex.quote(name)}={shlex.quote(value)}")
    return {"changed": changed}


def m_hostname(ctx, a):
    n = shlex.quote(str(a["name"]))
    cur = ctx.run("hostname").stdout.strip()
    if cur == str(a["name"]):
        return {"changed": False}
    cmd = f"hostnamectl set-hostname {n} 2>/dev/null || hostname {n}"
    return _cmd_result(ctx.run(cmd), cmd)


def m_authorized_key(ctx: ModuleContext, a: dict) -> dict:
    user = str(a.get("user", "root"))
    key = str(a["key"]).strip()
    home = "/root" if user == "root" else f"/home/{user}"
    path = f"{home}/.ssh/authorized_keys"
    old = (_read_remote(ctx, path) or b"").decode()
    if key in old.splitlines():
        return {"changed": False}
    new = old + ("" if old.endswith("\n") or not old else "\n") + key + "\n"
    ctx.run(f"mkdir -p {home}/.ssh && chmod 700 {home}/.ssh")
    return {"changed": _write_if_changed(ctx, path, new.encode(), {"mode": 0o600})}


def m_wait_for(ctx: ModuleContext, a: dict) -> dict:
    timeout = int(a.get("timeout", 300))
    delay = int(a.get("delay", 0))
    host = a.get("host", "127.0.0.1")
    if "port" in a:
        probe = f"(echo > /dev/tcp/{host}/{int(a['port'])}) >/dev/null 2>&1"
        if a.get("state") in ("stopped", "absent"):
            probe = "! " + probe
    elif "path" in a:
        probe = f"test -e {shlex.quote(str(a['path']))}"
        if a.get("search_regex"):
            probe += f" && grep -qE {shlex.quote(a['search_regex'])} {shlex.quote(str(a['path']))}"
    else:
        probe = "true"
    cmd = f"sleep {delay}; for i in $(seq 1 {max(1, timeout)}); do if {probe}; then exit 0; fi; sleep 1; done; exit 1"
    if isinstance(ctx.transport, FakeTransport):
        cmd = f"wait_for {probe}"
    r = ctx.run(cmd, timeout=timeout + delay + 30)
    out = _cmd_result(r, cmd, changed=False)
    if r.rc != 0:
        out["msg"] = f"Timeout when waiting for {a}"
    return out


BOOT_ID = "cat /proc/sys/kernel/random/boot_id"


def m_reboot(ctx: ModuleContext, a: dict) -> dict:
    """Reboot the host and wait until it is back (Ansible ``reboot``): the boot id before, a detached
    ``systemctl reboot`` (so the command returns before the connection drops), then the boot id polled until
    it changes or ``reboot_timeout`` runs out; an unreachable host while it restarts is expected."""
    from .transport import Unreachable

    timeout = float(a.get("reboot_timeout", 600))
    fake = isinstance(ctx.transport, FakeTransport)
    poll = 0.0 if fake else float(a.get("poll_interval", 5))
    t0 = time.time()
    before = ctx.run(BOOT_ID).stdout.strip()
    cmd = str(a.get("reboot_command", "systemctl reboot"))
    ctx.run(f"nohup sh -c 'sleep 2; {cmd}' >/dev/null 2>&1 &")
    if not fake:
        time.sleep(float(a.get("pre_reboot_delay", 0)) + 5)
    tries = 0
    while time.time() - t0 < timeout and (not fake or tries < 50):
        tries += 1
        try:
            r = ctx.run(BOOT_ID, timeout=30)
        except (Unreachable, OSError, TimeoutError):
            time.sleep(poll)
            continue
        now = r.stdout.strip()
        if r.rc == 0 and now and now != before:
            if not fake:
                time.sleep(float(a.get("post_reboot_delay", 0)))
            return {"changed": True, "rebooted": True, "elapsed": round(time.time() - t0, 1)}
        time.sleep(poll)
    return {"changed": True, "failed": True, "rebooted": False,
            "msg": f"host did not come back within {timeout:.0f} s (boot id unchanged)"}


_FACTS_PROBE = r"""
echo "hostname=$(hostname -s 2>/dev/null || hostname)"
echo "fqdn=$(hostname -f 2>/dev/null || hostname)"
. /etc/os-release 2>/dev/null; echo "distribution=${NAME%% *}"; echo "distribution_version=${VERSION_ID}"; echo "os_family=${ID_LIKE:-$ID}"
echo "kernel=$(uname -r)"; echo "architecture=$(uname -m)"
echo "memtotal_mb=$(( $(awk '/MemTotal/{print $2}' /proc/meminfo) / 1024 ))"
echo "processor_vcpus=$(nproc 2>/dev/null || grep -c ^processor /proc/cpuinfo)"
echo "processor_cores=$(lscpu 2>/dev/null | awk -F: '/^Core\(s\) per socket/{c=$2}/^Socket\(s\)/{s=$2}END{print c*s}')"
echo "default_ipv4=$(ip -4 route get 1.1.1.1 2>/dev/null | awk '{for(i=1;i<=NF;i++) if($i=="src") print $(i+1)}')"
for d in $(lsblk -dn -o NAME,TYPE 2>/dev/null | awk '$2=="disk"{print $1}'); do echo "device_$d=$(lsblk -dn -b -o SIZE /dev/$d)"; done
"""


def m_setup(ctx: ModuleContext, a: dict) -> dict:
    r = ctx.run(_FACTS_PROBE)
    kv = {}
    for line in r.stdout.splitlines():
        if "=" in line:
            k, v = line.split("=", 1)
            kv[k.strip()] = v.strip()
    if isinstance(ctx.transport, FakeTransport) and not kv:
        kv = ctx.transport.facts.get(ctx.host) or {
            "hostname": ctx.host.split(".")[0], "fqdn": ctx.host, "distribution": "Ubuntu",
            "distribution_version": "22.04", "os_family": "debian", "kernel": "5.15.0", "architecture": "x86_64",
            "memtotal_mb": "524288", "processor_vcpus": "128", "processor_cores": "64",
            "default_ipv4": ctx.conn.address, "device_nvme0n1": str(3840 * 1024 ** 3)}
    def _int(x, d=0):
        try:
            return int(float(x))
        except (TypeError, ValueError):
            return d
    ver = kv.get("distribution_version", "")
    facts = {
        "ansible_hostname": kv.get("hostname", ctx.host), "ansible_nodename": kv.get("hostname", ctx.host),
        "ansible_fqdn": kv.get("fqdn", ctx.host), "ansible_distribution": kv.get("distribution", ""),
        "ansible_distribution_version": ver, "ansible_distribution_major_version": ver.split(".")[0] if ver else "",
        "ansible_os_family": kv.get("os_family", ""), "ansible_kernel": kv.get("kernel", ""),
        "ansible_architecture": kv.get("architecture", ""), "ansible_memtotal_mb": _int(kv.get("memtotal_mb")),
        "ansible_processor_vcpus": _int(kv.get("processor_vcpus")),
        "ansible_processor_cores": _int(kv.get("processor_cores")),
        "ansible_default_ipv4": {"address": kv.get("default_ipv4") or ctx.conn.address},
        "ansible_devices": {k[7:]: {"size": _int(v)} for k, v in kv.items() if k.startswith("device_")},
    }
    ctx.facts_out.update(facts)
    ctx.facts_out["ansible_facts"] = {k[len("ansible_"):]: v for k, v in facts.items()}
    return {"changed": False, "ansible_facts": facts, "failed": r.rc != 0 and not kv}


# ------------------------------------------------------------------------------------------- control
def m_set_fact(ctx: ModuleContext, a: dict) -> dict:
    facts = {k: v for k, v in a.items() if k != "cacheable"}
    ctx.facts_out.update(facts)
    return {"changed": False, "ansible_facts": facts}


def m_debug(ctx: ModuleContext, a: dict) -> dict:
    if "var" in a:
        from .templating import render

        try:
            val = render("{{ " + str(a["var"]) + " }}", ctx.variables)
        except Exception as e:  # noqa: BLE001
            val = f"VARIABLE IS NOT DEFINED! ({e})"
        return {"changed": False, str(a["var"]): val, "msg": json.dumps(val, default=str)}
    return {"changed": False, "msg": a.get("msg", "Hello world!")}


def m_fail(ctx, a):
    return {"changed": False, "failed": True, "msg": a.get("msg", "Failed as requested from task")}


def m_assert(ctx: ModuleContext, a: dict) -> dict:
    from .templating import evaluate

    that = a.get("that", [])
    that = that if isinstance(that, list) else [that]
    for cond in that:
        if not evaluate(cond, ctx.variables):
            return {"changed": False, "failed": True, "assertion": cond,
                    "msg": a.get("fail_msg") or a.get("msg") or f"Assertion failed: {cond}"}
    return {"changed": False, "msg": a.get("success_msg", "All assertions passed")}


def m_include_vars(ctx: ModuleContext, a: dict) -> dict:
    import yaml

    path = ctx.find(str(a.get("file") or a.get("_raw_params")), "vars")
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    ctx.facts_out.update(data)
    return {"changed": False, "ansible_facts": data}


def m_meta(ctx, a):
    return {"changed": False, "msg": f"meta {a.get('_raw_params', '')}"}


MODULES = {
    "command": m_command, "shell": m_command, "raw": m_command, "script": m_command,
    "copy": m_copy, "template": m_template, "file": m_file, "lineinfile": m_lineinfile, "replace": m_replace,
    "blockinfile": m_blockinfile, "stat": m_stat, "slurp": m_slurp, "fetch": m_fetch, "unarchive": m_unarchive,
    "get_url": m_get_url, "synchronize": m_synchronize,
    "service": m_service, "systemd": m_service, "package": m_package, "yum": m_package, "apt": m_package,
    "dnf": m_package, "modprobe": m_modprobe, "sysctl": m_sysctl, "hostname": m_hostname,
    "authorized_key": m_authorized_key, "wait_for": m_wait_for, "reboot": m_reboot, "setup": m_setup, "gather_facts": m_setup,
    "set_fact": m_set_fact, "debug": m_debug, "fail": m_fail, "assert": m_assert, "include_vars": m_include_vars,
    "meta": m_meta, "pause": m_pause, "ping": lambda ctx, a: {"changed": False, "ping": "pong"},
}


def module_names() -> list[str]:
    """Module catalogue (reference ansible_api/ansible/modules.py)."""
    return sorted(MODULES)
