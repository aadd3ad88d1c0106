"""Host transports of the execution engine: how a task's command / file reaches a machine.

* ``SSHTransport`` -- OpenSSH client subprocess with connection multiplexing (ControlMaster/ControlPersist,
  one TCP+auth handshake per host per run instead of one per task), key auth, or password auth through an
  SSH_ASKPASS helper (no sshpass / paramiko needed). Replaces paramiko + Ansible's ssh plugin
  (common/ssh.py:13-70, ansible_api/ansible/runner.py:32-81).
* ``LocalTransport`` -- run on the controller itself (Ansible ``connection: local``; the reference uses it
  for the ``localhost`` node, models/cluster.py:308-315). An optional ``root`` re-bases every absolute
  path into a sandbox directory so plumbing tests never touch the real filesystem.
* ``FakeTransport`` -- a scripted host farm for CI: every command is recorded, answered by the first
  matching rule (regex -> rc/stdout/stderr or callable), files live in an in-memory filesystem per host,
  and faults can be injected (unreachable hosts, failing commands, nth-call failures, latency).

Every command runs under ``bash -o pipefail`` (``SHELL``): a pipeline such as ``kubeadm init ... | tail`` fails
when ``kubeadm`` fails instead of reporting ``tail``'s status -- Ansible's ``shell`` module (``/bin/sh -c``)
masks those failures, and the provisioning roles are written for the stricter shell.
"""
from __future__ import annotations

import os
import re
import shlex
import stat
import subprocess
import tempfile
import threading
import time
from dataclasses import dataclass, field


SHELL = ["/bin/bash", "-o", "pipefail", "-c"]
SHELL_STR = "/bin/bash -o pipefail -c "


class Unreachable(Exception):
    pass


@dataclass
class CmdResult:
    rc: int
    stdout: str = ""
    stderr: str = ""
    delta: float = 0.0


@dataclass
class HostConn:
    name: str
    address: str
    port: int = 22
    user: str = "root"
    password: str = ""
    private_key: str = ""  # key material or a path
    become: bool = False
    extra: dict = field(default_factory=dict)


class Transport:
    name = "base"

    def run(self, conn: HostConn, cmd: str, timeout: float = 3600, env: dict | None = None,
            stdin: str | None = None) -> CmdResult:
        raise NotImplementedError

    def put(self, conn: HostConn, data: bytes, dest: str, mode: int | None = None) -> None:
        raise NotImplementedError

    def get(self, conn: HostConn, src: str) -> bytes:
        raise NotImplementedError

    def ping(self, conn: HostConn) -> bool:
        try:
            return self.run(conn, "true", timeout=30).rc == 0
        except Unreachable:
            return False

    def close(self) -> None:
        pass


def _env_prefix(env: dict | None) -> str:
    if not env:
        return ""
    return " ".join(f"{k}={shlex.quote(str(v))}" for k, v in env.items()) + " "


# ---------------------------------------------------------------------------------------------------- local
class LocalTransport(Transport):
    name = "local"

    def __init__(self, root: str | None = None):
        self.root = root

    def _path(self, p: str) -> str:
        if self.root and os.path.isabs(p):
            return os.path.join(self.root, p.lstrip("/"))
        return p

    def run(self, conn, cmd, timeout=3600, env=None, stdin=None):
        t0 = time.time()
        e = dict(os.environ)
        if env:
            e.update({k: str(v) for k, v in env.items()})
        if self.root:
            e["KOP_SANDBOX_ROOT"] = self.root
        p = subprocess.run([*SHELL, cmd], input=stdin, capture_output=True, text=True, timeout=timeout,
                           env=e, cwd=self.root or None)
        return CmdResult(p.returncode, p.stdout, p.stderr, time.time() - t0)

    def put(self, conn, data, dest, mode=None):
        d = self._path(dest)
        os.makedirs(os.path.dirname(d) or ".", exist_ok=True)
        with open(d, "wb") as f:
            f.write(data)
        if mode is not None:
            os.chmod(d, mode)

    def get(self, conn, src):
        with open(self._path(src), "rb") as f:
            return f.read()


# ---------------------------------------------------------------------------------------------------- ssh
class SSHTransport(Transport):
    name = "ssh"

    def __init__(self, control_dir: str | None = None, connect_timeout: int = 10, ssh_bin: str = "ssh",
                 scp_bin: str = "scp", known_hosts_dir: str | None = None):
        self.control_dir = control_dir or tempfile.mkdtemp(prefix="kop-ssh-")
        os.makedirs(self.control_dir, mode=0o700, exist_ok=True)
        # host keys are recorded on first contact (trust on first use) and checked afterwards, one
        # known_hosts file per host:port so re-provisioned hosts can be reset individually
        self.known_hosts_dir = known_hosts_dir or os.path.join(self.control_dir, "known_hosts")
        os.makedirs(self.known_hosts_dir, mode=0o700, exist_ok=True)
        self.connect_timeout = connect_timeout
        self.ssh_bin, self.scp_bin = ssh_bin, scp_bin
        self._keys: dict[str, str] = {}
        self._lock = threading.Lock()

    def _keyfile(self, conn: HostConn) -> str | None:
        k = conn.private_key
        if not k:
            return None
        if "PRIVATE KEY" not in k and os.path.exists(k):
            return k
        import hashlib

        h = hashlib.md5(k.encode()).hexdigest()
        with self._lock:
            if h not in self._keys:
                p = os.path.join(self.control_dir, f".{h}")
                with open(p, "w") as f:
                    f.write(k if k.endswith("\n") else k + "\n")
                os.chmod(p, 0o400)
                self._keys[h] = p
            return self._keys[h]

    def known_hosts_file(self, conn: HostConn) -> str:
        safe = re.sub(r"[^A-Za-z0-9_.:-]", "_", f"{conn.address}_{conn.port}")
        return os.path.join(self.known_hosts_dir, safe)

    def forget_host_key(self, conn: HostConn) -> None:
        """Drop a host's recorded key (after the machine was legitimately re-installed)."""
        try:
            os.unlink(self.known_hosts_file(conn))
        except FileNotFoundError:
            pass

    @staticmethod
    def _cred_tag(conn: HostConn) -> str:
        # multiplexed masters are keyed by the credential too: after a password/key change a live master
        # opened with the old credential is never reused
        import hashlib

        h = hashlib.sha256(f"{conn.user}\0{conn.password or ''}\0{conn.private_key or ''}".encode())
        return h.hexdigest()[:10]

    def _base(self, conn: HostConn) -> tuple[list[str], dict]:
        opts = ["-o", "StrictHostKeyChecking=accept-new", "-o", f"UserKnownHostsFile={self.known_hosts_file(conn)}",
                "-o", "LogLevel=ERROR", "-o", f"ConnectTimeout={self.connect_timeout}", "-o", "ControlMaster=auto",
                "-o", "ControlPersist=120s", "-o", f"ControlPath={self.control_dir}/{self._cred_tag(conn)}-%C",
                "-o", "ServerAliveInterval=30"]
        env = dict(os.environ)
        kf = self._keyfile(conn)
        if kf:
            opts += ["-i", kf, "-o", "IdentitiesOnly=yes"]
        if conn.password and not kf:
            askpass = os.path.join(self.control_dir, "askpass.sh")
            if not os.path.exists(askpass):
                with open(askpass, "w") as f:
                    f.write("#!/bin/sh\nprintf '%s\\n' \"$KOP_SSH_PASSWORD\"\n")
                os.chmod(askpass, stat.S_IRWXU)
            env.update({"SSH_ASKPASS": askpass, "SSH_ASKPASS_REQUIRE": "force", "DISPLAY": env.get("DISPLAY", ":0"),
                        "KOP_SSH_PASSWORD": conn.password})
            opts += ["-o", "PreferredAuthentications=password,keyboard-interactive", "-o", "NumberOfPasswordPrompts=1"]
        else:
            opts += ["-o", "BatchMode=yes"]
        return opts, env

    def run(self, conn, cmd, timeout=3600, env=None, stdin=None):
        opts, penv = self._base(conn)
        remote = _env_prefix(env) + cmd
        if conn.become and conn.user != "root":
            remote = "sudo -H -n " + SHELL_STR + shlex.quote(remote)
        else:
            remote = SHELL_STR + shlex.quote(remote)
        argv = [self.ssh_bin, *opts, "-p", str(conn.port), f"{conn.user}@{conn.address}", remote]
        t0 = time.time()
        try:
            p = subprocess.run(argv, input=stdin, capture_output=True, text=True, timeout=timeout, env=penv)
        except subprocess.TimeoutExpired as e:
            return CmdResult(124, e.stdout or "", f"timeout after {timeout}s", time.time() - t0)
        if p.returncode == 255:
            raise Unreachable(p.stderr.strip() or f"ssh to {conn.address}:{conn.port} failed")
        return CmdResult(p.returncode, p.stdout, p.stderr, time.time() - t0)

    def put(self, conn, data, dest, mode=None):
        q = shlex.quote(dest)
        cmd = f"mkdir -p $(dirname {q}) && cat > {q}"
        if mode is not None:
            cmd += f" && chmod {mode:o} {q}"
        opts, penv = self._base(conn)
        remote = SHELL_STR + shlex.quote(cmd)
        if conn.become and conn.user != "root":
            remote = "sudo -H -n " + remote
        argv = [self.ssh_bin, *opts, "-p", str(conn.port), f"{conn.user}@{conn.address}", remote]
        p = subprocess.run(argv, input=data, capture_output=True, timeout=3600, env=penv)
        if p.returncode == 255:
            raise Unreachable(p.stderr.decode(errors="replace"))
        if p.returncode != 0:
            raise IOError(f"put {dest} on {conn.name}: {p.stderr.decode(errors='replace')}")

    def get(self, conn, src):
        opts, penv = self._base(conn)
        argv = [self.ssh_bin, *opts, "-p", str(conn.port), f"{conn.user}@{conn.address}", f"cat {shlex.quote(src)}"]
        p = subprocess.run(argv, capture_output=True, timeout=3600, env=penv)
        if p.returncode == 255:
            raise Unreachable(p.stderr.decode(errors="replace"))
        if p.returncode != 0:
            raise IOError(f"fetch {src} from {conn.name}: {p.stderr.decode(errors='replace')}")
        return p.stdout

    def close(self):
        for name in os.listdir(self.control_dir) if os.path.isdir(self.control_dir) else []:
            path = os.path.join(self.control_dir, name)
            if not name.startswith(".") and name not in ("askpass.sh", "known_hosts"):
                subprocess.run([self.ssh_bin, "-o", f"ControlPath={path}", "-O", "exit", "dummy"],
                               capture_output=True, timeout=10)


# ---------------------------------------------------------------------------------------------------- fake
@dataclass
class Rule:
    pattern: str
    rc: int = 0
    stdout: str = ""
    stderr: str = ""
    hosts: tuple = ()  # empty = every host
    times: int = -1  # how many matches this rule serves (-1 = forever)
    fn: object = None  # callable(host, cmd, fs) -> CmdResult | tuple


class FakeTransport(Transport):
    """Deterministic host farm for CI (no sockets, no root, no real package managers)."""

    name = "fake"

    def __init__(self, rules: list[Rule] | None = None, default_rc: int = 0, latency_s: float = 0.0):
        self.rules = list(rules or [])
        self.default_rc = default_rc
        self.latency_s = latency_s
        self.log: list[tuple[str, str]] = []  # (host, command)
        self.fs: dict[str, dict[str, bytes]] = {}
        self.unreachable: set[str] = set()
        self.fail_after: dict[str, int] = {}  # host -> fail every command after N calls
        self._calls: dict[str, int] = {}
        self._lock = threading.Lock()
        self.facts: dict[str, dict] = {}

    def add_rule(self, pattern, rc=0, stdout="", stderr="", hosts=(), times=-1, fn=None):
        self.rules.insert(0, Rule(pattern, rc, stdout, stderr, tuple(hosts), times, fn))

    def commands(self, host: str | None = None) -> list[str]:
        return [c for h, c in self.log if host is None or h == host]

    def _match(self, host: str, cmd: str) -> CmdResult:
        for r in self.rules:
            if r.hosts and host not in r.hosts:
                continue
            if r.times == 0:
                continue
            if re.search(r.pattern, cmd):
                if r.times > 0:
                    r.times -= 1
                if r.fn is not None:
                    out = r.fn(host, cmd, self.fs.setdefault(host, {}))
                    if isinstance(out, CmdResult):
                        return out
                    rc, so, se = (tuple(out) + ("", ""))[:3]
                    return CmdResult(rc, so, se)
                return CmdResult(r.rc, r.stdout, r.stderr)
        return CmdResult(self.default_rc, "", "")

    def run(self, conn, cmd, timeout=3600, env=None, stdin=None):
        if conn.name in self.unreachable or conn.address in self.unreachable:
            raise Unreachable(f"{conn.name}: host unreachable (injected)")
        with self._lock:
            n = self._calls.get(conn.name, 0) + 1
            self._calls[conn.name] = n
            self.log.append((conn.name, cmd))
        lim = self.fail_after.get(conn.name)
        if lim is not None and n > lim:
            return CmdResult(1, "", "injected failure")
        if self.latency_s:
            time.sleep(self.latency_s)
        return self._match(conn.name, cmd)

    def put(self, conn, data, dest, mode=None):
        if conn.name in self.unreachable:
            raise Unreachable(conn.name)
        with self._lock:
            self.fs.setdefault(conn.name, {})[dest] = bytes(data)
            self.log.append((conn.name, f"#put {dest}"))

    def get(self, conn, src):
        if conn.name in self.unreachable:
            raise Unreachable(conn.name)
        d = self.fs.get(conn.name, {})
        if src not in d:
            raise IOError(f"{conn.name}: {src}: no such file (fake)")
        return d[src]


_SIM = None


def make_transport(kind: str, **kw) -> Transport:
    if kind == "ssh":
        return SSHTransport(**kw)
    if kind == "local":
        return LocalTransport(**kw)
    if kind == "fake":
        return FakeTransport(**kw)
    if kind == "sim":  # one simulated farm per process, so host state persists across operations
        global _SIM
        if _SIM is None:
            from .simfarm import SimFarm

            gpu = [h for h in os.environ.get("KOP_SIM_GPU_HOSTS", "*").split(",") if h]
            from ..conf import get_config

            _SIM = SimFarm(gpu_hosts=set(gpu), latency_s=float(os.environ.get("KOP_SIM_LATENCY_S", "0")),
                           state_path=os.path.join(get_config().data_dir, "simfarm.json"))
        return _SIM
    raise ValueError(f"unknown transport {kind!r}")
