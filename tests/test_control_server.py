"""The control plane's own ASGI server over real sockets: HTTP keep-alive + chunked responses, the
progress websocket (RFC 6455 handshake, masked client frames, close), and the kubeopsctl service launcher
(start -d / status / stop with pidfiles, reference core/kubeops.py)."""
import asyncio
import base64
import json
import os
import socket
import struct
import subprocess
import sys
import threading
import time

import httpx
import pytest

from kubeoperator_amd.control.api import create_app
from kubeoperator_amd.control.api.server import Server


@pytest.fixture
def live(control):
    srv = Server(create_app(), "127.0.0.1", 0)
    loop = asyncio.new_event_loop()
    ready = threading.Event()

    def run():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(srv.start())
        ready.set()
        loop.run_forever()

    t = threading.Thread(target=run, daemon=True)
    t.start()
    assert ready.wait(10)
    yield f"127.0.0.1:{srv.port}"
    asyncio.run_coroutine_threadsafe(srv.stop(), loop).result(10)
    loop.call_soon_threadsafe(loop.stop)
    t.join(5)


def _ws_connect(addr, path):
    host, port = addr.split(":")
    s = socket.create_connection((host, int(port)), timeout=10)
    key = base64.b64encode(os.urandom(16)).decode()
    s.sendall((f"GET {path} HTTP/1.1\r\nHost: {addr}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
               f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n\r\n").encode())
    head = b""
    while b"\r\n\r\n" not in head:
        head += s.recv(1)
    assert head.startswith(b"HTTP/1.1 101"), head
    return s


def _ws_recv(s):
    b1, b2 = s.recv(2, socket.MSG_WAITALL)
    n = b2 & 0x7F
    if n == 126:
        n = struct.unpack("!H", s.recv(2, socket.MSG_WAITALL))[0]
    elif n == 127:
        n = struct.unpack("!Q", s.recv(8, socket.MSG_WAITALL))[0]
    data = s.recv(n, socket.MSG_WAITALL) if n else b""
    return b1 & 0x0F, data


def _ws_send_close(s):
    mask = os.urandom(4)
    payload = struct.pack("!H", 1000)
    s.sendall(bytes([0x88, 0x80 | len(payload)]) + mask + bytes(b ^ mask[i & 3] for i, b in enumerate(payload)))


def test_http_keepalive_and_auth(live):
    with httpx.Client(base_url=f"http://{live}") as c:
        assert c.get("/healthz").json()["ok"]
        tok = c.post("/api/v1/token/auth/", json={"username": "admin", "password": "kubeoperator@admin123"}).json()["token"]
        c.headers["Authorization"] = f"JWT {tok}"
        for _ in range(3):  # same connection
            assert c.get("/api/v1/packages/").status_code == 200
        assert c.get("/api/v1/clusters/nope/").status_code == 404
        r = c.get("/ui/")
        assert r.status_code == 200 and "<html" in r.text.lower()


def test_progress_websocket(live, control):
    from kubeoperator_amd.control.domain import clusters, deploy, hosts
    hosts.create_host({"name": "m1", "ip": "10.0.0.1", "password": "pw"})
    clusters.create_cluster({"name": "demo", "template": "single-master"})
    clusters.add_node("demo", {"name": "m1", "host": "m1", "roles": ["master"]})
    e = deploy.create("demo", "uninstall", run="inline")
    from kubeoperator_amd.control.domain import users
    tok = users.authenticate("admin", "kubeoperator@admin123")["token"]
    s = _ws_connect(live, f"/ws/progress/{e['id']}/?token={tok}")
    op, data = _ws_recv(s)
    assert op == 1
    msg = json.loads(data)
    assert msg["id"] == e["id"] and msg["state"] == e["state"]
    op, _ = _ws_recv(s)  # server closes after a finished execution
    assert op == 8
    _ws_send_close(s)
    s.close()


def test_service_launcher(tmp_path):
    cfgp = tmp_path / "config.yml"
    cfgp.write_text(f"DATA_DIR: {tmp_path}/data\nHTTP_LISTEN_PORT: 0\nHTTP_BIND_HOST: 127.0.0.1\n")
    env = dict(os.environ, KUBEOPERATOR_CONFIG=str(cfgp), KOP_PBKDF2_ITERS="1000")
    run = lambda *a: subprocess.run([sys.executable, "-m", "kubeoperator_amd.control.cli", *a], env=env,  # noqa: E731
                                    capture_output=True, text=True, timeout=60)
    r = run("start", "worker", "-d")
    assert r.returncode == 0, r.stdout + r.stderr
    try:
        r = run("status", "worker")
        assert "running" in r.stdout
    finally:
        r = run("stop", "worker")
    assert "stopped" in r.stdout
    for _ in range(50):
        if "stopped" in run("status", "worker").stdout:
            break
        time.sleep(0.1)
    assert "stopped" in run("status", "worker").stdout


def test_operator_lifecycle_verbs(tmp_path):
    """kubeopsctl install / db / python / upgrade / reload / tail / down / uninstall --purge (reference
    kubeopsctl.sh verbs, re-done for a process-based deployment)."""
    cfgp = tmp_path / "config.yml"
    data = tmp_path / "data"
    cfgp.write_text(f"DATA_DIR: {data}\nHTTP_LISTEN_PORT: 0\nHTTP_BIND_HOST: 127.0.0.1\n")
    env = dict(os.environ, KUBEOPERATOR_CONFIG=str(cfgp), KOP_PBKDF2_ITERS="1000")
    run = lambda *a: subprocess.run([sys.executable, "-m", "kubeoperator_amd.control.cli", *a], env=env,  # noqa: E731
                                    capture_output=True, text=True, timeout=60)
    r = run("install")
    assert r.returncode == 0, r.stderr
    unit = (data / "kubeops.service").read_text()
    assert "ExecStart=" in unit and "start all" in unit and str(cfgp) in unit
    r = run("db", "-c", "select username from users")
    assert r.returncode == 0 and "admin" in r.stdout, r.stdout + r.stderr
    r = run("python", "-c", "from sqlalchemy import select\nwith session_scope() as s: print(len(s.scalars(select(M.User)).all()))")
    assert r.returncode == 0 and r.stdout.strip() == "1", r.stdout + r.stderr
    r = run("upgrade")
    assert r.returncode == 0 and "backed up" in r.stdout, r.stdout + r.stderr
    r = run("reload", "worker")
    assert r.returncode == 0, r.stdout + r.stderr
    try:
        assert "running" in run("status", "worker").stdout
        time.sleep(0.5)
        r = run("tail", "-n", "5")
        assert r.returncode in (0, 1)
    finally:
        r = run("down", "worker")
    for _ in range(50):
        if "stopped" in run("status", "worker").stdout:
            break
        time.sleep(0.1)
    assert not list((data / "tmp").glob("*.pid"))
    r = run("uninstall", "--purge")
    assert r.returncode == 0 and not data.exists()


def test_ui_script_parses_and_covers_the_reference_modules():
    """The single-page UI parses (node, when present) and has a view for every reference UI module
     plus the MI355X additions (apps / training)."""
    import re
    import shutil

    path = os.path.join(os.path.dirname(__file__), "..", "kubeoperator_amd", "control", "ui", "app.js")
    src = open(path).read()
    views = set(re.findall(r"^views(?:\.|\[\")([\w-]+)", src, re.M))
    assert {"dashboard", "clusters", "cluster-create", "cluster", "hosts", "credentials", "packages", "regions", "zones",
            "plans", "storage", "items", "users", "settings", "messages", "logs", "profile", "training", "tasks"} <= views, views
    for tab in ("overview", "nodes", "deploy", "apps", "health", "events", "storage", "backup", "grade", "configs",
                "f5", "terminal"):
        assert f'tab === "{tab}"' in src or tab == "overview", tab
    assert "/trace/?view=summary" in src  # deploy tab: time breakdown of the execution's span trace
    node = shutil.which("node")
    if node:
        r = subprocess.run([node, "--harmony-nullish", "--harmony-optional-chaining", "--check", path],
                           capture_output=True, text=True)
        if "bad option" not in r.stderr:
            assert r.returncode == 0, r.stderr


def test_kubeopsctl_cluster_create_install_and_trace(tmp_path):
    """kubeopsctl cluster create -f <plan> --install on the simulated farm, then ``cluster trace``: the per-step
    time breakdown and the Chrome trace file of the install."""
    cfgp = tmp_path / "config.yml"
    cfgp.write_text(f"DATA_DIR: {tmp_path}/data\nDEFAULT_TRANSPORT: sim\n")
    env = dict(os.environ, KUBEOPERATOR_CONFIG=str(cfgp), KOP_PBKDF2_ITERS="1000")
    run = lambda *a: subprocess.run([sys.executable, "-m", "kubeoperator_amd.control.cli", *a], env=env,  # noqa: E731
                                    capture_output=True, text=True, timeout=300)
    plan = os.path.join(os.path.dirname(__file__), "..", "examples", "cluster-plan-mi355x.yml")
    r = run("cluster", "create", "-f", plan, "--install")
    assert r.returncode == 0 and "install: SUCCESS" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    r = run("cluster", "trace", "mi355x-demo")
    assert r.returncode == 0, r.stderr
    for step in ("config", "prepare", "master", "worker", "addon"):
        assert f"\n{step}: " in r.stdout, r.stdout
    assert "cp-1" in r.stdout and "gpu-1" in r.stdout
    out = tmp_path / "install.trace.json"
    r = run("cluster", "trace", "mi355x-demo", "-o", str(out))
    assert r.returncode == 0, r.stderr
    import json as _json
    ev = _json.loads(out.read_text())["traceEvents"]
    assert any(e.get("cat") == "host" for e in ev) and any(e.get("cat") == "step" for e in ev)
    r = run("host", "gpu-check", "gpu-1")  # the plan registered its hosts; gpu-1 is an 8x MI355X node of the farm
    assert r.returncode == 0 and "gpu-1: ok" in r.stdout and "kfd GPUs=8" in r.stdout, r.stdout + r.stderr
