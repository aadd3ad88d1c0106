"""The web UI's main flows, executed: tests/ui/flows.js runs the served index.html + app.js under node 12 over a
small DOM (tests/ui/dom.js) against a live control plane (own ASGI server + job workers) on the simulated farm --
sign in, cluster-create wizard with device checks, create & install followed over the progress / log websockets,
a PyTorch-ROCm training-chart deploy from the apps tab, then Day 2 through the forms: host registration, add-worker,
backup storage + backup, LDAP settings, a new user, and the task monitor."""
import asyncio
import json
import os
import shutil
import subprocess
import threading

import pytest

from kubeoperator_amd.control.api import create_app
from kubeoperator_amd.control.api.server import Server
from kubeoperator_amd.control.domain import hosts
from kubeoperator_amd.control.runtime import jobs
from kubeoperator_amd.control.store import models as M
from kubeoperator_amd.control.store.db import session_scope

HERE = os.path.dirname(os.path.abspath(__file__))
NODE = shutil.which("node")


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_ui_flows_against_a_live_control_plane(control):
    for hn, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2"), ("tiny", "10.0.0.7")):
        hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
    with session_scope() as s:  # a host below the worker role's 8 GB memory minimum
        s.query(M.Host).filter_by(name="tiny").one().memory = 2048
    pool = jobs.WorkerPool(concurrency=2, poll_s=0.05).start()
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
    try:
        r = subprocess.run([NODE, "--harmony-nullish", "--harmony-optional-chaining", os.path.join(HERE, "ui", "flows.js"),
                            f"http://127.0.0.1:{srv.port}", control.cfg["ADMIN_PASSWORD"], str(control.tmp / "bk")],
                           capture_output=True, text=True, timeout=240)
    finally:
        asyncio.run_coroutine_threadsafe(srv.stop(), loop).result(10)
        loop.call_soon_threadsafe(loop.stop)
        t.join(5)
        pool.stop()
    recs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and recs and recs[-1].get("step") == "done", r.stdout[-4000:] + r.stderr[-4000:]
    by = {x["step"]: x for x in recs}
    assert "Invalid" in by["login-refused"]["error"] or by["login-refused"]["error"]
    assert "role master: needs = 1 node(s), selected 2" in by["device-checks"]["messages"]
    assert "tiny: Memory 2 < 8 GB" in by["device-checks"]["messages"]
    inst = by["installed"]
    assert [s[0] for s in inst["steps"]][:5] == ["config", "prepare", "master", "worker", "addon"]
    assert all(s[1] == "success" for s in inst["steps"][:5]) and not inst["socket_errors"]
    assert inst["log_bytes"] > 1000
    assert "llama-train" in by["app-deployed"]["row"] and "tokens/s" in by["app-deployed"]["row"]
    assert "10.0.0.9" in by["host-registered"]["row"]
    assert by["worker-added"]["nodes"] == 3 and "10.0.0.9" in by["worker-added"]["row"]
    assert by["backup-done"]["backups"] == 1 and os.listdir(control.tmp / "bk" / "uiflow")
    assert {"Cluster status", "Capacity", "Statistics", "Pods failing"} <= set(by["dashboard"]["cards"])
    assert by["task-monitor"]["recent_jobs"] >= 4  # install, app deploy, add-worker, backup
