"""REST /api/v1 + WebSocket API through Starlette's TestClient (no sockets): JWT auth, RBAC, the cluster
lifecycle driven over HTTP exactly as the UI does (reference call stack SURVEY.md §3.1-3.3), progress and
log websockets, CRUD resources, multipart host import."""
import json
import time

import pytest

pytest.importorskip("httpx")
from fastapi.testclient import TestClient  # noqa: E402

from kubeoperator_amd.control.api import create_app  # noqa: E402


@pytest.fixture
def client(control):
    c = TestClient(create_app())
    tok = c.post("/api/v1/token/auth/", json={"username": "admin", "password": "kubeoperator@admin123"}).json()["token"]
    c.headers["Authorization"] = f"JWT {tok}"
    return c


def test_auth_required_and_bad_login(control):
    c = TestClient(create_app())
    assert c.get("/api/v1/clusters/").status_code == 401
    assert c.post("/api/v1/token/auth/", json={"username": "admin", "password": "nope"}).status_code == 401
    assert c.get("/api/v1/version/").json()["arch"] == "gfx950"
    r = c.get("/api/v1/clusters/", headers={"Authorization": "JWT garbage.token.here"})
    assert r.status_code == 401


def test_token_refresh_and_profile(client):
    tok = client.headers["Authorization"].split()[1]
    r = client.post("/api/v1/token/refresh/", json={"token": tok})
    assert r.status_code == 200 and r.json()["token"]
    p = client.get("/api/v1/profile/").json()
    assert p["username"] == "admin" and p["is_superuser"]


def _register_hosts(client):
    for name, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2"), ("w2", "10.0.0.3")):
        r = client.post("/api/v1/host/", json={"name": name, "ip": ip, "password": "pw"})
        assert r.status_code == 201, r.text


def test_cluster_lifecycle_over_http_and_ws(client):
    _register_hosts(client)
    hosts = client.get("/api/v1/host/", params={"page": 1, "size": 2}).json()
    assert hosts["count"] == 3 and len(hosts["results"]) == 2
    w1 = [h for h in client.get("/api/v1/host/").json() if h["name"] == "w1"][0]
    assert w1["gpu_num"] == 8 and "MI355X" in w1["gpu_info"]

    r = client.post("/api/v1/clusters/", json={
        "name": "demo", "template": "single-master", "network_plugin": "flannel", "persistent_storage": "local-volume",
        "package": "mi355x-k8s", "item_name": "KubeOperator",
        "nodes": [{"name": "m1", "host": "m1", "roles": ["master"]}, {"name": "w1", "host": "w1", "roles": ["worker"]}]})
    assert r.status_code == 201, r.text
    assert client.get("/api/v1/clusters/demo/").json()["node_size"] == 2
    assert {n["name"] for n in client.get("/api/v1/clusters/demo/nodes/").json()} == {"m1", "w1"}
    roles = {g["name"] for g in client.get("/api/v1/clusters/demo/roles/").json()}
    assert {"kube-master", "etcd", "gpu_nodes"} <= roles
    client.post("/api/v1/clusters/demo/configs/", json={"key": "MAX_PODS", "value": 200})
    assert client.get("/api/v1/clusters/demo/configs/MAX_PODS/").json()["value"] == 200

    r = client.post("/api/v1/clusters/demo/executions/", json={"operation": "install", "params": {}})
    assert r.status_code == 201, r.text
    eid = r.json()["id"]
    # worker pool is not running in tests: execute the queued job in-process, then watch the progress socket
    from kubeoperator_amd.control.runtime import jobs
    jobs.run_claimed(jobs.claim_pending(eid))
    tok = client.headers["Authorization"].split()[1]
    with pytest.raises(Exception):
        with TestClient(create_app()).websocket_connect(f"/ws/progress/{eid}/") as ws:
            ws.receive_text()
    with client.websocket_connect(f"/ws/progress/{eid}/?interval=0.05&token={tok}") as ws:
        msg = json.loads(ws.receive_text())
    assert msg["state"] == "SUCCESS" and all(s["status"] == "success" for s in msg["steps"])
    with client.websocket_connect(f"/ws/tasks/{eid}/log/?token={tok}") as ws:
        first = json.loads(ws.receive_text())["message"]
    assert "PLAY" in first or "Start task" in first
    log = client.get(f"/api/v1/tasks/{eid}/log/").json()
    assert "kubeadm" in log["data"] and log["end"]
    assert client.get(f"/api/v1/tasks/{eid}/result/").json()["state"] == "SUCCESS"
    assert client.get("/api/v1/clusters/demo/").json()["status"] == "RUNNING"
    assert "apiVersion" in client.get("/api/v1/cluster/demo/download/").text
    execs = client.get("/api/v1/clusters/demo/executions/").json()
    assert execs[0]["operation"] == "install"

    # span trace of the install: steps -> playbooks -> plays -> tasks -> per-host module runs
    tr = client.get(f"/api/v1/clusters/demo/executions/{eid}/trace/").json()
    evs = [e for e in tr["traceEvents"] if e["ph"] == "X"]
    cats = {e["cat"] for e in evs}
    assert {"step", "playbook", "play", "task", "host"} <= cats
    tracks = {e["args"]["name"] for e in tr["traceEvents"] if e["ph"] == "M" and e["name"] == "thread_name"}
    assert {"controller", "m1", "w1"} <= tracks
    steps = [e for e in evs if e["cat"] == "step"]
    assert [e["name"] for e in steps] == [s["name"] for s in msg["steps"]]
    for a, b in zip(steps, steps[1:]):  # steps run back to back, each inside the execution's wall time
        assert b["ts"] >= a["ts"] + a["dur"] - 1
    summ = client.get(f"/api/v1/clusters/demo/executions/{eid}/trace/", params={"view": "summary"}).json()
    assert [s["step"] for s in summ["steps"]] == [s["name"] for s in msg["steps"]]
    assert all(s["task_count"] > 0 and s["tasks"] and set(s["hosts"]) <= {"m1", "w1", "localhost"}
               for s in summ["steps"])
    assert client.get(f"/api/v1/clusters/demo/executions/{eid}/trace/", params={"view": "x"}).status_code == 400
    assert client.get("/api/v1/clusters/demo/executions/nope/trace/").status_code == 404
    assert b"kubeoperator_task_seconds_bucket" in client.get("/metrics").content

    # a second operation while one is queued is rejected
    client.post("/api/v1/clusters/demo/executions/", json={"operation": "gpu-validate"})
    r = client.post("/api/v1/clusters/demo/executions/", json={"operation": "gpu-validate"})
    assert r.status_code == 400


def test_rbac_viewer_cannot_operate(client, control):
    _register_hosts(client)
    client.post("/api/v1/clusters/", json={"name": "c1", "template": "single-master", "item_name": "KubeOperator"})
    client.post("/api/v1/clusters/", json={"name": "c2", "template": "single-master"})
    client.post("/api/v1/users/", json={"username": "bob", "password": "pw123456"})
    client.post("/api/v1/item/profiles/KubeOperator/", json=[{"username": "bob", "role": "VIEWER"}])
    c = TestClient(create_app())
    tok = c.post("/api/v1/token/auth/", json={"username": "bob", "password": "pw123456"}).json()["token"]
    c.headers["Authorization"] = f"JWT {tok}"
    assert [x["name"] for x in c.get("/api/v1/clusters/").json()] == ["c1"]
    assert c.get("/api/v1/clusters/c2/").status_code == 404
    assert c.post("/api/v1/clusters/c1/executions/", json={"operation": "install"}).status_code == 403
    assert c.delete("/api/v1/clusters/c1/").status_code == 403
    assert c.post("/api/v1/credential/", json={"name": "x"}).status_code == 403
    client.post("/api/v1/item/profiles/KubeOperator/", json=[{"username": "bob", "role": "MANAGER"}])
    assert c.post("/api/v1/clusters/c1/configs/", json={"key": "a", "value": 1}).status_code == 201


def test_crud_resources_and_secrets(client):
    r = client.post("/api/v1/credential/", json={"name": "root-pw", "username": "root", "password": "s3cret"})
    assert r.status_code == 201 and r.json()["password"] == ""
    assert client.get("/api/v1/credential/root-pw/").json()["username"] == "root"
    assert client.post("/api/v1/credential/", json={"name": "root-pw"}).status_code == 400
    client.patch("/api/v1/credential/root-pw/", json={"username": "ubuntu"})
    assert client.get("/api/v1/credential/root-pw/").json()["username"] == "ubuntu"
    assert client.delete("/api/v1/credential/root-pw/").status_code == 204
    assert client.get("/api/v1/credential/root-pw/").status_code == 404

    r = client.post("/api/v1/regions/", json={"name": "r1", "vars": {"provider": "fake"}})
    rid = r.json()["id"]
    z = client.post("/api/v1/zones/", json={"name": "z1", "region_id": rid,
                                            "vars": {"ip_start": "10.1.0.10", "ip_end": "10.1.0.20"}})
    assert z.status_code == 201
    assert client.post("/api/v1/plans/", json={"name": "p1", "region_id": rid, "zone_ids": [z.json()["id"]]}).status_code == 201
    assert len(client.get("/api/v1/cloud/compute/").json()) >= 3
    assert client.get("/api/v1/provider/template/").json()

    r = client.post("/api/v1/backupStorage/", json={"name": "local", "type": "LOCAL",
                                                    "credentials": {"path": "/tmp/kop-bk", "secretKey": "x"}})
    assert r.status_code == 201 and r.json()["credentials"]["secretKey"] == ""
    assert client.post("/api/v1/backupStorage/check", json={"type": "LOCAL", "credentials": {"path": "/tmp/kop-bk"}}).json()["message"] == "OK"

    client.post("/api/v1/settings?tab=system", json={"local_hostname": "10.0.0.100", "SMTP_PASSWORD": "x"})
    st = client.get("/api/v1/settings", params={"tab": "system"}).json()
    assert st["local_hostname"] == "10.0.0.100" and st["SMTP_PASSWORD"] == ""

    # DNS page (ui/src/app/dns): stored as the "dns" settings tab, carried to the nameserver role via extra vars
    assert client.get("/api/v1/dns/").json() == {"id": "dns", "dns1": "", "dns2": ""}
    assert client.post("/api/v1/dns/update/", json={"dns1": "10.0.0.53", "dns2": "not-an-ip"}).status_code == 400
    assert client.post("/api/v1/dns/update/", json={"dns1": "10.0.0.53", "dns2": ""}).json()["dns1"] == "10.0.0.53"
    assert client.get("/api/v1/dns/").json()["dns1"] == "10.0.0.53"
    from kubeoperator_amd.control.domain import context as ctx
    assert ctx.get_settings()["dns1"] == "10.0.0.53"  # clusters.extra_vars merges every settings tab

    pk = client.get("/api/v1/packages/").json()
    assert {"mi355x-k8s", "mi355x-k8s-next"} <= {p["name"] for p in pk}
    assert client.get("/api/v1/cluster/config").json()["templates"]


def test_host_import_multipart(client):
    csv = b"name,ip,port,credential,username,password\nh1,10.0.0.2,22,,root,pw\nh2,10.0.0.3,22,,root,pw\n"
    bnd = "XyZbOuNdArY"
    payload = (f"--{bnd}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"hosts.csv\"\r\n"
               f"Content-Type: text/csv\r\n\r\n").encode() + csv + f"\r\n--{bnd}--\r\n".encode()
    r = client.post("/api/v1/host/import/", content=payload,
                    headers={"Content-Type": f"multipart/form-data; boundary={bnd}"})
    assert r.status_code == 200, r.text
    assert sorted(r.json()["created"]) == ["h1", "h2"]


def test_host_gpu_check_route(client):
    h = client.post("/api/v1/host/", json={"name": "w1", "ip": "10.0.0.2", "password": "pw"}).json()
    assert h["gpu_num"] == 8
    r = client.post(f"/api/v1/host/{h['id']}/gpu-check/")
    assert r.status_code == 200, r.text
    d = r.json()
    assert d["summary"]["success"] and d["kfd_gpus"] == "8" and d["rocminfo_gpus"] == "8"


def test_messages_and_log_search(client):
    from kubeoperator_amd.control.domain import messages
    messages.insert_message({"title": "hello", "content": {"detail": "x"}}, sync=True)
    assert client.get("/api/v1/notification/userMessage/unread/").json()["unread"] >= 1
    ms = client.get("/api/v1/notification/userMessage/").json()
    assert ms["count"] >= 1 and ms["results"][0]["message_detail"]["title"] == "hello"
    client.put("/api/v1/notification/userMessage/", json={"ids": None})
    assert client.get("/api/v1/notification/userMessage/unread/").json()["unread"] == 0
    import logging

    from kubeoperator_amd.control.domain.monitor import JsonlLogHandler
    lg = logging.getLogger("kop-test")
    lg.addHandler(JsonlLogHandler())
    lg.error("disk pressure on node-7")
    res = client.post("/api/v1/log/", json={"level": "ERROR", "keywords": "pressure"}).json()
    assert res["total"] >= 1


def test_ui_served(control):
    c = TestClient(create_app())
    r = c.get("/ui/")
    assert r.status_code == 200 and "<html" in r.text.lower()


def test_api_explorer_is_offline(control):
    """/swagger/, /docs/ and /redoc/ serve one self-contained explorer page (no http(s) asset URL: the offline
    install has no CDN) that reads the schema from this server; /docs.json and /docs.yaml serve the schema itself
    (reference kubeoperator/urls.py:44-47)."""
    import re

    import yaml

    c = TestClient(create_app())
    for path in ("/swagger/", "/docs/", "/redoc/"):
        r = c.get(path)
        assert r.status_code == 200 and r.headers["content-type"].startswith("text/html")
        assert not re.search(r"""(src|href)\s*=\s*["']?(https?:)?//""", r.text), path
        assert "http://" not in r.text and "https://" not in r.text
        assert "/swagger.json" in r.text
    j = c.get("/docs.json").json()
    assert "/api/v1/clusters/{name}/executions/" in j["paths"]
    y = yaml.safe_load(c.get("/docs.yaml").text)
    assert y["paths"].keys() == j["paths"].keys()
    assert c.get("/swagger.json").json()["info"]["title"] == j["info"]["title"]


def test_prometheus_metrics(client, control):
    from kubeoperator_amd.control.domain import deploy
    _register_hosts(client)
    client.post("/api/v1/clusters/", json={"name": "mx", "template": "single-master",
                                          "nodes": [{"name": "m1", "host": "m1", "roles": ["master"]},
                                                    {"name": "w1", "host": "w1", "roles": ["worker"]}]})
    e = deploy.create("mx", "install", run="inline")
    assert e["state"] == "SUCCESS"
    assert all("seconds" in s for s in e["steps"])
    text = TestClient(create_app()).get("/metrics").text
    assert 'kubeoperator_execution_seconds_count{operation="install",state="SUCCESS"}' in text
    assert 'kubeoperator_step_seconds_count{operation="install",status="success",step="master"}' in text
    assert 'kubeoperator_clusters{status="RUNNING"} 1.0' in text
    assert 'kubeoperator_gpus{model="AMD Instinct MI355X"}' in text


def test_app_catalog_and_deploy_over_http(client):
    """Bundled chart catalog, app-deploy execution over REST (validated names), recorded releases."""
    from kubeoperator_amd.control.runtime import jobs

    cat = {c["name"]: c for c in client.get("/api/v1/apps/catalog/").json()}
    assert {"nginx", "pytorch-rocm-train"} <= set(cat)
    assert cat["pytorch-rocm-train"]["values"]["model"] == "llama3_8b"
    _register_hosts(client)
    client.post("/api/v1/clusters/", json={
        "name": "demo", "template": "single-master", "item_name": "KubeOperator",
        "nodes": [{"name": "m1", "host": "m1", "roles": ["master"]}, {"name": "w1", "host": "w1", "roles": ["worker"]}]})
    eid = client.post("/api/v1/clusters/demo/executions/", json={"operation": "install"}).json()["id"]
    jobs.run_claimed(jobs.claim_pending(eid))
    r = client.post("/api/v1/clusters/demo/executions/",
                    json={"operation": "app-deploy", "params": {"chart": "nginx", "release": "Bad Name"}})
    assert r.status_code == 400
    r = client.post("/api/v1/clusters/demo/executions/",
                    json={"operation": "app-deploy", "params": {"chart": "pytorch-rocm-train", "release": "gpt2",
                                                                "values": {"model": "gpt2_small"}, "wait_job": True}})
    assert r.status_code == 201, r.text
    jobs.run_claimed(jobs.claim_pending(r.json()["id"]))
    e = client.get(f"/api/v1/clusters/demo/executions/{r.json()['id']}/").json()
    assert e["state"] == "SUCCESS" and e["result_summary"]["training"]["tokens_per_s"] > 0
    apps = client.get("/api/v1/clusters/demo/apps/").json()
    assert [a["release"] for a in apps] == ["gpt2"] and apps[0]["values"]["model"] == "gpt2_small"


def test_task_monitor_workers_stats_revoke_retry(client):
    """The Flower equivalent (reference core/kubeops.py:197-213, /flower/ proxy): worker heartbeats, per-task
    statistics, recent jobs, revoke of a queued job, retry of a failed one."""
    from kubeoperator_amd.control.runtime import jobs

    calls = []

    @jobs.task("monitor_probe")
    def probe(job_id, logger, fail=False):
        calls.append(job_id)
        logger.info("probe ran")
        if fail:
            raise RuntimeError("probe failed on purpose")
        return {"ok": True}

    queued = jobs.submit("monitor_probe", {})
    r = client.post(f"/api/v1/tasks/{queued}/revoke/")
    assert r.status_code == 200 and r.json()["state"] == "REVOKED"
    assert client.post(f"/api/v1/tasks/{queued}/revoke/").status_code == 409  # not PENDING any more
    ok = jobs.submit("monitor_probe", {})
    bad = jobs.submit("monitor_probe", {"fail": True})
    pool = jobs.WorkerPool(concurrency=2, poll_s=0.02, heartbeat_s=0.05).start()
    try:
        for _ in range(200):
            if jobs.get(ok).state == "SUCCESS" and jobs.get(bad).state == "FAILURE":
                break
            time.sleep(0.02)
        for _ in range(200):  # the heartbeat follows the job's end
            w = client.get("/api/v1/tasks/workers/").json()
            if any(x["online"] and x["name"] == pool.name and x["processed"] >= 2 for x in w):
                break
            time.sleep(0.02)
        assert any(x["online"] and x["name"] == pool.name and x["processed"] >= 2 for x in w), w
        assert queued not in calls  # revoked: never ran
        st = {t["task"]: t for t in client.get("/api/v1/tasks/stats/").json()["tasks"]}
        p = st["monitor_probe"]
        assert p["total"] == 3 and p["success"] == 1 and p["failure"] == 1 and p["revoked"] == 1
        assert p["runtime_avg_s"] is not None
        fails = client.get("/api/v1/tasks/?state=failure&name=monitor_probe").json()
        assert [j["id"] for j in fails] == [bad] and "on purpose" in fails[0]["error"]
        r = client.post(f"/api/v1/tasks/{bad}/retry/")
        assert r.status_code == 200 and r.json()["retry_of"] == bad
        again = r.json()["id"]
        for _ in range(200):
            if jobs.get(again).state in ("SUCCESS", "FAILURE"):
                break
            time.sleep(0.02)
        assert jobs.get(again).state == "FAILURE" and jobs.get(again).args == {"fail": True}
        assert "probe ran" in client.get(f"/api/v1/tasks/{again}/log/").json()["data"]
    finally:
        pool.stop()
    w = client.get("/api/v1/tasks/workers/").json()
    assert not next(x for x in w if x["name"] == pool.name)["online"]  # stopped
    assert client.get("/flower/", follow_redirects=False).headers["location"] == "/ui/#/tasks"
    assert isinstance(client.get("/api/v1/tasks/periodic/").json(), list)
