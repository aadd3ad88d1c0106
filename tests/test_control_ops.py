"""Day-2 / auxiliary control-plane paths: AUTOMATIC (IaaS) clusters with IP pools, Terraform rendering,
scale out/in and destroy; the periodic scheduler; S3 backup storage against a local SigV4-checking stub;
cluster monitoring (data blob with AMD GPU metrics, events -> messages, health, grade) with stub clients."""
import datetime as dt
import hashlib
import http.server
import json
import os
import threading

import pytest

from kubeoperator_amd.control.domain import backup, cloud, clusters, deploy, monitor
from kubeoperator_amd.control.store import models as M
from kubeoperator_amd.control.store.db import session_scope


# ------------------------------------------------------------------------------------------------ IaaS
def _plan(provider="fake", n_ips=20, template="SINGLE"):
    with session_scope() as s:
        tmpl = s.query(M.CloudProviderTemplate).filter_by(name=provider).first()
        r = M.Region(name="r1", cloud_region="dc1", template_id=tmpl.id if tmpl else None,
                     vars={"provider": provider, "vc_host": "vc.local", "vc_username": "u", "vc_password": "p",
                           "datacenter": "dc1"})
        s.add(r)
        s.flush()
        z1 = M.Zone(name="z1", region_id=r.id, cloud_zone="cluster-a",
                    vars={"ip_start": "10.1.0.10", "ip_end": f"10.1.0.{9 + n_ips // 2}", "net_mask": "255.255.255.0",
                          "gateway": "10.1.0.1", "dns1": "10.1.0.2", "provider": provider, "cluster": "cluster-a",
                          "datastore": "ds1", "network": "vm-net", "image_name": "ubuntu-22.04-rocm"})
        z2 = M.Zone(name="z2", region_id=r.id, cloud_zone="cluster-b",
                    vars={"ip_start": "10.2.0.10", "ip_end": f"10.2.0.{9 + n_ips // 2}", "net_mask": "255.255.255.0",
                          "gateway": "10.2.0.1", "dns1": "10.2.0.2", "provider": provider, "cluster": "cluster-b",
                          "datastore": "ds1", "network": "vm-net", "image_name": "ubuntu-22.04-rocm"})
        s.add_all([z1, z2])
        s.flush()
        p = M.Plan(name="p1", region_id=r.id, zone_ids=[z1.id, z2.id], deploy_template=template,
                   vars={"master_model": "large", "worker_model": "mi355x-8gpu"})
        s.add(p)
        s.flush()
        return p.id, z1.id, z2.id


def test_ip_pool_and_allocation(control):
    _, z1, _ = _plan(n_ips=4)
    got = {cloud.allocate_ip(z1), cloud.allocate_ip(z1)}
    assert got == {"10.1.0.10", "10.1.0.11"}
    cloud.recover_ip(z1, "10.1.0.10")
    assert cloud.allocate_ip(z1) == "10.1.0.10"


def test_automatic_cluster_install_scale_destroy(control):
    pid, z1, z2 = _plan()
    clusters.create_cluster({"name": "auto", "template": "single-master", "deploy_type": "AUTOMATIC", "plan": pid,
                             "worker_size": 2, "cluster_doamin_suffix": "lab.local"})
    e = deploy.create("auto", "install", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert e["steps"][0]["name"] == "create-resource"
    nodes = sorted(n["name"] for n in clusters.list_nodes("auto"))
    assert nodes == ["master1.auto.lab.local", "worker1.auto.lab.local", "worker2.auto.lab.local"]
    tf = open(os.path.join(control.cfg.data_dir, "terraform", "auto", "main.tf")).read()
    assert "worker2" in tf and "10.1.0." in tf
    with session_scope() as s:
        ips = {h.name: h.ip for h in s.query(M.Host)}
    assert ips["worker1.auto.lab.local"].startswith("10.2.") or ips["worker1.auto.lab.local"].startswith("10.1.")
    # multi-AZ round robin: the two workers land in different zones
    assert ips["worker1.auto.lab.local"].split(".")[1] != ips["worker2.auto.lab.local"].split(".")[1]

    e = deploy.create("auto", "scale", {"num": 3}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert len(clusters.list_nodes("auto")) == 4
    e = deploy.create("auto", "scale", {"num": 1}, run="inline")
    assert e["state"] == "SUCCESS"
    assert len(clusters.list_nodes("auto")) == 2

    e = deploy.create("auto", "uninstall", run="inline")
    assert e["state"] == "SUCCESS"
    assert clusters.list_nodes("auto") == []
    with session_scope() as s:
        assert all(not z.ip_used for z in s.query(M.Zone))


def test_capacity_check(control):
    pid, _, _ = _plan(n_ips=2)
    clusters.create_cluster({"name": "big", "template": "single-master", "deploy_type": "AUTOMATIC", "plan": pid,
                             "worker_size": 5})
    with pytest.raises(Exception):
        deploy.create("big", "scale", {"num": 10}, run="none")


@pytest.mark.parametrize("provider", ["vsphere", "openstack"])
def test_terraform_templates_render(control, provider):
    hosts = [{"name": "master1.c.local", "short_name": "master1", "role": "master", "ip": "10.0.0.5", "cpu": 8,
              "memory": 32768, "gpu": 0, "gpu_model": "", "zone": {"cluster": "a", "datastore": "d", "network": "n",
                                                                    "net_mask": "255.255.255.0", "gateway": "10.0.0.1",
                                                                    "dns1": "10.0.0.2", "image_name": "img",
                                                                    "zone_name": "z1", "key": "z1", "name": "a",
                                                                    "network_id": "net", "floating_network": "pub"},
              "zone_name": "z1", "domain": "c.local"}]
    variables = {"vc_host": "vc", "vc_username": "u", "vc_password": "p", "datacenter": "dc", "region": "r",
                 "auth_url": "http://keystone:5000/v3", "username": "u", "password": "p", "project_name": "p",
                 "user_domain": "Default", "project_domain": "Default", "flavor": "m1.xlarge", "image_name": "img"}
    variables["zones"] = [hosts[0]["zone"]]
    path = cloud.render_terraform("c", provider, variables, hosts)
    text = open(path).read()
    assert "master1" in text and "10.0.0.5" in text


# ------------------------------------------------------------------------------------------------ scheduler
def test_cron_and_due(control):
    from kubeoperator_amd.control.runtime import scheduler
    t = dt.datetime(2026, 10, 15, 1, 0)
    assert scheduler.cron_match("0 1 * * *", t)
    assert not scheduler.cron_match("0 2 * * *", t)
    assert scheduler.cron_match("*/15 * * * *", t.replace(minute=45))
    assert scheduler.cron_match("0 0-3 * * 1-5", t)  # Thursday
    scheduler.seed_defaults()
    fired = {n for n, _, _ in scheduler.due(t)}
    assert {"cluster-backup-daily", "save-cluster-data", "host-health-check"} <= fired
    again = {n for n, _, _ in scheduler.due(t + dt.timedelta(seconds=30))}
    assert "cluster-backup-daily" not in again and "save-cluster-data" not in again
    later = {n for n, _, _ in scheduler.due(t + dt.timedelta(minutes=6))}
    assert "save-cluster-data" in later


def test_scheduler_tick_submits_jobs(control):
    from kubeoperator_amd.control.domain import tasks  # noqa: F401  (registers jobs)
    from kubeoperator_amd.control.runtime import jobs, scheduler
    scheduler.seed_defaults()
    fired = scheduler.Scheduler().tick(dt.datetime(2026, 10, 15, 1, 0))
    assert "cluster-backup-daily" in fired
    with session_scope() as s:
        names = {j.name for j in s.query(M.Job)}
    assert "cluster_backup_all" in names
    pool = jobs.WorkerPool(concurrency=2, poll_s=0.05).start()
    try:
        for _ in range(200):
            with session_scope() as s:
                if all(j.state in ("SUCCESS", "FAILURE") for j in s.query(M.Job)):
                    break
            import time
            time.sleep(0.05)
    finally:
        pool.stop()
    with session_scope() as s:
        assert all(j.state == "SUCCESS" for j in s.query(M.Job)), [(j.name, j.result) for j in s.query(M.Job)]


# ------------------------------------------------------------------------------------------------ S3 backup
class _S3Stub(http.server.BaseHTTPRequestHandler):
    store = {}

    def _ok_sig(self):
        auth = self.headers.get("Authorization", "")
        body_hash = self.headers.get("x-amz-content-sha256", "")
        return auth.startswith("AWS4-HMAC-SHA256 Credential=AK/") and "Signature=" in auth and len(body_hash) == 64

    def do_PUT(self):
        n = int(self.headers.get("Content-Length", 0))
        data = self.rfile.read(n)
        if not self._ok_sig() or hashlib.sha256(data).hexdigest() != self.headers["x-amz-content-sha256"]:
            self.send_response(403)
            self.end_headers()
            return
        self.store[self.path] = data
        self.send_response(200)
        self.end_headers()

    def do_GET(self):
        if self.path not in self.store:
            self.send_response(404)
            self.end_headers()
            return
        self.send_response(200)
        self.send_header("Content-Length", str(len(self.store[self.path])))
        self.end_headers()
        self.wfile.write(self.store[self.path])

    def do_HEAD(self):
        self.send_response(200 if self.path in self.store or self.path.count("/") == 1 else 404)
        self.end_headers()

    def do_DELETE(self):
        self.store.pop(self.path, None)
        self.send_response(204)
        self.end_headers()

    def log_message(self, *a):
        pass


def test_s3_storage_roundtrip(tmp_path):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _S3Stub)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        st = backup.S3Storage("AK", "SK", "bkt", "us-east-1", f"http://127.0.0.1:{srv.server_port}")
        src = tmp_path / "a.zip"
        src.write_bytes(b"PK" + os.urandom(1000))
        st.upload(str(src), "demo/a.zip")
        assert st.exists("demo/a.zip") and st.check()
        st.download("demo/a.zip", str(tmp_path / "b.zip"))
        assert (tmp_path / "b.zip").read_bytes() == src.read_bytes()
        st.delete("demo/a.zip")
        assert not st.exists("demo/a.zip")
    finally:
        srv.shutdown()


def test_backup_retention(control, tmp_path):
    clusters.create_cluster({"name": "c", "template": "single-master"})
    c = clusters.get_cluster("c")
    with session_scope() as s:
        st = M.BackupStorage(name="l", type="LOCAL", credentials={"path": str(tmp_path / "bk")})
        s.add(st)
        s.flush()
        for i in range(5):
            s.add(M.ClusterBackup(name=f"c-{i}.zip", cluster_id=c.id, backup_storage_id=st.id,
                                  date_created=dt.datetime(2026, 1, 1 + i)))
    removed = backup.apply_retention(c.id, 2)
    assert len(removed) == 3
    with session_scope() as s:
        assert sorted(b.name for b in s.query(M.ClusterBackup)) == ["c-3.zip", "c-4.zip"]


# ------------------------------------------------------------------------------------------------ monitor
class _K8s:
    def get(self, path, params=None):
        if path == "/api/v1/nodes":
            return {"items": [{"metadata": {"name": "w1"}, "status": {
                "addresses": [{"type": "InternalIP", "address": "10.0.0.2"}],
                "allocatable": {"amd.com/gpu": "8"}, "capacity": {"amd.com/gpu": "8"},
                "conditions": [{"type": "Ready", "status": "True"}], "nodeInfo": {"kubeletVersion": "v1.30.6"}}}]}
        if path == "/api/v1/pods":
            return {"items": [{"metadata": {"name": "p1", "namespace": "default"},
                               "status": {"phase": "Failed", "containerStatuses": [{"restartCount": 3}]}}]}
        if path == "/api/v1/namespaces":
            return {"items": [{"metadata": {"name": "default"}, "status": {"phase": "Active"}}]}
        if path in ("/apis/apps/v1/deployments", "/apis/apps/v1/daemonsets"):
            return {"items": [{"kind": "Deployment", "metadata": {"name": "train", "namespace": "ml"},
                               "spec": {"template": {"spec": {"containers": [{
                                   "name": "trainer", "image": "kop/train:latest",
                                   "resources": {"requests": {"amd.com/gpu": 8}}}]}}}}]}
        if path == "/api/v1/events":
            return {"items": [{"metadata": {"uid": "e1", "namespace": "ml"}, "type": "Warning", "reason": "OOMKilled",
                               "message": "container trainer OOM", "involvedObject": {"kind": "Pod", "name": "p1"},
                               "lastTimestamp": "2026-10-15T01:00:00Z"}]}
        if path == "/api/v1/componentstatuses":
            return {"items": []}
        return {}


class _Prom:
    def scalar(self, q, default=0.0):
        if "gpu_ecc_uncorrect_total" in q:
            return 2.0
        if "gpu_health" in q or "gpu_junction_temperature" in q:
            return 0.0
        if "gpu_gfx_activity" in q and q.startswith("avg"):
            return 87.0
        if "count(gpu_gfx_activity" in q:
            return 8
        if "mem" in q.lower():
            return 0.5
        return 0.25


def test_monitor_with_stub_clients(control):
    clusters.create_cluster({"name": "mon", "template": "single-master"})
    monitor.set_clients("mon", k8s=_K8s(), prom=_Prom())
    d = monitor.set_cluster_data("mon")
    assert d["gpu_total"] == 8 and d["gpu_allocatable"] == 8
    assert d["nodes"][0]["gpu_util"] == pytest.approx(0.87) and d["nodes"][0]["gpu_count"] == 8
    assert d["error_pods"][0]["name"] == "p1" and d["restart_pods"]
    assert monitor.get_cluster_data("mon")["name"] == "mon"
    assert monitor.save_events("mon") == 1
    assert monitor.save_events("mon") == 0  # dedup by uid
    ev = monitor.search_events("mon", type_="Warning")
    assert ev["total"] == 1 and ev["items"][0]["reason"] == "OOMKilled"
    with session_scope() as s:
        assert s.query(M.Message).filter(M.Message.level == "WARNING").count() >= 1
    h = monitor.cluster_health("mon")
    assert h["available_rate"] == pytest.approx(25.0)
    g = monitor.grade("mon")
    ids = {r["id"] for r in g["results"][0]["results"] if not r["success"]}
    assert {"tagNotSpecified", "gpuLimitMissing", "livenessProbeMissing"} <= ids
    cond = monitor.gpu_condition(_K8s().get("/api/v1/nodes")["items"][0], _Prom())
    assert cond["type"] == "AMDGPUHealthy" and cond["status"] == "False" and "ECC" in cond["message"]
    ok = monitor.gpu_condition(_K8s().get("/api/v1/nodes")["items"][0], None)
    assert ok["status"] == "True"
    monitor.record_availability("mon", 99.0)
    assert monitor.availability_history(clusters.get_cluster("mon").id)[0]["available_rate"] == 99.0


def test_monitoring_content_matches_exported_metrics():
    """Grafana dashboards, alert rules and the NPD GPU monitor shipped by the cluster-addon role: valid JSON /
    YAML, and every training series they query is one the training chart's exporter defines."""
    import json
    import re

    import yaml

    from kubeoperator_amd.control.domain.plan import PLAYBOOK_DIR
    from kubeoperator_amd.control.engine.templating import render_text

    role = os.path.join(PLAYBOOK_DIR, "roles", "cluster-addon")
    src = open(os.path.join(os.path.dirname(PLAYBOOK_DIR), "..", "..", "train", "metrics.py")).read()
    exported = set(re.findall(r'"(kop_train_[a-z_]+)"', src))
    queried = set()
    for name in ("amd-gpu.json", "training.json", "cluster.json"):
        d = json.load(open(os.path.join(role, "files", "dashboards", name)))
        assert d["uid"].startswith("kop-") and d["panels"]
        for p in d["panels"]:
            for t in p["targets"]:
                queried |= set(re.findall(r"kop_train_[a-z_]+", t["expr"]))
    vals = yaml.safe_load(render_text(open(os.path.join(role, "templates", "prometheus-values.yaml.j2")).read(),
                                      {"prometheus_retention_days": 7, "APP_DOMAIN": "apps.example"}))
    rules = [r for g in vals["serverFiles"]["alerting_rules.yml"]["groups"] for r in g["rules"]]
    names = {r["alert"] for r in rules}
    assert {"TargetDown", "ContainerMemoryHigh", "GPUUncorrectableECC", "GPUUnhealthy", "TrainingStalled"} <= names
    for r in rules:
        queried |= set(re.findall(r"kop_train_[a-z_]+", r["expr"]))
    assert "{{ $labels" in open(os.path.join(role, "templates", "prometheus-values.yaml.j2")).read().replace(
        "{% raw %}", "")
    exported_series = exported | {f"{m}_total" for m in exported}
    assert queried and queried <= exported_series, queried - exported_series
    npd = yaml.safe_load(render_text(open(os.path.join(role, "templates", "npd-values.yaml.j2")).read(), {}))
    mon = json.loads(npd["settings"]["custom_monitor_definitions"]["amdgpu-monitor.json"])
    assert mon["conditions"][0]["type"] == "AMDGPUProblem"
    for rule in mon["rules"]:
        re.compile(rule["pattern"])
    assert re.search(mon["rules"][0]["pattern"], "[drm:amdgpu_job_timedout [amdgpu]] *ERROR* ring gfx_0.0.0 timeout")


# ------------------------------------------------------------------------------------------- cloud APIs
class _CloudStub(http.server.BaseHTTPRequestHandler):
    """Just enough of Keystone v3 / Nova / Neutron / Cinder / Glance v2 and the vCenter REST API."""
    uploads: dict = {}

    def _send(self, code, body=None, headers=None):
        data = json.dumps(body).encode() if body is not None else b""
        self.send_response(code)
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def do_POST(self):
        base = f"http://127.0.0.1:{self.server.server_port}"
        p = self.path.split("?")[0]
        self._body()
        if p == "/identity/v3/auth/tokens":
            cat = [{"type": t, "endpoints": [{"interface": "public", "region": "RegionOne", "url": f"{base}/{u}"}]}
                   for t, u in (("compute", "compute"), ("network", "network"), ("volumev3", "volume"),
                                ("image", "image"))]
            return self._send(201, {"token": {"catalog": cat}}, {"X-Subject-Token": "tok-1"})
        if p == "/image/v2/images":
            return self._send(201, {"id": "img-1", "status": "queued"})
        if p == "/api/session":
            return self._send(201, "sess-1")
        if p == "/api/content/local-library":
            return self._send(201, "lib-1")
        if p == "/api/content/library/item":
            return self._send(201, "item-1")
        if p == "/api/content/library/item/update-session":
            return self._send(201, "us-1")
        if p == "/api/content/library/item/update-session/us-1/file":
            return self._send(200, {"upload_endpoint": {"uri": f"{base}/upload/item-1"}})
        if p == "/api/content/library/item/update-session/us-1":
            return self._send(204)
        self._send(404, {"path": p})

    def do_PUT(self):
        _CloudStub.uploads[self.path] = len(self._body())
        self._send(204)

    def do_GET(self):
        p = self.path.split("?")[0]
        hdr = self.headers
        if p.startswith(("/compute", "/network", "/volume", "/image", "/identity")) and hdr.get("X-Auth-Token") != "tok-1":
            return self._send(401, {})
        if p.startswith("/api/") and hdr.get("vmware-api-session-id") != "sess-1":
            return self._send(401, {})
        table = {
            "/identity/v3/regions": {"regions": [{"id": "RegionOne"}]},
            "/compute/os-availability-zone": {"availabilityZoneInfo": [{"zoneName": "nova",
                                                                        "zoneState": {"available": True}}]},
            "/compute/flavors/detail": {"flavors": [{"id": "1", "name": "m1.small", "vcpus": 2, "ram": 4096, "disk": 40},
                                                    {"id": "2", "name": "gpu.8x", "vcpus": 128, "ram": 2097152,
                                                     "disk": 960}]},
            "/network/v2.0/networks": {"networks": [{"id": "n1", "name": "private"},
                                                    {"id": "n2", "name": "public", "router:external": True}]},
            "/network/v2.0/subnets": {"subnets": [{"id": "s1", "network_id": "n1", "cidr": "10.0.0.0/24"}]},
            "/network/v2.0/security-groups": {"security_groups": [{"name": "default"}]},
            "/volume/types": {"volume_types": [{"id": "v1", "name": "ssd"}]},
            "/image/v2/images": {"images": []},
            "/api/vcenter/datacenter": [{"datacenter": "datacenter-1", "name": "dc1"}],
            "/api/vcenter/network": [{"name": "VM Network"}],
            "/api/vcenter/datastore": [{"datastore": "ds-1", "name": "ds1", "free_space": 10 ** 12, "type": "VMFS"}],
            "/api/vcenter/cluster": [{"cluster": "domain-c1", "name": "gpu-cluster"}],
            "/api/vcenter/resource-pool": [{"name": "Resources"}],
            "/api/content/library": [],
            "/api/content/library/item": [],
        }
        if p in table:
            return self._send(200, table[p])
        self._send(404, {"path": p})

    def log_message(self, *a):
        pass


def test_openstack_and_vsphere_rest_clients(tmp_path):
    from kubeoperator_amd.control.domain import cloud_clients as cc

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _CloudStub)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_port}"
    img = tmp_path / "node.qcow2"
    img.write_bytes(b"Q" * 4096)
    try:
        os_ = cc.OpenStackClient({"auth_url": f"{base}/identity/v3", "user_name": "u", "password": "p",
                                  "project_name": "kube"}, region="RegionOne")
        assert os_.list_regions() == ["RegionOne"]
        (z,) = os_.list_zones()
        assert z["cluster"] == "nova" and [n["name"] for n in z["networkList"]] == ["private"]
        assert [n["name"] for n in z["floatingNetworkList"]] == ["public"] and z["securityGroups"] == ["default"]
        assert z["networkList"][0]["subnetList"][0]["cidr"] == "10.0.0.0/24" and z["storages"][0]["name"] == "ssd"
        assert [f["name"] for f in os_.get_flavors()] == ["gpu.8x"]  # >= 4C / 8G / 60G only
        assert os_.create_image("node", str(img)) == "img-1"
        assert _CloudStub.uploads["/image/v2/images/img-1/file"] == 4096
        vc = cc.VSphereClient({"vc_host": "127.0.0.1", "vc_port": srv.server_port, "vc_scheme": "http",
                               "vc_username": "administrator", "vc_password": "pw"})
        assert vc.list_regions() == ["dc1"]
        (vz,) = vc.list_zones("dc1")
        assert vz == {"cluster": "gpu-cluster", "networks": ["VM Network"], "resourcePools": ["Resources"],
                      "storages": [{"name": "ds1", "free": 10 ** 12, "type": "VMFS"}]}
        assert vc.create_image("node", str(img), "ds1") == "item-1"
        assert _CloudStub.uploads["/upload/item-1"] == 4096
        with pytest.raises(cc.CloudError):
            cc.OpenStackClient({"auth_url": f"{base}/nope", "user_name": "u", "password": "p", "project_name": "k"})
    finally:
        srv.shutdown()


def test_zone_create_imports_image_through_the_cloud_api(control, tmp_path):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _CloudStub)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    img = tmp_path / "node.qcow2"
    img.write_bytes(b"Q" * 100)
    try:
        with session_scope() as s:
            reg = M.Region(name="os1", cloud_region="RegionOne", vars={
                "provider": "openstack", "auth_url": f"http://127.0.0.1:{srv.server_port}/identity/v3",
                "user_name": "u", "password": "p", "project_name": "kube", "image_name": "node",
                "image_path": str(img)})
            s.add(reg)
            s.flush()
            z = M.Zone(name="z1", region_id=reg.id, vars={"ip_start": "10.0.0.10", "ip_end": "10.0.0.20"})
            off = M.Zone(name="z2", region_id=reg.id)
            s.add_all([z, off])
            s.flush()
            zid = z.id
        cloud.on_zone_create(zid, run="inline")
        with session_scope() as s:
            z = s.get(M.Zone, zid)
            assert z.status == "READY" and z.vars["image_id"] == "img-1"
        assert [r["cluster"] for r in cloud.list_zones_from_cloud(
            {"provider": "openstack", "auth_url": f"http://127.0.0.1:{srv.server_port}/identity/v3", "user_name": "u",
             "password": "p", "project_name": "kube"}, "RegionOne")] == ["nova"]
    finally:
        srv.shutdown()


# ------------------------------------------------------------------------------------------------ LDAP
def _ldap_server(directory: dict):
    """A tiny LDAPv3 server (simple bind + subtree search with and / or / not / equality / presence /
    initial-substring filters) speaking BER through the client's own codec."""
    import socket as so

    from kubeoperator_amd.control.domain import ldap_client as lc

    def match(f, attrs):
        tag, val, _ = lc.decode(f)
        kids = [bytes([t]) + lc._len(len(v)) + v for t, v in lc.children(val)] if tag in (0xA0, 0xA1, 0xA2) else []
        if tag == 0xA0:
            return all(match(k, attrs) for k in kids)
        if tag == 0xA1:
            return any(match(k, attrs) for k in kids)
        if tag == 0xA2:
            return not match(kids[0], attrs)
        if tag == 0x87:
            return val.decode().lower() in attrs
        a, v = [x for _, x in lc.children(val)][:2]
        vals = [x.lower() for x in attrs.get(a.decode().lower(), [])]
        if tag == 0xA3:
            return v.decode().lower() in vals
        if tag == 0xA4:
            init = [x for t, x in lc.children(v) if t == 0x80]
            return any(x.startswith(init[0].decode().lower()) for x in vals) if init else bool(vals)
        return False

    def handle(c):
        buf = b""
        while True:
            data = c.recv(65536)
            if not data:
                return
            buf += data
            while buf:
                try:
                    _, msg, end = lc.decode(buf)
                except IndexError:
                    break
                if end > len(buf):
                    break
                buf = buf[end:]
                (_, mid), (op, body) = lc.children(msg)[:2]
                mid = lc.as_int(mid)
                if op == 0x60:
                    _, dn, pw = [v for _, v in lc.children(body)][:3]
                    ok = directory.get(dn.decode(), {}).get("_pw") == pw.decode()
                    res = lc.seq(lc.ber_int(0 if ok else 49, 0x0A), lc.ber_str(""), lc.ber_str("" if ok else "bad"), tag=0x61)
                    c.sendall(lc.seq(lc.ber_int(mid), res))
                elif op == 0x63:
                    parts = lc.children(body)
                    base = parts[0][1].decode()
                    f = bytes([parts[6][0]]) + lc._len(len(parts[6][1])) + parts[6][1]
                    want = [v.decode() for _, v in lc.children(parts[7][1])]
                    for dn, ent in directory.items():
                        attrs = {k.lower(): v for k, v in ent.items() if k != "_pw"}
                        if dn.endswith(base) and match(f, attrs):
                            al = [lc.seq(lc.ber_str(k), lc.seq(*[lc.ber_str(x) for x in attrs.get(k.lower(), [])],
                                                               tag=0x31)) for k in want if k.lower() in attrs]
                            c.sendall(lc.seq(lc.ber_int(mid), lc.seq(lc.ber_str(dn), lc.seq(*al), tag=0x64)))
                    c.sendall(lc.seq(lc.ber_int(mid), lc.seq(lc.ber_int(0, 0x0A), lc.ber_str(""), lc.ber_str(""),
                                                             tag=0x65)))
                elif op == 0x42:
                    c.close()
                    return

    srv = so.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(8)

    def loop():
        while True:
            try:
                c, _ = srv.accept()
            except OSError:
                return
            threading.Thread(target=handle, args=(c,), daemon=True).start()

    threading.Thread(target=loop, daemon=True).start()
    return srv


def test_ldap_login_and_sync_with_builtin_client(control):
    """LDAP login (service bind, search with an escaped user name, user bind) and sync through the
    control plane's own LDAPv3 client (no ldap3 on the controller image)."""
    from kubeoperator_amd.control.domain import context, ldap_client, users

    assert ldap_client.encode_filter("(uid=alice)") == bytes.fromhex("a30c04037569640405616c696365")
    people = "ou=people,dc=ex,dc=org"
    srv = _ldap_server({
        "cn=admin,dc=ex,dc=org": {"_pw": "adminpw"},
        f"uid=alice,{people}": {"_pw": "alicepw", "uid": ["alice"], "mail": ["alice@ex.org"], "objectClass": ["person"]},
        f"uid=bob,{people}": {"_pw": "bobpw", "uid": ["bob"], "mail": ["bob@ex.org"], "objectClass": ["inetOrgPerson"]},
    })
    try:
        context.set_settings({"AUTH_LDAP_ENABLE": "true", "AUTH_LDAP_SERVER_URI": f"ldap://127.0.0.1:{srv.getsockname()[1]}",
                              "AUTH_LDAP_BIND_DN": "cn=admin,dc=ex,dc=org", "AUTH_LDAP_BIND_PASSWORD": "adminpw",
                              "AUTH_LDAP_SEARCH_OU": f"ou=nobody,dc=ex,dc=org|{people}",
                              "AUTH_LDAP_SEARCH_FILTER": "(&(objectClass=*)(uid=%(user)s))"}, tab="ldap")
        tok = users.authenticate("alice", "alicepw")
        assert tok["token"] and tok["user"]["username"] == "alice"
        with session_scope() as s:
            u = s.query(M.User).filter_by(username="alice").one()
            assert u.source == "ldap" and u.email == "alice@ex.org"
        with pytest.raises(users.AuthError):
            users.authenticate("alice", "wrong")
        with pytest.raises(users.AuthError):
            users.authenticate("*)(uid=*", "x")  # escaped: matches nobody
        assert users.sync_ldap_users() == 1  # bob (alice exists already)
        with session_scope() as s:
            assert s.query(M.User).filter_by(username="bob", source="ldap").count() == 1
    finally:
        srv.close()


def test_ldap_login_refuses_an_ambiguous_search(control):
    """Two entries match the user name (one per search base): the login is refused rather than binding as
    whichever DN the server returns first (django-auth-ldap behaviour, which the reference builds on)."""
    from kubeoperator_amd.control.domain import context, users

    srv = _ldap_server({
        "cn=admin,dc=ex,dc=org": {"_pw": "adminpw"},
        "uid=carol,ou=people,dc=ex,dc=org": {"_pw": "pw1", "uid": ["carol"], "objectClass": ["person"]},
        "uid=carol,ou=staff,dc=ex,dc=org": {"_pw": "pw2", "uid": ["carol"], "objectClass": ["person"]},
    })
    try:
        context.set_settings({"AUTH_LDAP_ENABLE": "true", "AUTH_LDAP_SERVER_URI": f"ldap://127.0.0.1:{srv.getsockname()[1]}",
                              "AUTH_LDAP_BIND_DN": "cn=admin,dc=ex,dc=org", "AUTH_LDAP_BIND_PASSWORD": "adminpw",
                              "AUTH_LDAP_SEARCH_OU": "ou=people,dc=ex,dc=org|ou=staff,dc=ex,dc=org",
                              "AUTH_LDAP_SEARCH_FILTER": "(uid=%(user)s)"}, tab="ldap")
        for pw in ("pw1", "pw2"):
            with pytest.raises(users.AuthError, match="more than one"):
                users.authenticate("carol", pw)
    finally:
        srv.close()
