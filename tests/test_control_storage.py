"""Every storage back-end the cluster plan offers (resources/cluster/config.yml ``storages``) installs on the
simulated farm through its own role (reference roles/cluster-storage/tasks/{nfs-client,rook-ceph,external-ceph,
local-volume,vsphere-client,cinder-client}.yml), renders its manifests with no unexpanded Jinja, makes its
StorageClass the default, passes the verification pod, and keeps working through a scale-out (reference
roles/scale/tasks/scale-{ceph,vsan}.yml)."""
import re

import pytest

from kubeoperator_amd.control.domain import clusters, deploy, hosts, plan, storage
from kubeoperator_amd.control.store import models as M
from kubeoperator_amd.control.store.db import session_scope


def _hosts():
    for hn, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2"), ("w2", "10.0.0.3")):
        try:
            hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
        except Exception:
            pass


def _manual(name, storage_name, configs=None):
    _hosts()
    clusters.create_cluster({"name": name, "template": "single-master", "network_plugin": "calico",
                             "persistent_storage": storage_name, "configs": configs or {}})
    clusters.add_node(name, {"name": "m1", "host": "m1", "roles": ["master"]})
    clusters.add_node(name, {"name": "w1", "host": "w1", "roles": ["worker"]})


def _automatic(name, storage_name, region_vars, zone_vars):
    with session_scope() as s:
        r = M.Region(name="r-" + name, cloud_region="dc1", vars={"provider": "fake", **region_vars})
        s.add(r)
        s.flush()
        z = M.Zone(name="z-" + name, region_id=r.id, cloud_zone="cluster-a",
                   vars={"ip_start": "10.1.0.10", "ip_end": "10.1.0.30", "net_mask": "255.255.255.0",
                         "gateway": "10.1.0.1", "provider": "fake", **zone_vars})
        s.add(z)
        s.flush()
        p = M.Plan(name="p-" + name, region_id=r.id, zone_ids=[z.id], deploy_template="SINGLE", vars={})
        s.add(p)
        s.flush()
        pid = p.id
    clusters.create_cluster({"name": name, "template": "single-master", "deploy_type": "AUTOMATIC", "plan": pid,
                             "worker_size": 1, "persistent_storage": storage_name})


def _setup_nfs(name):
    storage.create_nfs({"name": "nfs1", "vars": {"external": True, "storage_nfs_server": "10.0.0.9",
                                                 "storage_nfs_server_path": "/exports"}}, run="none")
    _manual(name, "nfs", {"nfs_storage": "nfs1"})


def _setup_external_ceph(name):
    _manual(name, "external-ceph")
    storage.create_ceph({"name": "ceph1", "vars": {"ceph_cluster_id": "b6f1c2d4-0000-4000-8000-000000000001",
                                                   "ceph_monitors": ["10.0.0.20:6789", "10.0.0.21:6789"],
                                                   "ceph_key": "AQBsecretkey==", "ceph_pool": "kube"}})
    storage.bind_ceph(clusters.get_cluster(name).id, "ceph1")


SETUPS = {
    "nfs": (_setup_nfs, ["nfs.yaml"], "nfs-client-provisioner"),
    "rook-ceph": (lambda n: _manual(n, "rook-ceph"), ["rook/cluster.yaml", "rook/blockpool.yaml"],
                  "helm upgrade --install rook-ceph"),
    "external-ceph": (_setup_external_ceph, ["ceph-csi-values.yaml"], "helm upgrade --install ceph-csi-rbd"),
    "local-volume": (lambda n: _manual(n, "local-volume"), ["local-volume.yaml"], "kubeoperator.io/storage=local-volume"),
    "vSphere DataStore": (lambda n: _automatic(n, "vSphere DataStore",
                                               {"vc_host": "vc.lab", "vc_username": "admin@vsphere.local",
                                                "vc_password": "vc-secret", "datacenter": "dc1"},
                                               {"datastore": "nvme-ds1", "cluster": "cluster-a"}),
                          ["csi-vsphere.conf", "vsphere-sc.yaml"], "vsphere-csi-driver.yaml"),
    "openstack Cinder": (lambda n: _automatic(n, "openstack Cinder",
                                              {"auth_url": "https://keystone.lab:5000/v3", "user_name": "kube",
                                               "password": "os-secret", "project_name": "gpu"},
                                              {"volume_type": "nvme"}),
                         ["cloud.conf", "cinder-sc.yaml"], "helm upgrade --install cinder-csi"),
}


def test_every_plan_storage_has_a_role_and_a_test():
    assert {s["name"] for s in plan.load_plan()["storages"]} == set(SETUPS)


def _files(farm, suffix):
    return {h: fs[p] for h, fs in farm.fs.items() for p in fs if p.endswith(suffix)}


@pytest.mark.parametrize("storage_name", list(SETUPS))
def test_storage_backend_installs(control, storage_name):
    setup, manifests, marker = SETUPS[storage_name]
    name = "st" + re.sub(r"[^a-z0-9]", "", storage_name.lower())[:10]
    setup(name)
    e = deploy.create(name, "install", run="inline")
    assert e["state"] == "SUCCESS", (e["result_summary"].get("dark"), e["result_summary"].get("failed"))
    farm = control.farm
    log = "\n".join(c for _, c in farm.log)
    assert marker in log
    for m in manifests:
        got = _files(farm, "/manifests/storage/" + m)
        assert got, m
        for data in got.values():
            assert not re.search(rb"\{\{\s*[A-Za-z_]|\{%", data), m
    if storage_name != "local-volume":  # local NVMe volumes are scratch, not the default class
        assert "kubectl apply -f /opt/kubeoperator/manifests/test-sc.yaml" in log
        assert "is-default-class" in log
    cfg = clusters.get_cluster(name).configs
    if storage_name in ("vSphere DataStore", "openstack Cinder"):
        # cloud credentials reach the run but are never copied into the stored cluster configs
        assert not any(k in cfg for k in ("vc_password", "password"))
        conf = next(iter(_files(farm, "csi-vsphere.conf" if storage_name.startswith("vSphere") else "cloud.conf").values()))
        assert (b"vc-secret" if storage_name.startswith("vSphere") else b"os-secret") in conf
        kubelet = [c for c in farm.log if "KUBELET_EXTRA_ARGS" in c[1] or "/etc/default/kubelet" in c[1]]
        env = [fs.get("/etc/default/kubelet", b"") for fs in farm.fs.values()]
        assert any(b"--cloud-provider=external" in x for x in env), kubelet
    if storage_name == "external-ceph":
        vals = next(iter(_files(farm, "ceph-csi-values.yaml").values())).decode()
        assert "10.0.0.20:6789" in vals and "AQBsecretkey==" in vals


def test_rook_ceph_scale_out_adds_osd_node(control):
    _manual("rk", "rook-ceph")
    assert deploy.create("rk", "install", run="inline")["state"] == "SUCCESS"
    e = deploy.create("rk", "add-worker", {"host": "w2"}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    new = [n["name"] for n in clusters.list_nodes("rk") if n["name"] not in ("m1", "w1")]
    assert len(new) == 1
    cl = next(iter(_files(control.farm, "/manifests/storage/rook/cluster.yaml").values())).decode()
    assert '- name: "w1"' in cl and f'- name: "{new[0]}"' in cl
    assert any(f"app=rook-ceph-osd-prepare --field-selector spec.nodeName={new[0]}" in c for _, c in control.farm.log)


def test_vsphere_scale_out_sets_disk_uuid_on_new_vms(control):
    SETUPS["vSphere DataStore"][0]("vs")
    assert deploy.create("vs", "install", run="inline")["state"] == "SUCCESS"
    before = sum(1 for _, c in control.farm.log if "vsphere-enable-uuid.sh" in c and c.startswith("bash"))
    e = deploy.create("vs", "scale", {"num": 2}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    after = sum(1 for _, c in control.farm.log if "vsphere-enable-uuid.sh" in c and c.startswith("bash"))
    assert after == before + 1
    assert any("{.spec.providerID}" in c and "worker2" in c for _, c in control.farm.log)


def test_storage_failure_fails_the_install(control):
    """No masking: a storage back-end that does not come up fails the addon step (the reference swallowed
    errors of the rook applies with ignore_errors)."""
    _manual("bad", "rook-ceph")
    control.farm.add_rule(r"helm upgrade --install rook-ceph", rc=1, stderr="chart not found")
    e = deploy.create("bad", "install", run="inline")
    assert e["state"] == "FAILURE"
    assert [s["status"] for s in e["steps"]][-1] == "error"
