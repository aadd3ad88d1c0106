"""The provisioning content as the hosts receive it, parsed by structure rather than matched by regex (VERDICT r5
Missing #3): after a full install on the SimFarm every file a host received is parsed by type -- TOML (containerd
config.toml, every registry hosts.toml), YAML (manifests, Helm values, the kubeadm configuration), JSON (Grafana
dashboards) -- and the kubeadm / kubelet / kube-proxy documents are checked key by key against the committed schema
(resources/schemas/kubernetes_config_keys.yml). Negative controls: a TOML file with an unclosed table and a kubeadm
configuration with a misspelt key fail the checker, and a template rendering broken TOML fails the install at its
template step. The control-plane unit file passes ``systemd-analyze verify``.

Reference behaviour: the kubeasz roles hand rendered files straight to the tools on the host
(core/resource/kubeasz/roles/kube-master/tasks/main.yml:1-127), which is where a typo surfaced."""
import json
import os
import shutil
import subprocess

import pytest
import tomli
import yaml

from kubeoperator_amd.control.domain import clusters, deploy, hosts
from kubeoperator_amd.control.engine import filecheck

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cluster():
    """1 master (m1) + 1 GPU worker (w1) on the SimFarm of the ``control`` fixture."""
    for hn, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2")):
        hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
    clusters.create_cluster({"name": "demo", "template": "single-master", "network_plugin": "flannel",
                             "persistent_storage": "local-volume"})
    clusters.add_node("demo", {"name": "m1", "host": "m1", "roles": ["master"]})
    clusters.add_node("demo", {"name": "w1", "host": "w1", "roles": ["worker"]})


def _install(control):
    _cluster()
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    return control.farm


def test_every_received_file_parses_by_type(control):
    farm = _install(control)
    kinds = {"toml": 0, "yaml": 0, "json": 0}
    for host, files in farm.fs.items():
        for path, data in files.items():
            if "/charts/" in path and "/templates/" in path:  # Helm templates: Go-template payload, not YAML yet
                continue
            got = filecheck.check(path, data)
            if got:
                kinds[got] += 1
    assert kinds["toml"] >= 2 * 6 and kinds["yaml"] >= 10 and kinds["json"] >= 3, kinds

    # containerd: the structure containerd 1.7 / 2.x reads (CRI plugin, runc with systemd cgroups, config_path hosts)
    for host in ("m1", "w1"):
        cfg = tomli.loads(farm.fs[host]["/etc/containerd/config.toml"].decode())
        assert cfg["version"] == 2 and cfg["root"].startswith("/")
        cri = cfg["plugins"]["io.containerd.grpc.v1.cri"]
        assert cri["sandbox_image"].endswith("/pause:3.9")
        runc = cri["containerd"]["runtimes"]["runc"]
        assert runc["runtime_type"] == "io.containerd.runc.v2" and runc["options"]["SystemdCgroup"] is True
        assert cri["registry"] == {"config_path": "/etc/containerd/certs.d"}
        certs = {p: tomli.loads(d.decode()) for p, d in farm.fs[host].items()
                 if p.startswith("/etc/containerd/certs.d/") and p.endswith("/hosts.toml")}
        assert len(certs) >= 5
        for p, doc in certs.items():
            assert doc["server"].startswith(("http://", "https://")), p
            assert list(doc["host"]) == [doc["server"]] and doc["host"][doc["server"]]["capabilities"] == ["pull", "resolve"]

    # kubeadm: four documents, each a known apiVersion / kind with known keys only
    docs = list(yaml.safe_load_all(farm.fs["m1"]["/etc/kubernetes/kubeadm-config.yaml"].decode()))
    assert [(d["apiVersion"], d["kind"]) for d in docs] == [
        ("kubeadm.k8s.io/v1beta3", "InitConfiguration"), ("kubeadm.k8s.io/v1beta3", "ClusterConfiguration"),
        ("kubelet.config.k8s.io/v1beta1", "KubeletConfiguration"),
        ("kubeproxy.config.k8s.io/v1alpha1", "KubeProxyConfiguration")]
    init, clus, kubelet, proxy = docs
    assert init["localAPIEndpoint"] == {"advertiseAddress": "10.0.0.1", "bindPort": 6443}
    assert init["nodeRegistration"]["criSocket"] == "unix:///run/containerd/containerd.sock"
    assert clus["kubernetesVersion"].startswith("v1.") and "10.0.0.1" in clus["apiServer"]["certSANs"]
    assert kubelet["cgroupDriver"] == "systemd" and isinstance(kubelet["maxPods"], int)
    assert proxy["mode"] in ("ipvs", "iptables")

    for path in ("/opt/kubeoperator/dashboards/amd-gpu.json",):
        assert json.loads(farm.fs["m1"][path])["panels"]


def test_checker_rejects_broken_toml_and_misspelt_kubeadm_key(control):
    farm = _install(control)
    good = farm.fs["w1"]["/etc/containerd/config.toml"].decode()
    assert filecheck.check("/etc/containerd/config.toml", good.encode()) == "toml"
    broken = good.replace('[plugins."io.containerd.grpc.v1.cri".registry]', '[plugins."io.containerd.grpc.v1.cri".registry')
    with pytest.raises(filecheck.FileCheckError, match="config.toml"):
        filecheck.check("/etc/containerd/config.toml", broken.encode())
    kcfg = farm.fs["m1"]["/etc/kubernetes/kubeadm-config.yaml"].decode()
    assert "kubernetesVersion:" in kcfg
    with pytest.raises(filecheck.FileCheckError, match="kubernetesVerison"):
        filecheck.check("/etc/kubernetes/kubeadm-config.yaml", kcfg.replace("kubernetesVersion:", "kubernetesVerison:").encode())
    with pytest.raises(filecheck.FileCheckError, match="nodeRegistration.criSockett"):
        filecheck.check("/x/kubeadm.yaml", kcfg.replace("criSocket:", "criSockett:").encode())
    with pytest.raises(filecheck.FileCheckError, match="unknown kind"):
        filecheck.check("/x/k.yaml", b"apiVersion: kubeadm.k8s.io/v1beta3\nkind: InitConfig\n")
    with pytest.raises(filecheck.FileCheckError):
        filecheck.check("/x/d.json", b'{"panels": [}')
    with pytest.raises(filecheck.FileCheckError):
        filecheck.check("/x/m.yaml", b"a: [1, 2\n")
    assert filecheck.check("/etc/chrony/chrony.conf", b"server x iburst\n") is None  # unstructured: not parsed


def test_broken_template_fails_the_install_at_its_step(control, monkeypatch):
    """End to end: a containerd template that renders an unclosed TOML table fails the install at the template
    step, before any host receives the file."""
    from kubeoperator_amd.control.engine import modules

    real = modules.render_text

    def broken(text, variables):
        out = real(text, variables)
        return out.replace("[plugins.", "[plugins", 1) if "SystemdCgroup" in out else out

    monkeypatch.setattr(modules, "render_text", broken)
    _cluster()
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "FAILURE"
    assert "rendered file does not parse" in json.dumps(e["result_summary"])
    assert not any("/etc/containerd/config.toml" in files for files in control.farm.fs.values())


@pytest.mark.skipif(shutil.which("systemd-analyze") is None, reason="no systemd-analyze")
def test_control_plane_unit_file_verifies():
    r = subprocess.run(["systemd-analyze", "verify", os.path.join(ROOT, "scripts", "kubeops.service")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
