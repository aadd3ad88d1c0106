"""Cluster lifecycle on simulated hosts (SimFarm): register hosts with GPU discovery, create a cluster
from a plan template, install -> gpu-validate -> add-worker -> upgrade -> backup -> restore ->
remove-worker -> uninstall, plus failure / resume / busy-lock paths. Mirrors the reference's deploy
state machine (kubeops_api/models/deploy.py:55-230) and its per-step status tracking."""
import os
import re

import pytest

from kubeoperator_amd.control.domain import clusters, deploy, hosts
from kubeoperator_amd.control.store import models as M
from kubeoperator_amd.control.store.db import session_scope


def _cluster(template="single-master", name="demo", workers=("w1",)):
    for hn, ip in (("m1", "10.0.0.1"), ("m2", "10.0.0.4"), ("m3", "10.0.0.5"), ("w1", "10.0.0.2"),
                   ("w2", "10.0.0.3")):
        try:
            hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
        except Exception:
            pass
    clusters.create_cluster({"name": name, "template": template, "network_plugin": "flannel",
                             "persistent_storage": "local-volume"})
    masters = ["m1"] if template == "single-master" else ["m1", "m2", "m3"]
    for m in masters:
        clusters.add_node(name, {"name": m, "host": m, "roles": ["master"]})
    for w in workers:
        clusters.add_node(name, {"name": w, "host": w, "roles": ["worker"]})


def test_host_gpu_discovery(control):
    h = hosts.create_host({"name": "w1", "ip": "10.0.0.2", "password": "pw"})
    assert h["status"] == "RUNNING"
    assert h["gpu_num"] == 8 and h["gpu_info"] == "AMD Instinct MI355X"
    c = hosts.create_host({"name": "m1", "ip": "10.0.0.1", "password": "pw"})
    assert c["gpu_num"] == 0


def test_lspci_parsing():
    text = "\n".join([
        "05:00.0 Processing accelerators [1200]: Advanced Micro Devices, Inc. [AMD/ATI] Device [1002:75a3]",
        "15:00.0 Processing accelerators [1200]: Advanced Micro Devices, Inc. [AMD/ATI] Device [1002:74a1]",
        "65:00.0 VGA compatible controller [0300]: ASPEED Technology, Inc. ASPEED Graphics Family [1a03:2000]",
    ])
    gpus = hosts.parse_lspci_amd(text)
    names = [g["name"] for g in gpus]
    assert names == ["AMD Instinct MI355X", "AMD Instinct MI300X"]


def test_gpu_discovery_without_pciutils_uses_sysfs_and_kfd(control):
    """No lspci on the node: the sysfs PCI scan finds the GPUs, the kfd topology names the architecture."""
    control.farm.no_pciutils.add("w1")
    h = hosts.create_host({"name": "w1", "ip": "10.0.0.2", "password": "pw"})
    assert h["gpu_num"] == 8 and h["gpu_info"] == "AMD Instinct MI355X"
    g = h["gpus"][0]
    assert g["pci"] == "0000:05:00.0" and g["device_id"] == "1002:75a3" and g["arch"] == "gfx950"
    assert g["cu_count"] == 256 and g["numa_node"] == 0 and h["gpus"][-1]["numa_node"] == 1
    assert all(x["pci"] != "0000:04:00.0" for x in h["gpus"])  # the AMD bridge function is not a GPU


def test_kfd_topology_parsing():
    text = "\n".join([
        "node 0 cpu_cores_count 96 simd_count 0 gfx_target_version 0 location_id 0 domain 0",
        "node 1 cpu_cores_count 0 simd_count 1024 gfx_target_version 90500 vendor_id 4098 device_id 30115 "
        "location_id 1280 domain 0 local_mem_size 309237645312",
        "node 2 simd_count 440 gfx_target_version 90010 vendor_id 4098 device_id 29711 location_id 49417 domain 1"])
    agents = hosts.parse_kfd_topology(text)
    assert [a["arch"] for a in agents] == ["gfx950", "gfx90a"]
    assert agents[0]["pci"] == "0000:05:00.0" and agents[0]["device_id"] == "1002:75a3"
    assert agents[1]["pci"] == "0001:c1:01.1"
    assert hosts.gfx_name(90402) == "gfx942"


def test_unknown_device_id_takes_arch_from_kfd():
    probe = ("--amd-smi--\n--sysfs--\n0000:05:00.0 0x120000 0x75b0 0\n--kfd--\n"
             "node 1 simd_count 1024 gfx_target_version 90500 vendor_id 4098 device_id 30128 location_id 1280 domain 0")
    (g,) = hosts.detect_gpus(probe)
    assert g["arch"] == "gfx950" and g["device_id"] == "1002:75b0" and "75b0" in g["name"]


def test_gpu_node_check_runs_only_read_only_tasks(control):
    h = hosts.create_host({"name": "w1", "ip": "10.0.0.2", "password": "pw"})
    r = hosts.check_gpu_node(h["id"])
    assert r["summary"]["success"], r
    assert r["kfd_gpus"] == "8" and r["rocminfo_gpus"] == "8", r["tasks"]
    cmds = control.farm.commands("w1")
    assert not any(c.startswith(("apt-get", "dnf", "modprobe", "udevadm")) or "amdgpu-dkms" in c for c in cmds)


def _upgrade_slice(farm, op):
    start = len(farm.log)
    e = op()
    return e, farm.log[start:]


def _first(log, host, pattern):
    for i, (h, c) in enumerate(log):
        if h == host and re.search(pattern, c):
            return i
    raise AssertionError(f"no {pattern!r} on {host}")


def test_upgrade_moves_the_gpu_pool_to_the_package_versions(control):
    """drain -> device plugin off -> pinned install -> reload -> kfd / rocminfo -> plugin back
    -> validation pod -> uncordon, on the GPU worker only; a no-op for the GPU stack when versions are equal."""
    _cluster()
    farm = control.farm
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    assert farm.gpu_stack["w1"] == {"dkms": "6.14.14", "rocm": "7.0.0", "boot": 0}
    assert "m1" not in farm.gpu_stack  # the control node never gets the GPU stack

    # same package: the Kubernetes part runs, the GPU stack is left alone
    e, log = _upgrade_slice(farm, lambda: deploy.create("demo", "upgrade", {"package": "mi355x-k8s"}, run="inline"))
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    gpu_ops = r"amdgpu-dkms[=-]|rocm-core[=-]|modprobe -r amdgpu|systemctl reboot|kubeoperator\.io/gpu-|rocminfo-w1"
    assert not [c for _, c in log if re.search(gpu_ops, c)]
    assert any(h == "m1" and "kubectl uncordon w1" in c for h, c in log)

    # ROCm 7.0 -> 7.1, amdgpu-dkms 6.14 -> 6.16
    e, log = _upgrade_slice(farm, lambda: deploy.create("demo", "upgrade", {"package": "mi355x-k8s-next"},
                                                        run="inline"))
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert farm.gpu_stack["w1"]["dkms"] == "6.16.6" and farm.gpu_stack["w1"]["rocm"] == "7.1.0"
    order = [
        _first(log, "w1", r"/repository/rocm/apt/7\.1|sources\.list\.d|apt-get update"),  # repository re-run
        _first(log, "m1", r"kubectl drain w1"),
        _first(log, "m1", r"kubectl label node w1 kubeoperator\.io/gpu-$"),
        _first(log, "m1", r"amdgpu-dp-ds --field-selector spec\.nodeName=w1"),
        _first(log, "w1", r"^apt-mark unhold amdgpu-dkms rocm-core$"),
        _first(log, "w1", r"'amdgpu-dkms=1:6\.16\.6\*' 'rocm-core=7\.1\*'"),  # apt pins carry the epoch
        _first(log, "w1", r"^apt-mark hold amdgpu-dkms rocm-core$"),
        _first(log, "w1", r"modprobe -r amdgpu && modprobe amdgpu"),
        _first(log, "w1", r"kfd/topology/nodes/\*/gpu_id"),
        _first(log, "w1", r"rocminfo \| awk"),
        _first(log, "m1", r"kubectl label node w1 kubeoperator\.io/gpu=true"),
        _first(log, "m1", r"kubectl apply -f /opt/kubeoperator/manifests/rocminfo-w1\.yaml"),
        _first(log, "m1", r"get pod rocminfo-upgrade-w1"),
        _first(log, "m1", r"kubectl uncordon w1"),
    ]
    assert order == sorted(order), order
    assert not any(re.search(r"systemctl reboot", c) for _, c in log)  # no holders: reload, not reboot
    assert farm.apt_installed["w1"]["amdgpu-dkms"] == "1:6.16.6.30300000-2204"
    assert {"amdgpu-dkms", "rocm-core", "kubeadm", "kubelet", "kubectl"} <= farm.apt_held["w1"]
    # kubeadm upgrade semantics: each Kubernetes package is released, moved and held again
    for pkg in ("kubeadm", "kubelet"):
        assert (_first(log, "w1", rf"^apt-mark unhold {pkg}\b") < _first(log, "w1", rf"'{pkg}=1\.31\.2\*'")
                < _first(log, "w1", rf"^apt-mark hold {pkg}\b"))
    # masters: no GPU-stack commands at all
    assert not [c for h, c in log if h == "m1" and re.search(r"amdgpu-dkms|rocm-core|modprobe .*amdgpu", c)]
    # the node's apt sources now name the new ROCm and driver repositories
    src = farm.fs["w1"]["/etc/apt/sources.list.d/kubeoperator.list"].decode()
    assert "/rocm/apt/7.1 " in src and "/amdgpu/apt/7.1.70100-1 " in src

    # running it again is a no-op for the GPU stack
    e, log = _upgrade_slice(farm, lambda: deploy.create("demo", "upgrade", {"package": "mi355x-k8s-next"},
                                                        run="inline"))
    assert e["state"] == "SUCCESS" and not [c for _, c in log if re.search(gpu_ops, c)]


def test_gpu_upgrade_reboots_when_the_module_is_held(control):
    _cluster()
    farm = control.farm
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    farm.amdgpu_holders = 3
    e, log = _upgrade_slice(farm, lambda: deploy.create("demo", "upgrade", {"package": "mi355x-k8s-next"},
                                                        run="inline"))
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert farm.gpu_stack["w1"]["boot"] == 1
    assert not any("modprobe -r amdgpu" in c for _, c in log)
    assert _first(log, "w1", r"systemctl reboot") < _first(log, "w1", r"kfd/topology/nodes/\*/gpu_id") \
        < _first(log, "m1", r"kubectl uncordon w1")


def test_gpu_upgrade_reboots_when_the_reload_fails(control):
    """a holder that appears between the refcount read and the unload makes ``modprobe -r`` fail; the
    node reboots instead of staying cordoned without GPUs."""
    _cluster()
    farm = control.farm
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    farm.add_rule(r"^modprobe -r amdgpu && modprobe amdgpu$", rc=1, stderr="modprobe: FATAL: Module amdgpu is in use.")
    e, log = _upgrade_slice(farm, lambda: deploy.create("demo", "upgrade", {"package": "mi355x-k8s-next"},
                                                        run="inline"))
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert farm.gpu_stack["w1"]["boot"] == 1
    assert _first(log, "w1", r"modprobe -r amdgpu") < _first(log, "w1", r"systemctl reboot") \
        < _first(log, "m1", r"kubectl uncordon w1")


def test_full_lifecycle(control):
    _cluster()
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert [s["status"] for s in e["steps"]] == ["success"] * len(e["steps"])
    assert clusters.get_cluster("demo").status == "RUNNING"
    farm = control.farm
    assert any(c.startswith("kubeadm init --config") for c in farm.commands("m1"))
    assert any(c.startswith("kubeadm join") for c in farm.commands("w1"))
    # GPU stack only on GPU nodes
    assert any("amdgpu" in c for c in farm.commands("w1"))
    assert not any("amdgpu-dkms" in c for c in farm.commands("m1"))
    assert "apiVersion" in clusters.fetch_kubeconfig("demo")
    # every templated file and command is fully expanded (role defaults that reference other vars included)
    for h, files in farm.fs.items():
        for path, data in files.items():
            if "/charts/" in path or "/dashboards/" in path:  # Helm charts / Grafana legends are copied verbatim
                continue
            # (Go / Prometheus / Grafana templates -- {{ $labels.x }}, {{ .Values.x }} -- are payload, not Jinja)
            assert not re.search(rb"\{\{\s*[A-Za-z_]|\{%", data), (h, path)
    assert not [c for _, c in farm.log if re.search(r"\{\{\s*[A-Za-z_]|\{%", c)]
    cfg = farm.fs["w1"]["/etc/containerd/config.toml"].decode()
    assert re.search(r'^root = "/[^"{]+"$', cfg, re.M) and 'sandbox_image = "' in cfg
    # GPU repositories only on GPU nodes (a package without a GPU tree must not break apt on the others)
    src_m1 = farm.fs["m1"]["/etc/apt/sources.list.d/kubeoperator.list"].decode()
    src_w1 = farm.fs["w1"]["/etc/apt/sources.list.d/kubeoperator.list"].decode()
    assert "/rocm/" not in src_m1 and "/amdgpu/" not in src_m1
    assert "/rocm/apt/7.0 " in src_w1 and "/amdgpu/apt/7.0.70000-1 " in src_w1
    assert any("/amdgpu/apt/7.0.70000-1/Packages" in c for c in farm.commands("w1"))  # preflight checked the tree
    # registry hosts in the config_path form containerd 2.x requires (no deprecated registry.mirrors table)
    assert 'config_path = "/etc/containerd/certs.d"' in cfg and "registry.mirrors" not in cfg
    hosts = {p: d.decode() for p, d in farm.fs["w1"].items() if p.startswith("/etc/containerd/certs.d/")}
    assert {"/etc/containerd/certs.d/docker.io/hosts.toml", "/etc/containerd/certs.d/registry.k8s.io/hosts.toml"} <= set(hosts)
    for body in hosts.values():
        srv = re.search(r'^server = "(http://[^"]+)"$', body, re.M).group(1)
        assert f'[host."{srv}"]' in body and 'capabilities = ["pull", "resolve"]' in body

    assert deploy.create("demo", "gpu-validate", run="inline")["state"] == "SUCCESS"

    e = deploy.create("demo", "add-worker", {"host": "w2"}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    assert len(clusters.list_nodes("demo")) == 3

    e = deploy.create("demo", "upgrade", {"package": "mi355x-k8s-next"}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    c = clusters.get_cluster("demo")
    assert c.package == "mi355x-k8s-next" and c.configs["kube_version"] == "v1.31.2"

    with session_scope() as s:
        st = M.BackupStorage(name="local", type="LOCAL", credentials={"path": str(control.tmp / "bk")})
        s.add(st)
        s.flush()
        sid = st.id
    e = deploy.create("demo", "backup", {"backupStorageId": sid}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    with session_scope() as s:
        b = s.query(M.ClusterBackup).one()
        bid = b.id
    assert os.listdir(control.tmp / "bk" / "demo")
    e = deploy.create("demo", "restore", {"clusterBackupId": bid}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")

    names = [n["name"] for n in clusters.list_nodes("demo")]
    node = [n for n in names if n not in ("m1", "w1")][0]
    e = deploy.create("demo", "remove-worker", {"node": node}, run="inline")
    assert e["state"] == "SUCCESS"
    assert len(clusters.list_nodes("demo")) == 2

    e = deploy.create("demo", "uninstall", run="inline")
    assert e["state"] == "SUCCESS"
    assert clusters.get_cluster("demo").status == "READY"
    assert "/etc/kubernetes/admin.conf" not in farm.fs["m1"]


def test_multi_master_install(control):
    _cluster(template="multiple-master", name="ha")
    e = deploy.create("ha", "install", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    joins = [h for h in ("m2", "m3") if any("--control-plane" in c for c in control.farm.commands(h))]
    assert joins == ["m2", "m3"]


def test_install_failure_then_resume(control):
    _cluster()
    control.farm.add_rule(r"^kubeadm join", rc=1, stderr="connection refused", times=1)
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "FAILURE"
    st = {s["name"]: s["status"] for s in e["steps"]}
    assert st["master"] == "success" and st["worker"] == "error" and st["addon"] == "pending"
    assert clusters.get_cluster("demo").status == "ERROR"
    n_init = sum(c.startswith("kubeadm init --config") for c in control.farm.commands("m1"))
    e = deploy.create("demo", "install", {"resume": True}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    # resumed run skipped the finished steps: kubeadm init did not run again
    assert sum(c.startswith("kubeadm init --config") for c in control.farm.commands("m1")) == n_init


def test_unreachable_host_fails_install(control):
    _cluster()
    control.farm.unreachable.add("w1")
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "FAILURE"
    assert "w1" in e["result_summary"]["dark"]


def test_busy_cluster_rejects_second_operation(control):
    _cluster()
    deploy.create("demo", "install", run="queue")  # no worker running: stays PENDING
    with pytest.raises(clusters.Conflict):
        deploy.create("demo", "gpu-validate", run="none")
    # an execution that never got a job (client died) does not lock the cluster
    clusters.create_cluster({"name": "demo2", "template": "single-master"})
    deploy.create("demo2", "install", run="none")
    deploy.create("demo2", "gpu-validate", run="none")


def test_unknown_operation(control):
    _cluster()
    with pytest.raises(ValueError):
        deploy.create("demo", "explode", run="none")


def test_app_deploy_nginx_and_training_chart(control):
    """BASELINE config #1 (deploy the nginx chart) and #3/#4 (the bundled PyTorch-ROCm training chart)
    through ``app-deploy`` executions: helm command lines, rendered values, recorded releases, the training
    run's last step record attached to the execution, removal, and input validation."""
    _cluster()
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    e = deploy.create("demo", "app-deploy", {"chart": "nginx", "values": {"replicas": 2, "note": "{{ inventory_hostname }}"}},
                      run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"]
    m1 = control.farm.commands("m1")
    helm = [c for c in m1 if c.startswith("helm upgrade --install nginx /opt/kubeoperator/charts/nginx")]
    assert helm and "-n default --create-namespace" in helm[0] and "--wait --timeout 10m" in helm[0]
    vals = control.farm.fs["m1"]["/opt/kubeoperator/charts/values/nginx.yaml"]
    assert b"replicas: 2" in vals and b"note: '{{ inventory_hostname }}'" in vals  # user data, never templated
    assert "/opt/kubeoperator/charts/nginx/templates/deployment.yaml" in control.farm.fs["m1"]

    e = deploy.create("demo", "app-deploy", {"chart": "pytorch-rocm-train", "release": "llama-8x", "namespace": "train",
                                             "values": {"model": "llama3_8b", "gpusPerNode": 8, "steps": 20},
                                             "wait_job": True}, run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"]
    assert e["result_summary"]["training"]["tokens_per_s"] > 0 and e["result_summary"]["training"]["step"] == 20
    assert any(c.startswith("kubectl -n train wait --for=condition=complete job -l app.kubernetes.io/instance=llama-8x")
               for c in control.farm.commands("m1"))
    apps = {a["release"]: a for a in clusters.list_apps("demo")}
    assert set(apps) == {"nginx", "llama-8x"} and apps["llama-8x"]["training"]["tokens_per_s"] > 0

    # the serving chart (Deployment + Service around kubeoperator_amd.serve.server)
    e = deploy.create("demo", "app-deploy", {"chart": "pytorch-rocm-serve", "release": "llama-serve",
                                             "namespace": "serve", "values": {"maxBatch": 32, "fp8": True}},
                      run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"]
    assert any(c.startswith("helm upgrade --install llama-serve /opt/kubeoperator/charts/pytorch-rocm-serve")
               for c in control.farm.commands("m1"))
    assert b"maxBatch: 32" in control.farm.fs["m1"]["/opt/kubeoperator/charts/values/llama-serve.yaml"]
    assert deploy.create("demo", "app-remove", {"release": "llama-serve", "namespace": "serve"},
                         run="inline")["state"] == "SUCCESS"

    assert deploy.create("demo", "app-remove", {"release": "nginx"}, run="inline")["state"] == "SUCCESS"
    assert [a["release"] for a in clusters.list_apps("demo")] == ["llama-8x"]
    assert clusters.get_cluster("demo").status == "RUNNING"
    for bad in ({"release": "x; rm -rf /"}, {"chart": "../etc"}, {"namespace": "A B"}, {"values": [1]}):
        with pytest.raises(ValueError):
            deploy.create("demo", "app-deploy", bad, run="none")


def test_bigip_config_attaches_virtual_servers(control):
    """F5 BIG-IP (reference roles/f5/tasks/main.yml:1-39): controller with RBAC, readiness poll, then a virtual
    server on every add-on ingress (HTTP annotations; HTTPS: client-SSL TLS patch + server-SSL annotation), and
    the ingresses report the BIG-IP address."""
    _cluster()
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    clusters.set_config("demo", "bigip_url", "https://10.9.9.9")
    clusters.set_config("demo", "public_ip", "10.9.9.100")
    evil = "p w;$(touch /tmp/pwned)'\""
    clusters.set_config("demo", "bigip_password", evil)
    start = len(control.farm.log)
    e = deploy.create("demo", "bigip-config", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    log = [c for _, c in control.farm.log]
    # the credentials reach the secret through 0600 files, never through a shell command line
    assert not [c for c in log[start:] if "touch /tmp/pwned" in c]
    assert any("--from-file=password=/opt/kubeoperator/secrets/bigip/password" in c for c in log[start:])
    ann = [c for c in log if "annotate ingress" in c]
    for name in ("f2c-grafana", "registry-ui", "weave-scope", "kubeapps-plus", "dashboard-kubernetes-dashboard"):
        assert any(f" {name} " in c and "virtual-server.f5.com/ip=10.9.9.100" in c for c in ann), name
    assert any("serverssl=/Common/serverssl" in c and "dashboard" in c for c in ann)
    assert any("patch ingress dashboard-kubernetes-dashboard" in c and "/Common/clientssl" in c for c in log)
    assert any("get deploy k8s-bigip-ctlr" in c for c in log)
    ctlr = control.farm.fs["m1"]["/opt/kubeoperator/manifests/bigip-ctlr.yaml"].decode()
    assert "serviceAccountName: bigip-ctlr" in ctlr and "--bigip-url=https://10.9.9.9" in ctlr
    # without the endpoint the operation refuses (cluster state unchanged: bigip errors are ignored)
    clusters.set_config("demo", "bigip_url", "")
    assert deploy.create("demo", "bigip-config", run="inline")["state"] == "FAILURE"
    assert clusters.get_cluster("demo").status == "RUNNING"


def test_addons_include_weave_scope_and_the_kubeapps_store(control):
    _cluster()
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    log = [c for _, c in control.farm.log]
    assert any("kubectl apply -f /opt/kubeoperator/manifests/weave-scope.yaml" in c for c in log)
    assert any("helm upgrade --install kubeapps-plus kubeoperator/kubeapps" in c for c in log)
    vals = control.farm.fs["m1"]["/opt/kubeoperator/manifests/kubeapps-values.yaml"].decode()
    assert "chartmuseum.kube-operator.svc.cluster.local:8080" in vals and "apps." in vals
    uploads = [c for c in log if "api/charts?force" in c]
    assert {u.split("helm package ")[1].split()[0] for u in uploads} >= {"pytorch-rocm-train", "pytorch-rocm-serve"}


def test_os_hardening_is_opt_in_and_kubernetes_safe(control):
    """OS hardening (reference roles/os-harden, dormant there): off by default; with os_hardening_enabled the
    prepare step writes the sysctl / login / pam / limits / modprobe / audit policy on every node, keeps the
    forwarding and bridge settings Kubernetes needs (checked), and the install still succeeds."""
    _cluster()
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    assert not any("90-kubeoperator-hardening" in p for fs in control.farm.fs.values() for p in fs)
    clusters.set_config("demo", "os_hardening_enabled", True)
    e = deploy.create("demo", "install", run="inline")
    assert e["state"] == "SUCCESS", e["result_summary"].get("dark")
    for h in ("m1", "w1"):
        fs = control.farm.fs[h]
        sysctl = fs["/etc/sysctl.d/90-kubeoperator-hardening.conf"].decode()
        assert "kernel.kptr_restrict = 2" in sysctl and "ip_forward" not in sysctl
        mp = fs["/etc/modprobe.d/kubeoperator-hardening.conf"].decode()
        assert "install cramfs /bin/true" in mp and "amdgpu" not in mp and "squashfs" not in mp
        assert b"-w /etc/kubernetes/ -p wa -k kubernetes" in fs["/etc/audit/rules.d/kubeoperator.rules"]
        assert b"* hard core 0" in fs["/etc/security/limits.d/10-kubeoperator-hardening.conf"]
    cmds = control.farm.commands("w1")
    assert "sysctl -n net.ipv4.ip_forward net.bridge.bridge-nf-call-iptables" in cmds
    assert any(c.startswith("usermod -s /usr/sbin/nologin daemon") for c in cmds)
    assert not any("usermod -s /usr/sbin/nologin root" in c for c in cmds)
    # a node whose forwarding the hardening would break fails the step instead of continuing
    control.farm.add_rule(r"^sysctl -n net\.ipv4\.ip_forward", stdout="0\n1")
    assert deploy.create("demo", "install", run="inline")["state"] == "FAILURE"
