"""A simulated host farm for CPU-only plumbing runs (BASELINE config #1) and the test-suite.

``SimFarm`` is a :class:`FakeTransport` pre-loaded with rules that answer the commands the provisioning
roles issue the way real Ubuntu 22.04 nodes with kubeadm / containerd / ROCm would: kubeadm init creates
``admin.conf`` (stateful, so re-runs are idempotent), join commands are printed, nodes report Ready,
GPU nodes expose 8 x AMD Instinct MI355X over lspci / kfd topology / rocminfo and ``amd.com/gpu: 8``,
validation pods succeed, etcd snapshots produce an archive that ``fetch`` can pull. Every command is
recorded, so tests assert on the exact command stream; fault injection comes from FakeTransport
(``unreachable``, ``fail_after``, extra rules inserted first).
"""
from __future__ import annotations

import base64
import fnmatch
import json
import os
import re
import shlex
import time

from .transport import CmdResult, FakeTransport

MI355X_BUSES = (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)
MI355X_LSPCI = "\n".join(
    f"{b:02x}:00.0 Processing accelerators [1200]: Advanced Micro Devices, Inc. [AMD/ATI] Device [1002:75a3]"
    for b in MI355X_BUSES)
# the probe's sysfs sections as a node with 8 MI355X shows them (hosts.GPU_PROBE): PCI functions of vendor
# 0x1002 (the GPUs plus a non-GPU function that must be skipped) and the kfd topology (2 CPU nodes, 8 GPUs)
MI355X_SYSFS = "\n".join(
    [f"0000:{b:02x}:00.0 0x120000 0x75a3 {0 if i < 4 else 1}" for i, b in enumerate(MI355X_BUSES)]
    + ["0000:04:00.0 0x060400 0x14a0 0"])
MI355X_KFD = "\n".join(
    ["node 0 cpu_cores_count 64 simd_count 0 gfx_target_version 0 vendor_id 0 device_id 0 location_id 0 domain 0",
     "node 1 cpu_cores_count 64 simd_count 0 gfx_target_version 0 vendor_id 0 device_id 0 location_id 0 domain 0"]
    + [f"node {2 + i} cpu_cores_count 0 simd_count 1024 gfx_target_version 90500 vendor_id 4098 device_id 30115 "
       f"location_id {b << 8} domain 0 local_mem_size {288 * 2 ** 30}" for i, b in enumerate(MI355X_BUSES)])
KUBECONFIG = """apiVersion: v1
kind: Config
clusters:
- cluster: {server: 'https://%s:6443', insecure-skip-tls-verify: true}
  name: kubernetes
contexts:
- context: {cluster: kubernetes, user: kubernetes-admin}
  name: kubernetes-admin@kubernetes
current-context: kubernetes-admin@kubernetes
users:
- name: kubernetes-admin
  user: {token: sim-admin-token}
"""


def _apt_install_args(cmd: str) -> list[str] | None:
    """Package arguments of the apt-get install in a command (the package module's apt branch), or None."""
    m = re.search(r"apt-get install (.*?)(?:;|&&|\|\||$)", cmd)
    if not m:
        return None
    try:
        words = shlex.split(m.group(1))
    except ValueError:
        return None
    return [w for w in words if not w.startswith("-")]


def _upstream3(v: str) -> str:
    """'1:6.14.14.30200000-2204' -> '6.14.14', '7.0.0.70000-17~22.04' -> '7.0.0'."""
    return ".".join(v.split(":", 1)[-1].split("-", 1)[0].split(".")[:3])


def _dkms_probe_sed(v: str) -> str:
    """What upgrade-gpu's version probe pipeline prints for a dpkg version string (its sed, in Python)."""
    v = re.sub(r"^[0-9]+:", "", v)
    return re.sub(r"^([0-9]+(\.[0-9]+)*).*", r"\1", v)


class SimFarm(FakeTransport):
    def __init__(self, gpu_hosts: set | None = None, gpus_per_host: int = 8, latency_s: float = 0.0,
                 state_path: str | None = None):
        super().__init__(latency_s=latency_s)
        self.state_path = state_path  # persist host file systems across processes (kubeopsctl sim mode)
        if state_path and os.path.exists(state_path):
            with open(state_path) as f:
                st = json.load(f)
            self.fs = {h: {p: base64.b64decode(v) for p, v in files.items()} for h, files in st["fs"].items()}
            self._addr = dict(st.get("addr", {}))
        self.gpu_hosts = set(gpu_hosts or ())  # inventory names or addresses of the GPU machines
        self._addr: dict[str, str] = getattr(self, "_addr", {})
        self.gpus_per_host = gpus_per_host
        self.no_pciutils: set = set()  # hosts whose probe has no lspci section (pciutils not installed)
        # AMD GPU stack per host: installed amdgpu-dkms / ROCm versions (None: not installed), amdgpu module
        # holders (a non-zero count makes the upgrade reboot instead of reloading) and the boot counter
        self.gpu_stack: dict[str, dict] = {}
        self.amdgpu_holders = 0
        # Debian package state per host: installed version strings and apt-mark holds
        self.apt_installed: dict[str, dict] = {}
        self.apt_held: dict[str, set] = {}
        self._install_rules()

    # The offline repository's versions of the pinned packages, ascending, as the vendors publish them: AMD's
    # amdgpu-dkms carries epoch 1, rocm-core and the pkgs.k8s.io packages none (tests/test_apt_resolve.py builds
    # real .debs with these strings and resolves the roles' pins with apt-get).
    APT_CATALOG = {
        "amdgpu-dkms": ["1:6.14.14.30200000-2204", "1:6.16.6.30300000-2204"],
        "rocm-core": ["7.0.0.70000-17~22.04", "7.1.0.70100-20~22.04"],
        "kubeadm": ["1.30.6-1.1", "1.31.2-1.1"],
        "kubelet": ["1.30.6-1.1", "1.31.2-1.1"],
        "kubectl": ["1.30.6-1.1", "1.31.2-1.1"],
    }

    BASE_FILES = {
        "/etc/ssh/sshd_config": b"#UseDNS yes\nPermitRootLogin yes\n",
        "/etc/hosts": b"127.0.0.1 localhost\n",
        "/etc/resolv.conf": b"nameserver 127.0.0.53\n",
        "/etc/fstab": b"UUID=0 / ext4 defaults 0 1\n",
        "/etc/exports": b"",
        "/etc/login.defs": b"MAIL_DIR /var/mail\nPASS_MAX_DAYS\t99999\nPASS_MIN_DAYS\t0\nUMASK\t\t022\n",
        "/etc/passwd": b"root:x:0:0:root:/root:/bin/bash\ndaemon:x:1:1:daemon:/usr/sbin:/bin/sh\n",
        "/etc/group": b"root:x:0:\n",
        "/etc/shadow": b"root:*:19000:0:99999:7:::\n",
        "/etc/gshadow": b"root:*::\n",
    }

    def _seed(self, host: str) -> dict:
        fs = self.fs.setdefault(host, {})
        if "/etc/hosts" not in fs:
            fs.update(self.BASE_FILES)
        return fs

    def is_gpu(self, host: str) -> bool:
        return "*" in self.gpu_hosts or host in self.gpu_hosts or self._addr.get(host) in self.gpu_hosts

    def run(self, conn, cmd, timeout=3600, env=None, stdin=None):
        self._addr[conn.name] = conn.address
        self._seed(conn.name)
        try:
            return super().run(conn, cmd, timeout, env, stdin)
        finally:
            self._save()

    def put(self, conn, data, dest, mode=None):
        try:
            return super().put(conn, data, dest, mode)
        finally:
            self._save()

    def _save(self):
        if not self.state_path:
            return
        with self._lock:
            st = {"fs": {h: {p: base64.b64encode(v).decode() for p, v in files.items()} for h, files in self.fs.items()},
                  "addr": self._addr}
            tmp = self.state_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(st, f)
            os.replace(tmp, self.state_path)

    def get(self, conn, src):
        self._seed(conn.name)
        return super().get(conn, src)

    GPU_LABEL = "/etc/kubernetes/.sim-label-gpu"  # the node's kubeoperator.io/gpu=true label (reset drops it)

    def _n_gpu_nodes(self) -> int:
        """Nodes that ``kubectl get nodes -l kubeoperator.io/gpu=true`` lists with GPUs: GPU machines that joined,
        were labelled by the kube-node role and were not reset since."""
        return sum(1 for h, fs in self.fs.items()
                   if self.is_gpu(h) and "/etc/kubernetes/kubelet.conf" in fs and self.GPU_LABEL in fs)

    def _joined(self, workers_only: bool = False) -> int:
        """Machines that joined the simulated cluster (kubelet.conf present); workers hold no admin.conf."""
        return sum(1 for fs in self.fs.values() if "/etc/kubernetes/kubelet.conf" in fs
                   and not (workers_only and "/etc/kubernetes/admin.conf" in fs))

    def _install_rules(self):
        R = self.add_rule

        def stat(host, cmd, fs):
            path = cmd.split("stat -c '%F|%s|%a|%U|%Y' ", 1)[1].split(" ")[0].strip("'\"")
            if path in fs:
                return 0, f"regular file|{len(fs[path])}|600|root|{int(time.time())}", ""
            return 1, "", ""

        def kinit(host, cmd, fs):
            fs["/etc/kubernetes/admin.conf"] = (KUBECONFIG % host).encode()
            fs["/etc/kubernetes/kubelet.conf"] = b"kubelet"
            return 0, "Your Kubernetes control-plane has initialized successfully!", ""

        def kjoin(host, cmd, fs):
            fs["/etc/kubernetes/kubelet.conf"] = b"kubelet"
            if "--control-plane" in cmd:
                fs["/etc/kubernetes/admin.conf"] = (KUBECONFIG % host).encode()
            return 0, "This node has joined the cluster", ""

        def reset(host, cmd, fs):
            for p in list(fs):
                if p.startswith("/etc/kubernetes/"):
                    del fs[p]
            return 0, "", ""

        def label_gpu(host, cmd, fs):
            node = cmd.split("kubectl label node ", 1)[1].split()[0]
            with self._lock:
                self.fs.setdefault(node, {})[self.GPU_LABEL] = b"true"
            return 0, f"node/{node} labeled", ""

        def cat_conf(host, cmd, fs):
            data = fs.get("/etc/kubernetes/admin.conf")
            return (0, data.decode(), "") if data else (1, "", "No such file")

        def gpu_probe(host, cmd, fs):
            if not self.is_gpu(host):
                return 0, "--amd-smi--\n--sysfs--\n--kfd--\n" + MI355X_KFD.split("\n")[0] + "\n", ""
            lspci = "" if host in self.no_pciutils else MI355X_LSPCI + "\n"
            return 0, lspci + "--amd-smi--\n--sysfs--\n" + MI355X_SYSFS + "\n--kfd--\n" + MI355X_KFD + "\n", ""

        def stack(host):
            with self._lock:
                return self.gpu_stack.setdefault(host, {"dkms": None, "rocm": None, "boot": 0})

        def pkg_install(host, cmd, fs):
            """apt-get install as apt resolves it: a "name=<pattern>" argument must match one of the repository's
            version strings of that package WHOLE (epoch included) as a glob, and a held package may not change
            version; otherwise apt's error and status 100. Installed versions are recorded per host."""
            args = _apt_install_args(cmd)
            if args is None:
                return 0, "", ""
            chosen = {}
            for a in args:
                name, _, pat = a.partition("=")
                vers = self.APT_CATALOG.get(name)
                if vers is None:  # a package the catalogue does not model: any name / version installs
                    continue
                hit = [v for v in vers if fnmatch.fnmatchcase(v, pat)] if pat else list(vers)
                if not hit:
                    return 100, "", f"E: Version '{pat}' for '{name}' was not found"
                chosen[name] = hit[-1]  # catalogue order is ascending: apt's candidate is the highest match
            with self._lock:
                inst = self.apt_installed.setdefault(host, {})
                held = self.apt_held.setdefault(host, set())
                for name, v in chosen.items():
                    if name in held and inst.get(name) not in (None, v):
                        return 100, "", ("E: Held packages were changed and -y was used without "
                                         "--allow-change-held-packages.")
                inst.update(chosen)
            if "amdgpu-dkms" in chosen:
                stack(host)["dkms"] = _upstream3(chosen["amdgpu-dkms"])
            if "rocm-core" in chosen:
                stack(host)["rocm"] = _upstream3(chosen["rocm-core"])
            return 0, "", ""

        def apt_mark(host, cmd, fs):
            words = cmd.split()
            op, names = words[1], words[2:]
            with self._lock:
                held = self.apt_held.setdefault(host, set())
                for n in names:
                    (held.add if op == "hold" else held.discard)(n)
            return 0, "".join(f"{n} set on hold.\n" if op == "hold" else f"Canceled hold on {n}.\n" for n in names), ""

        def dkms_version(host, cmd, fs):  # dpkg-query's full version string; the probe strips it with sed
            v = self.apt_installed.get(host, {}).get("amdgpu-dkms")
            if "sed" in cmd:
                return 0, _dkms_probe_sed(v) if v else "none", ""
            return (0, v, "") if v else (1, "", "no packages found matching amdgpu-dkms")

        def rocm_version(host, cmd, fs):
            v = stack(host)["rocm"]
            if "sed" in cmd:
                return 0, v or "none", ""
            return (0, f"{v}-17", "") if v else (1, "", "No such file")

        def reboot(host, cmd, fs):
            stack(host)["boot"] += 1
            return 0, "", ""

        def boot_id(host, cmd, fs):
            return 0, f"00000000-0000-4000-8000-{stack(host)['boot']:012d}", ""

        def snapshot_zip(host, cmd, fs):
            fs["/opt/kubeoperator/backup/cluster-backup.zip"] = b"PK\x05\x06" + b"\x00" * 18
            return 0, "", ""

        def train_log(host, cmd, fs):
            # simulated: shaped like the per-step JSON records rank 0 of the training chart prints
            rec = {"step": 20, "loss": 12.16, "grad_norm": 1.0, "lr": 6e-5, "step_s": 1.645, "tokens_per_s": 19915.5,
                   "tflops_per_gpu": 1025.1}
            return 0, "\n".join([json.dumps(dict(rec, step=10, step_s=1.66)), json.dumps(rec)]), ""

        # order: later add_rule calls win (inserted first), so generic rules go first
        R(r"stat -c", fn=stat)
        R(r"ctr version", stdout="ready")
        R(r"kubectl get --raw=/readyz", stdout="ok")
        R(r"kubeadm init phase upload-certs|--print-join-command.*--control-plane", stdout=(
            "kubeadm join 127.0.0.1:6443 --token sim.token --discovery-token-ca-cert-hash sha256:00 --control-plane "
            "--certificate-key 00"))
        R(r"^kubeadm token create --print-join-command$",
          stdout="kubeadm join 10.0.0.1:6443 --token sim.token --discovery-token-ca-cert-hash sha256:00")
        R(r"^echo \$\(kubeadm token create", stdout=(
            "kubeadm join 10.0.0.1:6443 --token sim.token --discovery-token-ca-cert-hash sha256:00 --control-plane "
            "--certificate-key 00"))
        R(r"^kubeadm init --config", fn=kinit)
        R(r"^kubeadm join", fn=kjoin)
        R(r"kubeadm reset", fn=reset)
        R(r"kubectl get node (\S+) --no-headers",
          fn=lambda h, c, fs: (0, f"{c.split('get node ')[1].split()[0]} Ready worker 1m v1.30.6", ""))
        R(r"get ds \S+ -o jsonpath='\{\.status\.numberReady\}/\{\.status\.desiredNumberScheduled\}'",
          fn=lambda h, c, fs: (0, f"{self._joined()}/{self._joined()}", ""))
        R(r"get deploy \S+ -o jsonpath='\{\.status\.readyReplicas\}'", stdout="2")
        R(r"test-sc-pod -o jsonpath", stdout="Succeeded")
        R(r"is-default-class\}'", stdout="true")
        R(r"get cephcluster rook-ceph -o jsonpath", stdout="Ready/HEALTH_OK")
        R(r"-l app=rook-ceph-osd --no-headers -o name \| wc -l", fn=lambda h, c, fs: (0, str(self._joined(True)), ""))
        R(r"app=rook-ceph-osd-prepare", stdout="Succeeded")
        R(r"\{\.spec\.providerID\}.*grep -c '\^(vsphere|openstack)://'",
          fn=lambda h, c, fs: (0, str(self._joined()), ""))
        R(r"get node \S+ -o jsonpath='\{\.spec\.providerID\}'$", stdout="vsphere://4211aa00-sim")
        R(r"get node \S+ -o jsonpath='\{\.status\.conditions", stdout="True")
        R(r"get apprepositories (\S+) -o jsonpath='\{\.metadata\.name\}'",
          fn=lambda h, c, fs: (0, c.split("get apprepositories ")[1].split()[0], ""))
        R(r"get ingress \S+ -o name --ignore-not-found",
          fn=lambda h, c, fs: (0, "ingress.networking.k8s.io/" + c.split("get ingress ")[1].split()[0], ""))

        def f5_annotate(host, cmd, fs):
            ip = cmd.split("virtual-server.f5.com/ip=", 1)[1].split()[0]
            fs["/sim/f5-virtual-servers"] = fs.get("/sim/f5-virtual-servers", b"") + ip.encode() + b"\n"
            return 0, "annotated", ""

        R(r"annotate ingress .*virtual-server\.f5\.com/ip=", fn=f5_annotate)
        R(r"get ingress -A -o jsonpath=.*loadBalancer",
          fn=lambda h, c, fs: (0, fs.get("/sim/f5-virtual-servers", b"").decode(), ""))
        R(r"^sysctl -n net\.ipv4\.ip_forward net\.bridge\.bridge-nf-call-iptables$", stdout="1\n1")
        R(r"awk -F: '\$3 < \d+ .*/etc/passwd", stdout="daemon\nbin\nsync")
        R(r"get pv -l kubeoperator\.io/storage=local-volume",
          fn=lambda h, c, fs: (0, "Available " * self._joined(True), ""))
        R(r"awk '\$2 != \"Ready\"' \| wc -l", stdout="0")
        R(r"/sys/class/kfd/kfd/topology", fn=lambda h, c, fs: (0, str(self.gpus_per_host if self.is_gpu(h) else 0), ""))
        R(r"rocminfo \| awk", fn=lambda h, c, fs: (0, str(self.gpus_per_host if self.is_gpu(h) else 0), ""))
        R(r"allocatable\.amd", fn=lambda h, c, fs: (0, " ".join([str(self.gpus_per_host)] * self._n_gpu_nodes()) + " ", ""))
        R(r"app=rocminfo-validate -o jsonpath", fn=lambda h, c, fs: (0, "Succeeded " * self._n_gpu_nodes(), ""))
        R(r"kubectl -n kube-system logs", stdout="Marketing Name: AMD Instinct MI355X\n  Name: gfx950")
        R(r"lspci -nn -d 1002:", fn=gpu_probe)
        R(r"cat /etc/kubernetes/admin.conf", fn=cat_conf)
        R(r"kubectl label node \S+ .*kubeoperator\.io/gpu=true", fn=label_gpu)
        R(r"date \+%s", fn=lambda h, c, fs: (0, str(int(time.time())), ""))
        R(r"create token kubeoperator-admin", stdout="sim-sa-token")
        R(r"zip -qr cluster-backup.zip", fn=snapshot_zip)
        R(r"^hostname$", fn=lambda h, c, fs: (0, h, ""))
        R(r"helm version", stdout="v3.15.4+g0")
        R(r"^helm status \S+ -n \S+ -o json", stdout="deployed")
        R(r"kubectl -n \S+ logs -l app.kubernetes.io/instance=", fn=train_log)
        R(r"systemctl is-active", rc=3)
        R(r"apt-get install ", fn=pkg_install)
        R(r"^apt-mark (un)?hold ", fn=apt_mark)
        R(r"dpkg-query -W -f='\$\{Version\}' amdgpu-dkms", fn=dkms_version)
        R(r"^d=\$\( \(dpkg-query", fn=lambda h, c, fs: (
            (0, f"{self.apt_installed[h]['amdgpu-dkms'].split(':', 1)[-1]} {stack(h)['rocm']}", "")
            if stack(h)["dkms"] else (1, "", "not installed")))
        R(r"cat /opt/rocm/\.info/version", fn=rocm_version)
        R(r"awk '\$1 == \"amdgpu\" \{print \$3\}' /proc/modules", fn=lambda h, c, fs: (0, str(self.amdgpu_holders), ""))
        R(r"nohup sh -c 'sleep 2; systemctl reboot'", fn=reboot)
        R(r"^cat /proc/sys/kernel/random/boot_id$", fn=boot_id)
        R(r"get node \S+ -o jsonpath='\{\.status\.allocatable\.amd", stdout="8")
        R(r"get pod rocminfo-upgrade-\S+ -o jsonpath='\{\.status\.phase\}'", stdout="Succeeded")

    def is_sim(self) -> bool:
        return True


def sim_result(rc: int = 0, stdout: str = "") -> CmdResult:
    return CmdResult(rc, stdout, "")
