"""The provisioning content against REAL tools (VERDICT r4 items 1 / Weak #3-#4).

The SimFarm answers every command with rules, so a rule that accepts what the real tool rejects hides a broken
role (round 4: ``amdgpu-dkms=6.14.14*`` -- apt matches a pin against the whole version string, and AMD's
amdgpu-dkms carries epoch 1, so that pin is "not found" on every Ubuntu node). Here:

* every ``package`` task that the install, upgrade and add-worker plays render for the built-in packages is
  resolved by the container's real ``apt-get`` (2.4) in simulate mode, against a throwaway repository of stub
  ``.deb`` files (``dpkg-deb`` / ``dpkg-scanpackages -m``) that carry the vendors' real version strings -- the
  pinned packages must resolve to the version the package's ``meta.yml`` names;
* every rendered ``shell`` / ``command`` string of those plays and of ``clean.yml`` passes ``bash -n``.

Reference: the kubeasz roles install through real yum and fail the step on a bad command
(``core/resource/kubeasz/roles/gpu-driver/tasks/main.yml:15-22``, ``roles/upgrade-worker/tasks/main.yml:1-20``).
No root, no network: apt runs with every ``Dir::`` option pointed into ``tmp_path``.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

from kubeoperator_amd.control.domain import deploy
from kubeoperator_amd.control.engine.simfarm import SimFarm, _apt_install_args

pytestmark = pytest.mark.skipif(not (shutil.which("apt-get") and shutil.which("dpkg-deb")
                                     and shutil.which("dpkg-scanpackages")), reason="needs apt-get / dpkg tools")

# (package version var in meta.yml, its Debian package) -> the upstream version every pin must land on
_META = {
    "mi355x-k8s": {"amdgpu-dkms": "6.14.14", "rocm-core": "7.0.0", "kubeadm": "1.30.6", "kubelet": "1.30.6",
                   "kubectl": "1.30.6"},
    "mi355x-k8s-next": {"amdgpu-dkms": "6.16.6", "rocm-core": "7.1.0", "kubeadm": "1.31.2", "kubelet": "1.31.2",
                        "kubectl": "1.31.2"},
}


class AptRepo:
    """A file: apt repository of stub packages plus an apt configuration rooted in one directory."""

    def __init__(self, root, packages: dict[str, list[str]]):
        self.root = str(root)
        repo = os.path.join(self.root, "repo")
        for d in ("repo", "build", "state/lists/partial", "cache/archives/partial", "etc/apt.conf.d",
                  "etc/preferences.d", "etc/sources.list.d"):
            os.makedirs(os.path.join(self.root, d), exist_ok=True)
        for name, versions in packages.items():
            for v in versions:
                src = os.path.join(self.root, "build", f"{name}_{v.replace(':', '_')}")
                os.makedirs(os.path.join(src, "DEBIAN"))
                with open(os.path.join(src, "DEBIAN", "control"), "w") as f:
                    f.write(f"Package: {name}\nVersion: {v}\nArchitecture: amd64\nMaintainer: kop <kop@example.com>\n"
                            f"Description: stub of {name}\n")
                subprocess.run(["dpkg-deb", "-b", src, os.path.join(repo, f"{name}_{v.replace(':', '%3a')}_amd64.deb")],
                               check=True, capture_output=True)
        # -m: keep every version of a package in the index (the repository serves the old and the new one)
        idx = subprocess.run(["dpkg-scanpackages", "-m", ".", "/dev/null"], cwd=repo, check=True, capture_output=True)
        with open(os.path.join(repo, "Packages"), "wb") as f:
            f.write(idx.stdout)
        with open(os.path.join(self.root, "etc", "sources.list"), "w") as f:
            f.write(f"deb [trusted=yes] file:{repo} ./\n")
        open(os.path.join(self.root, "state", "status"), "w").close()
        r = self.root
        self.opts = [f"-oDir::State={r}/state", f"-oDir::State::status={r}/state/status", f"-oDir::Cache={r}/cache",
                     f"-oDir::Etc={r}/etc", f"-oDir::Etc::SourceList={r}/etc/sources.list",
                     f"-oDir::Etc::SourceParts={r}/etc/sources.list.d", f"-oDir::Etc::Parts={r}/etc/apt.conf.d",
                     f"-oDir::Etc::Preferences={r}/etc/preferences", f"-oDir::Etc::PreferencesParts={r}/etc/preferences.d",
                     "-oDebug::NoLocking=1", "-oAPT::Architecture=amd64", "-oAPT::Sandbox::User=root"]
        up = subprocess.run(["apt-get", *self.opts, "update"], capture_output=True, text=True)
        assert up.returncode == 0, up.stderr

    def simulate(self, args: list[str]) -> tuple[int, dict[str, str], str]:
        """apt-get -s install: (status, {package: version apt would install}, stderr)."""
        p = subprocess.run(["apt-get", *self.opts, "-s", "install", "-y", "--no-install-recommends", *args],
                           capture_output=True, text=True)
        inst = dict(re.findall(r"^Inst (\S+) \((\S+) ", p.stdout, re.M))
        return p.returncode, inst, p.stderr


def _cluster():
    from kubeoperator_amd.control.domain import clusters, hosts

    for hn, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2"), ("w2", "10.0.0.3")):
        hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
    clusters.create_cluster({"name": "demo", "template": "single-master", "network_plugin": "flannel",
                             "persistent_storage": "local-volume"})
    clusters.add_node("demo", {"name": "m1", "host": "m1", "roles": ["master"]})
    clusters.add_node("demo", {"name": "w1", "host": "w1", "roles": ["worker"]})


def _run_plays(control):
    """install (mi355x-k8s) -> add-worker -> upgrade (mi355x-k8s-next) -> uninstall; the farm's log slice of each."""
    farm = control.farm
    _cluster()
    out = {}
    for key, op, params in (("install", "install", None), ("add-worker", "add-worker", {"host": "w2"}),
                            ("upgrade", "upgrade", {"package": "mi355x-k8s-next"}), ("clean", "uninstall", None)):
        start = len(farm.log)
        e = deploy.create("demo", op, params, run="inline")
        assert e["state"] == "SUCCESS", (op, e["result_summary"].get("dark"))
        out[key] = farm.log[start:]
    return out


def _package_commands(log):
    """Package-module commands (the rendered apt branch), with their argument lists."""
    return [(h, c, _apt_install_args(c)) for h, c in log
            if c.startswith("if command -v apt-get") and "apt-get install" in c]


def test_every_rendered_package_task_resolves_with_real_apt(control, tmp_path):
    logs = _run_plays(control)
    cmds = {k: _package_commands(v) for k, v in logs.items()}
    assert cmds["install"] and cmds["upgrade"] and cmds["add-worker"]
    names = {a.partition("=")[0] for v in cmds.values() for _, _, args in v for a in args}
    pkgs = {n: list(SimFarm.APT_CATALOG.get(n, ["1.0-1"])) for n in names}
    assert {"amdgpu-dkms", "rocm-core", "kubeadm", "kubelet", "kubectl"} <= set(pkgs)
    repo = AptRepo(tmp_path / "apt", pkgs)

    # negative control: the round-4 pin (no epoch) is what real apt rejects
    rc, _, err = repo.simulate(["amdgpu-dkms=6.14.14*"])
    assert rc != 0 and "Version '6.14.14*' for 'amdgpu-dkms' was not found" in err

    seen = set()
    for play, want in (("install", _META["mi355x-k8s"]), ("add-worker", _META["mi355x-k8s"]),
                       ("upgrade", _META["mi355x-k8s-next"])):
        for host, cmd, args in cmds[play]:
            rc, inst, err = repo.simulate(args)
            assert rc == 0, (play, host, args, err)
            for a in args:
                name, _, pat = a.partition("=")
                if not pat:
                    continue
                assert name in want, (play, a)  # every pinned package is one the package meta versions
                got = inst[name]
                # the resolved Debian version's upstream part is the meta.yml version
                assert re.match(re.escape(want[name]) + r"[.-]", got.split(":", 1)[-1]), (play, host, a, got)
                seen.add((play, name))
    assert {("install", "amdgpu-dkms"), ("install", "rocm-core"), ("install", "kubeadm"),
            ("upgrade", "amdgpu-dkms"), ("upgrade", "rocm-core"), ("upgrade", "kubeadm"),
            ("upgrade", "kubelet"), ("add-worker", "kubeadm")} <= seen, seen


def test_every_rendered_shell_command_passes_bash_syntax_check(control):
    logs = _run_plays(control)
    bad = []
    checked = 0
    for play, log in logs.items():
        for host, cmd in log:
            p = subprocess.run(["bash", "-n"], input=cmd, capture_output=True, text=True)
            checked += 1
            if p.returncode != 0:
                bad.append((play, host, cmd[:200], p.stderr.strip()[:200]))
    assert checked > 300
    assert not bad, bad[:5]


def test_simfarm_apt_rejects_what_real_apt_rejects():
    """The farm's apt model follows the resolver: an epoch-less amdgpu-dkms pin is 'not found' (status 100), a
    held package cannot change version, an unheld one can; unknown packages install at any version."""
    from kubeoperator_amd.control.engine.transport import HostConn

    farm = SimFarm(gpu_hosts={"*"})
    c = HostConn(name="w1", address="10.0.0.2")

    def apt(*pkgs):
        return farm.run(c, "DEBIAN_FRONTEND=noninteractive apt-get install -y --no-install-recommends "
                        + " ".join(f"'{p}'" for p in pkgs))

    r = apt("amdgpu-dkms=6.14.14*")
    assert r.rc == 100 and "Version '6.14.14*' for 'amdgpu-dkms' was not found" in r.stderr
    assert apt("amdgpu-dkms=1:6.14.14*", "rocm-core=7.0*", "rocminfo").rc == 0
    assert farm.apt_installed["w1"]["amdgpu-dkms"] == "1:6.14.14.30200000-2204"
    assert farm.gpu_stack["w1"]["dkms"] == "6.14.14" and farm.gpu_stack["w1"]["rocm"] == "7.0.0"
    assert farm.run(c, "apt-mark hold amdgpu-dkms rocm-core").rc == 0
    r = apt("amdgpu-dkms=1:6.16.6*")
    assert r.rc == 100 and "--allow-change-held-packages" in r.stderr
    assert apt("amdgpu-dkms=1:6.14.14*").rc == 0  # same version: nothing changes, the hold does not matter
    assert farm.run(c, "apt-mark unhold amdgpu-dkms").rc == 0
    assert apt("amdgpu-dkms=1:6.16.6*").rc == 0 and farm.gpu_stack["w1"]["dkms"] == "6.16.6"
    assert apt("kubeadm=1.29*").rc == 100
