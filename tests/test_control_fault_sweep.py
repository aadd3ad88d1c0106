"""Provisioning fails loudly: replay the install's command stream on the simulated farm, then inject ``rc=1``
ONCE into each distinct shell / command task in turn. The execution must end FAILURE -- unless the task declares
how it handles a failure: ``until`` (the retry absorbs a single failure, so the install must then SUCCEED),
``failed_when`` or ``ignore_errors`` (its own rule; not asserted). A command that fails without failing the
install is a masked failure (the reference's ``| tail`` / ``|| true`` patterns)."""
import threading

from kubeoperator_amd.control.domain import clusters, context, deploy, hosts
from kubeoperator_amd.control.engine import runner as R
from kubeoperator_amd.control.engine.simfarm import SimFarm
from kubeoperator_amd.control.store import db


def _fresh(cfg):
    db.reset_for_tests("sqlite://")  # in-memory: a new empty database per injected run
    db.init_db()
    farm = SimFarm(gpu_hosts={"10.0.0.2"})
    context.set_transport_factory(lambda: farm)
    for hn, ip in (("m1", "10.0.0.1"), ("w1", "10.0.0.2")):
        hosts.create_host({"name": hn, "ip": ip, "password": "pw"})
    clusters.create_cluster({"name": "demo", "template": "single-master", "network_plugin": "flannel",
                             "persistent_storage": "local-volume"})
    clusters.add_node("demo", {"name": "m1", "host": "m1", "roles": ["master"]})
    clusters.add_node("demo", {"name": "w1", "host": "w1", "roles": ["worker"]})
    return farm


def _policy(t: dict) -> str:
    if "failed_when" in t or t.get("ignore_errors"):
        return "own"
    return "retry" if "until" in t else "fail"


def test_every_install_command_failure_fails_the_install(control, monkeypatch):
    cur = threading.local()
    seen: dict[str, dict] = {}  # command -> task of its first occurrence
    orig = R.Runner._execute_once

    def execute_once(self, h, t, mod, raw, v, base):
        if not getattr(cur, "install", False):  # host registration etc. before the install: not swept
            return orig(self, h, t, mod, raw, v, base)
        cur.cmds = []
        try:
            return orig(self, h, t, mod, raw, v, base)
        finally:
            if mod in ("shell", "command") and cur.cmds:
                seen.setdefault(cur.cmds[-1], t)  # the module's own command (after any creates / removes test)
            cur.cmds = None

    monkeypatch.setattr(R.Runner, "_execute_once", execute_once)
    orig_run = SimFarm.run

    def run(self, conn, cmd, *a, **k):
        if getattr(cur, "cmds", None) is not None:
            cur.cmds.append(cmd)
        return orig_run(self, conn, cmd, *a, **k)

    monkeypatch.setattr(SimFarm, "run", run)
    _fresh(control.cfg)
    cur.install = True
    assert deploy.create("demo", "install", run="inline")["state"] == "SUCCESS"
    cur.install = False
    baseline = dict(seen)
    assert len(baseline) > 30
    masked, unexpected = [], []
    for cmd, task in baseline.items():
        pol = _policy(task)
        if pol == "own":
            continue
        farm = _fresh(control.cfg)
        farm.add_rule("^" + __import__("re").escape(cmd) + "$", rc=1, stderr="injected", times=1)
        state = deploy.create("demo", "install", run="inline")["state"]
        if pol == "fail" and state != "FAILURE":
            masked.append((task.get("name"), cmd[:120]))
        if pol == "retry" and state != "SUCCESS":
            unexpected.append((task.get("name"), cmd[:120]))
    assert not masked, f"failures that did not fail the install: {masked}"
    assert not unexpected, f"retried tasks that did not recover from one failure: {unexpected}"
