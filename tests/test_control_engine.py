"""Playbook engine: inventory patterns / variable precedence, templating, free-form args and the
Ansible constructs the provisioning roles use (mirrors the reference's ansible_api tests of
inventory + runner, ansible_api/tests/test_inventory.py / test_runner.py)."""
import os
import textwrap

import pytest

from kubeoperator_amd.control.engine import FakeTransport, Inventory, Runner
from kubeoperator_amd.control.engine.runner import _parse_free_form, _split_top_level
from kubeoperator_amd.control.engine.templating import evaluate, render


def _inv():
    return Inventory.from_dict({
        "hosts": [{"name": "m1", "ip": "10.0.0.1", "vars": {"role": "m"}},
                  {"name": "m2", "ip": "10.0.0.2"},
                  {"name": "w1", "ip": "10.0.0.3", "vars": {"gpu": 8}},
                  {"name": "w2", "ip": "10.0.0.4"}],
        "groups": [{"name": "kube-master", "hosts": ["m1", "m2"], "vars": {"x": "master"}},
                   {"name": "kube-worker", "hosts": ["w1", "w2"], "vars": {"x": "worker"}, "children": ["gpu_nodes"]},
                   {"name": "gpu_nodes", "hosts": ["w1"], "vars": {"x": "gpu"}},
                   {"name": "k8s", "children": ["kube-master", "kube-worker"], "vars": {"x": "k8s", "y": 1}},
                   {"name": "all", "vars": {"y": 0, "z": "all"}}],
    })


def test_inventory_patterns():
    inv = _inv()
    assert inv.match("all") == ["m1", "m2", "w1", "w2"]
    assert inv.match("kube-master:kube-worker") == ["m1", "m2", "w1", "w2"]
    assert inv.match("k8s:!gpu_nodes") == ["m1", "m2", "w2"]
    assert inv.match("kube-worker:&gpu_nodes") == ["w1"]
    assert inv.match("kube-master[0]") == ["m1"]
    assert inv.match("kube-master[1:]") == ["m2"]
    assert inv.match("w*") == ["w1", "w2"]
    assert inv.match("nope") == []


def test_inventory_var_precedence():
    inv = _inv()
    v = inv.host_vars("w1")
    assert v["x"] == "gpu"            # child group (depth 3) beats parent groups
    assert v["y"] == 1                # parent group beats all
    assert v["z"] == "all"
    assert v["gpu"] == 8              # host var
    assert v["ansible_host"] == "10.0.0.3"
    assert set(v["group_names"]) == {"gpu_nodes", "k8s", "kube-worker"}
    assert inv.host_vars("m1")["x"] == "master"
    rt = Inventory.from_dict(inv.to_dict())
    assert rt.match("k8s") == inv.match("k8s") and rt.host_vars("w1")["x"] == "gpu"


def test_templating_filters_and_tests():
    v = {"a": [3, 1, 2], "s": "v1.30.6", "d": {"k": "v"}, "n": None}
    assert render("{{ a | max }}", v) == 3
    assert render("{{ s | regex_replace('^v', '') }}", v) == "1.30.6"
    assert render("{{ n | default('x', true) }}", v) == "x"
    assert render("{{ d | dict2items | map(attribute='key') | list }}", v) == ["k"]
    assert evaluate("s is search('30')", v)
    assert evaluate(["a | length == 3", "d.k == 'v'"], v)
    assert render("prefix-{{ s }}", v) == "prefix-v1.30.6"


def test_free_form_parsing_keeps_jinja_and_quotes():
    assert _split_top_level("a=1 b='x y' c={{ foo | default('a b') }}") == ["a=1", "b='x y'", "c={{ foo | default('a b') }}"]
    assert _parse_free_form("hostname", "name={{ inventory_hostname }}") == {"name": "{{ inventory_hostname }}"}
    assert _parse_free_form("copy", 'dest=/x content="a b"') == {"dest": "/x", "content": "a b"}
    assert _parse_free_form("shell", "echo a=b c")["_raw_params"] == "echo a=b c"


def _play(tmp_path, text, inv=None, transport=None, **kw):
    p = tmp_path / "site.yml"
    p.write_text(textwrap.dedent(text))
    t = transport or FakeTransport()
    r = Runner(inv or _inv(), t, **kw)
    return r.run_playbook(str(p)), t, r


def test_runner_loops_register_when_handlers(tmp_path):
    res, t, _ = _play(tmp_path, """
    - hosts: kube-worker
      gather_facts: false
      handlers:
        - name: restart svc
          shell: "systemctl restart svc"
      tasks:
        - name: loop
          shell: "echo {{ item }}"
          loop: [a, b]
        - name: reg
          shell: "echo hello"
          register: out
        - name: only gpu
          shell: "gpu-only {{ gpu }}"
          when: gpu is defined
        - name: notify
          copy: dest=/etc/svc.conf content="x={{ inventory_hostname }}"
          notify: restart svc
        - set_fact: seen={{ out.rc }}
        - assert:
            that: ["seen | int == 0"]
    """)
    assert res["summary"]["success"]
    w1 = t.commands("w1")
    assert "echo a" in w1 and "echo b" in w1 and "gpu-only 8" in w1
    assert "gpu-only 8" not in " ".join(t.commands("w2"))
    assert t.fs["w1"]["/etc/svc.conf"] == b"x=w1"
    assert "systemctl restart svc" in w1


def test_runner_failure_rescue_ignore_until(tmp_path):
    t = FakeTransport()
    t.add_rule(r"^boom$", rc=1, stderr="bad")
    t.add_rule(r"^flaky$", rc=1, times=2)
    res, t, r = _play(tmp_path, """
    - hosts: kube-master
      gather_facts: false
      tasks:
        - block:
            - shell: boom
          rescue:
            - shell: "echo rescued"
          always:
            - shell: "echo always"
        - shell: boom
          ignore_errors: true
        - shell: flaky
          register: f
          until: f.rc == 0
          retries: 3
          delay: 0
        - shell: "echo after"
    """, transport=t)
    assert res["summary"]["success"], res["summary"]["dark"]
    cmds = t.commands("m1")
    assert cmds.count("flaky") == 3 and "echo rescued" in cmds and "echo always" in cmds and "echo after" in cmds


def test_until_met_does_not_hide_a_failing_command(tmp_path):
    """Ansible semantics: ``until`` ends the retries, but a command that exits non-zero still fails the task
    unless ``failed_when`` says otherwise (the count is printed, then the pipeline fails)."""
    t = FakeTransport()
    t.add_rule(r"^count$", rc=1, stdout="8")
    t.add_rule(r"^count2$", rc=1, stdout="8")
    res, t, _ = _play(tmp_path, """
    - hosts: kube-master
      gather_facts: false
      tasks:
        - shell: count2
          register: c2
          until: c2.stdout | int >= 8
          failed_when: c2.stdout | int < 8
        - shell: count
          register: c
          until: c.stdout | int >= 8
          retries: 2
          delay: 0
        - shell: "echo after"
    """, transport=t)
    assert not res["summary"]["success"]
    assert "echo after" not in t.commands("m1") and t.commands("m1").count("count") == 1


def test_runner_failure_stops_host_and_unreachable(tmp_path):
    t = FakeTransport()
    t.add_rule(r"^boom$", rc=2, hosts=("w1",))
    t.unreachable.add("w2")
    res, t, _ = _play(tmp_path, """
    - hosts: k8s
      gather_facts: false
      tasks:
        - shell: boom
        - shell: "echo next"
    """, transport=t)
    s = res["summary"]
    assert not s["success"]
    assert "w1" in s["dark"] and "w2" in s["dark"]
    assert "echo next" in t.commands("m1") and "echo next" not in t.commands("w1")
    assert res["raw"]["unreachable"].get("w2")


def test_runner_span_trace_nests_and_records_host_status(tmp_path):
    """Execution tracing: playbook -> play -> task spans on the controller track, one host span per
    module run under its task, with the result status; exported as Chrome trace events and a summary."""
    from kubeoperator_amd.control.engine.trace import Tracer, chrome_trace, summary

    t = FakeTransport()
    t.add_rule(r"^boom$", rc=3, hosts=("w1",))
    seen = []
    tr = Tracer(on_host_span=seen.append)
    sid = tr.begin("install", "step")
    res, t, _ = _play(tmp_path, """
    - name: workers
      hosts: kube-worker
      gather_facts: false
      tasks:
        - name: first
          shell: "echo hi"
        - name: boom
          shell: boom
          ignore_errors: true
        - name: skipped on w2
          shell: "echo gpu"
          when: gpu is defined
    """, transport=t, tracer=tr)
    tr.end(sid, "success")
    spans = tr.to_list()
    by = {}
    for s in spans:
        by.setdefault(s["kind"], []).append(s)
    assert [s["name"] for s in by["playbook"]] == ["site.yml"] and by["playbook"][0]["parent"] == sid
    assert [s["name"] for s in by["play"]] == ["workers"] and by["play"][0]["parent"] == by["playbook"][0]["id"]
    assert [s["name"] for s in by["task"]] == ["first", "boom", "skipped on w2"]
    assert all(s["parent"] == by["play"][0]["id"] for s in by["task"])
    hosts = {(s["name"], s["host"]): s for s in by["host"]}
    assert hosts[("boom", "w1")]["status"] == "failed" and hosts[("boom", "w1")]["attrs"]["rc"] == 3
    assert hosts[("boom", "w2")]["status"] in ("ok", "changed")
    assert hosts[("skipped on w2", "w2")]["status"] == "skipped"
    assert all(s["end"] is not None and s["end"] >= s["start"] for s in spans)
    assert len(seen) == len(by["host"]) == 6
    ct = chrome_trace(spans)
    x = [e for e in ct["traceEvents"] if e["ph"] == "X"]
    assert len(x) == len(spans) and {e["tid"] for e in x if e["cat"] == "host"} == {1, 2}
    sm = summary(spans)
    assert sm["steps"][0]["step"] == "install" and sm["steps"][0]["task_count"] == 3
    assert set(sm["steps"][0]["hosts"]) == {"w1", "w2"}


def test_tracer_closes_spans_an_exception_left_open():
    from kubeoperator_amd.control.engine.trace import Tracer

    tr = Tracer()
    with pytest.raises(RuntimeError):
        with tr.span("step", "step"):
            tr.begin("pb", "playbook")
            tr.begin("t", "task")
            raise RuntimeError("x")
    st = {s["kind"]: s["status"] for s in tr.to_list()}
    assert st == {"step": "error", "playbook": "aborted", "task": "aborted"} and tr.current() is None


def test_runner_delegate_run_once_serial_tags(tmp_path):
    res, t, _ = _play(tmp_path, """
    - hosts: k8s
      gather_facts: false
      serial: 2
      tasks:
        - shell: "echo once"
          run_once: true
        - shell: "echo on-master for {{ inventory_hostname }}"
          delegate_to: "{{ groups['kube-master'][0] }}"
        - shell: "echo tagged"
          tags: [skipme]
    """, skip_tags=["skipme"])
    assert res["summary"]["success"]
    m1 = t.commands("m1")
    assert sum(c == "echo once" for _, c in t.log) == 2  # once per serial batch
    assert "echo on-master for w2" in m1
    assert not any(c == "echo tagged" for _, c in t.log)


def test_roles_defaults_templates_and_include(tmp_path):
    role = tmp_path / "roles" / "demo"
    for d in ("tasks", "defaults", "templates", "handlers"):
        (role / d).mkdir(parents=True)
    (role / "defaults" / "main.yml").write_text("port: 80\nname_suffix: d\n")
    (role / "templates" / "conf.j2").write_text("listen {{ port }} {{ inventory_hostname }}-{{ name_suffix }}\n")
    (role / "tasks" / "main.yml").write_text(
        "- template: src=conf.j2 dest=/etc/demo.conf\n- include_tasks: extra.yml\n")
    (role / "tasks" / "extra.yml").write_text("- shell: 'echo extra {{ port }}'\n")
    res, t, _ = _play(tmp_path, """
    - hosts: gpu_nodes
      gather_facts: false
      roles:
        - role: demo
          vars: {port: 8080}
    """, roles_path=[str(tmp_path / "roles")])
    assert res["summary"]["success"], res["summary"]
    assert t.fs["w1"]["/etc/demo.conf"] == b"listen 8080 w1-d\n"
    assert "echo extra 8080" in t.commands("w1")


def test_role_default_referencing_other_vars_is_expanded(tmp_path):
    """A role default whose value is a template (Ansible's lazy var templating) must be rendered wherever it
    is used: in a template file, a shell command, a hostvars lookup and a dict-valued var."""
    role = tmp_path / "roles" / "rt"
    for d in ("tasks", "defaults", "templates"):
        (role / d).mkdir(parents=True)
    (role / "defaults" / "main.yml").write_text(textwrap.dedent("""
        root: "{{ STORAGE_DIR | default('/var/lib/c') }}"
        state: "{{ root }}/state"
        max_pods: "{{ MAX_PODS | default(110) }}"
        opts: {dir: "{{ state }}", pods: "{{ max_pods }}"}
    """))
    (role / "templates" / "c.conf.j2").write_text("root = \"{{ root }}\"\nstate = \"{{ state }}\"\n"
                                                  "pods = {{ max_pods | int + 1 }}\ndir = {{ opts.dir }}\n")
    (role / "tasks" / "main.yml").write_text(textwrap.dedent("""
        - template: src=c.conf.j2 dest=/etc/c.conf
        - shell: "mkdir -p {{ root }} && echo {{ hostvars[inventory_hostname]['hv'] }}"
    """))
    inv = _inv()
    inv.groups["all"].vars["hv"] = "{{ z }}-{{ STORAGE_DIR }}"
    res, t, _ = _play(tmp_path, """
    - hosts: gpu_nodes
      gather_facts: false
      roles: [rt]
    """, inv=inv, roles_path=[str(tmp_path / "roles")], extra_vars={"STORAGE_DIR": "/data/ctr", "MAX_PODS": 200})
    assert res["summary"]["success"], res["summary"]
    assert t.fs["w1"]["/etc/c.conf"] == b'root = "/data/ctr"\nstate = "/data/ctr/state"\npods = 201\n' \
                                        b'dir = /data/ctr/state\n'
    assert "mkdir -p /data/ctr && echo all-/data/ctr" in t.commands("w1")


def test_templates_are_sandboxed_and_recursion_bounded():
    from kubeoperator_amd.control.engine.templating import TemplateError, render_text

    evil = "{{ cycler.__init__.__globals__.os.popen('echo pwned').read() }}"
    v = {"CLUSTER_CIDR": evil, "a": "{{ b }}", "b": "{{ a }}"}
    for text in (evil, "{{ CLUSTER_CIDR }}", "x {{ ''.__class__.__mro__[1].__subclasses__() }}"):
        with pytest.raises(TemplateError):
            render(text, v)
    with pytest.raises(TemplateError):
        render_text("cidr={{ CLUSTER_CIDR }}\n", v)
    with pytest.raises(TemplateError, match="recursive"):
        render("{{ a }}", v)


def test_connection_secrets_are_not_template_visible(tmp_path):
    """Host passwords / keys reach the transport but never the templating namespace (so a cluster config
    such as ``x: "{{ hostvars['w1'].ansible_ssh_pass }}"`` cannot read them)."""
    inv = _inv()
    inv.hosts["w1"].vars["ansible_ssh_pass"] = "hunter2"
    res, t, r = _play(tmp_path, """
    - hosts: gpu_nodes
      gather_facts: false
      tasks:
        - shell: "echo {{ ansible_ssh_pass | default('hidden') }} {{ hostvars['w1']['ansible_ssh_pass'] | default('hidden') }}"
    """, inv=inv)
    assert res["summary"]["success"], res["summary"]
    assert "echo hidden hidden" in t.commands("w1")
    assert r._conn("w1", {}).password == "hunter2"


def test_adhoc():
    t = FakeTransport()
    t.add_rule(r"uptime", stdout="up 1 day")
    r = Runner(_inv(), t)
    res = r.run_adhoc("kube-master", "shell", "uptime")
    assert res["summary"]["success"]
    assert set(res["raw"]["ok"]) == {"m1", "m2"}


def test_all_bundled_playbooks_parse():
    import yaml

    from kubeoperator_amd.control.domain.plan import PLAYBOOK_DIR
    n = 0
    for root, _, files in os.walk(PLAYBOOK_DIR):
        for f in files:
            if f.endswith((".yml", ".yaml")) and "charts" not in root:
                with open(os.path.join(root, f)) as fh:
                    yaml.safe_load(fh)
                n += 1
    assert n > 40
