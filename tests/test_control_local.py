"""Playbook modules against the real local machine (LocalTransport, files under a temp dir): the file
modules' idempotence and change reporting, templates, line/block edits, fetch/slurp/stat, archives,
facts and ad-hoc shell. The fake/sim transports cover the provisioning roles; this covers the module
implementations doing real work."""
import os
import tarfile
import textwrap

from kubeoperator_amd.control.engine import Inventory, Runner
from kubeoperator_amd.control.engine.transport import LocalTransport


def _run(tmp_path, tasks, extra=None):
    inv = Inventory.from_dict({"hosts": [{"name": "localhost", "vars": {"ansible_connection": "local"}}],
                               "groups": [{"name": "nodes", "hosts": ["localhost"]}]})
    pb = tmp_path / "site.yml"
    pb.write_text(textwrap.dedent(tasks))
    (tmp_path / "templates").mkdir(exist_ok=True)
    r = Runner(inv, LocalTransport(), extra_vars={"d": str(tmp_path / "out"), **(extra or {})},
               controller_dir=str(tmp_path / "ctl"))
    return r.run_playbook(str(pb))


def _changed(res, task):
    return res["raw"]["ok"]["localhost"][task].get("changed")


def test_file_copy_template_idempotent(tmp_path):
    (tmp_path / "templates").mkdir()
    (tmp_path / "templates" / "app.conf.j2").write_text("port={{ port }}\nhost={{ inventory_hostname }}\n")
    play = """
    - hosts: nodes
      gather_facts: false
      vars: {port: 6443}
      tasks:
        - name: dir
          file: path={{ d }}/etc state=directory mode=0755
        - name: copy
          copy: dest={{ d }}/etc/a.txt content="hello"
        - name: template
          template: src=app.conf.j2 dest={{ d }}/etc/app.conf
        - name: link
          file: src={{ d }}/etc/a.txt dest={{ d }}/etc/b.txt state=link
    """
    res = _run(tmp_path, play)
    assert res["summary"]["success"], res["summary"]["dark"]
    out = tmp_path / "out" / "etc"
    assert (out / "a.txt").read_text() == "hello"
    assert (out / "app.conf").read_text() == "port=6443\nhost=localhost\n"
    assert os.path.islink(out / "b.txt")
    assert _changed(res, "copy") and _changed(res, "template")
    res2 = _run(tmp_path, play)
    assert res2["summary"]["success"]
    assert not _changed(res2, "copy") and not _changed(res2, "template")


def test_lineinfile_replace_blockinfile(tmp_path):
    cfg = tmp_path / "out" / "sshd_config"
    cfg.parent.mkdir(parents=True)
    cfg.write_text("#UseDNS yes\nPermitRootLogin yes\nPort 22\n")
    res = _run(tmp_path, """
    - hosts: nodes
      gather_facts: false
      tasks:
        - name: usedns
          lineinfile: path={{ d }}/sshd_config regexp='^#?UseDNS' line='UseDNS no'
        - name: port
          replace: path={{ d }}/sshd_config regexp='^Port 22$' replace='Port 2222'
        - name: block
          blockinfile:
            path: "{{ d }}/sshd_config"
            block: |
              Match User kop
                AllowTcpForwarding no
        - name: new line
          lineinfile: path={{ d }}/sshd_config line='MaxSessions 32'
    """)
    assert res["summary"]["success"], res["summary"]["dark"]
    text = cfg.read_text()
    assert "UseDNS no" in text and "#UseDNS" not in text
    assert "Port 2222" in text
    assert "Match User kop" in text and "BEGIN KUBEOPERATOR MANAGED BLOCK" in text
    assert text.rstrip().endswith("MaxSessions 32")


def test_stat_slurp_fetch_shell_register(tmp_path):
    f = tmp_path / "out" / "data.bin"
    f.parent.mkdir(parents=True)
    f.write_bytes(b"\x00\x01payload")
    res = _run(tmp_path, """
    - hosts: nodes
      gather_facts: false
      tasks:
        - stat: path={{ d }}/data.bin
          register: st
        - stat: path={{ d }}/missing
          register: nost
        - slurp: src={{ d }}/data.bin
          register: sl
        - fetch: src={{ d }}/data.bin dest={{ d }}/fetched/ flat=yes
        - shell: "echo $((6 * 7))"
          register: calc
        - assert:
            that:
              - st.stat.exists
              - not nost.stat.exists
              - st.stat.size == 9
              - calc.stdout | int == 42
              - (sl.content | b64decode | length) > 0
    """)
    assert res["summary"]["success"], res["summary"]["dark"]
    assert (tmp_path / "out" / "fetched" / "data.bin").read_bytes() == b"\x00\x01payload"


def test_unarchive_and_setup_facts(tmp_path):
    src = tmp_path / "files"
    src.mkdir()
    (src / "bin").mkdir()
    (src / "bin" / "tool").write_text("#!/bin/sh\necho tool\n")
    with tarfile.open(tmp_path / "tool.tgz", "w:gz") as tf:
        tf.add(src / "bin", arcname="bin")
    res = _run(tmp_path, """
    - hosts: nodes
      gather_facts: true
      tasks:
        - file: path={{ d }}/opt state=directory
        - unarchive: src={{ tgz }} dest={{ d }}/opt remote_src=yes
        - debug: msg="{{ ansible_facts.processor_vcpus | default(ansible_processor_vcpus) }}"
        - assert:
            that: ["ansible_memtotal_mb | int > 0"]
    """, extra={"tgz": str(tmp_path / "tool.tgz")})
    assert res["summary"]["success"], res["summary"]["dark"]
    assert (tmp_path / "out" / "opt" / "bin" / "tool").exists()


def test_ssh_transport_pins_host_keys_and_keys_masters_by_credential(tmp_path):
    """SSH options: trust-on-first-use host keys in a per-host known_hosts file (not disabled checking), and
    a ControlPath that changes with the credential so a master opened with an old password is not reused."""
    import json
    import stat as st

    from kubeoperator_amd.control.engine.transport import HostConn, SSHTransport

    rec = tmp_path / "argv.jsonl"
    fake_ssh = tmp_path / "ssh"
    fake_ssh.write_text("#!/usr/bin/env python3\nimport json, sys\n"
                        f"open({str(rec)!r}, 'a').write(json.dumps(sys.argv[1:]) + '\\n')\n")
    fake_ssh.chmod(fake_ssh.stat().st_mode | st.S_IEXEC)
    t = SSHTransport(control_dir=str(tmp_path / "ctl"), ssh_bin=str(fake_ssh),
                     known_hosts_dir=str(tmp_path / "kh"))
    a = HostConn("n1", "10.1.2.3", 2222, "root", password="old")
    t.run(a, "true")
    t.run(HostConn("n1", "10.1.2.3", 2222, "root", password="new"), "true")
    argvs = [json.loads(line) for line in rec.read_text().splitlines()]

    def opt(argv, key):
        return [argv[i + 1].split("=", 1)[1] for i, x in enumerate(argv) if x == "-o" and
                argv[i + 1].startswith(key + "=")][0]

    assert opt(argvs[0], "StrictHostKeyChecking") == "accept-new"
    assert opt(argvs[0], "UserKnownHostsFile") == str(tmp_path / "kh" / "10.1.2.3_2222")
    assert opt(argvs[0], "ControlPath") != opt(argvs[1], "ControlPath")
    assert "/dev/null" not in " ".join(argvs[0])
    t.forget_host_key(a)  # no file yet: a no-op
