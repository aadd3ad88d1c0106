"""Host registry: registration with SSH validation, fact gathering, AMD GPU detection, health, bulk import.

Reference: kubeops_api/models/host.py:17-159 (gather_info :96-142, GPU via ``lspci | grep -i nvidia``
:122-131), utils/gpu.py:4-9, serializers/host.py:28-43 (IP unique + SSH ping), host_import.py:12-63
(xlsx import), models/health/host_health.py:9-42.

GPU detection is AMD-first and needs no extra tool on the node: ``lspci -nn -d 1002:`` when pciutils is
there, else ``/sys/bus/pci/devices/*/{vendor,class,device}``; PCI class 0380/0300/0302/1200 rows are matched
against the AMD Instinct device-ID table (MI355X = 1002:75a3 ...). The kfd topology
(``/sys/class/kfd/kfd/topology/nodes/*/properties``) supplies the architecture the ROCm runtime will report
(``gfx_target_version`` 90500 -> gfx950), the CU count and VRAM; ``amd-smi list`` adds GPU indices / UUIDs.
"""
from __future__ import annotations

import csv
import io
import re
import zipfile
from xml.etree import ElementTree as ET

from sqlalchemy import select

from ..engine import Inventory, ResultCallback, Runner
from ..store import models as M
from ..store.db import session_scope
from . import context

# AMD Instinct accelerators by PCI device id (vendor 0x1002): name, architecture, HBM GiB
AMD_INSTINCT = {
    "75a3": ("AMD Instinct MI355X", "gfx950", 288),
    "75a0": ("AMD Instinct MI350X", "gfx950", 288),
    "74a5": ("AMD Instinct MI325X", "gfx942", 256),
    "74a1": ("AMD Instinct MI300X", "gfx942", 192),
    "74a9": ("AMD Instinct MI300X HF", "gfx942", 192),
    "74a2": ("AMD Instinct MI308X", "gfx942", 128),
    "74a0": ("AMD Instinct MI300A", "gfx942", 128),
    "74b5": ("AMD Instinct MI300X VF", "gfx942", 192),
    "740c": ("AMD Instinct MI250X/MI250", "gfx90a", 128),
    "740f": ("AMD Instinct MI210", "gfx90a", 64),
    "738c": ("AMD Instinct MI100", "gfx908", 32),
}

LSPCI_RE = re.compile(r"^(?P<slot>\S+)\s+(?P<cls>[^\[]*)\[(?P<code>[0-9a-fA-F]{4})\]:\s+(?P<desc>.*?)\s*"
                      r"\[1002:(?P<dev>[0-9a-fA-F]{4})\]")


def parse_lspci_amd(text: str) -> list[dict]:
    """Accelerators from ``lspci -nn -d 1002:`` (display / processing-accelerator classes only)."""
    gpus = []
    for line in text.splitlines():
        m = LSPCI_RE.search(line.strip())
        if not m:
            continue
        if m.group("code").lower() not in ("0380", "0300", "0302", "1200"):
            continue  # skip audio / bridges / PSP
        dev = m.group("dev").lower()
        name, arch, vram = AMD_INSTINCT.get(dev, (m.group("desc").strip(), "", 0))
        gpus.append({"name": name, "vendor": "amd", "pci": m.group("slot"), "device_id": f"1002:{dev}",
                     "arch": arch, "vram_gb": vram})
    return gpus


def parse_amd_smi_list(text: str) -> list[dict]:
    """``amd-smi list`` -> [{gpu, bdf, uuid}] (used to cross-check lspci and for the node labeller)."""
    out, cur = [], {}
    for line in text.splitlines():
        line = line.strip()
        m = re.match(r"^GPU:\s*(\d+)", line)
        if m:
            if cur:
                out.append(cur)
            cur = {"gpu": int(m.group(1))}
            continue
        m = re.match(r"^(BDF|UUID|KFD_ID|NODE_ID):\s*(\S+)", line)
        if m and cur is not None:
            cur[m.group(1).lower()] = m.group(2)
    if cur:
        out.append(cur)
    return out


# One shell round trip, four sections. lspci and amd-smi are optional tools; the two sysfs sections are always
# there on a Linux host with the amdgpu driver bound, so a node without pciutils is still discovered.
#   --sysfs--  one line per PCI function of vendor 0x1002: "<bdf> <class> <device> <numa_node>"
#   --kfd--    one line per kfd topology node: "node <id> <key> <value> ..." (the node's properties file)
GPU_PROBE = (
    "(lspci -nn -d 1002: 2>/dev/null || true); echo '--amd-smi--'; (amd-smi list 2>/dev/null || true); "
    "echo '--sysfs--'; for d in /sys/bus/pci/devices/*; do "
    "[ \"$(cat $d/vendor 2>/dev/null)\" = 0x1002 ] && "
    "echo \"${d##*/} $(cat $d/class) $(cat $d/device) $(cat $d/numa_node 2>/dev/null || echo -1)\"; done; "
    "echo '--kfd--'; for n in /sys/class/kfd/kfd/topology/nodes/*; do "
    "[ -f $n/properties ] && echo \"node ${n##*/} $(tr '\\n' ' ' < $n/properties)\"; done; true")

GPU_CLASSES = ("0380", "0300", "0302", "1200")  # display / 3D / processing accelerator; skips audio, PSP, bridges


def parse_sysfs_pci(text: str) -> list[dict]:
    """Accelerators from the ``--sysfs--`` section: ``<bdf> 0x<class24> 0x<device> <numa>`` per AMD function."""
    gpus = []
    for line in text.splitlines():
        parts = line.split()
        if len(parts) < 3 or not parts[1].startswith("0x"):
            continue
        bdf, cls, dev = parts[0], parts[1][2:].rjust(6, "0")[:4].lower(), parts[2].lower().replace("0x", "")
        if cls not in GPU_CLASSES:
            continue
        name, arch, vram = AMD_INSTINCT.get(dev, (f"AMD GPU [1002:{dev}]", "", 0))
        g = {"name": name, "vendor": "amd", "pci": bdf, "device_id": f"1002:{dev}", "arch": arch, "vram_gb": vram}
        if len(parts) > 3 and parts[3].lstrip("-").isdigit() and int(parts[3]) >= 0:
            g["numa_node"] = int(parts[3])
        gpus.append(g)
    return gpus


def gfx_name(target_version: int) -> str:
    """kfd ``gfx_target_version`` (major*10000 + minor*100 + stepping) -> ``gfx950`` / ``gfx942`` / ``gfx90a``."""
    major, minor, step = target_version // 10000, (target_version // 100) % 100, target_version % 100
    return f"gfx{major}{minor:x}{step:x}"


def parse_kfd_topology(text: str) -> list[dict]:
    """GPU agents from the ``--kfd--`` section (CPU nodes have gfx_target_version 0)."""
    out = []
    for line in text.splitlines():
        parts = line.split()
        if len(parts) < 2 or parts[0] != "node":
            continue
        props = {}
        for k, v in zip(parts[2::2], parts[3::2]):
            try:
                props[k] = int(v)
            except ValueError:
                continue
        tv = props.get("gfx_target_version", 0)
        if not tv:
            continue
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        out.append({"node": int(parts[1]), "arch": gfx_name(tv), "vendor_id": props.get("vendor_id", 0),
                    "device_id": f"{props.get('vendor_id', 0):04x}:{props.get('device_id', 0):04x}",
                    "pci": f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}",
                    "simd_count": props.get("simd_count", 0), "cu_count": props.get("simd_count", 0) // 4,
                    "vram_bytes": props.get("local_mem_size", 0)})
    return out


def _same_bdf(a: str, b: str) -> bool:
    """``05:00.0`` (lspci, no domain) matches ``0000:05:00.0`` (sysfs / amd-smi)."""
    a, b = a.lower(), b.lower()
    return a == b or a.endswith(b) or b.endswith(a)


def detect_gpus(probe_stdout: str) -> list[dict]:
    """Merge the probe's sections: lspci rows if pciutils is installed, else sysfs rows; then amd-smi indices /
    UUIDs and the kfd topology's architecture (authoritative: it is what the ROCm runtime will report)."""
    lspci, _, rest = probe_stdout.partition("--amd-smi--")
    smi, _, rest = rest.partition("--sysfs--")
    sysfs, _, kfd = rest.partition("--kfd--")
    gpus = parse_lspci_amd(lspci)
    sys_rows = parse_sysfs_pci(sysfs)
    if not gpus:
        gpus = sys_rows
    else:
        for g in gpus:  # full BDF and NUMA node from sysfs
            for r in sys_rows:
                if _same_bdf(r["pci"], g["pci"]):
                    g["pci"] = r["pci"]
                    if "numa_node" in r:
                        g["numa_node"] = r["numa_node"]
    agents = parse_kfd_topology(kfd)
    for g in gpus:
        for a in agents:
            if _same_bdf(a["pci"], g["pci"]):
                g["arch"] = a["arch"]
                g["kfd_node"] = a["node"]
                g["cu_count"] = a["cu_count"]
                if not g.get("vram_gb") and a["vram_bytes"]:
                    g["vram_gb"] = round(a["vram_bytes"] / 2 ** 30)
        for row in parse_amd_smi_list(smi):
            if _same_bdf(row.get("bdf", ""), g["pci"]):
                g["index"] = row["gpu"]
                g["uuid"] = row.get("uuid", "")
    return gpus


# ------------------------------------------------------------------------------------------- registry
def _conn_inventory(h: M.Host) -> Inventory:
    inv = Inventory()
    user, pw, key = h.username, context.dec(h.password), context.dec(h.private_key)
    if h.credential_id:
        with session_scope() as s:
            c = s.get(M.Credential, h.credential_id)
            if c is not None:
                user, pw, key = c.username, context.dec(c.password), context.dec(c.private_key)
    hv = {"ansible_host": h.ip, "ansible_port": h.port, "ansible_user": user}
    if pw:
        hv["ansible_ssh_pass"] = pw
    if key:
        hv["ansible_ssh_private_key_file"] = key
    inv.add_host(h.name, hv)
    return inv


def create_host(data: dict, gather: bool = True, check_ssh: bool = True) -> dict:
    """Register a host (IP unique, SSH reachable), then gather facts + GPUs."""
    with session_scope() as s:
        if s.scalar(select(M.Host).where(M.Host.ip == data["ip"])) is not None:
            raise ValueError(f"host with ip {data['ip']} already exists")
        if s.scalar(select(M.Host).where(M.Host.name == data["name"])) is not None:
            raise ValueError(f"host {data['name']} already exists")
        h = M.Host(name=data["name"], ip=data["ip"], port=int(data.get("port", 22)),
                   credential_id=data.get("credential") or data.get("credential_id"),
                   username=data.get("username", "root"), password=context.enc(data.get("password", "")),
                   private_key=context.enc(data.get("private_key", "")), zone_id=data.get("zone"),
                   status="CREATING", auto_gather_info=data.get("auto_gather_info", True))
        s.add(h)
        s.flush()
        hid = h.id
    if check_ssh and not test_host(hid):
        with session_scope() as s:
            s.delete(s.get(M.Host, hid))
        raise ValueError(f"host {data['ip']}:{data.get('port', 22)} is not reachable over SSH")
    if gather:
        gather_info(hid)
    return host_dict(hid)


def test_host(host_id: str) -> bool:
    with session_scope() as s:
        h = s.get(M.Host, host_id)
    inv = _conn_inventory(h)
    r = Runner(inv, context.transport(), forks=1, callback=ResultCallback())
    res = r.run_adhoc(h.name, "command", {"_raw_params": "pwd"}, name="ping")
    return bool(res["summary"]["success"])


def gather_info(host_id: str, retry: int = 1) -> dict:
    """Facts (memory, cores, distro, disks) + AMD GPUs (reference Host.gather_info, retry=5 w/ 5 s sleeps)."""
    with session_scope() as s:
        h = s.get(M.Host, host_id)
    inv = _conn_inventory(h)
    facts = {}
    for _ in range(max(1, retry)):
        r = Runner(inv, context.transport(), forks=1, callback=ResultCallback())
        r.run_adhoc(h.name, "setup", {}, name="gather facts")
        facts = r.state[h.name].facts
        if facts.get("ansible_memtotal_mb"):
            break
    r2 = Runner(inv, context.transport(), forks=1, callback=ResultCallback())
    res = r2.run_adhoc(h.name, "shell", {"_raw_params": GPU_PROBE}, name="gpu probe")
    probe = (res["raw"]["ok"].get(h.name, {}).get("gpu probe", {}) or {}).get("stdout", "")
    gpus = detect_gpus(probe)
    with session_scope() as s:
        h = s.get(M.Host, host_id)
        if facts:
            h.memory = int(facts.get("ansible_memtotal_mb", 0))
            h.cpu_core = int(facts.get("ansible_processor_vcpus", 0))
            h.os = facts.get("ansible_distribution", "")
            h.os_version = facts.get("ansible_distribution_version", "")
            h.volumes = [{"name": k, "size": round(v.get("size", 0) / 1024 ** 3)}
                         for k, v in (facts.get("ansible_devices") or {}).items()]
            h.info = {k: facts[k] for k in ("ansible_kernel", "ansible_architecture", "ansible_hostname") if k in facts}
            h.status = "RUNNING"
        else:
            h.status = "UNKNOWN"
        h.gpus = gpus
        h.gpu_vendor = "amd" if gpus else ""
    return host_dict(host_id)


def check_gpu_node(host_id: str, gpu_num: int | None = None) -> dict:
    """Read-only GPU check on a registered host: the ``gpu-check`` tagged tasks of ``amdgpu-driver`` (kfd count)
    and ``rocm-runtime`` (rocminfo agents, amd-smi inventory) through the engine -- no package tasks run.
    Returns the engine summary plus the registered outputs."""
    import os

    from .plan import PLAYBOOK_DIR

    with session_scope() as s:
        h = s.get(M.Host, host_id)
        n = gpu_num if gpu_num is not None else len(h.gpus or []) or 1
    inv = _conn_inventory(h)
    inv.add_group("gpu_nodes", {"gpu_num": n})
    inv.add_host(h.name, groups=["gpu_nodes"])
    cb = ResultCallback()
    r = Runner(inv, context.transport(), forks=1, callback=cb, tags=["gpu-check"])
    res = r.run_playbook(os.path.join(PLAYBOOK_DIR, "gpu-check.yml"))
    ok = res["raw"]["ok"].get(h.name, {})
    out = lambda name: next((str(v.get("stdout", "")).strip() for k, v in ok.items()  # noqa: E731
                             if k.split(" : ")[-1] == name), "")
    return {"summary": res["summary"], "kfd_gpus": out("count bound Instinct devices"),
            "rocminfo_gpus": out("rocminfo sees every GPU agent"), "amd_smi": out("record GPU inventory"),
            "tasks": sorted(ok)}


def host_dict(host_id: str) -> dict:
    with session_scope() as s:
        h = s.get(M.Host, host_id)
        d = h.to_dict(exclude=("password", "private_key"))
    d["has_gpu"] = bool(d.get("gpus"))
    d["gpu_num"] = len(d.get("gpus") or [])
    d["gpu_info"] = ", ".join(sorted({g["name"] for g in d.get("gpus") or []}))
    return d


def host_health_check() -> dict:
    """SSH reachability of every host -> condition + status (reference host_health.py:24-42)."""
    out = {}
    with session_scope() as s:
        ids = [h.id for h in s.scalars(select(M.Host))]
    for hid in ids:
        ok = test_host(hid)
        with session_scope() as s:
            h = s.get(M.Host, hid)
            cond = {"type": "Ready", "status": str(ok), "message": "" if ok else "ssh unreachable",
                    "reason": "" if ok else "HostUnreachable", "last_time": M.now().isoformat()}
            h.conditions = [c for c in (h.conditions or []) if c.get("type") != "Ready"] + [cond]
            if not ok:
                h.status = "UNKNOWN"
            elif h.status == "UNKNOWN":
                h.status = "RUNNING"
            out[h.name] = ok
    return out


# ------------------------------------------------------------------------------------------- import
def _xlsx_rows(data: bytes) -> list[list[str]]:
    """Minimal .xlsx reader (first sheet; shared + inline strings) -- no openpyxl needed."""
    z = zipfile.ZipFile(io.BytesIO(data))
    ns = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
    shared = []
    if "xl/sharedStrings.xml" in z.namelist():
        root = ET.fromstring(z.read("xl/sharedStrings.xml"))
        for si in root.findall("m:si", ns):
            shared.append("".join(t.text or "" for t in si.iter("{%s}t" % ns["m"])))
    sheet = sorted(n for n in z.namelist() if n.startswith("xl/worksheets/sheet"))[0]
    root = ET.fromstring(z.read(sheet))
    rows = []
    for row in root.iter("{%s}row" % ns["m"]):
        vals = []
        for c in row.findall("m:c", ns):
            t = c.get("t")
            v = c.find("m:v", ns)
            if t == "s" and v is not None:
                vals.append(shared[int(v.text)])
            elif t == "inlineStr":
                vals.append("".join(x.text or "" for x in c.iter("{%s}t" % ns["m"])))
            else:
                vals.append(v.text if v is not None else "")
        rows.append(vals)
    return rows


def import_hosts(filename: str, data: bytes, check_ssh: bool = True) -> dict:
    """Bulk import (columns: name, ip, port, credential[, username, password]) from .xlsx or .csv."""
    if filename.endswith(".xlsx"):
        rows = _xlsx_rows(data)
    else:
        rows = list(csv.reader(io.StringIO(data.decode())))
    if not rows:
        return {"created": [], "errors": ["empty file"]}
    header = [c.strip().lower() for c in rows[0]]
    created, errors = [], []
    for r in rows[1:]:
        if not any(r):
            continue
        rec = dict(zip(header, r))
        cred = rec.get("credential", "")
        if cred:
            with session_scope() as s:
                c = s.scalar(select(M.Credential).where(M.Credential.name == cred))
                rec["credential"] = c.id if c else None
        try:
            created.append(create_host({"name": rec["name"], "ip": rec["ip"], "port": int(rec.get("port") or 22),
                                        "credential": rec.get("credential"), "username": rec.get("username", "root"),
                                        "password": rec.get("password", "")}, check_ssh=check_ssh)["name"])
        except Exception as e:  # noqa: BLE001 - per-row errors are reported, not raised
            errors.append(f"{rec.get('name')}: {e}")
    return {"created": created, "errors": errors}
