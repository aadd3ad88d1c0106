"""IaaS provisioning for AUTOMATIC clusters: regions / zones / plans, IP pools, host plans, Terraform.

Reference: cloud_provider/models.py:19-259 (Zone.allocate_ip :140-144, ip_pools :167-190, Plan.mixed_vars
:229-237), kubeops_api/cloud_provider.py:12-210 (create/scale/delete, multi-AZ round robin
``index % len(zones)``), cloud_provider/cloud_client.py + clients/{vsphere,openstack}.py,
resource/clouds/*/terraform/terraform.tf.j2, compute_model_meta.yml.

Providers: ``vsphere`` and ``openstack`` render ``resources/clouds/<provider>/terraform/main.tf.j2`` and run
the ``terraform`` binary (streamed to the execution log); ``baremetal`` allocates idle registered hosts
(e.g. 8x MI355X servers) from the zone's pool instead of creating VMs; ``fake`` renders the Terraform file
and returns the planned hosts without calling any API (CI). IP allocation is transactional (the zone's read-modify-write
runs under the store's write lock, ``store.db.write_scope``, so allocators in other threads and processes are
serialised; the reference's ``Zone.allocate_ip`` could double-allocate under concurrent installs).
"""
from __future__ import annotations

import ipaddress
import os
import shutil
import subprocess

import jinja2
import yaml
from sqlalchemy import select

from ..conf import RESOURCE_DIR, get_config
from ..runtime import jobs
from ..store import models as M
from ..store.db import session_scope, write_scope
from . import clusters


def _provider_meta(provider: str) -> dict:
    path = os.path.join(RESOURCE_DIR, "clouds", provider, "meta.yml")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return yaml.safe_load(f) or {}


def compute_models() -> list[dict]:
    with open(os.path.join(RESOURCE_DIR, "clouds", "compute_model_meta.yml")) as f:
        return yaml.safe_load(f)


def compute_model(name: str) -> dict:
    for m in compute_models():
        if m["name"] == name:
            return m["meta"]
    raise clusters.NotFound(f"compute model {name} not found")


# ------------------------------------------------------------------------------------------- zones / IPs
def ip_pool(zone: M.Zone, provider: str) -> list[str]:
    v = zone.vars or {}
    if not v.get("ip_start") or not v.get("ip_end"):
        return []
    start, end = ipaddress.ip_address(v["ip_start"]), ipaddress.ip_address(v["ip_end"])
    if provider == "openstack" or not v.get("net_mask"):
        pool = [str(ipaddress.ip_address(int(start) + i)) for i in range(int(end) - int(start) + 1)]
    else:
        net = ipaddress.ip_interface(f"{start}/{v['net_mask']}").network
        pool = [str(h) for h in net.hosts() if start <= h <= end]
    used = set(zone.ip_used or [])
    return [ip for ip in pool if ip not in used]


def zone_provider(s, zone: M.Zone) -> str:
    r = s.get(M.Region, zone.region_id)
    if r is None:
        return "fake"
    if r.template_id:
        t = s.get(M.CloudProviderTemplate, r.template_id)
        if t is not None:
            return t.name
    return (r.vars or {}).get("provider", "fake")


def allocate_ip(zone_id: str) -> str:
    """Take the zone's first free address. The zone row's read-modify-write runs under the store's write lock
    (``write_scope``: BEGIN IMMEDIATE on SQLite, SELECT ... FOR UPDATE elsewhere), so concurrent allocators in
    other threads or processes never hand out one address twice."""
    with write_scope() as s:
        z = s.get(M.Zone, zone_id, with_for_update=True)
        pool = ip_pool(z, zone_provider(s, z))
        if not pool:
            raise RuntimeError(f"zone {z.name}: no available ip address")
        ip = pool[0]
        z.ip_used = list(z.ip_used or []) + [ip]
        return ip


def recover_ip(zone_id: str, ip: str) -> None:
    with write_scope() as s:
        z = s.get(M.Zone, zone_id, with_for_update=True)
        z.ip_used = [x for x in (z.ip_used or []) if x != ip]


def zone_dict(s, z: M.Zone) -> dict:
    d = {"key": "z" + z.id.split("-")[3], "name": z.cloud_zone, "zone_name": z.name, "id": z.id}
    d.update(z.vars or {})
    v = z.vars or {}
    if v.get("ip_start") and v.get("net_mask"):
        d["net_mask"] = ipaddress.ip_interface(f"{v['ip_start']}/{v['net_mask']}").network.prefixlen
    else:
        d["net_mask"] = 24
    d["ip_available"] = len(ip_pool(z, zone_provider(s, z)))
    return d


def plan_zones(s, p: M.Plan) -> list[M.Zone]:
    return [z for z in (s.get(M.Zone, zid) for zid in (p.zone_ids or [])) if z is not None]


def count_ip_available(plan_id: str) -> int:
    with session_scope() as s:
        p = s.get(M.Plan, plan_id)
        return sum(len(ip_pool(z, zone_provider(s, z))) for z in plan_zones(s, p))


def check_capacity(c: M.Cluster, need: int) -> None:
    if not c.plan_id:
        raise ValueError("AUTOMATIC cluster has no plan")
    have = count_ip_available(c.plan_id)
    if have < need:
        raise ValueError(f"plan has {have} free IP addresses, {need} needed")


def mixed_vars(plan_id: str) -> dict:
    with session_scope() as s:
        p = s.get(M.Plan, plan_id)
        r = s.get(M.Region, p.region_id) if p.region_id else None
        v = dict(p.vars or {})
        if r is not None:
            v.update(r.vars or {})
            v["region"] = r.cloud_region
            v["provider"] = zone_provider(s, plan_zones(s, p)[0]) if p.zone_ids else (r.vars or {}).get("provider", "fake")
        v["zones"] = [zone_dict(s, z) for z in plan_zones(s, p)]
        v["deploy_template"] = p.deploy_template
        return v


# ------------------------------------------------------------------------------------------- host plans
def _pick_zone(zones: list[str], index: int) -> str:
    """Multi-AZ round robin by node index, skipping exhausted zones (fixes get_zone's pop-by-object)."""
    if not zones:
        raise RuntimeError("plan has no zones")
    order = zones[index % len(zones):] + zones[:index % len(zones)]
    for zid in order:
        with session_scope() as s:
            z = s.get(M.Zone, zid)
            if ip_pool(z, zone_provider(s, z)):
                return zid
    raise RuntimeError("Can not find available ip address!")


def create_cluster_hosts_dict(c: M.Cluster) -> list[dict]:
    with session_scope() as s:
        p = s.get(M.Plan, c.plan_id)
        zone_ids = list(p.zone_ids or [])
        tmpl = p.deploy_template
        models = {"master": (p.vars or {}).get("master_model", "medium"),
                  "worker": (p.vars or {}).get("worker_model", "large")}
    roles = {"master": 3 if tmpl == "MULTIPLE" else 1, "worker": c.worker_size}
    domain = c.name + (f".{c.cluster_doamin_suffix}" if c.cluster_doamin_suffix else "")
    hosts = []
    for role, size in roles.items():
        cm = compute_model(models[role])
        for i in range(1, size + 1):
            name = f"{role}{i}.{domain}"
            with session_scope() as s:
                existing = s.scalar(select(M.Host).where(M.Host.name == name))
            zid = existing.zone_id if existing is not None and existing.zone_id else _pick_zone(zone_ids, i)
            with session_scope() as s:
                zd = zone_dict(s, s.get(M.Zone, zid))
            h = {"role": role, "cpu": cm["cpu"], "memory": cm["memory"] * 1024, "gpu": cm.get("gpu", 0),
                 "gpu_model": cm.get("gpu_model", ""), "name": name, "short_name": f"{role}{i}", "domain": domain,
                 "zone": zd, "zone_name": zd["zone_name"], "zone_id": zid}
            if existing is not None:
                h["ip"] = existing.ip
            else:
                h["ip"] = allocate_ip(zid)
                h["new"] = True
            hosts.append(h)
    return hosts


# ------------------------------------------------------------------------------------------- terraform
def terraform_dir(cluster_name: str) -> str:
    d = os.path.join(get_config().data_dir, "terraform", cluster_name)
    os.makedirs(d, exist_ok=True)
    return d


def render_terraform(cluster_name: str, provider: str, variables: dict, hosts: list[dict]) -> str:
    tpl = os.path.join(RESOURCE_DIR, "clouds", provider if provider != "fake" else "vsphere", "terraform",
                       "main.tf.j2")
    env = jinja2.Environment(undefined=jinja2.StrictUndefined, trim_blocks=True, lstrip_blocks=True)
    with open(tpl) as f:
        text = env.from_string(f.read()).render(cluster_name=cluster_name, hosts=hosts, **variables)
    path = os.path.join(terraform_dir(cluster_name), "main.tf")
    with open(path, "w") as f:
        f.write(text)
    return path


def _terraform(cluster_name: str, args: list[str], logger=None) -> bool:
    tf = shutil.which(get_config()["TERRAFORM_BIN"])
    if tf is None:
        raise RuntimeError("terraform binary not found; install it or use the baremetal / fake provider")
    proc = subprocess.Popen([tf, *args], cwd=terraform_dir(cluster_name), stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    for line in proc.stdout:
        if logger:
            logger(line.rstrip("\n"))
    return proc.wait() == 0


def _register_hosts(c: M.Cluster, hosts: list[dict], variables: dict) -> None:
    from . import hosts as hostmod

    cred = variables.get("credential") or {}
    for h in hosts:
        with session_scope() as s:
            if s.scalar(select(M.Host).where(M.Host.name == h["name"])) is None:
                s.add(M.Host(name=h["name"], ip=h["ip"], zone_id=h["zone_id"], status="CREATING",
                             username=cred.get("username", get_config()["DEFAULT_HOST_USER"]),
                             password=hostmod.context.enc(cred.get("password", get_config()["DEFAULT_HOST_PASSWORD"]))))
        with session_scope() as s:
            hid = s.scalar(select(M.Host).where(M.Host.name == h["name"])).id
        try:
            hostmod.gather_info(hid)
        except Exception:  # noqa: BLE001 - a fresh VM may still be booting; health check retries later
            pass
        nodes = {n["name"] for n in clusters.list_nodes(c.name)}
        if h["name"] not in nodes:
            roles = [h["role"]] + (["new_node"] if h["role"] == "worker" and c.status == "SCALING" else [])
            clusters.add_node(c.name, {"name": h["name"], "host": h["name"], "roles": roles})


def create_resources(cluster_name: str, logger=None) -> list[dict]:
    c = clusters.get_cluster(cluster_name)
    variables = mixed_vars(c.plan_id)
    hosts = create_cluster_hosts_dict(c)
    provider = variables.get("provider", "fake")
    if provider == "baremetal":
        hosts = _allocate_baremetal(hosts)
    else:
        render_terraform(cluster_name, provider, variables, hosts)
        if provider != "fake":
            ok = _terraform(cluster_name, ["init", "-input=false"], logger) and \
                _terraform(cluster_name, ["apply", "-auto-approve", "-input=false"], logger)
            if not ok:
                raise RuntimeError("terraform apply failed")
        elif logger:
            logger(f"[fake provider] rendered {os.path.join(terraform_dir(cluster_name), 'main.tf')} "
                   f"for {len(hosts)} hosts")
    _register_hosts(c, hosts, variables)
    zone_vars = hosts[0]["zone"] if hosts else {}
    with session_scope() as s:
        row = s.get(M.Cluster, c.id)
        row.configs = {**(row.configs or {}), **{k: v for k, v in zone_vars.items() if k not in ("id", "key")}}
    return hosts


def _allocate_baremetal(hosts: list[dict]) -> list[dict]:
    """Bind planned nodes to idle registered hosts of the zone (GPU workers first for worker roles)."""
    out = []
    with session_scope() as s:
        for h in hosts:
            q = select(M.Host).where(M.Host.node_id.is_(None), M.Host.zone_id == h["zone_id"])
            cands = [x for x in s.scalars(q) if x.name not in {o["name"] for o in out}]
            if h["role"] == "worker":
                cands.sort(key=lambda x: -len(x.gpus or []))
            if not cands:
                raise RuntimeError(f"zone {h['zone_name']}: no idle bare-metal host for {h['name']}")
            pick = cands[0]
            recover = h.get("new")
            out.append({**h, "name": pick.name, "ip": pick.ip})
            if recover:
                z = s.get(M.Zone, h["zone_id"])
                z.ip_used = [x for x in (z.ip_used or []) if x != h["ip"]]
    return out


def scale_to(cluster_name: str, num: int, logger=None) -> None:
    """Scale the worker pool to ``num`` (reference scale_compute_resource, cloud_provider.py:17-48)."""
    c = clusters.get_cluster(cluster_name)
    workers = [n for n in clusters.list_nodes(cluster_name) if "worker" in (n.get("groups") or [])]
    if num < len(workers):
        remove = sorted(workers, key=lambda n: n["name"])[num:]
        m = clusters.first_master(c)
        for n in remove:
            clusters.run_adhoc(c, m, "shell", {"_raw_params": f"kubectl drain {n['name']} --ignore-daemonsets "
                                                              f"--delete-emptydir-data --force; kubectl delete node {n['name']}"},
                               logger=logger)
            clusters.remove_node_record(cluster_name, n["name"])
            with session_scope() as s:
                h = s.scalar(select(M.Host).where(M.Host.name == n["name"]))
                if h is not None:
                    if h.zone_id:
                        z = s.get(M.Zone, h.zone_id)
                        z.ip_used = [x for x in (z.ip_used or []) if x != h.ip]
                    s.delete(h)
    with session_scope() as s:
        s.get(M.Cluster, c.id).worker_size = num
    if num > len(workers):
        create_resources(cluster_name, logger=logger)
        for n in clusters.list_nodes(cluster_name):
            if "worker" in n["groups"] and n["name"] not in {w["name"] for w in workers}:
                clusters.set_node_groups(cluster_name, n["name"], ["worker", "new_node"])


def destroy_resources(cluster_name: str, logger=None) -> None:
    c = clusters.get_cluster(cluster_name)
    variables = mixed_vars(c.plan_id) if c.plan_id else {"provider": "fake"}
    provider = variables.get("provider", "fake")
    if provider not in ("fake", "baremetal"):
        if not _terraform(cluster_name, ["destroy", "-auto-approve", "-input=false"], logger):
            raise RuntimeError("Destroy nodes error!")
    for n in clusters.list_nodes(cluster_name):
        clusters.remove_node_record(cluster_name, n["name"])
        if provider == "baremetal":
            continue
        with session_scope() as s:
            h = s.scalar(select(M.Host).where(M.Host.name == n["name"]))
            if h is not None:
                if h.zone_id:
                    z = s.get(M.Zone, h.zone_id)
                    z.ip_used = [x for x in (z.ip_used or []) if x != h.ip]
                s.execute(M.ItemResource.__table__.delete().where(M.ItemResource.resource_id == h.id))
                s.delete(h)


# ------------------------------------------------------------------------------------------- cloud API
def list_regions_from_cloud(provider_vars: dict) -> list[str]:
    """Regions visible with the given credentials (reference cloud/region/): OpenStack Keystone regions or
    vSphere datacenters through their REST APIs (``cloud_clients``); offline plans: the configured ones."""
    from . import cloud_clients as cc

    prov = provider_vars.get("provider", "")
    if cc.has_endpoint(prov, provider_vars):
        return cc.client_for(prov, provider_vars).list_regions()
    return list(provider_vars.get("regions") or ([provider_vars["region"]] if provider_vars.get("region") else []))


def list_zones_from_cloud(region_vars: dict, cloud_region: str | None = None) -> list:
    """Zones of a region: OpenStack availability zones / vSphere compute clusters with their networks,
    storages and security groups or resource pools (reference cloud/<region>/zone/)."""
    from . import cloud_clients as cc

    prov = region_vars.get("provider", "")
    if cc.has_endpoint(prov, region_vars):
        cli = cc.client_for(prov, region_vars, cloud_region)
        return cli.list_zones() if prov == "openstack" else cli.list_zones(cloud_region or region_vars["datacenter"])
    return list(region_vars.get("zones") or region_vars.get("clusters") or [])


def list_flavors(region_vars: dict, cloud_region: str | None = None) -> list[dict]:
    """Compute flavors >= 4C/8G/60G (reference openstack client get_flavors); vSphere and offline plans use the
    built-in compute models."""
    from . import cloud_clients as cc

    if region_vars.get("provider") == "openstack" and cc.has_endpoint("openstack", region_vars):
        return cc.client_for("openstack", region_vars, cloud_region).get_flavors()
    return [m for m in compute_models() if m["meta"]["cpu"] >= 4 and m["meta"]["memory"] >= 8]


def create_image(region_vars: dict, zone_vars: dict, cloud_region: str | None = None) -> str:
    """Import the node OS image for a zone (reference ``CloudClient.create_image``): Glance upload or a
    vSphere content-library OVA item. Returns the image / library item id."""
    from . import cloud_clients as cc

    prov = region_vars.get("provider", "")
    meta = _provider_meta(prov).get("image", {})
    name = region_vars.get("image_name") or meta.get("name")
    path = region_vars.get("image_path") or meta.get("path")
    if prov == "openstack":
        return cc.client_for(prov, region_vars, cloud_region).create_image(name, path)
    if prov == "vsphere":
        return cc.VSphereClient(region_vars).create_image(name, path, zone_vars.get("datastore") or
                                                         region_vars.get("datastore"))
    raise cc.CloudError(f"provider {prov!r} has no image import")


# ------------------------------------------------------------------------------------- zone image import
def on_zone_create(zone_id: str, run: str = "queue") -> None:
    """Reference ``Zone.on_zone_create``: upload the node OS image for the zone in the background (Glance /
    vSphere content library); the zone is INITIALIZING meanwhile, then READY or ERROR. Offline providers
    (no API endpoint configured) are READY at once."""
    from . import cloud_clients as cc

    with session_scope() as s:
        z = s.get(M.Zone, zone_id)
        r = s.get(M.Region, z.region_id)
        prov = zone_provider(s, z)
        online = r is not None and cc.has_endpoint(prov, dict(r.vars or {}))
        z.status = "INITIALIZING" if online else "READY"
    if online:
        if run == "queue":
            jobs.submit("zone_create_image", {"zone_id": zone_id})
        else:
            jobs.run_inline("zone_create_image", {"zone_id": zone_id})


def init_zone_image(zone_id: str, logger=None) -> dict:
    with session_scope() as s:
        z = s.get(M.Zone, zone_id)
        r = s.get(M.Region, z.region_id)
        rvars = dict(r.vars or {}, provider=zone_provider(s, z))
        zvars, cloud_region = dict(z.vars or {}), r.cloud_region
    try:
        image = create_image(rvars, zvars, cloud_region)
        status, out = "READY", {"image_id": image}
    except Exception as e:  # noqa: BLE001 -- recorded on the zone
        if logger:
            logger(f"image import failed: {type(e).__name__}: {e}")
        status, out = "ERROR", {"error": f"{type(e).__name__}: {e}"}
    with session_scope() as s:
        z = s.get(M.Zone, zone_id)
        z.status = status
        z.vars = {**(z.vars or {}), **({"image_id": out["image_id"]} if "image_id" in out else {})}
    return dict(out, status=status)


@jobs.task("zone_create_image")
def _job_zone_create_image(job_id, logger, zone_id):
    return init_zone_image(zone_id, logger=logger)
