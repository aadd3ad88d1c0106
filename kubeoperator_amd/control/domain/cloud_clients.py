"""IaaS API clients behind the region / zone / flavor lookups and the VM image import of the IaaS plans.

Reference: ``cloud_provider/clients/openstack.py:13-146`` (openstacksdk: regions, availability zones with their
networks / floating networks / security groups / volume types, flavors >= 4C/8G/60G, Glance image create)
and ``cloud_provider/clients/vsphere.py:16-190`` (pyVmomi: datacenters, compute clusters with networks and
datastores, OVF import through an ``HttpNfcLease``). Neither SDK is a dependency here: both clients speak the
services' REST APIs directly with ``httpx``:

* OpenStack: Keystone v3 password auth (token + service catalog), Nova ``/os-availability-zone`` and
  ``/flavors/detail``, Neutron ``/v2.0/networks`` / ``/v2.0/subnets`` / ``/v2.0/security-groups``, Cinder
  ``/types``, Glance v2 image create + binary upload.
* vSphere: the vCenter Automation REST API (``/api/session``, ``/api/vcenter/{datacenter,cluster,network,
  datastore,resource-pool}``) and the content library for the image import (local library, library item,
  update session, file upload, complete) -- the Terraform vSphere provider clones from a content-library
  OVF template.

With no endpoint configured (an offline plan) the lookups fall back to the values configured on the region
/ zone, so plans can still be written by hand.
"""
from __future__ import annotations

import os

import httpx

TIMEOUT = 30


class CloudError(Exception):
    pass


def _check(r: httpx.Response, what: str) -> httpx.Response:
    if r.status_code >= 400:
        raise CloudError(f"{what}: HTTP {r.status_code} {r.text[:200]}")
    return r


# ---------------------------------------------------------------------------------------------- OpenStack
class OpenStackClient:
    """``vars``: auth_url (Keystone v3 base, e.g. https://keystone:5000/v3), user_name, password, project_name,
    domain_name (default "Default"), optional region."""

    def __init__(self, vars: dict, region: str | None = None, http: httpx.Client | None = None):
        self.vars = vars
        self.region = region or vars.get("region")
        self.http = http or httpx.Client(timeout=TIMEOUT, verify=bool(vars.get("verify_tls", False)))
        self.token, self.catalog = self._auth()

    def _auth(self):
        v = self.vars
        base = str(v["auth_url"]).rstrip("/")
        if not base.endswith("/v3"):
            base += "/v3"
        dom = v.get("domain_name") or "Default"
        body = {"auth": {"identity": {"methods": ["password"], "password": {"user": {
            "name": v["user_name"], "password": v["password"], "domain": {"name": dom}}}},
            "scope": {"project": {"name": v["project_name"], "domain": {"name": dom}}}}}
        r = _check(self.http.post(f"{base}/auth/tokens", json=body), "keystone auth")
        self.identity = base
        return r.headers["X-Subject-Token"], r.json()["token"].get("catalog", [])

    def endpoint(self, service_type: str) -> str:
        for svc in self.catalog:
            if svc.get("type") != service_type:
                continue
            eps = [e for e in svc.get("endpoints", []) if e.get("interface") == "public"]
            if self.region:
                eps = [e for e in eps if e.get("region") in (self.region, None) or e.get("region_id") == self.region] \
                    or eps
            if eps:
                return eps[0]["url"].rstrip("/")
        raise CloudError(f"no public {service_type} endpoint in the service catalog")

    def _get(self, service: str, path: str, **params) -> dict:
        r = self.http.get(f"{self.endpoint(service)}{path}", headers={"X-Auth-Token": self.token}, params=params)
        return _check(r, f"{service} GET {path}").json()

    def list_regions(self) -> list[str]:
        r = self.http.get(f"{self.identity}/regions", headers={"X-Auth-Token": self.token})
        return [x["id"] for x in _check(r, "keystone regions").json().get("regions", [])]

    def list_zones(self) -> list[dict]:
        """Availability zones shaped like the reference's zone dicts (cluster, networkList,
        floatingNetworkList, securityGroups, storages, ipType)."""
        azs = [z["zoneName"] for z in self._get("compute", "/os-availability-zone").get("availabilityZoneInfo", [])
               if z.get("zoneState", {}).get("available", True)]
        nets = self._get("network", "/v2.0/networks").get("networks", [])
        subnets = self._get("network", "/v2.0/subnets").get("subnets", [])
        sgs = self._get("network", "/v2.0/security-groups").get("security_groups", [])
        try:
            types = self._get("volumev3", "/types").get("volume_types", [])
        except CloudError:
            types = []
        by_net: dict[str, list] = {}
        for sn in subnets:
            by_net.setdefault(sn["network_id"], []).append({"id": sn["id"], "name": sn.get("name", ""),
                                                           "cidr": sn.get("cidr", "")})
        zones = []
        for az in azs:
            z = {"cluster": az, "networkList": [], "floatingNetworkList": [], "securityGroups": [s["name"] for s in sgs],
                 "storages": [{"id": t["id"], "name": t["name"]} for t in types], "ipType": ["private", "floating"]}
            for n in nets:
                entry = {"id": n["id"], "name": n.get("name", ""), "subnetList": by_net.get(n["id"], [])}
                (z["floatingNetworkList"] if n.get("router:external") else z["networkList"]).append(entry)
            zones.append(z)
        return zones

    def get_flavors(self) -> list[dict]:
        out = []
        for f in self._get("compute", "/flavors/detail").get("flavors", []):
            if f.get("vcpus", 0) >= 4 and f.get("ram", 0) / 1024 >= 8 and f.get("disk", 0) >= 60:
                out.append({"name": f["name"], "meta": {"id": f["id"], "cpu": f["vcpus"], "memory": f["ram"] / 1024,
                                                        "disk": f["disk"]}})
        return out

    def create_image(self, name: str, path: str, disk_format: str = "qcow2") -> str:
        """Glance v2: create the image record (unless one with that name exists) and upload the file."""
        glance = self.endpoint("image")
        hdr = {"X-Auth-Token": self.token}
        found = _check(self.http.get(f"{glance}/v2/images", headers=hdr, params={"name": name}), "glance list")
        imgs = found.json().get("images", [])
        if imgs and imgs[0].get("status") == "active":
            return imgs[0]["id"]
        img = _check(self.http.post(f"{glance}/v2/images", headers=hdr, json={
            "name": name, "disk_format": disk_format, "container_format": "bare", "visibility": "private"}),
            "glance create").json()
        with open(path, "rb") as f:
            _check(self.http.put(f"{glance}/v2/images/{img['id']}/file", content=f,
                                 headers=dict(hdr, **{"Content-Type": "application/octet-stream"})), "glance upload")
        return img["id"]


# ------------------------------------------------------------------------------------------------ vSphere
class VSphereClient:
    """``vars``: vc_host, vc_username, vc_password, optional vc_port (443)."""

    def __init__(self, vars: dict, http: httpx.Client | None = None):
        self.vars = vars
        port = int(vars.get("vc_port") or 443)
        scheme = vars.get("vc_scheme") or "https"
        self.base = f"{scheme}://{vars['vc_host']}:{port}"
        self.http = http or httpx.Client(timeout=TIMEOUT, verify=bool(vars.get("verify_tls", False)))
        r = _check(self.http.post(f"{self.base}/api/session", auth=(vars["vc_username"], vars["vc_password"])),
                   "vcenter login")
        self.session = r.json()
        self.hdr = {"vmware-api-session-id": self.session}

    def _get(self, path: str, **params):
        return _check(self.http.get(f"{self.base}{path}", headers=self.hdr, params=params), f"GET {path}").json()

    def _post(self, path: str, body=None, **params):
        r = _check(self.http.post(f"{self.base}{path}", headers=self.hdr, json=body, params=params), f"POST {path}")
        return r.json() if r.content else None

    def _dc_id(self, name: str) -> str:
        for d in self._get("/api/vcenter/datacenter", names=name):
            return d["datacenter"]
        raise CloudError(f"datacenter {name!r} not found")

    def list_regions(self) -> list[str]:
        return [d["name"] for d in self._get("/api/vcenter/datacenter")]

    def list_zones(self, datacenter: str) -> list[dict]:
        """Compute clusters of a datacenter with the networks, datastores and resource pools usable there
        (reference vsphere.py list_zone: cluster -> networks / datastores)."""
        dc = self._dc_id(datacenter)
        nets = [n["name"] for n in self._get("/api/vcenter/network", datacenters=dc)]
        stores = [{"name": s["name"], "free": s.get("free_space"), "type": s.get("type")}
                  for s in self._get("/api/vcenter/datastore", datacenters=dc)]
        zones = []
        for c in self._get("/api/vcenter/cluster", datacenters=dc):
            pools = [p["name"] for p in self._get("/api/vcenter/resource-pool", clusters=c["cluster"])]
            zones.append({"cluster": c["name"], "networks": nets, "storages": stores, "resourcePools": pools})
        return zones

    def create_image(self, name: str, ova_path: str, datastore: str, library: str = "kubeoperator") -> str:
        """Import an OVA into a local content library (created on first use): item + update session + upload
        + complete. Returns the library item id (what the Terraform provider clones from)."""
        ds = [d["datastore"] for d in self._get("/api/vcenter/datastore", names=datastore)]
        if not ds:
            raise CloudError(f"datastore {datastore!r} not found")
        libs = [lib for lib in (self._get(f"/api/content/library/{i}") for i in self._get("/api/content/library"))
                if lib.get("name") == library]
        lib_id = libs[0]["id"] if libs else self._post("/api/content/local-library", {
            "name": library, "type": "LOCAL", "storage_backings": [{"type": "DATASTORE", "datastore_id": ds[0]}]})
        for iid in self._get("/api/content/library/item", library_id=lib_id):
            if self._get(f"/api/content/library/item/{iid}").get("name") == name:
                return iid
        item = self._post("/api/content/library/item", {"library_id": lib_id, "name": name, "type": "ovf"})
        sess = self._post("/api/content/library/item/update-session", {"library_item_id": item})
        f = self._post(f"/api/content/library/item/update-session/{sess}/file", {
            "name": os.path.basename(ova_path), "source_type": "PUSH", "size": os.path.getsize(ova_path)}, action="add")
        uri = f["upload_endpoint"]["uri"].replace("*", self.vars["vc_host"])
        with open(ova_path, "rb") as fh:
            _check(self.http.put(uri, content=fh, headers=dict(self.hdr, **{"Content-Type": "application/octet-stream"})),
                   "content library upload")
        self._post(f"/api/content/library/item/update-session/{sess}", None, action="complete")
        return item


# -------------------------------------------------------------------------------------------- dispatcher
def client_for(provider: str, vars: dict, region: str | None = None):
    if provider == "openstack":
        return OpenStackClient(vars, region)
    if provider == "vsphere":
        return VSphereClient(vars)
    raise CloudError(f"provider {provider!r} has no cloud API")


def has_endpoint(provider: str, vars: dict) -> bool:
    return bool(vars.get("auth_url")) if provider == "openstack" else bool(vars.get("vc_host")) \
        if provider == "vsphere" else False
