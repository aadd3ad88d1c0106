"""Per-package offline endpoints: a file repository and a read-only OCI distribution registry.

The reference starts one Nexus container per package at scan time (``Package.lookup``,
core/apps/kubeops_api/models/package.py:41-62; ports ``repo_port`` -> 8081 yum/raw and ``registry_port`` ->
8092 docker, core/apps/kubeops_api/package_manage.py:31-45). Here the control plane serves the package
directory itself -- no Docker daemon, no Nexus image:

* ``RepoServer`` on ``repo_port``: ``<package>/repo/**`` under the Nexus-style ``/repository/`` prefix
  (apt / yum trees, Helm ``index.yaml`` + chart tarballs, kube / ROCm binaries, manifests), plus ``/healthz``.
* ``RegistryServer`` on ``registry_port``: the package's ``registry/`` directory, an OCI image layout
  (``oci-layout``, ``index.json``, ``blobs/sha256/*``) holding every image the roles pull, exposed through the
  read-only half of the OCI distribution API that containerd / nerdctl / kubelet use to pull:

  - ``GET /v2/`` (API version check), ``GET /v2/_catalog``, ``GET /v2/<name>/tags/list``;
  - ``HEAD`` / ``GET /v2/<name>/manifests/<tag|digest>`` with ``Accept`` negotiation (OCI index / manifest,
    Docker schema2 manifest / manifest list; an index is resolved to its linux/amd64 child for a client that
    accepts only single-image manifests);
  - ``HEAD`` / ``GET /v2/<name>/blobs/<digest>``, digest-verified before the first byte is sent (the sha256 of
    each blob file is computed once and cached by size + mtime), with ``Range`` support;
  - every response carries ``Docker-Content-Digest`` where a digest applies and
    ``Docker-Distribution-API-Version: registry/2.0``; writes are refused (``UNSUPPORTED``).

Image names come from the layout's ``index.json`` annotations: ``org.opencontainers.image.ref.name`` as
``<name>:<tag>`` (skopeo ``oci:<dir>:<name>:<tag>``), or ``io.containerd.image.name`` (``ctr image export``; the
registry host is stripped, so ``docker.io/flannel/flannel:v0.25.6`` is served as ``flannel/flannel:v0.25.6``).
"""
from __future__ import annotations

import hashlib
import http.server
import json
import logging
import os
import re
import threading
import urllib.parse

log = logging.getLogger("kubeops.packages")

OCI_INDEX = "application/vnd.oci.image.index.v1+json"
OCI_MANIFEST = "application/vnd.oci.image.manifest.v1+json"
DOCKER_LIST = "application/vnd.docker.distribution.manifest.list.v2+json"
DOCKER_MANIFEST = "application/vnd.docker.distribution.manifest.v2+json"
INDEX_TYPES = (OCI_INDEX, DOCKER_LIST)
MANIFEST_TYPES = (OCI_MANIFEST, DOCKER_MANIFEST)
REF_NAME = "org.opencontainers.image.ref.name"
CTR_NAME = "io.containerd.image.name"
_DIGEST_RE = re.compile(r"^sha256:[0-9a-f]{64}$")
_NAME_RE = re.compile(r"^[a-z0-9]+(?:(?:[._]|__|-+)[a-z0-9]+)*(?:/[a-z0-9]+(?:(?:[._]|__|-+)[a-z0-9]+)*)*$")


def split_ref(ref: str) -> tuple[str, str] | None:
    """``[host/]name:tag`` -> (name, tag) with the registry host dropped; None if there is no tag."""
    if "@" in ref:
        return None
    slash = ref.rfind("/")
    colon = ref.rfind(":")
    if colon <= slash:
        return None
    name, tag = ref[:colon], ref[colon + 1:]
    first, _, rest = name.partition("/")
    if rest and ("." in first or ":" in first or first == "localhost"):
        name = rest
    return name, tag


class OCILayout:
    """An OCI image layout on disk, indexed by repository name and tag.

    ``index.json`` must be replaced by an atomic rename (write a temporary file, ``os.replace``): a reload parses the
    new index completely, builds the tag, reachability and media-type tables aside and swaps all three in at once; an
    index that does not parse (caught mid-write) leaves the previous tables in place and is re-read on the next
    request."""

    def __init__(self, root: str):
        self.root = root
        self.tags: dict[str, dict[str, dict]] = {}  # name -> tag -> descriptor
        # name -> every digest a client may pull under that name: manifests / indexes (by digest) and the config and
        # layer blobs they reference -- a blob of another repository is refused (BLOB_UNKNOWN)
        self.reachable: dict[str, set[str]] = {}
        self.media: dict[str, str] = {}  # manifest digest -> media type
        self._hash_cache: dict[str, tuple[int, float, str]] = {}
        self._hash_lock = threading.Lock()
        self._hashing: dict[str, threading.Event] = {}  # blob path -> set when its in-flight hash is done
        self._load_lock = threading.Lock()
        self._index_mtime = None
        self.load()

    def refresh(self) -> None:
        """Re-read ``index.json`` when it changed (images added to the package while it is served)."""
        try:
            m = os.stat(os.path.join(self.root, "index.json")).st_mtime_ns
        except OSError:
            return
        if m != self._index_mtime:
            with self._load_lock:
                if m != self._index_mtime:
                    try:
                        self.load()
                    except (OSError, ValueError) as e:  # mid-write: keep serving the old index, retry next request
                        log.warning("registry %s: index.json not loadable yet (%s); keeping the previous index",
                                    self.root, e)

    def blob_path(self, digest: str) -> str:
        algo, _, hexd = digest.partition(":")
        return os.path.join(self.root, "blobs", algo, hexd)

    def load(self) -> None:
        path = os.path.join(self.root, "index.json")
        m = os.stat(path).st_mtime_ns
        with open(path) as f:
            index = json.load(f)  # parse first: a failure leaves every table (and the recorded mtime) as it was
        # build the new tables aside, then swap them in: a request in flight sees the old or the new index, whole
        tags: dict[str, dict[str, dict]] = {}
        reach: dict[str, set[str]] = {}
        media: dict[str, str] = {}
        self._index(index, tags, reach, media)
        self.tags, self.reachable, self.media = tags, reach, media
        self._index_mtime = m

    def _index(self, index: dict, tags: dict, reach: dict, media: dict) -> None:
        for d in index.get("manifests", []):
            ann = d.get("annotations") or {}
            parsed = None
            for key in (CTR_NAME, REF_NAME):
                if ann.get(key):
                    parsed = split_ref(ann[key])
                    if parsed:
                        break
            if not parsed or not _DIGEST_RE.match(d.get("digest", "")):
                continue
            name, tag = parsed
            tags.setdefault(name, {})[tag] = d
            media[d["digest"]] = d.get("mediaType", OCI_MANIFEST)
            self._walk(name, d["digest"], reach, media)

    def _walk(self, name: str, digest: str, reach: dict, media: dict) -> None:
        seen = reach.setdefault(name, set())
        if digest in seen:
            return
        seen.add(digest)
        kind = media.get(digest)
        if kind not in INDEX_TYPES and kind not in MANIFEST_TYPES:
            return  # a config or layer blob
        try:
            with open(self.blob_path(digest), "rb") as f:
                body = json.load(f)
        except (OSError, ValueError):
            return
        if kind in INDEX_TYPES:
            for child in body.get("manifests", []):
                if _DIGEST_RE.match(child.get("digest", "")):
                    media[child["digest"]] = child.get("mediaType", OCI_MANIFEST)
                    self._walk(name, child["digest"], reach, media)
            return
        for desc in [body.get("config") or {}] + list(body.get("layers") or []):
            if _DIGEST_RE.match(desc.get("digest", "")):
                seen.add(desc["digest"])

    def verified_digest(self, digest: str) -> bool:
        """True if the blob file exists and hashes to ``digest`` (hash cached by size + mtime). One thread hashes a
        given blob at a time: concurrent requests for a blob that is being hashed (many nodes pulling the same
        multi-GB layer at once) wait for that result instead of each reading and hashing the whole file."""
        p = self.blob_path(digest)
        while True:
            try:
                st = os.stat(p)
            except OSError:
                return False
            with self._hash_lock:
                c = self._hash_cache.get(p)
                if c is not None and c[0] == st.st_size and c[1] == st.st_mtime:
                    return c[2] == digest
                busy = self._hashing.get(p)
                if busy is None:
                    mine = self._hashing[p] = threading.Event()
            if busy is not None:
                busy.wait()
                continue  # re-check the cache the hashing thread filled (or hash it now if it failed)
            try:
                h = hashlib.sha256()
                with open(p, "rb") as f:
                    for chunk in iter(lambda: f.read(1 << 20), b""):
                        h.update(chunk)
                c = (st.st_size, st.st_mtime, "sha256:" + h.hexdigest())
                with self._hash_lock:
                    self._hash_cache[p] = c
                return c[2] == digest
            except OSError:
                return False
            finally:
                with self._hash_lock:
                    self._hashing.pop(p, None)
                mine.set()

    def blob_reachable(self, name: str, digest: str) -> bool:
        return digest in self.reachable.get(name, ())

    def resolve_manifest(self, name: str, ref: str) -> str | None:
        if name not in self.tags:
            return None
        if _DIGEST_RE.match(ref):
            # a manifest / index of this repository (its config and layer digests are reachable too, as blobs only)
            return ref if ref in self.reachable.get(name, ()) and ref in self.media else None
        d = self.tags[name].get(ref)
        return d["digest"] if d else None

    def platform_child(self, index_digest: str, accept: list[str]) -> str | None:
        """linux/amd64 child (else the first) of an index, among the media types the client accepts."""
        with open(self.blob_path(index_digest), "rb") as f:
            body = json.load(f)
        kids = [c for c in body.get("manifests", []) if c.get("mediaType", OCI_MANIFEST) in accept]
        for c in kids:
            p = c.get("platform") or {}
            if p.get("os") == "linux" and p.get("architecture") == "amd64":
                return c["digest"]
        return kids[0]["digest"] if kids else None


class _RegistryHandler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "kubeoperator-registry/1.0"
    layout: OCILayout = None  # set by RegistryServer

    def log_message(self, fmt, *args):  # route access logs through logging, not stderr
        log.debug("registry %s: " + fmt, self.address_string(), *args)

    # ---------------------------------------------------------------------------------------- replies
    def _send(self, code: int, body: bytes = b"", ctype: str = "application/json", headers: dict | None = None,
              head: bool = False) -> None:
        self.send_response(code)
        self.send_header("Docker-Distribution-API-Version", "registry/2.0")
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        self.end_headers()
        if body and not head:
            self.wfile.write(body)

    def _error(self, code: int, err: str, msg: str, head: bool = False) -> None:
        body = json.dumps({"errors": [{"code": err, "message": msg, "detail": {}}]}).encode()
        self._send(code, b"" if head else body, headers=None, head=head)

    def _accept(self) -> list[str]:
        out = []
        for h in self.headers.get_all("Accept") or []:
            out += [t.split(";")[0].strip() for t in h.split(",") if t.strip()]
        return out

    # ---------------------------------------------------------------------------------------- routing
    def _route(self, head: bool) -> None:
        self.layout.refresh()
        path = urllib.parse.urlsplit(self.path).path
        if path in ("/v2", "/v2/"):
            return self._send(200, b"{}", head=head)
        if path == "/v2/_catalog":
            return self._send(200, json.dumps({"repositories": sorted(self.layout.tags)}).encode(), head=head)
        m = re.match(r"^/v2/(?P<name>.+)/(?P<kind>manifests|blobs|tags)/(?P<ref>[^/]+)$", path)
        if not m or not _NAME_RE.match(m.group("name")):
            return self._error(404, "NAME_UNKNOWN", "repository name not known to registry", head)
        name, kind, ref = m.group("name"), m.group("kind"), urllib.parse.unquote(m.group("ref"))
        if name not in self.layout.tags:
            return self._error(404, "NAME_UNKNOWN", f"repository {name} not known to registry", head)
        if kind == "tags":
            if ref != "list":
                return self._error(404, "NAME_UNKNOWN", "unknown endpoint", head)
            body = {"name": name, "tags": sorted(self.layout.tags[name])}
            return self._send(200, json.dumps(body).encode(), head=head)
        if kind == "manifests":
            return self._manifest(name, ref, head)
        return self._blob(name, ref, head)

    def _manifest(self, name: str, ref: str, head: bool) -> None:
        digest = self.layout.resolve_manifest(name, ref)
        if digest is None:
            return self._error(404, "MANIFEST_UNKNOWN", f"manifest unknown: {name}:{ref}", head)
        mtype = self.layout.media.get(digest, OCI_MANIFEST)
        accept = self._accept()
        if accept and "*/*" not in accept and mtype not in accept:
            child = self.layout.platform_child(digest, accept) if mtype in INDEX_TYPES else None
            if child is None:
                return self._error(404, "MANIFEST_UNKNOWN",
                                   f"{name}:{ref} is {mtype}; not in Accept ({', '.join(accept)})", head)
            digest, mtype = child, self.layout.media.get(child, OCI_MANIFEST)
        if not self.layout.verified_digest(digest):
            log.error("registry: manifest %s of %s fails its digest check", digest, name)
            return self._error(404, "MANIFEST_UNKNOWN", f"manifest {digest} missing or corrupt", head)
        with open(self.layout.blob_path(digest), "rb") as f:
            body = f.read()
        self._send(200, body, ctype=mtype, headers={"Docker-Content-Digest": digest, "ETag": f'"{digest}"'},
                   head=head)

    def _blob(self, name: str, digest: str, head: bool) -> None:
        if not _DIGEST_RE.match(digest):
            return self._error(400, "DIGEST_INVALID", f"invalid digest {digest}", head)
        # only blobs an image of THIS repository references (distribution spec: a blob is scoped to its repository)
        if not self.layout.blob_reachable(name, digest) or not self.layout.verified_digest(digest):
            return self._error(404, "BLOB_UNKNOWN", f"blob unknown to registry: {digest}", head)
        p = self.layout.blob_path(digest)
        size = os.path.getsize(p)
        start, end, code = 0, size - 1, 200
        rng = self.headers.get("Range")
        if rng:
            m = re.match(r"^bytes=(\d*)-(\d*)$", rng.strip())
            if not m or (not m.group(1) and not m.group(2)):
                return self._error(416, "BLOB_UNKNOWN", f"bad range {rng}", head)
            if m.group(1):
                start = int(m.group(1))
                end = min(int(m.group(2)), size - 1) if m.group(2) else size - 1
            else:  # suffix range: the last N bytes
                start = max(0, size - int(m.group(2)))
            if start > end or start >= size:
                self.send_response(416)
                self.send_header("Content-Range", f"bytes */{size}")
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            code = 206
        self.send_response(code)
        self.send_header("Docker-Distribution-API-Version", "registry/2.0")
        self.send_header("Content-Type", "application/octet-stream")
        self.send_header("Docker-Content-Digest", digest)
        self.send_header("Accept-Ranges", "bytes")
        self.send_header("Content-Length", str(end - start + 1))
        if code == 206:
            self.send_header("Content-Range", f"bytes {start}-{end}/{size}")
        self.end_headers()
        if head:
            return
        with open(p, "rb") as f:
            f.seek(start)
            left = end - start + 1
            while left > 0:
                chunk = f.read(min(left, 1 << 20))
                if not chunk:
                    break
                self.wfile.write(chunk)
                left -= len(chunk)

    def do_GET(self):  # noqa: N802
        self._route(head=False)

    def do_HEAD(self):  # noqa: N802
        self._route(head=True)

    def _readonly(self):
        n = int(self.headers.get("Content-Length") or 0)
        if n:
            self.rfile.read(n)
        self._error(405, "UNSUPPORTED", "this registry serves an offline package read-only")

    do_PUT = do_POST = do_PATCH = do_DELETE = _readonly  # noqa: N815


class _RepoHandler(http.server.SimpleHTTPRequestHandler):
    """``/repository/<path>`` -> ``<package>/repo/<path>``; ``/healthz`` for the install preflight."""

    def log_message(self, fmt, *args):
        log.debug("repo %s: " + fmt, self.address_string(), *args)

    def translate_path(self, path):
        p = urllib.parse.urlsplit(path).path
        if p == "/repository" or p.startswith("/repository/"):
            return super().translate_path(p[len("/repository"):] or "/")
        return os.path.join(self.directory, ".no-such-path")  # only /repository/ is served

    def do_GET(self):  # noqa: N802
        if urllib.parse.urlsplit(self.path).path == "/healthz":
            body = b"ok\n"
            self.send_response(200)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
            return
        super().do_GET()


class _Server:
    def __init__(self, handler, host: str, port: int, name: str):
        self.httpd = http.server.ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, name=name, daemon=True)
        self.thread.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


class RepoServer(_Server):
    def __init__(self, root: str, host: str = "0.0.0.0", port: int = 8081, name: str = "repo"):
        handler = type("RepoHandler", (_RepoHandler,), {})
        super().__init__(lambda *a, **k: handler(*a, directory=root, **k), host, port, f"pkg-repo-{name}")
        self.root = root


class RegistryServer(_Server):
    def __init__(self, root: str, host: str = "0.0.0.0", port: int = 8082, name: str = "registry"):
        self.layout = OCILayout(root)
        handler = type("RegistryHandler", (_RegistryHandler,), {"layout": self.layout})
        super().__init__(handler, host, port, f"pkg-registry-{name}")
