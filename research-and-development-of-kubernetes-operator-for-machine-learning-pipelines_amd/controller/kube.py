"""Kubernetes API access for the operator: an async interface with two backends.

* ``RestKube`` — async HTTP client for a real kube-apiserver (in-cluster
  service-account token or a token/cert kubeconfig), custom objects, status
  subresource, merge-patch, events, watch streams.  Constructed lazily: unlike
  the reference (``config.load_incluster_config()`` at import,
  mlflow_operator.py:13) nothing touches the cluster until used.
* ``FakeKube`` — an in-memory apiserver with the semantics the operator
  relies on: resourceVersion + 409 Conflict on stale replace, the status
  subresource (main-resource writes ignore ``status``; status writes ignore
  everything else), ``metadata.generation`` bumps on spec change, JSON merge
  patch, ownerReference garbage collection (cascade on delete), watch
  streams and an Events log.  Fault injection: ``fail_next(verb, status)``.

The reference called the blocking ``kubernetes`` client inside coroutines
(mlflow_operator.py:73,111,247,262,273,465), stalling every CR; here every
call is awaitable.
"""
from __future__ import annotations

import asyncio
import copy
import datetime as _dt
import itertools
import json
import os
import ssl
import uuid
from collections import defaultdict


class ApiError(Exception):
    def __init__(self, status: int, reason: str = "", message: str = ""):
        super().__init__(f"{status} {reason}: {message}")
        self.status, self.reason, self.message = status, reason, message


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch (None deletes a key)."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _now_iso() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


# ------------------------------------------------------------------ fake --

class FakeKube:
    STATUS_SUBRESOURCE = {("mlflow.nizepart.com", "mlflowmodels"),
                          ("machinelearning.seldon.io", "seldondeployments")}

    def __init__(self, validate: bool = True):
        self._objs: dict[tuple, dict] = {}
        self._rv = itertools.count(1)
        self._watchers: list[tuple[tuple, asyncio.Queue]] = []
        self.events: list[dict] = []
        self._faults: dict[str, list[int]] = defaultdict(list)
        self.calls = defaultdict(int)
        # structural schemas of installed CRDs: bodies are validated (422 Invalid) and
        # pruned like the real apiserver does (crd.admit)
        self.schemas: dict[tuple, tuple[str, dict]] = {}
        if validate:
            from .crd import crd_schema
            self.register_crd("mlflow.nizepart.com", "mlflowmodels", "MlflowModel", crd_schema())

    def register_crd(self, group: str, plural: str, kind: str, schema: dict) -> None:
        self.schemas[(group, plural)] = (kind, schema)

    def _admit(self, group, plural, body, name, status_only: bool = False):
        ent = self.schemas.get((group, plural))
        if ent is None:
            return body
        from .crd import admit
        kind, schema = ent
        if status_only:  # /status writes: only .status is taken from the body
            schema = {"type": "object", "properties": {"status": schema.get("properties", {}).get("status", {})}}
            body = {k: v for k, v in body.items() if k in ("apiVersion", "kind", "metadata", "status")}
        pruned, errs = admit(body, schema)
        if errs:
            raise ApiError(422, "Invalid", f'{kind}.{group} "{name}" is invalid: ' + "; ".join(errs))
        return pruned

    def _next_rv(self) -> int:
        self._last_rv = next(self._rv)
        return self._last_rv

    def current_rv(self) -> int:
        """The newest resourceVersion handed out (a List's metadata.resourceVersion)."""
        return getattr(self, "_last_rv", 0)

    def subscribe(self, group, plural, ns=None):
        """Raw event queue of (type, object) for a watch front-end; returns (queue, unsubscribe)."""
        q: asyncio.Queue = asyncio.Queue()
        entry = ((group, plural, ns), q)
        self._watchers.append(entry)
        return q, lambda: self._watchers.remove(entry) if entry in self._watchers else None

    # -- fault injection --
    def fail_next(self, verb: str, status: int = 500, times: int = 1):
        self._faults[verb].extend([status] * times)

    def _maybe_fail(self, verb):
        self.calls[verb] += 1
        if self._faults.get(verb):
            st = self._faults[verb].pop(0)
            raise ApiError(st, "Injected", f"injected failure for {verb}")

    def _key(self, group, plural, ns, name):
        return (group, plural, ns, name)

    def _emit(self, etype, group, plural, obj):
        for (g, p, ns), q in self._watchers:
            if g == group and p == plural and (ns is None or ns == obj["metadata"].get("namespace")):
                q.put_nowait((etype, copy.deepcopy(obj)))

    # -- CRUD --
    async def get(self, group, version, ns, plural, name):
        self._maybe_fail("get")
        obj = self._objs.get(self._key(group, plural, ns, name))
        if obj is None:
            raise ApiError(404, "NotFound", f'{plural} "{name}" not found')
        return copy.deepcopy(obj)

    async def list(self, group, version, ns, plural, label_selector: dict | None = None):
        self._maybe_fail("list")
        out = []
        for (g, p, n, _), o in self._objs.items():
            if g == group and p == plural and (ns is None or n == ns):
                labels = o["metadata"].get("labels", {})
                if label_selector and any(labels.get(k) != v for k, v in label_selector.items()):
                    continue
                out.append(copy.deepcopy(o))
        return out

    async def create(self, group, version, ns, plural, body):
        self._maybe_fail("create")
        body = copy.deepcopy(body)
        md = body.setdefault("metadata", {})
        name = md.get("name")
        key = self._key(group, plural, ns, name)
        if key in self._objs:
            raise ApiError(409, "AlreadyExists", f'{plural} "{name}" already exists')
        body = self._admit(group, plural, body, name)
        md.update(namespace=ns, uid=str(uuid.uuid4()), resourceVersion=str(self._next_rv()),
                  generation=1, creationTimestamp=_now_iso())
        md.pop("deletionTimestamp", None)
        if (group, plural) in self.STATUS_SUBRESOURCE:
            body.pop("status", None)
        self._objs[key] = body
        self._emit("ADDED", group, plural, body)
        return copy.deepcopy(body)

    def _write(self, group, plural, key, new, status_only: bool):
        cur = self._objs[key]
        new = self._admit(group, plural, new, key[3], status_only)
        sub = (group, plural) in self.STATUS_SUBRESOURCE
        if sub and status_only:
            obj = copy.deepcopy(cur)
            if "status" in new:
                obj["status"] = new["status"]
            else:
                obj.pop("status", None)
        elif sub:
            obj = copy.deepcopy(new)
            if "status" in cur:
                obj["status"] = copy.deepcopy(cur["status"])
            else:
                obj.pop("status", None)
        else:
            obj = copy.deepcopy(new)
        md = obj.setdefault("metadata", {})
        for k in ("uid", "creationTimestamp", "namespace", "name"):
            if k in cur["metadata"]:
                md[k] = cur["metadata"][k]
        gen = cur["metadata"].get("generation", 1)
        if not status_only and obj.get("spec") != cur.get("spec"):
            gen += 1
        md["generation"] = gen
        md["resourceVersion"] = str(self._next_rv())
        self._objs[key] = obj
        self._emit("MODIFIED", group, plural, obj)
        return copy.deepcopy(obj)

    async def replace(self, group, version, ns, plural, name, body, status: bool = False):
        self._maybe_fail("replace_status" if status else "replace")
        key = self._key(group, plural, ns, name)
        if key not in self._objs:
            raise ApiError(404, "NotFound", f'{plural} "{name}" not found')
        rv = (body.get("metadata") or {}).get("resourceVersion")
        if rv is not None and rv != self._objs[key]["metadata"]["resourceVersion"]:
            raise ApiError(409, "Conflict", "the object has been modified; please apply your changes "
                                            "to the latest version and try again")
        return self._write(group, plural, key, body, status_only=status)

    async def patch(self, group, version, ns, plural, name, patch, status: bool = False):
        self._maybe_fail("patch_status" if status else "patch")
        key = self._key(group, plural, ns, name)
        if key not in self._objs:
            raise ApiError(404, "NotFound", f'{plural} "{name}" not found')
        return self._write(group, plural, key, merge_patch(self._objs[key], patch), status_only=status)

    async def patch_status(self, group, version, ns, plural, name, patch):
        return await self.patch(group, version, ns, plural, name, patch, status=True)

    async def delete(self, group, version, ns, plural, name):
        self._maybe_fail("delete")
        key = self._key(group, plural, ns, name)
        obj = self._objs.pop(key, None)
        if obj is None:
            raise ApiError(404, "NotFound", f'{plural} "{name}" not found')
        self._emit("DELETED", group, plural, obj)
        await self._gc(obj["metadata"]["uid"])
        return obj

    async def _gc(self, owner_uid):
        """Cascade-delete dependents (ownerReferences), like the K8s garbage collector."""
        for key, o in list(self._objs.items()):
            refs = o["metadata"].get("ownerReferences") or []
            if any(r.get("uid") == owner_uid for r in refs):
                g, p, ns, name = key
                await self.delete(g, None, ns, p, name)

    # -- events --
    async def create_event(self, ns, event: dict):
        self._maybe_fail("event")
        ev = copy.deepcopy(event)
        ev.setdefault("metadata", {}).setdefault("name", f"ev-{self._next_rv()}")
        ev["metadata"]["namespace"] = ns
        self.events.append(ev)
        return ev

    def events_for(self, name: str | None = None, reason: str | None = None):
        return [e for e in self.events
                if (name is None or e["involvedObject"]["name"] == name)
                and (reason is None or e["reason"] == reason)]

    # -- watch --
    async def watch(self, group, version, plural, ns=None, send_initial: bool = True):
        q: asyncio.Queue = asyncio.Queue()
        entry = ((group, plural, ns), q)
        self._watchers.append(entry)
        try:
            if send_initial:
                for o in await self.list(group, version, ns, plural):
                    q.put_nowait(("ADDED", o))
            while True:
                yield await q.get()
        finally:
            self._watchers.remove(entry)


# ------------------------------------------------------------------ REST --

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class RestKube:
    """Async kube-apiserver client (aiohttp).  ``RestKube.from_environment()``
    picks in-cluster credentials, else ``$KUBECONFIG`` / ``~/.kube/config``
    (bearer-token or client-cert contexts)."""

    def __init__(self, server: str, token: str | None = None, ca_file: str | None = None,
                 client_cert: tuple | None = None, insecure: bool = False):
        self.server = server.rstrip("/")
        self.token, self.ca_file, self.client_cert, self.insecure = token, ca_file, client_cert, insecure
        self._session = None

    @classmethod
    def from_environment(cls) -> "RestKube":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if host and os.path.exists(f"{SA_DIR}/token"):
            with open(f"{SA_DIR}/token") as f:
                token = f.read().strip()
            return cls(f"https://{host}:{port}", token=token, ca_file=f"{SA_DIR}/ca.crt")
        import yaml

        path = os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cl = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        us = next(u["user"] for u in kc["users"] if u["name"] == ctx["user"])
        cert = (us["client-certificate"], us["client-key"]) if "client-certificate" in us else None
        return cls(cl["server"], token=us.get("token"), ca_file=cl.get("certificate-authority"),
                   client_cert=cert, insecure=cl.get("insecure-skip-tls-verify", False))

    async def _sess(self):
        import aiohttp

        if self._session is None or self._session.closed:
            sslctx = None
            if self.server.startswith("https"):
                sslctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
                if self.insecure:
                    sslctx.check_hostname = False
                    sslctx.verify_mode = ssl.CERT_NONE
                if self.client_cert:
                    sslctx.load_cert_chain(*self.client_cert)
            headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
            self._session = aiohttp.ClientSession(headers=headers, connector=aiohttp.TCPConnector(ssl=sslctx))
        return self._session

    async def close(self):
        if self._session is not None:
            await self._session.close()

    @staticmethod
    def _path(group, version, ns, plural, name=None, status=False):
        base = f"/apis/{group}/{version}" if group else f"/api/{version}"
        p = f"{base}/namespaces/{ns}/{plural}" if ns else f"{base}/{plural}"
        if name:
            p += f"/{name}"
        if status:
            p += "/status"
        return p

    async def _req(self, method, path, body=None, content_type="application/json", params=None):
        s = await self._sess()
        data = json.dumps(body) if body is not None else None
        async with s.request(method, self.server + path, data=data, params=params,
                             headers={"Content-Type": content_type}) as r:
            txt = await r.text()
            if r.status >= 400:
                try:
                    j = json.loads(txt)
                    raise ApiError(r.status, j.get("reason", ""), j.get("message", txt))
                except ValueError:
                    raise ApiError(r.status, "", txt) from None
            return json.loads(txt) if txt else {}

    async def get(self, group, version, ns, plural, name):
        return await self._req("GET", self._path(group, version, ns, plural, name))

    async def list(self, group, version, ns, plural, label_selector=None):
        params = {"labelSelector": ",".join(f"{k}={v}" for k, v in label_selector.items())} if label_selector else None
        return (await self._req("GET", self._path(group, version, ns, plural), params=params)).get("items", [])

    async def create(self, group, version, ns, plural, body):
        return await self._req("POST", self._path(group, version, ns, plural), body)

    async def replace(self, group, version, ns, plural, name, body, status=False):
        return await self._req("PUT", self._path(group, version, ns, plural, name, status), body)

    async def patch(self, group, version, ns, plural, name, patch, status=False):
        return await self._req("PATCH", self._path(group, version, ns, plural, name, status), patch,
                               content_type="application/merge-patch+json")

    async def patch_status(self, group, version, ns, plural, name, patch):
        return await self.patch(group, version, ns, plural, name, patch, status=True)

    async def delete(self, group, version, ns, plural, name):
        return await self._req("DELETE", self._path(group, version, ns, plural, name),
                               {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": "Background"})

    async def create_event(self, ns, event):
        return await self._req("POST", f"/api/v1/namespaces/{ns}/events", event)

    async def watch(self, group, version, plural, ns=None, send_initial=True):
        s = await self._sess()
        rv = None
        if send_initial:
            lst = await self._req("GET", self._path(group, version, ns, plural))
            rv = lst.get("metadata", {}).get("resourceVersion")
            for o in lst.get("items", []):
                yield ("ADDED", o)
        while True:
            params = {"watch": "1", "allowWatchBookmarks": "true"}
            if rv:
                params["resourceVersion"] = rv
            async with s.get(self.server + self._path(group, version, ns, plural), params=params,
                             timeout=None) as r:
                if r.status == 410:  # expired: relist
                    rv = None
                    continue
                async for line in r.content:
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    obj = ev.get("object", {})
                    rv = obj.get("metadata", {}).get("resourceVersion", rv)
                    if ev.get("type") in ("ADDED", "MODIFIED", "DELETED"):
                        yield (ev["type"], obj)
            await asyncio.sleep(1.0)
