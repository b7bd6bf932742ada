"""A kube-apiserver wire front-end over ``FakeKube`` (aiohttp).

The operator's real-cluster client (``kube.RestKube``, what ``python -m
mlopamd.controller run`` uses) speaks the Kubernetes REST protocol; this serves
that protocol from the in-memory ``FakeKube`` so the whole real-cluster code path
(kubeconfig / bearer token, JSON bodies, merge-patch, the ``/status``
subresource, optimistic concurrency, ``ownerReferences`` GC, chunked
``?watch=1`` streams, Events, ``Status`` error objects) is exercised end to end
without a cluster (no kind / kubectl in this environment).

The reference relies on the real apiserver for all of this
(`mlflow_operator.py:73,111,247,262,273,465` via the kubernetes client; watch via
kopf, `:26-27`); the RBAC it needs is `rbac.yaml:14-31`.

Routes (namespaced and cluster-wide, custom groups under /apis, core under /api):
  GET/POST          {base}/namespaces/{ns}/{plural}            list (labelSelector) / watch=1 / create
  GET/PUT/PATCH/DEL {base}/namespaces/{ns}/{plural}/{name}     get / replace / merge-patch / delete
  GET/PUT/PATCH     {base}/namespaces/{ns}/{plural}/{name}/status
  GET               {base}/{plural}                            cluster-wide list / watch
  POST              /api/v1/namespaces/{ns}/events
"""
from __future__ import annotations

import asyncio
import json

from .kube import ApiError, FakeKube


def _status(code: int, reason: str, message: str) -> dict:
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
            "message": message, "reason": reason, "code": code}


def apiserver_app(kube: FakeKube, token: str | None = None):
    """aiohttp Application serving ``kube``; requests must carry ``Bearer <token>``
    when a token is set (401 Status otherwise)."""
    from aiohttp import web

    def err(e: ApiError):
        return web.json_response(_status(e.status, e.reason, e.message), status=e.status)

    @web.middleware
    async def auth(request, handler):
        if token is not None and request.headers.get("Authorization") != f"Bearer {token}":
            return web.json_response(_status(401, "Unauthorized", "Unauthorized"), status=401)
        try:
            return await handler(request)
        except ApiError as e:
            return err(e)
        except json.JSONDecodeError as e:
            return web.json_response(_status(400, "BadRequest", f"invalid JSON body: {e}"), status=400)

    def gv(request):
        m = request.match_info
        return m.get("group", ""), m["version"]

    def selector(request):
        sel = request.query.get("labelSelector")
        if not sel:
            return None
        return dict(kv.split("=", 1) for kv in sel.split(",") if "=" in kv)

    async def list_or_watch(request):
        group, version = gv(request)
        ns = request.match_info.get("ns")
        plural = request.match_info["plural"]
        if request.query.get("watch") in ("1", "true"):
            return await watch(request, group, plural, ns)
        items = await kube.list(group, version, ns, plural, label_selector=selector(request))
        return web.json_response({"kind": "List", "apiVersion": f"{group}/{version}".lstrip("/"),
                                  "metadata": {"resourceVersion": str(kube.current_rv())}, "items": items})

    async def watch(request, group, plural, ns):
        since = int(request.query.get("resourceVersion") or 0)
        timeout = float(request.query.get("timeoutSeconds") or 0) or None
        q, unsubscribe = kube.subscribe(group, plural, ns)
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        resp.enable_chunked_encoding()
        await resp.prepare(request)
        try:
            # objects changed after the client's list (the window between its list and
            # this watch): replayed as MODIFIED; the reconciler is level-triggered
            for o in await kube.list(group, None, ns, plural):
                if int(o["metadata"].get("resourceVersion", 0)) > since:
                    await resp.write((json.dumps({"type": "MODIFIED", "object": o}) + "\n").encode())
            loop = asyncio.get_running_loop()
            end = loop.time() + timeout if timeout else None
            while True:
                if end is not None and loop.time() >= end:
                    break
                tr = request.transport
                if tr is None or tr.is_closing():  # client went away: end the stream
                    break
                wait = 0.5 if end is None else max(0.0, min(0.5, end - loop.time()))
                try:
                    etype, obj = await asyncio.wait_for(q.get(), wait)
                except asyncio.TimeoutError:
                    continue
                await resp.write((json.dumps({"type": etype, "object": obj}) + "\n").encode())
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            unsubscribe()
        return resp

    async def create(request):
        group, version = gv(request)
        body = await request.json()
        o = await kube.create(group, version, request.match_info["ns"], request.match_info["plural"], body)
        return web.json_response(o, status=201)

    async def get(request):
        group, version = gv(request)
        m = request.match_info
        return web.json_response(await kube.get(group, version, m["ns"], m["plural"], m["name"]))

    def writer(status: bool):
        async def put(request):
            group, version = gv(request)
            m = request.match_info
            body = await request.json()
            return web.json_response(await kube.replace(group, version, m["ns"], m["plural"], m["name"], body,
                                                        status=status))

        async def patch(request):
            group, version = gv(request)
            m = request.match_info
            ctype = request.headers.get("Content-Type", "")
            if ctype.split(";")[0].strip() not in ("application/merge-patch+json", "application/json"):
                return web.json_response(_status(415, "UnsupportedMediaType",
                                                 f"patch type {ctype!r} not supported (merge-patch only)"),
                                         status=415)
            body = await request.json()
            return web.json_response(await kube.patch(group, version, m["ns"], m["plural"], m["name"], body,
                                                      status=status))
        return put, patch

    async def delete(request):
        group, version = gv(request)
        m = request.match_info
        o = await kube.delete(group, version, m["ns"], m["plural"], m["name"])
        return web.json_response(o)

    async def event(request):
        ev = await request.json()
        return web.json_response(await kube.create_event(request.match_info["ns"], ev), status=201)

    app = web.Application(middlewares=[auth])
    r = app.router
    r.add_post("/api/v1/namespaces/{ns}/events", event)
    put_main, patch_main = writer(False)
    put_status, patch_status = writer(True)
    for base in ("/apis/{group}/{version}", "/api/{version}"):
        ns_coll = base + "/namespaces/{ns}/{plural}"
        r.add_get(ns_coll, list_or_watch)
        r.add_post(ns_coll, create)
        r.add_get(ns_coll + "/{name}", get)
        r.add_put(ns_coll + "/{name}", put_main)
        r.add_patch(ns_coll + "/{name}", patch_main)
        r.add_delete(ns_coll + "/{name}", delete)
        r.add_get(ns_coll + "/{name}/status", get)
        r.add_put(ns_coll + "/{name}/status", put_status)
        r.add_patch(ns_coll + "/{name}/status", patch_status)
        r.add_get(base + "/{plural}", list_or_watch)
    return app


async def serve_apiserver(kube: FakeKube, host: str = "127.0.0.1", port: int = 0, token: str | None = None):
    """Start the front-end; returns (runner, base_url)."""
    from aiohttp import web

    runner = web.AppRunner(apiserver_app(kube, token), shutdown_timeout=2.0)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    sock = site._server.sockets[0]  # noqa: SLF001 - the bound port when port=0
    return runner, f"http://{host}:{sock.getsockname()[1]}"


def write_kubeconfig(path, server: str, token: str, namespace: str = "default") -> str:
    """A kubeconfig for ``RestKube.from_environment()`` pointing at ``server``."""
    import yaml

    kc = {"apiVersion": "v1", "kind": "Config", "current-context": "fake",
          "clusters": [{"name": "fake", "cluster": {"server": server}}],
          "users": [{"name": "operator", "user": {"token": token}}],
          "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "operator",
                                                    "namespace": namespace}}]}
    with open(path, "w") as f:
        yaml.safe_dump(kc, f)
    return str(path)
