"""MLflow model-registry access (the reference's ``MlflowClient`` usage,
mlflow_operator.py:44,59,131) without the ``mlflow`` package.

* ``MlflowRestClient`` — async REST client of the MLflow 2.x registry API:
  ``registered-models/alias`` (get/set/delete), ``model-versions/get|create|set-tag``,
  ``registered-models/create``.  Tracking URI / token from the same env vars the
  ``mlflow-creds`` secret provides to the reference (MLFLOW_TRACKING_URI,
  MLFLOW_TRACKING_TOKEN / _USERNAME / _PASSWORD).
* ``SqliteRegistry`` — a local sqlite-backed registry with the same interface
  (BASELINE config 1: "local sqlite MLFlow"); ``serve_registry`` exposes it over
  the same REST paths so the REST client can be tested end-to-end.

Error taxonomy (fixes the reference's "any exception = alias missing",
mlflow_operator.py:61): ``NotFound`` (alias / version really absent) vs
``RegistryUnavailable`` (5xx, connection errors, timeouts) — only NotFound
deletes a deployment.
"""
from __future__ import annotations

import asyncio
import json
import os
import sqlite3
import threading
import time
from dataclasses import dataclass, field


class RegistryError(Exception):
    pass


class NotFound(RegistryError):
    pass


class RegistryUnavailable(RegistryError):
    pass


@dataclass
class ModelVersion:
    name: str
    version: str
    source: str
    run_id: str = ""
    tags: dict = field(default_factory=dict)
    aliases: list = field(default_factory=list)
    status: str = "READY"

    @classmethod
    def from_json(cls, d: dict) -> "ModelVersion":
        tags = d.get("tags") or []
        if isinstance(tags, list):
            tags = {t["key"]: t["value"] for t in tags}
        return cls(name=d.get("name"), version=str(d.get("version")), source=d.get("source", ""),
                   run_id=d.get("run_id", ""), tags=tags, aliases=list(d.get("aliases") or []),
                   status=d.get("status", "READY"))

    def to_json(self) -> dict:
        return {"name": self.name, "version": self.version, "source": self.source,
                "run_id": self.run_id, "status": self.status, "aliases": self.aliases,
                "tags": [{"key": k, "value": v} for k, v in self.tags.items()]}


# ------------------------------------------------------------- sqlite fake --

class SqliteRegistry:
    """Thread-safe sqlite model registry (':memory:' or a file)."""

    def __init__(self, path: str = ":memory:"):
        self._db = sqlite3.connect(path, check_same_thread=False)
        self._lock = threading.Lock()
        self.fail_mode: str | None = None  # "unavailable" -> every call raises RegistryUnavailable
        with self._lock:
            self._db.executescript("""
                CREATE TABLE IF NOT EXISTS models (name TEXT PRIMARY KEY, created REAL);
                CREATE TABLE IF NOT EXISTS versions (name TEXT, version INTEGER, source TEXT,
                    run_id TEXT, tags TEXT, created REAL, PRIMARY KEY (name, version));
                CREATE TABLE IF NOT EXISTS aliases (name TEXT, alias TEXT, version INTEGER,
                    PRIMARY KEY (name, alias));
            """)

    def _check(self):
        if self.fail_mode == "unavailable":
            raise RegistryUnavailable("registry unavailable (injected)")

    def create_registered_model(self, name: str):
        self._check()
        with self._lock:
            self._db.execute("INSERT OR IGNORE INTO models VALUES (?, ?)", (name, time.time()))
            self._db.commit()

    def create_model_version(self, name: str, source: str, run_id: str = "", tags: dict | None = None) -> ModelVersion:
        self._check()
        self.create_registered_model(name)
        with self._lock:
            cur = self._db.execute("SELECT COALESCE(MAX(version), 0) FROM versions WHERE name=?", (name,))
            v = cur.fetchone()[0] + 1
            self._db.execute("INSERT INTO versions VALUES (?, ?, ?, ?, ?, ?)",
                             (name, v, source, run_id, json.dumps(tags or {}), time.time()))
            self._db.commit()
        return self._version(name, v)

    def set_tag(self, name, version, key, value):
        self._check()
        mv = self._version(name, int(version))
        mv.tags[key] = value
        with self._lock:
            self._db.execute("UPDATE versions SET tags=? WHERE name=? AND version=?",
                             (json.dumps(mv.tags), name, int(version)))
            self._db.commit()

    def set_alias(self, name: str, alias: str, version) -> None:
        self._check()
        self._version(name, int(version))
        with self._lock:
            self._db.execute("INSERT OR REPLACE INTO aliases VALUES (?, ?, ?)", (name, alias, int(version)))
            self._db.commit()

    def delete_alias(self, name: str, alias: str) -> None:
        self._check()
        with self._lock:
            self._db.execute("DELETE FROM aliases WHERE name=? AND alias=?", (name, alias))
            self._db.commit()

    def _version(self, name, v: int) -> ModelVersion:
        with self._lock:
            row = self._db.execute("SELECT source, run_id, tags FROM versions WHERE name=? AND version=?",
                                   (name, v)).fetchone()
            if row is None:
                raise NotFound(f"Model Version (name={name}, version={v}) not found")
            al = [r[0] for r in self._db.execute("SELECT alias FROM aliases WHERE name=? AND version=?", (name, v))]
        return ModelVersion(name, str(v), row[0], row[1], json.loads(row[2]), al)

    # -- client interface (sync core; async wrappers below) --
    def get_model_version(self, name: str, version) -> ModelVersion:
        self._check()
        return self._version(name, int(version))

    def get_model_version_by_alias(self, name: str, alias: str) -> ModelVersion:
        self._check()
        with self._lock:
            row = self._db.execute("SELECT version FROM aliases WHERE name=? AND alias=?", (name, alias)).fetchone()
        if row is None:
            raise NotFound(f"Registered model alias {alias} not found.")
        return self._version(name, row[0])


class LocalMlflowClient:
    """Async facade over a ``SqliteRegistry`` (same interface as the REST client)."""

    def __init__(self, registry: SqliteRegistry):
        self.registry = registry

    async def get_model_version_by_alias(self, name, alias) -> ModelVersion:
        return self.registry.get_model_version_by_alias(name, alias)

    async def get_model_version(self, name, version) -> ModelVersion:
        return self.registry.get_model_version(name, version)

    async def close(self):
        pass


# ------------------------------------------------------------- REST client --

class MlflowRestClient:
    def __init__(self, tracking_uri: str | None = None, token: str | None = None,
                 username: str | None = None, password: str | None = None, timeout_s: float = 10.0):
        self.uri = (tracking_uri or os.environ.get("MLFLOW_TRACKING_URI", "http://localhost:5000")).rstrip("/")
        self.token = token or os.environ.get("MLFLOW_TRACKING_TOKEN")
        self.auth = (username or os.environ.get("MLFLOW_TRACKING_USERNAME"),
                     password or os.environ.get("MLFLOW_TRACKING_PASSWORD"))
        self.timeout_s = timeout_s
        self._session = None

    async def _sess(self):
        import aiohttp

        if self._session is None or self._session.closed:
            headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
            auth = aiohttp.BasicAuth(*self.auth) if all(self.auth) else None
            self._session = aiohttp.ClientSession(headers=headers, auth=auth,
                                                  timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        return self._session

    async def close(self):
        if self._session is not None:
            await self._session.close()

    async def _call(self, method: str, path: str, params=None, body=None) -> dict:
        import aiohttp

        try:
            s = await self._sess()
            async with s.request(method, f"{self.uri}/api/2.0/mlflow/{path}", params=params,
                                 json=body) as r:
                txt = await r.text()
                if r.status == 404 or (r.status == 400 and "RESOURCE_DOES_NOT_EXIST" in txt):
                    raise NotFound(txt)
                if r.status >= 400:
                    if r.status >= 500 or r.status == 429:
                        raise RegistryUnavailable(f"{r.status}: {txt[:200]}")
                    if "RESOURCE_DOES_NOT_EXIST" in txt or "INVALID_PARAMETER_VALUE" in txt:
                        raise NotFound(txt)
                    raise RegistryError(f"{r.status}: {txt[:200]}")
                return json.loads(txt) if txt else {}
        except (aiohttp.ClientError, asyncio.TimeoutError, OSError) as e:
            raise RegistryUnavailable(str(e)) from e

    async def get_model_version_by_alias(self, name, alias) -> ModelVersion:
        d = await self._call("GET", "registered-models/alias", params={"name": name, "alias": alias})
        return ModelVersion.from_json(d["model_version"])

    async def get_model_version(self, name, version) -> ModelVersion:
        d = await self._call("GET", "model-versions/get", params={"name": name, "version": str(version)})
        return ModelVersion.from_json(d["model_version"])

    async def create_registered_model(self, name):
        return await self._call("POST", "registered-models/create", body={"name": name})

    async def create_model_version(self, name, source, run_id="", tags=None) -> ModelVersion:
        d = await self._call("POST", "model-versions/create",
                             body={"name": name, "source": source, "run_id": run_id,
                                   "tags": [{"key": k, "value": v} for k, v in (tags or {}).items()]})
        return ModelVersion.from_json(d["model_version"])

    async def set_alias(self, name, alias, version):
        return await self._call("POST", "registered-models/alias",
                                body={"name": name, "alias": alias, "version": str(version)})

    async def delete_alias(self, name, alias):
        return await self._call("DELETE", "registered-models/alias", params={"name": name, "alias": alias})


# --------------------------------------------------------- REST server --

def registry_app(registry: SqliteRegistry):
    """aiohttp application serving the registry subset of the MLflow REST API."""
    from aiohttp import web

    def err(status, code, msg):
        return web.json_response({"error_code": code, "message": msg}, status=status)

    async def wrap(fn):
        try:
            return web.json_response(fn())
        except NotFound as e:
            return err(404, "RESOURCE_DOES_NOT_EXIST", str(e))
        except RegistryUnavailable as e:
            return err(503, "TEMPORARILY_UNAVAILABLE", str(e))

    async def get_alias(req):
        q = req.query
        return await wrap(lambda: {"model_version": registry.get_model_version_by_alias(q["name"], q["alias"]).to_json()})

    async def set_alias(req):
        b = await req.json()
        return await wrap(lambda: registry.set_alias(b["name"], b["alias"], b["version"]) or {})

    async def del_alias(req):
        q = req.query
        return await wrap(lambda: registry.delete_alias(q["name"], q["alias"]) or {})

    async def get_version(req):
        q = req.query
        return await wrap(lambda: {"model_version": registry.get_model_version(q["name"], q["version"]).to_json()})

    async def create_model(req):
        b = await req.json()
        return await wrap(lambda: registry.create_registered_model(b["name"]) or {"registered_model": {"name": b["name"]}})

    async def create_version(req):
        b = await req.json()
        tags = {t["key"]: t["value"] for t in b.get("tags", [])}
        return await wrap(lambda: {"model_version": registry.create_model_version(
            b["name"], b["source"], b.get("run_id", ""), tags).to_json()})

    async def set_tag(req):
        b = await req.json()
        return await wrap(lambda: registry.set_tag(b["name"], b["version"], b["key"], b["value"]) or {})

    app = web.Application()
    p = "/api/2.0/mlflow/"
    app.router.add_get(p + "registered-models/alias", get_alias)
    app.router.add_post(p + "registered-models/alias", set_alias)
    app.router.add_delete(p + "registered-models/alias", del_alias)
    app.router.add_get(p + "model-versions/get", get_version)
    app.router.add_post(p + "registered-models/create", create_model)
    app.router.add_post(p + "model-versions/create", create_version)
    app.router.add_post(p + "model-versions/set-tag", set_tag)
    return app


async def serve_registry(registry: SqliteRegistry, host: str = "127.0.0.1", port: int = 0):
    """Start the REST server; returns (runner, base_url)."""
    from aiohttp import web

    runner = web.AppRunner(registry_app(registry))
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    sock = site._server.sockets[0]  # noqa: SLF001
    return runner, f"http://{host}:{sock.getsockname()[1]}"
