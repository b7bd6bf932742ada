"""A kopf-style operator framework (kopf itself is not installable offline).

Same programming model as the reference's kopf usage (mlflow_operator.py:26-27,
``kopf.event``): handlers registered per (group, version, plural) with
decorators, called with kopf-like kwargs (``spec, name, namespace, status,
body, meta, logger``), plus the daemon form that fixes the reference's
structural defect: the reference registered ONE never-returning coroutine for
both create and update, so updates were never processed.  Here each object
gets a *daemon* task that owns its reconcile loop; a spec change (generation
bump) cancels and restarts it with the new spec; deletion cancels it.

Handler failures are retried with exponential backoff (kopf's default
behaviour for unexpected errors); ``PermanentError`` stops retrying.
"""
from __future__ import annotations

import asyncio
import logging
import traceback
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable

from .clock import RealClock
from .kube import ApiError

log = logging.getLogger("mlopamd.operator")


class PermanentError(Exception):
    """Do not retry this handler for this object generation."""


class TemporaryError(Exception):
    def __init__(self, msg: str = "", delay: float = 10.0):
        super().__init__(msg)
        self.delay = delay


@dataclass
class _Resource:
    group: str
    version: str
    plural: str
    on_create: list = field(default_factory=list)
    on_update: list = field(default_factory=list)
    on_delete: list = field(default_factory=list)
    on_resume: list = field(default_factory=list)
    daemons: list = field(default_factory=list)
    on_event: list = field(default_factory=list)


def cr_logger(name: str, namespace: str) -> logging.Logger:
    """Per-CR logger named ``{name}-{namespace}`` (reference mlflow_operator.py:38-41)."""
    lg = logging.getLogger(f"{name}-{namespace}")
    lg.setLevel(logging.INFO)
    return lg


class Operator:
    def __init__(self, kube, clock=None, namespace: str | None = None,
                 backoff: tuple = (1.0, 2.0, 5.0, 10.0, 30.0, 60.0)):
        self.kube = kube
        self.clock = clock or RealClock()
        self.namespace = namespace
        self.backoff = backoff
        self._res: dict[tuple, _Resource] = {}
        self._daemons: dict[tuple, asyncio.Task] = {}
        self._stopped: dict[tuple, asyncio.Event] = {}
        self._generation: dict[tuple, int] = {}
        self._tasks: list[asyncio.Task] = []
        self.handler_errors: list[tuple] = []

    # ---------------------------------------------------- registration --
    def _r(self, group, version, plural) -> _Resource:
        return self._res.setdefault((group, version, plural), _Resource(group, version, plural))

    def on_create(self, group, version, plural):
        def deco(fn):
            self._r(group, version, plural).on_create.append(fn)
            return fn
        return deco

    def on_update(self, group, version, plural):
        def deco(fn):
            self._r(group, version, plural).on_update.append(fn)
            return fn
        return deco

    def on_delete(self, group, version, plural):
        def deco(fn):
            self._r(group, version, plural).on_delete.append(fn)
            return fn
        return deco

    def on_resume(self, group, version, plural):
        def deco(fn):
            self._r(group, version, plural).on_resume.append(fn)
            return fn
        return deco

    def event_handler(self, group, version, plural):
        """``async def fn(event_type, body, **kw)`` for EVERY watch event (incl. status-only
        changes, which do not bump ``generation``) — e.g. to react to owned objects."""
        def deco(fn):
            self._r(group, version, plural).on_event.append(fn)
            return fn
        return deco

    def daemon(self, group, version, plural):
        """``async def fn(stopped: asyncio.Event, **kwargs)`` runs while the object exists."""
        def deco(fn):
            self._r(group, version, plural).daemons.append(fn)
            return fn
        return deco

    # ---------------------------------------------------------- events --
    async def event(self, body: dict, type: str, reason: str, message: str):  # noqa: A002
        """Post a K8s Event about ``body`` (kopf.event equivalent)."""
        md = body.get("metadata", {})
        ev = {
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{md.get('name', 'obj')}."},
            "involvedObject": {"apiVersion": body.get("apiVersion"), "kind": body.get("kind"),
                               "name": md.get("name"), "namespace": md.get("namespace"),
                               "uid": md.get("uid")},
            "type": type, "reason": reason, "message": message,
            "source": {"component": "mlflow-operator"},
            "firstTimestamp": None, "count": 1,
        }
        try:
            await self.kube.create_event(md.get("namespace"), ev)
        except Exception as e:  # events are best-effort (kopf does the same)
            log.warning("event %s/%s failed: %s", reason, md.get("name"), e)

    # --------------------------------------------------------- running --
    def _kwargs(self, body: dict, logger: logging.Logger) -> dict:
        md = body.get("metadata", {})
        return dict(spec=body.get("spec", {}) or {}, status=body.get("status"), body=body, meta=md,
                    name=md.get("name"), namespace=md.get("namespace"), uid=md.get("uid"),
                    logger=logger, operator=self)

    async def _call(self, fn: Callable[..., Awaitable[Any]], body: dict, **extra):
        md = body.get("metadata", {})
        logger = cr_logger(md.get("name"), md.get("namespace"))
        attempt = 0
        while True:
            try:
                return await fn(**self._kwargs(body, logger), **extra)
            except asyncio.CancelledError:
                raise
            except PermanentError as e:
                logger.error("[%s/%s] handler %s failed permanently: %s", md.get("namespace"),
                             md.get("name"), fn.__name__, e)
                self.handler_errors.append((md.get("name"), fn.__name__, repr(e)))
                return None
            except Exception as e:  # noqa: BLE001 - kopf retries unexpected errors
                delay = e.delay if isinstance(e, TemporaryError) else self.backoff[min(attempt, len(self.backoff) - 1)]
                self.handler_errors.append((md.get("name"), fn.__name__, repr(e)))
                logger.warning("[%s/%s] handler %s failed (%s); retry in %.0fs\n%s", md.get("namespace"),
                               md.get("name"), fn.__name__, e, delay,
                               traceback.format_exc(limit=3) if not isinstance(e, (ApiError, TemporaryError)) else "")
                attempt += 1
                await self.clock.sleep(delay)
                try:  # re-read the object: it may have changed or gone
                    body = await self.kube.get(self._grp(body), self._ver(body), md.get("namespace"),
                                               self._plural_of(body), md.get("name"))
                except ApiError as ge:
                    if ge.status == 404:
                        return None

    def _grp(self, body):
        return body.get("apiVersion", "/").split("/")[0]

    def _ver(self, body):
        return body.get("apiVersion", "/").split("/")[-1]

    def _plural_of(self, body):
        for (g, v, p) in self._res:
            if g == self._grp(body):
                return p
        return None

    def _start_daemons(self, res: _Resource, key, body):
        if not res.daemons:
            return
        stopped = asyncio.Event()
        self._stopped[key] = stopped

        async def runner():
            await asyncio.gather(*(self._call(d, body, stopped=stopped) for d in res.daemons))

        self._daemons[key] = asyncio.get_running_loop().create_task(runner())

    async def _stop_daemons(self, key):
        task = self._daemons.pop(key, None)
        ev = self._stopped.pop(key, None)
        if ev:
            ev.set()
        if task and not task.done():
            task.cancel()
            try:
                await task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass

    async def _dispatch(self, res: _Resource, etype: str, body: dict):
        md = body["metadata"]
        key = (res.plural, md.get("namespace"), md.get("name"))
        gen = md.get("generation", 1)
        for h in res.on_event:
            try:
                await h(event_type=etype, body=body, operator=self)
            except Exception as e:  # noqa: BLE001 - observers never break dispatch
                log.warning("event handler %s failed: %s", h.__name__, e)
        if not (res.on_create or res.on_update or res.on_delete or res.on_resume or res.daemons):
            return
        if etype == "DELETED":
            self._generation.pop(key, None)
            await self._stop_daemons(key)
            for h in res.on_delete:
                await self._call(h, body)
            return
        known = key in self._generation
        if not known:
            self._generation[key] = gen
            resumed = bool(body.get("status"))
            for h in (res.on_resume if resumed and res.on_resume else res.on_create):
                await self._call(h, body)
            self._start_daemons(res, key, body)
        elif gen != self._generation[key]:
            self._generation[key] = gen
            await self._stop_daemons(key)
            for h in res.on_update:
                await self._call(h, body)
            self._start_daemons(res, key, body)

    async def _watch_loop(self, res: _Resource):
        async for etype, body in self.kube.watch(res.group, res.version, res.plural, self.namespace):
            try:
                await self._dispatch(res, etype, body)
            except Exception as e:  # noqa: BLE001 - never kill the watch loop
                log.exception("dispatch failed: %s", e)

    async def start(self):
        for res in self._res.values():
            self._tasks.append(asyncio.get_running_loop().create_task(self._watch_loop(res)))

    async def stop(self):
        for key in list(self._daemons):
            await self._stop_daemons(key)
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._tasks.clear()

    async def run(self):
        await self.start()
        try:
            await asyncio.gather(*self._tasks)
        finally:
            await self.stop()
