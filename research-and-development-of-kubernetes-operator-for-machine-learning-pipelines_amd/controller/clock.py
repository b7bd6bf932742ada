"""Injectable clocks.

The reference sleeps on the wall clock everywhere (poll 60 s, canary step
60 s, retries 10 s: mlflow_operator.py:154,294,352), which makes its flows
untestable.  Every wait in this control plane goes through a ``Clock``:
``RealClock`` for production, ``VirtualClock`` for tests, where a 540 s canary
runs in milliseconds (time only advances when every task is blocked on it).
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import time


class RealClock:
    def now(self) -> float:
        return time.time()

    def monotonic(self) -> float:
        return time.monotonic()

    async def sleep(self, seconds: float) -> None:
        await asyncio.sleep(max(0.0, seconds))


class VirtualClock:
    """Discrete-event clock for asyncio tests.

    ``sleep(s)`` parks the caller until virtual time reaches now + s.  A
    background driver advances time to the earliest deadline whenever the
    event loop has no other ready work (checked by yielding a few times),
    so real I/O done by fakes (in-process HTTP) still completes first."""

    def __init__(self, start: float = 1_700_000_000.0, idle_yields: int = 20):
        self._t = start
        self._heap: list = []
        self._seq = itertools.count()
        self._idle_yields = idle_yields
        self._driver: asyncio.Task | None = None

    def now(self) -> float:
        return self._t

    def monotonic(self) -> float:
        return self._t

    async def sleep(self, seconds: float) -> None:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        heapq.heappush(self._heap, (self._t + max(0.0, seconds), next(self._seq), fut))
        self._ensure_driver()
        await fut

    def _ensure_driver(self):
        if self._driver is None or self._driver.done():
            self._driver = asyncio.get_running_loop().create_task(self._drive())

    async def _drive(self):
        while self._heap:
            for _ in range(self._idle_yields):
                await asyncio.sleep(0)
            # drop cancelled sleepers
            while self._heap and self._heap[0][2].done():
                heapq.heappop(self._heap)
            if not self._heap:
                break
            t, _, fut = heapq.heappop(self._heap)
            self._t = max(self._t, t)
            if not fut.done():
                fut.set_result(None)

    def advance(self, seconds: float) -> None:
        """Manually move time forward (wakes every sleeper that is due)."""
        self._t += seconds
        while self._heap and self._heap[0][0] <= self._t:
            _, _, fut = heapq.heappop(self._heap)
            if not fut.done():
                fut.set_result(None)
