"""Lock-free shutdown signalling for the engine's long-running processes.

The reference engine stops through Spring's context close: Tomcat's
connector is paused and the request pool gets <= 20 s to drain before the
JVM is forced down (``engine/src/main/java/io/seldon/engine/App.java:
89-92``).  Here the same lifecycle is driven by POSIX signals, and a Python
signal handler runs on the main thread *between bytecodes of whatever that
thread was doing* -- including the inside of ``threading.Event.set()``.  A
handler that takes a lock (``Event.set``, ``Popen.wait``, ``logging``) can
therefore re-enter itself on a second SIGTERM/SIGINT and block forever on
its own non-reentrant lock; the supervisor's ``killpg`` + forwarded SIGTERM
delivers exactly that double signal.

:class:`StopSignal` is the only thing a handler here touches: it sets plain
attributes and writes one byte to a non-blocking self-pipe -- no lock, no
allocation that can block -- and the main loop waits on the pipe with
``select``.  Every consumer (worker, gang rank, microservice, supervisor)
observes the flag from its own loop and does the real work (forwarding,
draining, escalation) there, never inside the handler.
"""
from __future__ import annotations

import os
import select
import signal
import time
from typing import Iterable, Optional


class StopSignal:
    """A stop request set by signal handlers, waited on by the main loop."""

    POLL_S = 0.5

    def __init__(self) -> None:
        self._r, self._w = os.pipe()
        os.set_blocking(self._r, False)
        os.set_blocking(self._w, False)
        self.requested = False          # plain attribute: the handler's only state change
        self.first_signal: Optional[int] = None
        self.signals = 0                # how many stop signals arrived (best effort)
        self.first_at: Optional[float] = None

    # -- handler side: async-signal safe (attributes + one write) --------------
    def handler(self, signum, frame=None) -> None:  # noqa: ARG002
        self.signals += 1
        if not self.requested:
            self.first_signal = signum
            self.first_at = time.monotonic()
            self.requested = True
        try:
            os.write(self._w, b"\x01")
        except OSError:  # pipe full: a wake-up is already pending
            pass

    def install(self, signums: Iterable[int] = (signal.SIGTERM, signal.SIGINT)) -> "StopSignal":
        """Install the handlers (main thread only).  The pipe also becomes the
        interpreter's wakeup fd: a signal delivered to one of the engine's
        native threads runs CPython's C-level handler *there*, so the main
        thread's ``select`` is never interrupted; the byte the C handler
        writes to the wakeup fd is what wakes it."""
        for s in signums:
            signal.signal(s, self.handler)
        try:
            signal.set_wakeup_fd(self._w, warn_on_full_buffer=False)
        except (ValueError, OSError):  # not the main thread: the bounded wait still polls
            pass
        return self

    # -- main-loop side ----------------------------------------------------------
    def set(self) -> None:
        """Request a stop from ordinary code (same path as a signal)."""
        self.handler(0)

    def is_set(self) -> bool:
        return self.requested

    def _drain(self) -> None:
        try:
            while os.read(self._r, 4096):
                pass
        except (BlockingIOError, InterruptedError):
            pass
        except OSError:
            pass

    def wait(self, timeout: Optional[float] = None) -> bool:
        """Block until a stop was requested (or ``timeout`` s passed); returns
        the flag.  The wakeup-fd byte (or the handler's own) makes ``select``
        return; CPython runs the pending Python-level handler before the next
        bytecode, so the flag is set by the time the loop re-checks it."""
        deadline = None if timeout is None else time.monotonic() + timeout
        while not self.requested:
            left = None if deadline is None else deadline - time.monotonic()
            if left is not None and left <= 0:
                break
            # bounded: a lost wake-up costs at most one poll interval
            step = self.POLL_S if left is None else max(0.0, min(left, self.POLL_S))
            try:
                select.select([self._r], [], [], step)
            except (InterruptedError, ValueError):
                pass
            self._drain()
        return self.requested

    def fileno(self) -> int:
        return self._r

    def close(self) -> None:
        try:  # never leave the interpreter writing signal bytes into a closed (reusable) fd
            old = signal.set_wakeup_fd(-1)
            if old not in (-1, self._w):
                signal.set_wakeup_fd(old)
        except (ValueError, OSError):
            pass
        for fd in (self._r, self._w):
            try:
                os.close(fd)
            except OSError:
                pass
