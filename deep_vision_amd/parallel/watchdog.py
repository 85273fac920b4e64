"""Collective watchdog: turn a hung or failed collective into a prompt, whole-job exit.

The reference has no failure handling beyond Hourglass's NaN-skip
(R/Hourglass/tensorflow/train.py:126-130). In a one-process-per-GPU job a dead or wedged rank
leaves its peers blocked inside an RCCL all-reduce forever; this module bounds that:

* ``CommWatchdog.guard(name)`` brackets a region that issues / waits on collectives. A
  background thread checks the oldest open region; if it has been open longer than
  ``timeout`` seconds (``DV_COMM_TIMEOUT``), it dumps every thread's Python stack and ends the
  process with ``os._exit(EXIT_COMM_TIMEOUT)`` -- no Python cleanup that could block on the
  wedged communicator. The launcher (torch.distributed.run / deep_vision_amd.launch) sees a
  non-zero exit and tears the remaining ranks down. A restart is a fresh child process from
  the launcher; a GPU-initialised process is never re-exec'ed.
* Exceptions raised inside a guard by the backend (RCCL async errors surfaced by
  ``TORCH_NCCL_ASYNC_ERROR_HANDLING``, gloo "connection closed by peer") are reported and turned
  into ``os._exit(EXIT_COMM_ERROR)`` for the same reason.
* ``CommWatchdog.track(name, event)`` watches GPU-side completion instead of a host region: the
  caller records an event after the work it enqueued (a HIP-graph replay of a data-parallel step,
  whose captured RCCL all-reduces run with ProcessGroupNCCL's async error handling off, or an
  eager step whose ``work.wait()`` only made the compute stream wait). The thread polls
  ``event.query()``; an event not complete ``timeout`` seconds after it was recorded ends the
  process the same way. A dead or wedged peer therefore ends the job in graph mode too.
* ``install_backend_error_handling()`` sets the RCCL env knobs that make the process group
  surface async errors and abort the communicator instead of hanging (must run before the
  process group is created).
"""
from __future__ import annotations

import contextlib
import faulthandler
import os
import sys
import threading
import time

EXIT_COMM_TIMEOUT = 75
EXIT_COMM_ERROR = 76


def install_backend_error_handling(timeout_s: int | None = None) -> None:
    """RCCL (ProcessGroupNCCL) settings: async error handling tears the communicator down on a
    failed / timed-out collective; the desync debug report names the rank that fell behind."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "0")
    if timeout_s:
        os.environ.setdefault("DV_COMM_TIMEOUT", str(int(timeout_s)))


# Held by a watchdog while it queries its events, and by a HIP-graph capture for its whole
# duration (train/graph.py): event queries from another thread during a global-mode capture are
# illegal, so polling pauses while a step is being captured.
_POLL_LOCK = threading.Lock()


@contextlib.contextmanager
def suspend_polling():
    with _POLL_LOCK:
        yield


class CommWatchdog:
    def __init__(self, timeout: float | None = None, on_timeout=None, poll: float | None = None):
        self.timeout = float(timeout if timeout is not None else os.environ.get("DV_COMM_TIMEOUT", "600"))
        self.on_timeout = on_timeout
        self.poll = poll if poll is not None else max(0.05, min(2.0, self.timeout / 10))
        self._open = {}  # token -> (name, start)
        self._events = []  # (name, event, recorded-at), oldest first
        self._lock = threading.Lock()
        self._next = 0
        self._stop = threading.Event()
        self._t = None
        self.fired = None

    def start(self):
        if self.timeout > 0 and self._t is None:
            self._t = threading.Thread(target=self._run, name="dv-comm-watchdog", daemon=True)
            self._t.start()
        return self

    def stop(self):
        self._stop.set()

    @contextlib.contextmanager
    def guard(self, name: str):
        with self._lock:
            tok = self._next
            self._next += 1
            self._open[tok] = (name, time.monotonic())
        try:
            yield
        except Exception as e:  # backend error inside a collective region
            if self._is_comm_error(e):
                self._abort(EXIT_COMM_ERROR, f"collective '{name}' failed: {type(e).__name__}: {e}")
            raise
        finally:
            with self._lock:
                self._open.pop(tok, None)

    def track(self, name: str, event) -> None:
        """Watch ``event`` (anything with ``query() -> bool``, e.g. a torch.cuda.Event recorded
        after a graph replay): the process ends if it has not completed ``timeout`` s from now."""
        if self.timeout <= 0:
            return
        with self._lock:
            self._events.append((name, event, time.monotonic()))

    def pending(self) -> int:
        with self._lock:
            return len(self._events)

    def _check_events(self, now):
        """Drop completed events (in order); return the oldest incomplete one past the deadline."""
        while True:
            with self._lock:
                if not self._events:
                    return None
                name, ev, t0 = self._events[0]
            try:
                with _POLL_LOCK:
                    done = bool(ev.query())
            except Exception as e:  # a failed stream (aborted communicator): report it as a comm error
                return name, t0, f"{type(e).__name__}: {e}"
            if not done:
                return (name, t0, None) if now - t0 > self.timeout else None
            with self._lock:
                if self._events and self._events[0][1] is ev:
                    self._events.pop(0)

    @staticmethod
    def _is_comm_error(e: BaseException) -> bool:
        """By exception TYPE (torch.distributed's backend / network / store errors), plus gloo's
        transport failures, which surface as a RuntimeError raised from gloo's own sources (the
        message carries the ``gloo/transport`` source path). Anything else propagates normally
        (free-text keywords killed ranks on unrelated errors)."""
        import torch.distributed as dist

        types = tuple(t for t in (getattr(dist, n, None) for n in ("DistBackendError", "DistNetworkError",
                                                                  "DistStoreError", "DistError"))
                      if isinstance(t, type))
        if types and isinstance(e, types):
            return True
        return type(e) is RuntimeError and "gloo/transport" in str(e)

    def _abort(self, code: int, why: str):
        self.fired = why
        sys.stderr.write(f"[dv-comm-watchdog] {why}; aborting rank {os.environ.get('RANK', '0')}\n")
        try:
            faulthandler.dump_traceback(all_threads=True)
        except Exception:
            pass
        sys.stderr.flush()
        if self.on_timeout is not None:
            self.on_timeout(code, why)
            return
        os._exit(code)

    def _run(self):
        while not self._stop.wait(self.poll):
            now = time.monotonic()
            with self._lock:
                stale = [(n, t0) for n, t0 in self._open.values() if now - t0 > self.timeout]
            if stale:
                name, t0 = min(stale, key=lambda v: v[1])
                self._abort(EXIT_COMM_TIMEOUT, f"collective region '{name}' open for {now - t0:.1f}s "
                                               f"(> {self.timeout:.0f}s)")
                return
            late = self._check_events(now)
            if late is not None:
                name, t0, err = late
                if err is not None:
                    self._abort(EXIT_COMM_ERROR, f"GPU work '{name}' failed: {err}")
                else:
                    self._abort(EXIT_COMM_TIMEOUT, f"GPU work '{name}' not complete {now - t0:.1f}s after it was "
                                                   f"enqueued (> {self.timeout:.0f}s)")
                return
