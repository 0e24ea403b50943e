"""Race detection / debug helpers and a collective watchdog.

The reference has none of these: blocking P2P ops hang forever when a peer
dies, four ranks race on ``download=True``, and timers read host time while
collectives are in flight.  Here:

* :func:`debug_env` switches on serialised kernel launches
  (``AMD_SERIALIZE_KERNEL=3``, ``HIP_LAUNCH_BLOCKING=1``) and RCCL logging
  (``NCCL_DEBUG``) for reproducing a race -- it must run before the GPU is
  initialised;
* :func:`rank0_first` lets rank 0 do one-off work (dataset preparation) while
  the others wait at a barrier, then the others proceed;
* :class:`CommWatchdog` watches the native communicator's stream from a host
  thread and aborts the process (so torchrun can restart it) when a posted
  collective makes no progress for ``timeout_s`` -- instead of hanging
  every rank until the job's wall-clock limit;
* :class:`FailureBroadcast` propagates a failure that ONE rank detects (a
  broken pipeline shape contract on rank 0, an exception inside a stage) to
  every other rank through the rendezvous store, so ranks blocked in a
  point-to-point receive that will never be matched exit non-zero instead of
  hanging (RCCL has no peer-failure detection on xGMI).
"""
from __future__ import annotations

import contextlib
import itertools
import os
import sys
import threading
import time
from typing import Callable, Iterator, Optional

import torch
import torch.distributed as dist


def debug_env(serialize: bool = True, rccl_debug: str = "WARN") -> dict:
    """Set debug environment variables (call before any GPU work)."""
    env = {}
    if serialize:
        env.update(AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3", HIP_LAUNCH_BLOCKING="1")
    if rccl_debug:
        env["NCCL_DEBUG"] = rccl_debug
    env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.update(env)
    return env


@contextlib.contextmanager
def rank0_first(group=None) -> Iterator[None]:
    """``with rank0_first(): prepare_data()`` -- rank 0 runs first, others after a barrier."""
    init = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if init else 0
    if init and rank != 0:
        dist.barrier(group)
    try:
        yield
    finally:
        if init and rank == 0:
            dist.barrier(group)


class CommWatchdog:
    """Abort when the communicator stream stops making progress.

    ``poll()`` is cheap: it records an event on the comm stream and checks
    (hipEventQuery) whether the previous one has completed.  If an event has
    been pending for longer than ``timeout_s`` the watchdog calls
    ``on_timeout`` (default: print a diagnostic and ``os._exit(1)``).
    """

    def __init__(self, comm, timeout_s: float = 600.0, interval_s: float = 5.0,
                 on_timeout: Optional[Callable[[], None]] = None):
        self.comm = comm
        self.timeout_s = timeout_s
        self.interval_s = interval_s
        self.on_timeout = on_timeout or self._default_timeout
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._pending: Optional[torch.cuda.Event] = None
        self._since = 0.0

    def _default_timeout(self) -> None:
        print(f"[dmp watchdog] rank {getattr(self.comm, 'rank', '?')}: collective stream made no "
              f"progress for {self.timeout_s:.0f}s -- aborting so the launcher can restart",
              file=sys.stderr, flush=True)
        os._exit(1)

    def poll(self) -> bool:
        """One check; returns False if the timeout fired."""
        native = getattr(self.comm, "native", None)
        if native is None:
            return True
        now = time.monotonic()
        if self._pending is None:
            stream = torch.cuda.ExternalStream(native.stream_handle(), device=self.comm.device)
            ev = torch.cuda.Event()
            ev.record(stream)
            self._pending, self._since = ev, now
            return True
        if self._pending.query():
            self._pending = None
            return True
        if now - self._since > self.timeout_s:
            self.on_timeout()
            return False
        return True

    def _run(self) -> None:
        while not self._stop.wait(self.interval_s):
            if not self.poll():
                return

    def start(self) -> "CommWatchdog":
        self._thread = threading.Thread(target=self._run, name="dmp-comm-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.interval_s * 2)


_fail_counter = itertools.count()


class FailureBroadcast:
    """Out-of-band "this job has failed" flag shared by the ranks of a group.

    ``publish(msg)`` (on the failing rank) writes the message under a key of
    the rendezvous store, then waits -- at most ``ack_timeout_s`` -- until
    every other rank's watcher has acknowledged it, so its own exit (which may
    take the store server with it on rank 0) cannot race the others' polls.
    Every rank runs a daemon watcher thread that polls the key with a
    non-blocking ``store.check`` (a blocking ``store.wait`` would hold the
    store client's lock against the main thread); when another rank's flag
    appears it prints the message and ``os._exit(exit_code)`` -- the process
    may be stuck inside a receive (gloo) or a stream wait (RCCL) that no
    Python exception can interrupt.  Instances are keyed by construction
    order, which must be the same on every rank (like the communicators).
    A lost store (rank 0 exited normally) just stops the watcher."""

    def __init__(self, rank: int, world: int, store=None, interval_s: float = 0.5,
                 ack_timeout_s: float = 10.0, exit_code: int = 3, on_failure: Optional[Callable] = None):
        self.rank, self.world = rank, world
        self.store = store if store is not None else dist.distributed_c10d._get_default_store()
        n = next(_fail_counter)
        self.key, self.ack_key = f"dmp/failure/{n}", f"dmp/failure/{n}/ack"
        self.interval_s, self.ack_timeout_s, self.exit_code = interval_s, ack_timeout_s, exit_code
        self.on_failure = on_failure or self._default_failure
        self.published = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="dmp-failure-watch", daemon=True)
        self._thread.start()

    def _default_failure(self, msg: str) -> None:
        print(f"[dmp] rank {self.rank}: peer failure -- {msg}; exiting", file=sys.stderr, flush=True)
        os._exit(self.exit_code)

    def _run(self) -> None:
        while not self._stop.wait(self.interval_s):
            try:
                if self.published or not self.store.check([self.key]):
                    continue
                msg = self.store.get(self.key).decode(errors="replace")
                self.store.add(self.ack_key, 1)
            except Exception:  # noqa: BLE001 - store gone: the job is over either way
                return
            self.on_failure(msg)
            return

    def publish(self, msg: str) -> None:
        if self.published or self.world <= 1:
            return
        self.published = True
        try:
            self.store.set(self.key, f"rank {self.rank}: {msg}")
            deadline = time.monotonic() + self.ack_timeout_s
            while time.monotonic() < deadline:
                if self.store.add(self.ack_key, 0) >= self.world - 1:
                    break
                time.sleep(0.05)
        except Exception:  # noqa: BLE001 - best effort on the way out
            pass

    def stop(self) -> None:
        self._stop.set()

    @contextlib.contextmanager
    def guard(self) -> Iterator[None]:
        """Publish any exception escaping the block, then re-raise it."""
        try:
            yield
        except BaseException as e:  # noqa: BLE001
            self.publish(f"{type(e).__name__}: {e}")
            raise
