"""Utilities shared across the engine (role of tcb/cnn_util.py:26-251).

``log_fn`` is the single logging hook (tests monkey-patch it to capture the
output, as tcb/test_util.py does).  ``Barrier`` is a reusable thread barrier
with abort; ``ImageProducer`` is the background thread that keeps
``batch_group_size`` batches staged ahead of the consumer.
"""

from __future__ import annotations

import sys
import threading
from typing import Callable, List, Optional

import numpy as np


def log_fn(log):
    print(log)
    sys.stdout.flush()


def roll_numpy_batches(array, batch_size, shift_ratio):
    """Moves a proportion of the array from the start to the end
    (tcb/cnn_util.py:41-66); used to give workers different data orders."""
    num_items = array.shape[0]
    assert num_items % batch_size == 0
    num_batches = num_items // batch_size
    starting_batch = int(num_batches * shift_ratio)
    starting_item = starting_batch * batch_size
    return np.roll(array, -starting_item, axis=0)


class Barrier:
    """Re-usable barrier for ``parties`` threads with an abort that wakes all
    waiters (tcb/cnn_util.py:70-115)."""

    def __init__(self, parties):
        assert parties > 0
        self.parties = parties
        self._cond = threading.Condition()
        self._waiting = 0
        self._generation = 0
        self._aborted = False

    def wait(self):
        with self._cond:
            if self._aborted:
                return
            gen = self._generation
            self._waiting += 1
            if self._waiting == self.parties:
                self._waiting = 0
                self._generation += 1
                self._cond.notify_all()
                return
            while gen == self._generation and not self._aborted:
                self._cond.wait()

    def abort(self):
        with self._cond:
            self._aborted = True
            self._cond.notify_all()


class ImageProducer:
    """Runs ``put_fn`` in a background thread, staying at most
    ``batch_group_size`` batches ahead of the consumer
    (tcb/cnn_util.py:118-198)."""

    def __init__(self, put_fn: Callable[[], None], batch_group_size: int,
                 use_python32_barrier: bool = False):
        self.put_fn = put_fn
        self.batch_group_size = batch_group_size
        self.done_event = threading.Event()
        self._consumed = 0
        self._produced = 0
        self._cond = threading.Condition()
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None

    def start(self):
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def _loop(self):
        try:
            while not self.done_event.is_set():
                with self._cond:
                    while (self._produced - self._consumed >= 2 * self.batch_group_size
                           and not self.done_event.is_set()):
                        self._cond.wait(0.1)
                if self.done_event.is_set():
                    break
                for _ in range(self.batch_group_size):
                    self.put_fn()
                with self._cond:
                    self._produced += self.batch_group_size
                    self._cond.notify_all()
        except BaseException as e:  # surfaced on the consumer side
            self._error = e
            with self._cond:
                self._cond.notify_all()

    def notify_image_consumption(self):
        with self._cond:
            self._consumed += 1
            self._cond.notify_all()
        if self._error is not None:
            raise RuntimeError("image producer failed") from self._error

    def done(self):
        self.done_event.set()
        with self._cond:
            self._cond.notify_all()
        if self._thread is not None:
            self._thread.join(timeout=5)


class BaseClusterManager:
    """Cluster description from --ps_hosts / --worker_hosts
    (tcb/cnn_util.py:201-230)."""

    def __init__(self, params):
        self._ps = [h for h in (params.ps_hosts or "").split(",") if h]
        self._workers = [h for h in (params.worker_hosts or "").split(",") if h]
        self._cluster_spec = {"worker": list(self._workers)}
        if self._ps:
            self._cluster_spec["ps"] = list(self._ps)

    def get_target(self):
        return ""

    def get_cluster_spec(self):
        return self._cluster_spec

    def join_server(self):
        raise NotImplementedError("join must be implemented by subclass")

    def num_workers(self):
        return max(len(self._workers), 1)

    def num_ps(self):
        return len(self._ps)


DONE_KEY = "kfb/job_done"


class TorchClusterManager(BaseClusterManager):
    """The reference's gRPC cluster (tcb/cnn_util.py:232-251) mapped onto a
    torch.distributed world: each ``--job_name=worker --task_index=i`` task
    is rank i of ``len(worker_hosts)``; the first worker's host:port is the
    rendezvous (TCPStore) address.  Variables are replicated on every GPU,
    so ``ps`` and ``controller`` tasks hold no state: ``join_server`` blocks
    until worker 0 marks the job done in the store, so launch scripts that
    start ps tasks keep working."""

    def __init__(self, params, config_proto=None):
        super().__init__(params)
        del config_proto
        self.params = params
        if not self._workers:
            raise ValueError("--worker_hosts must be set with --job_name")
        host, port = self._workers[0].rsplit(":", 1)
        self.master_addr = "127.0.0.1" if host in ("localhost", "") else host
        self.master_port = int(port)

    def setup_worker_env(self):
        """Exports RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* for this task."""
        import os
        p = self.params
        if p.job_name != "worker":
            return
        me = self._workers[p.task_index].rsplit(":", 1)[0]
        local = sum(1 for h in self._workers[:p.task_index] if h.rsplit(":", 1)[0] == me)
        os.environ.setdefault("RANK", str(p.task_index))
        os.environ.setdefault("WORLD_SIZE", str(len(self._workers)))
        os.environ.setdefault("LOCAL_RANK", str(local))
        os.environ.setdefault("MASTER_ADDR", self.master_addr)
        os.environ.setdefault("MASTER_PORT", str(self.master_port))

    def join_server(self, timeout_s: float = 7 * 24 * 3600):
        import datetime
        from torch.distributed import TCPStore
        store = TCPStore(self.master_addr, self.master_port, is_master=False,
                         timeout=datetime.timedelta(seconds=timeout_s))
        try:
            store.wait([DONE_KEY])
        except RuntimeError:
            pass  # worker 0 closed the store: the job is over

    @staticmethod
    def mark_done():
        """Called by worker 0 at the end of the run."""
        import torch.distributed as dist
        if dist.is_initialized():
            try:
                dist.distributed_c10d._get_default_store().set(DONE_KEY, "1")
            except Exception:  # pragma: no cover - store already gone
                pass


GrpcClusterManager = TorchClusterManager
