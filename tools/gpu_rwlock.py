"""tools/gpu_rwlock.py -- a writer-preferring reader/writer lock over two lock files (flock), for sweep workers that
share one GPU.

Every phase of a worker that puts work on the GPU -- upload, plan (its device-to-host copies run as blit kernels),
fills, checks, frees -- holds the lock SHARED; a timed region holds it EXCLUSIVE, so no other process's GPU work runs
while it is timed.  Writer preference: a process that wants the exclusive lock takes the gate first, so readers
arriving after it wait instead of starving it.

    lk = GpuRWLock("/tmp/sweep.lock")
    with lk.shared():
        ...upload, plan...
    with lk.exclusive():
        ...warm-up and timed launches...
"""
import contextlib
import fcntl


class GpuRWLock:
    def __init__(self, path: str):
        self.gate = open(path + ".gate", "a+")
        self.data = open(path, "a+")

    @contextlib.contextmanager
    def shared(self):
        fcntl.flock(self.gate, fcntl.LOCK_EX)         # queue behind a waiting writer
        fcntl.flock(self.data, fcntl.LOCK_SH)
        fcntl.flock(self.gate, fcntl.LOCK_UN)
        try:
            yield
        finally:
            fcntl.flock(self.data, fcntl.LOCK_UN)

    @contextlib.contextmanager
    def exclusive(self):
        fcntl.flock(self.gate, fcntl.LOCK_EX)         # new readers now wait at the gate
        try:
            fcntl.flock(self.data, fcntl.LOCK_EX)     # the readers inside finish first
        finally:
            fcntl.flock(self.gate, fcntl.LOCK_UN)
        try:
            yield
        finally:
            fcntl.flock(self.data, fcntl.LOCK_UN)

    def close(self):
        self.gate.close()
        self.data.close()
