"""Stage deadlines for bench.py's multi-GPU first runs.

A step of the N-GPU bench waits on things no host code can interrupt: an RCCL communicator's
setup, a grouped ncclGather, a device that never finishes its render. A hang there used to end as a
kill at the driver's time limit that named no device and no stage. Here every such wait runs inside
a named stage with a deadline; a daemon thread watches the clock and, when a stage overruns, prints
ONE JSON line whose "error" names the stage (and, through `detail`, where the frame stands: which
device is still rendering, which has not gathered, whether the root has unpacked), then ends the
process with os._exit(3) — no re-exec, no retry.

Host-side waits on device work are polled (`wait_events`: event queries with a short sleep), so the
process is never parked inside a driver call when its deadline passes.
"""
import json
import os
import sys
import threading
import time


class Watchdog:
    EXIT_CODE = 3

    def __init__(self, metric, rank=0, poll_s=0.2, out=None):
        self.metric, self.rank, self.poll_s = metric, rank, poll_s
        self.out = out if out is not None else (sys.stdout if rank == 0 else sys.stderr)
        self._lock = threading.Lock()
        self._stage = None
        self._deadline = None
        self._limit = None
        self._detail = None
        self._t = threading.Thread(target=self._run, name="yart-watchdog", daemon=True)
        self._t.start()

    def stage(self, name, seconds, detail=None):
        """Context manager: `with wd.stage("gather", 30.0, detail_fn): ...`."""
        wd = self

        class _Stage:
            def __enter__(self):
                with wd._lock:
                    wd._stage, wd._limit, wd._detail = name, float(seconds), detail
                    wd._deadline = time.monotonic() + float(seconds)
                return self

            def __exit__(self, *exc):
                with wd._lock:
                    wd._stage = wd._deadline = wd._limit = wd._detail = None
                return False

        return _Stage()

    def _run(self):
        while True:
            time.sleep(self.poll_s)
            with self._lock:
                name, deadline, limit, detail = self._stage, self._deadline, self._limit, self._detail
            if name is None or time.monotonic() <= deadline:
                continue
            info = None
            if detail is not None:
                try:
                    info = detail()
                except Exception as e:  # the diagnosis must not stop the exit
                    info = f"detail unavailable: {e}"
            line = {"metric": self.metric, "value": None, "error": f"stage '{name}' exceeded its {limit:.0f} s deadline",
                    "stage": name, "detail": info, "rank": self.rank}
            try:
                print(json.dumps(line), file=self.out, flush=True)
            finally:
                os._exit(self.EXIT_CODE)


def wait_events(events, sleep_s=0.001):
    """Waits for every torch.cuda.Event in `events` by polling (the watchdog's stage decides how long)."""
    for ev in events:
        while not ev.query():
            time.sleep(sleep_s)
