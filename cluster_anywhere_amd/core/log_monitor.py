"""Stream worker stdout/stderr to the driver (reference: _private/log_monitor.py +
``init(log_to_driver=True)``). Workers write to ``<session>/worker-<id>.log``;
this thread tails every such file and re-prints new lines on the driver as
``(pid=<pid>) <line>``. Progress records from :mod:`experimental.tqdm_ray`
are rendered as one status line per bar instead of raw JSON."""
from __future__ import annotations

import glob
import json
import os
import sys
import threading
from typing import Dict, Optional

_TQDM = "__caamd_tqdm__"


class LogMonitor:
    def __init__(self, session_dir: str, out=None, interval: float = 0.1):
        self.session_dir = session_dir
        self.out = out
        self.interval = interval
        self.offsets: Dict[str, int] = {}
        self.partial: Dict[str, bytes] = {}
        self.pids: Dict[str, Optional[int]] = {}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="caamd-log-monitor", daemon=True)
        # lines already in files when we attach are not replayed
        for p in glob.glob(os.path.join(session_dir, "worker-*.log")):
            try:
                self.offsets[p] = os.path.getsize(p)
            except OSError:
                pass

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=2)
        self.poll()

    def _pid_of(self, path):
        key = os.path.basename(path)[len("worker-"):-len(".log")]
        pid = self.pids.get(key)
        if pid is None:
            try:
                from .api import _state

                for w in _state("workers") or []:
                    wid = w.get("worker_id") or ""
                    if wid.startswith(key):
                        pid = w.get("pid")
                        break
            except Exception:
                pid = None
            if pid is not None:
                self.pids[key] = pid
        return pid

    def _emit(self, path, line: str):
        out = self.out or sys.stdout
        if line.startswith(_TQDM):
            try:
                r = json.loads(line[len(_TQDM):])
                tot = f"/{r['total']}" if r.get("total") is not None else ""
                line = f"{r.get('desc', '')}: {r['x']}{tot} [{r.get('rate', 0)}{r.get('unit', 'it')}/s]" + \
                       (" (done)" if r.get("closed") else "")
            except Exception:
                pass
        pid = self._pid_of(path)
        print(f"(pid={pid if pid is not None else '?'}) {line}", file=out, flush=True)

    def poll(self):
        for p in glob.glob(os.path.join(self.session_dir, "worker-*.log")):
            off = self.offsets.get(p, 0)
            try:
                size = os.path.getsize(p)
                if size <= off:
                    continue
                with open(p, "rb") as f:
                    f.seek(off)
                    data = f.read(size - off)
            except OSError:
                continue
            self.offsets[p] = off + len(data)
            data = self.partial.pop(p, b"") + data
            lines = data.split(b"\n")
            if lines and lines[-1]:
                self.partial[p] = lines[-1]
            for ln in lines[:-1]:
                self._emit(p, ln.decode("utf-8", "replace"))

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self.poll()
            except Exception:
                pass
