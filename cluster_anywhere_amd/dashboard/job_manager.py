"""Job manager (reference: python/ray/dashboard/modules/job/job_manager.py,
job_supervisor.py): each submitted entrypoint runs as a shell subprocess whose
driver connects to this cluster (``CAAMD_ADDRESS``), with logs captured per
job and status PENDING -> RUNNING -> SUCCEEDED / FAILED / STOPPED."""
from __future__ import annotations

import json
import os
import signal
import subprocess
import threading
import time
import uuid
from typing import Dict, List, Optional


class JobManager:
    def __init__(self, control_address: str, log_dir: str):
        self.address = control_address
        self.log_dir = log_dir
        os.makedirs(log_dir, exist_ok=True)
        self.jobs: Dict[str, dict] = {}
        self.procs: Dict[str, subprocess.Popen] = {}
        self.lock = threading.Lock()

    def submit(self, entrypoint: str, submission_id: Optional[str] = None, runtime_env: Optional[dict] = None,
               metadata: Optional[dict] = None, num_cpus=None, num_gpus=None) -> str:
        sid = submission_id or f"raysubmit_{uuid.uuid4().hex[:16]}"
        with self.lock:
            if sid in self.jobs:
                raise ValueError(f"job {sid} already exists")
            self.jobs[sid] = {"submission_id": sid, "job_id": sid, "entrypoint": entrypoint, "status": "PENDING",
                              "message": "", "start_time": int(time.time() * 1000), "end_time": None,
                              "metadata": metadata or {}, "runtime_env": runtime_env or {},
                              "driver_exit_code": None, "type": "SUBMISSION"}
        env = dict(os.environ)
        env["CAAMD_ADDRESS"] = self.address
        env["CAAMD_JOB_SUBMISSION_ID"] = sid
        renv = runtime_env or {}
        for k, v in (renv.get("env_vars") or {}).items():
            env[k] = str(v)
        if renv:
            env["CAAMD_JOB_RUNTIME_ENV"] = json.dumps(renv)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        cwd = renv.get("working_dir") if renv.get("working_dir") and os.path.isdir(renv["working_dir"]) else None
        log = open(os.path.join(self.log_dir, f"{sid}.log"), "wb")
        p = subprocess.Popen(["bash", "-c", entrypoint], env=env, stdout=log, stderr=subprocess.STDOUT,
                             stdin=subprocess.DEVNULL, cwd=cwd, start_new_session=True)
        log.close()
        with self.lock:
            self.procs[sid] = p
            self.jobs[sid]["status"] = "RUNNING"
            self.jobs[sid]["driver_pid"] = p.pid
        threading.Thread(target=self._watch, args=(sid, p), daemon=True).start()
        return sid

    def _watch(self, sid, p):
        rc = p.wait()
        with self.lock:
            j = self.jobs[sid]
            j["driver_exit_code"] = rc
            j["end_time"] = int(time.time() * 1000)
            if j["status"] == "STOPPED":
                return
            j["status"] = "SUCCEEDED" if rc == 0 else "FAILED"
            if rc != 0:
                j["message"] = f"Job entrypoint command failed with exit code {rc}"

    def info(self, sid) -> Optional[dict]:
        with self.lock:
            j = self.jobs.get(sid)
            return dict(j) if j else None

    def list(self) -> List[dict]:
        with self.lock:
            return [dict(j) for j in self.jobs.values()]

    def logs(self, sid) -> Optional[str]:
        p = os.path.join(self.log_dir, f"{sid}.log")
        if sid not in self.jobs or not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return f.read().decode("utf-8", errors="replace")

    def stop(self, sid) -> bool:
        with self.lock:
            p = self.procs.get(sid)
            j = self.jobs.get(sid)
            if p is None or p.poll() is not None:
                return False
            j["status"] = "STOPPED"
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return False
        try:
            p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
        return True

    def delete(self, sid) -> bool:
        with self.lock:
            j = self.jobs.get(sid)
            if j is None or j["status"] in ("PENDING", "RUNNING"):
                return False
            del self.jobs[sid]
            self.procs.pop(sid, None)
            return True

    def stop_all(self):
        for sid in list(self.procs):
            self.stop(sid)
