"""Job submission client (reference: python/ray/job_submission/ —
JobSubmissionClient over the dashboard's /api/jobs/ REST API)."""
from __future__ import annotations

import enum
import json
import time
import urllib.error
import urllib.request
from dataclasses import dataclass
from typing import Any, Dict, Iterator, List, Optional


class JobStatus(str, enum.Enum):
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    STOPPED = "STOPPED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"

    def is_terminal(self):
        return self in (JobStatus.STOPPED, JobStatus.SUCCEEDED, JobStatus.FAILED)


@dataclass
class JobDetails:
    submission_id: str
    entrypoint: str
    status: JobStatus
    message: str = ""
    start_time: Optional[int] = None
    end_time: Optional[int] = None
    metadata: Optional[Dict[str, str]] = None
    runtime_env: Optional[Dict[str, Any]] = None
    driver_exit_code: Optional[int] = None

    @property
    def job_id(self):
        return self.submission_id


JobInfo = JobDetails


class JobSubmissionClient:
    def __init__(self, address: Optional[str] = None, headers: Optional[Dict[str, str]] = None, **_):
        import os

        address = address or os.environ.get("CAAMD_DASHBOARD_ADDRESS") or "http://127.0.0.1:8265"
        if not address.startswith("http"):
            address = "http://" + address
        self.address = address.rstrip("/")
        self.headers = headers or {}

    def _req(self, method, path, body=None):
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.address + path, data=data, method=method,
                                     headers=dict(self.headers, **({"content-type": "application/json"}
                                                                   if data else {})))
        try:
            with urllib.request.urlopen(req, timeout=60) as r:
                return json.loads(r.read())
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")
            raise RuntimeError(f"{method} {path} failed ({e.code}): {msg}") from None

    def submit_job(self, *, entrypoint: str, submission_id: Optional[str] = None, job_id: Optional[str] = None,
                   runtime_env: Optional[Dict] = None, metadata: Optional[Dict] = None,
                   entrypoint_num_cpus=None, entrypoint_num_gpus=None, **_) -> str:
        r = self._req("POST", "/api/jobs/", {"entrypoint": entrypoint, "submission_id": submission_id or job_id,
                                             "runtime_env": runtime_env, "metadata": metadata,
                                             "entrypoint_num_cpus": entrypoint_num_cpus,
                                             "entrypoint_num_gpus": entrypoint_num_gpus})
        return r["submission_id"]

    def get_job_info(self, job_id: str) -> JobDetails:
        r = self._req("GET", f"/api/jobs/{job_id}")
        return JobDetails(r["submission_id"], r["entrypoint"], JobStatus(r["status"]), r.get("message", ""),
                          r.get("start_time"), r.get("end_time"), r.get("metadata"), r.get("runtime_env"),
                          r.get("driver_exit_code"))

    def get_job_status(self, job_id: str) -> JobStatus:
        return self.get_job_info(job_id).status

    def get_job_logs(self, job_id: str) -> str:
        return self._req("GET", f"/api/jobs/{job_id}/logs")["logs"]

    def tail_job_logs(self, job_id: str) -> Iterator[str]:
        sent = 0
        while True:
            logs = self.get_job_logs(job_id)
            if len(logs) > sent:
                yield logs[sent:]
                sent = len(logs)
            if self.get_job_status(job_id).is_terminal():
                logs = self.get_job_logs(job_id)
                if len(logs) > sent:
                    yield logs[sent:]
                return
            time.sleep(0.5)

    def stop_job(self, job_id: str) -> bool:
        return self._req("POST", f"/api/jobs/{job_id}/stop")["stopped"]

    def delete_job(self, job_id: str) -> bool:
        return self._req("DELETE", f"/api/jobs/{job_id}")["deleted"]

    def list_jobs(self) -> List[JobDetails]:
        return [JobDetails(r["submission_id"], r["entrypoint"], JobStatus(r["status"]), r.get("message", ""),
                           r.get("start_time"), r.get("end_time"), r.get("metadata"), r.get("runtime_env"),
                           r.get("driver_exit_code")) for r in self._req("GET", "/api/jobs/")]

    def wait_until_finish(self, job_id: str, timeout: float = 600) -> JobStatus:
        deadline = time.time() + timeout
        while time.time() < deadline:
            s = self.get_job_status(job_id)
            if s.is_terminal():
                return s
            time.sleep(0.2)
        raise TimeoutError(f"job {job_id} still running after {timeout}s")


class JobType(str, enum.Enum):
    """How a job came to be: submitted through the job API, or a driver script
    that called ``init()`` itself."""

    SUBMISSION = "SUBMISSION"
    DRIVER = "DRIVER"


@dataclass
class DriverInfo:
    """The driver process of a job (reference: job_submission DriverInfo)."""

    id: str
    node_ip_address: str
    pid: str


__all__ = ["JobSubmissionClient", "JobStatus", "JobDetails", "JobInfo", "JobType", "DriverInfo"]
