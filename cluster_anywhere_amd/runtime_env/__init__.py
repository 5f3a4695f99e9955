"""Runtime environments (reference: python/ray/runtime_env/runtime_env.py).

A :class:`RuntimeEnv` is a validated dict applied by each worker before it runs
user code (``core/worker_main.py``): ``env_vars`` (exported before HIP starts, so
``HIP_VISIBLE_DEVICES``-style variables take effect), ``working_dir`` (chdir +
``sys.path``), ``py_modules`` (``sys.path``). Workers are pooled per runtime env
(a task only reuses a worker started with the same env). ``pip`` / ``uv`` entries
are INSTALLED offline into a cached virtualenv per requirements hash
(``runtime_env/pip.py``: ``--no-index`` from local wheels / ``find_links``, LRU URI
cache) and the env's workers run that env's interpreter; a failed install fails
the task with :class:`RuntimeEnvSetupError`. ``conda`` is not in the image, so its
dependencies are verified instead (they must already be importable).
"""
from __future__ import annotations

import importlib.util
import json
import os
import re
from typing import Any, Dict, List, Optional

SUPPORTED = {"env_vars", "working_dir", "py_modules", "pip", "conda", "uv", "config",
             "excludes", "worker_process_setup_hook", "nsight", "image_uri", "_validate"}


class RuntimeEnvConfig(dict):
    """Options of the environment itself (reference: runtime_env.py RuntimeEnvConfig)."""

    def __init__(self, setup_timeout_seconds: int = 600, eager_install: bool = True,
                 log_files: Optional[List[str]] = None):
        if not (setup_timeout_seconds == -1 or setup_timeout_seconds > 0):
            raise ValueError("setup_timeout_seconds must be -1 or > 0")
        super().__init__(setup_timeout_seconds=setup_timeout_seconds, eager_install=eager_install,
                         log_files=list(log_files or []))


def _pkg_name(req: str) -> str:
    return re.split(r"[<>=!~\[; ]", req.strip(), maxsplit=1)[0].replace("-", "_").lower()


_IMPORT_ALIASES = {"scikit_learn": "sklearn", "pyyaml": "yaml", "python_dateutil": "dateutil",
                   "protobuf": "google.protobuf", "pillow": "PIL", "opencv_python": "cv2"}


def missing_packages(reqs) -> List[str]:
    """Requirements of a ``pip`` field that are not importable here."""
    if isinstance(reqs, dict):
        reqs = reqs.get("packages", [])
    if isinstance(reqs, str):
        if os.path.isfile(reqs):
            with open(reqs) as f:
                reqs = [ln for ln in f.read().splitlines() if ln.strip() and not ln.startswith("#")]
        else:
            reqs = [reqs]
    out = []
    for r in reqs:
        name = _pkg_name(r)
        mod = _IMPORT_ALIASES.get(name, name)
        try:
            found = importlib.util.find_spec(mod) is not None
        except (ImportError, ValueError):
            found = False
        if not found:
            out.append(r)
    return out


class RuntimeEnv(dict):
    def __init__(self, *, py_modules=None, working_dir=None, pip=None, conda=None, uv=None,
                 env_vars: Optional[Dict[str, str]] = None, config=None, _validate: bool = True,
                 **kwargs: Any):
        super().__init__()
        fields = dict(py_modules=py_modules, working_dir=working_dir, pip=pip, conda=conda, uv=uv,
                      env_vars=env_vars, config=config, **kwargs)
        for k, v in fields.items():
            if v is not None:
                self[k] = v
        if _validate:
            self.validate()

    def validate(self):
        unknown = set(self) - SUPPORTED
        if unknown:
            raise ValueError(f"unknown runtime_env fields: {sorted(unknown)}")
        if "pip" in self and "conda" in self:
            raise ValueError("pip and conda cannot both be specified")
        ev = self.get("env_vars")
        if ev is not None:
            if not isinstance(ev, dict) or not all(isinstance(k, str) and isinstance(v, str)
                                                    for k, v in ev.items()):
                raise TypeError("env_vars must be a Dict[str, str]")
        wd = self.get("working_dir")
        if wd is not None and not isinstance(wd, str):
            raise TypeError("working_dir must be a path string")
        pm = self.get("py_modules")
        if pm is not None and not isinstance(pm, (list, tuple)):
            raise TypeError("py_modules must be a list of paths / modules")
        return self

    # reference accessors
    def env_vars(self) -> Dict[str, str]:
        return dict(self.get("env_vars") or {})

    def working_dir(self) -> str:
        return self.get("working_dir", "")

    def py_modules(self) -> List[str]:
        return [str(m) for m in self.get("py_modules") or []]

    def pip_config(self) -> Dict:
        p = self.get("pip")
        if p is None:
            return {}
        return p if isinstance(p, dict) else {"packages": p}

    def has_py_container(self) -> bool:
        return False

    def to_dict(self) -> Dict:
        return dict(self)

    def serialize(self) -> str:
        return json.dumps(self, sort_keys=True)

    @classmethod
    def deserialize(cls, s: str) -> "RuntimeEnv":
        return cls(**json.loads(s))


__all__ = ["RuntimeEnv", "RuntimeEnvConfig", "missing_packages"]
