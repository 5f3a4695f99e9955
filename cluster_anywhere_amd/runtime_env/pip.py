"""``pip`` / ``uv`` runtime environments without a package index.

Reference roles: ``python/ray/_private/runtime_env/pip.py:45`` (``PipProcessor``:
a virtualenv per requirements hash, ``pip install`` into it) and ``:216``
(``PipPlugin``: workers of that env start with the env's interpreter),
``uv.py`` (the same with ``uv pip install``) and ``uri_cache.py:9``
(``URICache``: built envs are reused by URI and evicted least-recently-used
beyond a size budget).

MI355X pods have no package index, so installs come from local wheels:
``find_links`` directories (in the ``pip`` dict, or ``CAAMD_PIP_FIND_LINKS``,
``os.pathsep``-separated) and wheel files listed directly as packages, always
with ``--no-index``. A virtualenv is created with ``--system-site-packages`` (the
image's torch / ROCm stack stays visible; packages installed into the env shadow
it), under ``CAAMD_RUNTIME_ENV_DIR`` (default ``<tmp>/caamd_runtime_envs``), one
directory per requirements hash, built once under a file lock (several workers /
heads may ask for the same env at once) and marked ready afterwards. When every
requirement is already satisfied by the running interpreter no env is built.

``uv`` entries use the ``uv`` binary when it is on PATH, otherwise pip with the
same cache (``uv`` is not in the image).
"""
from __future__ import annotations

import fcntl
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional

_MARKER = ".caamd_ready"


class EnvSetupError(RuntimeError):
    pass


def root_dir() -> str:
    return os.environ.get("CAAMD_RUNTIME_ENV_DIR") or os.path.join(tempfile.gettempdir(), "caamd_runtime_envs")


def normalize(value, kind: str = "pip") -> Dict:
    """``pip`` field (list / requirements-file path / dict) -> {"packages", "find_links",
    "pip_install_options", "installer"}."""
    if isinstance(value, dict):
        pkgs = value.get("packages", [])
        find_links = list(value.get("find_links") or value.get("pip_find_links") or [])
        opts = list(value.get("pip_install_options") or [])
    else:
        pkgs, find_links, opts = value, [], []
    if isinstance(pkgs, str):
        if os.path.isfile(pkgs):
            with open(pkgs) as f:
                pkgs = [ln.strip() for ln in f.read().splitlines() if ln.strip() and not ln.startswith("#")]
        else:
            pkgs = [pkgs]
    env_links = [p for p in os.environ.get("CAAMD_PIP_FIND_LINKS", "").split(os.pathsep) if p]
    return {"packages": [str(p) for p in pkgs], "find_links": find_links + env_links,
            "pip_install_options": opts, "installer": kind}


def env_hash(cfg: Dict) -> str:
    key = {"packages": sorted(cfg["packages"]), "find_links": cfg["find_links"],
           "options": cfg["pip_install_options"], "python": sys.version.split()[0],
           "executable": os.path.realpath(sys.executable)}
    return hashlib.sha1(json.dumps(key, sort_keys=True).encode()).hexdigest()[:20]


def satisfied(packages: List[str]) -> bool:
    """True when the running interpreter already satisfies every requirement (then
    no environment is built). Wheel files / paths always need an install."""
    try:
        from importlib import metadata

        from packaging.requirements import InvalidRequirement, Requirement
    except ImportError:
        return False
    for p in packages:
        if p.endswith(".whl") or os.path.sep in p:
            return False
        try:
            req = Requirement(p)
        except InvalidRequirement:
            return False
        try:
            ver = metadata.version(req.name)
        except metadata.PackageNotFoundError:
            return False
        if req.specifier and not req.specifier.contains(ver, prereleases=True):
            return False
    return True


def _dir_bytes(path: str) -> int:
    n = 0
    for dp, _dn, fns in os.walk(path):
        for f in fns:
            try:
                n += os.lstat(os.path.join(dp, f)).st_size
            except OSError:
                pass
    return n


class URICache:
    """Built environments by URI (directory), least-recently-used eviction beyond
    ``max_bytes`` (reference: uri_cache.py:9). Use is recorded as the ready
    marker's mtime; environments in use by a live worker are skipped."""

    def __init__(self, root: str, max_bytes: int):
        self.root = root
        self.max_bytes = max_bytes

    def entries(self):
        out = []
        if not os.path.isdir(self.root):
            return out
        for name in os.listdir(self.root):
            d = os.path.join(self.root, name)
            m = os.path.join(d, _MARKER)
            if os.path.isfile(m):
                out.append((os.path.getmtime(m), d))
        return sorted(out)

    def touch(self, d: str):
        try:
            os.utime(os.path.join(d, _MARKER))
        except OSError:
            pass

    def evict(self, keep: Optional[str] = None, in_use=()) -> List[str]:
        """Remove least-recently-used envs until the cache fits. An env is skipped
        when it is ``keep`` / in ``in_use``, when a live process registered as its
        user (:func:`mark_in_use`; any head's workers, not only this process's), or
        when another process holds its build lock."""
        ents = self.entries()
        sizes = {d: _dir_bytes(d) for _, d in ents}
        total = sum(sizes.values())
        gone = []
        for _, d in ents:  # oldest first
            if total <= self.max_bytes:
                break
            if d == keep or d in in_use or live_users(d):
                continue
            with open(d + ".lock", "w") as lk:
                try:
                    fcntl.flock(lk, fcntl.LOCK_EX | fcntl.LOCK_NB)
                except OSError:
                    continue  # being built or re-validated right now
                try:
                    if live_users(d):
                        continue
                    shutil.rmtree(d, ignore_errors=True)
                    shutil.rmtree(d + ".users", ignore_errors=True)
                finally:
                    fcntl.flock(lk, fcntl.LOCK_UN)
            total -= sizes[d]
            gone.append(d)
        return gone


def mark_in_use(env_dir: str, pid: Optional[int] = None) -> None:
    """Register ``pid`` (default: this process) as a user of ``env_dir`` so no
    cache eviction removes the env while it runs."""
    users = env_dir + ".users"
    os.makedirs(users, exist_ok=True)
    with open(os.path.join(users, str(pid or os.getpid())), "w"):
        pass


def live_users(env_dir: str) -> List[int]:
    """Pids registered as users of ``env_dir`` that are still running (stale
    registrations are dropped)."""
    users = env_dir + ".users"
    try:
        names = os.listdir(users)
    except OSError:
        return []
    live = []
    for n in names:
        try:
            pid = int(n)
            os.kill(pid, 0)
            live.append(pid)
        except ValueError:
            continue
        except ProcessLookupError:
            try:
                os.unlink(os.path.join(users, n))
            except OSError:
                pass
        except PermissionError:
            live.append(pid)
    return live


def _cache() -> URICache:
    mb = float(os.environ.get("CAAMD_RUNTIME_ENV_CACHE_MB", "10240"))
    return URICache(os.path.join(root_dir(), "pip"), int(mb * (1 << 20)))


def ensure_env(cfg: Dict, timeout_s: float = 600.0) -> str:
    """Python executable of the environment for ``cfg`` (built on first use)."""
    cache = _cache()
    os.makedirs(cache.root, exist_ok=True)
    h = env_hash(cfg)
    d = os.path.join(cache.root, h)
    py = os.path.join(d, "bin", "python")
    with open(d + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if os.path.isfile(os.path.join(d, _MARKER)):
                cache.touch(d)
                return py
            shutil.rmtree(d, ignore_errors=True)
            t0 = time.time()
            # --without-pip: the image's Python has no ensurepip; the env's interpreter
            # runs the system pip (visible through --system-site-packages), which
            # installs into the env and never touches the system site-packages
            r = subprocess.run([sys.executable, "-m", "venv", "--system-site-packages", "--without-pip", d],
                               capture_output=True, text=True, timeout=timeout_s)
            if r.returncode != 0:
                raise EnvSetupError(f"creating the virtualenv failed: {(r.stdout + r.stderr)[-2000:]}")
            links = []
            for fl in cfg["find_links"]:
                links += ["--find-links", fl]
            uv = shutil.which("uv") if cfg.get("installer") == "uv" else None
            if uv:
                cmd = [uv, "pip", "install", "--python", py, "--no-index", *links,
                       *cfg["pip_install_options"], *cfg["packages"]]
            else:
                cmd = [py, "-m", "pip", "install", "--no-index", "--disable-pip-version-check",
                       "--no-warn-script-location", "--no-input", *links, *cfg["pip_install_options"],
                       *cfg["packages"]]
            left = max(1.0, timeout_s - (time.time() - t0))
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=left,
                               env=dict(os.environ, PIP_NO_INPUT="1", PYTHONNOUSERSITE="1"))
            if r.returncode != 0:
                shutil.rmtree(d, ignore_errors=True)
                raise EnvSetupError("installing {} failed (offline, --no-index; find_links={}): {}".format(
                    cfg["packages"], cfg["find_links"], (r.stdout + r.stderr)[-3000:]))
            with open(os.path.join(d, _MARKER), "w") as f:
                json.dump({"packages": cfg["packages"], "built_s": round(time.time() - t0, 2)}, f)
        except subprocess.TimeoutExpired:
            shutil.rmtree(d, ignore_errors=True)
            raise EnvSetupError(f"runtime env setup exceeded {timeout_s:.0f}s")
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    cache.evict(keep=d)
    return py


def pip_field(renv) -> Optional[Dict]:
    """Normalized pip / uv config of a runtime env that needs its own interpreter."""
    if not renv:
        return None
    for kind in ("pip", "uv"):
        v = renv.get(kind)
        if v:
            cfg = normalize(v, kind)
            if not cfg["packages"] or satisfied(cfg["packages"]):
                return None
            return cfg
    return None


def setup_timeout(renv) -> float:
    c = (renv or {}).get("config") or {}
    t = c.get("setup_timeout_seconds", 600) if isinstance(c, dict) else 600
    return 1e9 if t == -1 else float(t)
