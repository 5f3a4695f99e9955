"""joblib ParallelBackend over our actor Pool (reference: util/joblib/ray_backend.py)."""
from __future__ import annotations

from joblib._parallel_backends import MultiprocessingBackend

from ...core import api as _core
from ..multiprocessing import Pool


class RayBackend(MultiprocessingBackend):
    supports_sharedmem = False
    supports_retrieve_callback = True

    def __init__(self, nesting_level=None, inner_max_num_threads=None, ray_remote_args=None, **kw):
        self.ray_remote_args = ray_remote_args
        super().__init__(nesting_level=nesting_level, inner_max_num_threads=inner_max_num_threads, **kw)

    def effective_n_jobs(self, n_jobs):
        if n_jobs == 0:
            raise ValueError("n_jobs == 0 in Parallel has no meaning")
        if n_jobs is None:
            return 1
        if n_jobs < 0:
            if not _core.is_initialized():
                _core.init()
            cpus = int(_core.cluster_resources().get("CPU", 1))
            n_jobs = max(cpus + 1 + n_jobs, 1)
        return n_jobs

    def configure(self, n_jobs=1, parallel=None, prefer=None, require=None, **memmappingpool_args):
        n_jobs = self.effective_n_jobs(n_jobs)
        if not _core.is_initialized():
            _core.init()
        self._pool = Pool(processes=n_jobs, ray_remote_args=self.ray_remote_args)
        self.parallel = parallel
        return n_jobs

    def terminate(self):
        if self._pool is not None:
            self._pool.terminate()
            self._pool = None
