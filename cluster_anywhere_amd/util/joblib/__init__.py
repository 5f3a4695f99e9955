"""joblib backend (reference: python/ray/util/joblib/): ``register_ray()`` then
``with joblib.parallel_backend("ray"): ...`` runs joblib batches (e.g. scikit-learn
``n_jobs``) on the cluster through :class:`util.multiprocessing.Pool` actors."""


def register_ray():
    try:
        from joblib.parallel import register_parallel_backend
    except ImportError as e:  # pragma: no cover
        raise ImportError("joblib is required for the ray joblib backend") from e
    from .ray_backend import RayBackend

    register_parallel_backend("ray", RayBackend)


__all__ = ["register_ray"]
