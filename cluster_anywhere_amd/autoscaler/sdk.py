"""``request_resources`` (reference: python/ray/autoscaler/sdk/sdk.py
``request_resources``): ask the autoscaler to keep enough TOTAL capacity for the
given bundles, independent of current load. Each call replaces the previous
request; ``request_resources()`` with no arguments clears it."""
from __future__ import annotations

import json
from typing import Dict, List, Optional

from .autoscaler import KV_NS, KV_REQUEST


def request_resources(num_cpus: Optional[int] = None, bundles: Optional[List[Dict[str, float]]] = None) -> None:
    from ..experimental import internal_kv as kv

    req: List[Dict[str, float]] = []
    if num_cpus:
        req += [{"CPU": 1.0}] * int(num_cpus)
    for b in bundles or []:
        req.append({k: float(v) for k, v in b.items()})
    kv._internal_kv_put(KV_REQUEST, json.dumps(req), overwrite=True, namespace=KV_NS)
