"""Use counting behind the LayerNorm backward's direct main-grad path
(ops/norm.py ``_Use``): a norm used once in the step may write dgamma / dbeta into
their main-grad views and signal readiness itself; a norm used twice must hand every
use's gradient to autograd (which sums them before the single post-accumulate hook);
a use whose graph is dropped without a backward must not leave the weight looking
shared for the next step."""
import gc

import torch

from cluster_anywhere_amd.ops.norm import _Use


def _p():
    p = torch.nn.Parameter(torch.ones(4))
    p.main_grad = torch.zeros(4)
    return p


def test_single_use_is_not_shared():
    p = _p()
    u = _Use(p)
    assert not u.shared()
    u.finish()
    assert p._ca_ln_uses == 0


def test_every_use_of_a_shared_norm_is_shared():
    p = _p()
    u1, u2 = _Use(p), _Use(p)
    # backward runs in reverse order: the second use first
    assert u2.shared()
    u2.finish()
    assert u1.shared()  # remembered for the rest of the step
    u1.finish()
    assert p._ca_ln_uses == 0 and not p._ca_ln_shared
    u3 = _Use(p)  # next step, single use
    assert not u3.shared()
    u3.finish()


def test_dropped_graph_releases_its_use():
    p = _p()
    u = _Use(p)
    del u
    gc.collect()
    assert p._ca_ln_uses == 0
    u2 = _Use(p)
    assert not u2.shared()
    u2.finish()
    u2.finish()  # idempotent
    assert p._ca_ln_uses == 0
