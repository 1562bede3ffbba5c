"""
Host logic of the guide draw made by the linear site launch (``engine.claim_linear_draws``,
``guide.PendingDraw``), without a GPU: which deferred draws a linear launch may make itself and
which are launched before planning. The kernels' side is ``tests/test_gpu_linear_draw.py``.
"""
import torch

from mininf_amd import engine, guide
from mininf_amd.particles import ParticleTrace, SiteRecord


def _pending(K=8, P=4):
    z = torch.empty(K, P)
    cfg = guide.DrawConfig(K=K, seed=1, step=0, stream_id=0, particle_offset=0, defer=True)
    rec = guide.PendingDraw(cfg, z, torch.zeros(P), 1, torch.ones(P), 1, None)
    guide._PENDING_DRAWS[guide._storage_of(z)] = rec
    return rec


def _linear_site(theta, name="y"):
    site = SiteRecord(name=name, family="normal", roles=[], site_shape=torch.Size([16]), scale=1.0,
                      mask=None, description="Normal")
    site.linear_X = torch.empty(16, theta.shape[1])
    site.linear_theta = theta
    site.tensors = [torch.empty(()), torch.ones(()), torch.empty(16)]
    return site


def _value_site(value, name="theta"):
    return SiteRecord(name=name, family="normal", roles=[], site_shape=torch.Size([value.shape[1]]),
                      scale=1.0, mask=None, description="Normal",
                      tensors=[torch.zeros(()), torch.ones(()), value])


def _launches(monkeypatch):
    calls = []

    def launch(self):
        if not self.done:
            self.done = True
            calls.append(self)
    monkeypatch.setattr(guide.PendingDraw, "launch", launch)
    return calls


def test_only_reader_is_one_linear_site(monkeypatch):
    calls = _launches(monkeypatch)
    rec = _pending()
    trace = ParticleTrace(sites=[_value_site(rec.z), _linear_site(rec.z)], checks=[], fallback=[],
                          K=8)
    claims = engine.claim_linear_draws(trace)
    assert list(claims.values()) == [rec] and rec.claimed and calls == []
    guide.flush_draws()            # ordinary flushes leave a claimed draw to its launch
    assert calls == []
    guide.take_draw(rec)           # the linear launch made it
    assert guide._PENDING_DRAWS == {} and rec.done


def test_two_linear_readers_launch_the_draw(monkeypatch):
    calls = _launches(monkeypatch)
    rec = _pending()
    trace = ParticleTrace(sites=[_linear_site(rec.z, "y1"), _linear_site(rec.z, "y2")], checks=[],
                          fallback=[], K=8)
    assert engine.claim_linear_draws(trace) == {}
    assert calls == [rec] and guide._PENDING_DRAWS == {}


def test_other_layout_reader_launches_the_draw(monkeypatch):
    calls = _launches(monkeypatch)
    rec = _pending()
    view = rec.z[:, :2]   # a site reading part of the draw: planning may copy it
    trace = ParticleTrace(sites=[_value_site(view), _linear_site(rec.z)], checks=[], fallback=[],
                          K=8)
    assert engine.claim_linear_draws(trace) == {}
    assert calls == [rec]


def test_release_flushes_claimed_draws(monkeypatch):
    calls = _launches(monkeypatch)
    rec = _pending()
    rec.claimed = True
    guide.release_lazy()   # the loss failed before its linear launch: the draw is still made
    assert calls == [rec] and guide._PENDING_DRAWS == {}


def test_pending_draw_seen_through_batched_views(monkeypatch):
    _launches(monkeypatch)
    rec = _pending()
    seen = []
    torch.func.vmap(lambda t: seen.append(guide.pending_draw(t)) or t)(rec.z)
    assert seen == [rec]
    guide.flush_draws()
