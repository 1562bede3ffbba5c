"""
Host-side shortcuts of the eager step (CPU): each one is checked against the torch call it
replaces.

* particles.vmap_tensors vs torch.func.vmap(randomness="different"): same outputs, batched and
  unbatched results alike; anything outside its fast path goes to torch (and raises torch's errors);
* particles.broadcast_shapes vs torch.broadcast_shapes, including size-0 dimensions and the error;
* optim.Adam.zero_grad vs torch.optim.Optimizer.zero_grad (set_to_none and zeroing);
* nn._float32 vs float(torch.tensor(v, dtype=torch.float32)).
"""
import pytest
import torch

from mininf_amd import nn, optim, particles


def _fn(a, b):
    return (a * 2, b.sum(), torch.ones(()), a + 1, b[0], a.new_zeros(3))


def test_vmap_tensors_matches_torch_vmap():
    a, b = torch.randn(7), torch.randn(7, 3)
    ours = particles.vmap_tensors(_fn, [a, b])
    ref = torch.func.vmap(_fn, randomness="different")(a, b)
    assert len(ours) == len(ref)
    for x, y in zip(ours, ref):
        assert x.shape == y.shape and torch.equal(x, y)


def test_vmap_tensors_randomness_differs_per_row():
    out, = particles.vmap_tensors(lambda a: (torch.rand(()) + 0 * a,), [torch.zeros(64)])
    assert out.shape == (64,) and out.unique().numel() > 1


@pytest.mark.parametrize("args", [[torch.randn(3), torch.randn(4)], [torch.randn(3), torch.tensor(1.0)]])
def test_vmap_tensors_hands_bad_inputs_to_torch(args):
    with pytest.raises(ValueError):
        particles.vmap_tensors(lambda a, b: (a + b,), args)


def test_vmap_tensors_rejects_non_tensor_outputs():
    with pytest.raises(ValueError):
        particles.vmap_tensors(lambda a: (a, 3), [torch.randn(4)])


@pytest.mark.parametrize("shapes", [((3, 1), (1, 4)), ((), (5,)), ((0,), (1,)), ((2, 3), (3,)),
                                    ((4, 1, 2), (3, 1)), ((1,), ()), ((2, 0, 1), (1, 5))])
def test_broadcast_shapes_matches_torch(shapes):
    assert particles.broadcast_shapes(*shapes) == tuple(torch.broadcast_shapes(*shapes))


def test_broadcast_shapes_mismatch_raises_torchs_error():
    with pytest.raises(RuntimeError):
        particles.broadcast_shapes((2,), (3,))


@pytest.mark.parametrize("set_to_none", [True, False])
def test_adam_zero_grad_matches_torch(set_to_none):
    params = [torch.nn.Parameter(torch.randn(3)), torch.nn.Parameter(torch.randn(2))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    for group in (params, ref):
        for p in group:
            p.grad = torch.ones_like(p)
    params[1].grad = None
    ref[1].grad = None
    optim.Adam(params).zero_grad(set_to_none=set_to_none)
    torch.optim.Adam(ref).zero_grad(set_to_none=set_to_none)
    for p, q in zip(params, ref):
        assert (p.grad is None) == (q.grad is None)
        if p.grad is not None:
            assert torch.equal(p.grad, q.grad)


@pytest.mark.parametrize("K", [1, 3, 7, 33, 1000, 4096, 123457])
def test_float32_rounding_matches_torch(K):
    assert nn._float32(-1.0 / K) == float(torch.tensor(-1.0 / K, dtype=torch.float32))


def test_eager_validation_words_are_fresh_zeroed_rows():
    """Every eager step gets validation words no earlier step wrote: rows of a zeroed block, a new
    block once the rows run out (the old block lives on while a step still holds its row)."""
    loss = nn.EvidenceLowerBoundLoss(num_particles=4)
    device = torch.device("cpu")
    rows = [loss._zeroed_flags(device) for _ in range(loss.FLAG_POOL + 2)]
    for r in rows:
        assert r.shape == (loss.FLAG_WORDS,) and r.dtype == torch.int32 and not r.any()
    ptrs = [r.data_ptr() for r in rows]
    assert len(set(ptrs)) == len(ptrs)   # (the first block is still alive through its rows)
    rows[0].fill_(7)                     # a step's kernels write its words ...
    assert not loss._zeroed_flags(device).any()   # ... and no later step sees them


def test_only_the_last_captured_step_mirrors_the_validation_words():
    """StepGraph(repeat=R) captures R steps whose sticky validation words are the same device
    words: only the last step's ELBO forward copies them to the pinned host mirror
    (graph.mirrors_flags); outside a capture every step does."""
    from mininf_amd import graph
    assert graph.mirrors_flags()
    seen = []
    for r in range(3):
        graph._STATE.capture_position = (r, 3)
        seen.append(graph.mirrors_flags())
    graph._STATE.capture_position = None
    assert seen == [False, False, True]
    assert graph.mirrors_flags()
