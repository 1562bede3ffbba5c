"""
The C-ABI library: it loads on a CPU-only host, exports every function include/mininf_amd.h
declares, its ctypes structs match the header's layout, and every site program the engine
specialises compiles (hiprtc needs no device). No kernel is launched here.
"""
import ctypes
import os
import re

import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd import _native as nat, engine, particles
from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mininf_amd.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^int (mi_\w+)\(", text, flags=re.M)))


def test_library_loads_and_exports_header():
    lib = nat.lib()
    names = declared_functions()
    assert len(names) >= 14
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(nat.EXPORTED_SYMBOLS)
    target = ctypes.create_string_buffer(16)
    assert lib.mi_abi_version(target, 16) == nat.ABI_VERSION == 18
    assert target.value == b"gfx950"


def test_struct_layout_matches_header():
    sizes = [ctypes.c_size_t() for _ in range(3)]
    assert nat.lib().mi_struct_sizes(*[ctypes.byref(s) for s in sizes]) == 0
    assert [s.value for s in sizes] == [ctypes.sizeof(nat.Operand), ctypes.sizeof(nat.Site),
                                        ctypes.sizeof(nat.Group)]
    assert nat.Site.scale.offset == 56 and nat.Site.mask.offset == 32
    assert nat.Group.sites.offset == 40
    elbo_sizes = [ctypes.c_size_t() for _ in range(2)]
    assert nat.lib().mi_elbo_struct_sizes(*[ctypes.byref(s) for s in elbo_sizes]) == 0
    assert [s.value for s in elbo_sizes] == [ctypes.sizeof(nat.Factor), ctypes.sizeof(nat.Elbo)]


def test_invalid_arguments_are_rejected():
    lib = nat.lib()
    size = ctypes.c_size_t()
    group = nat.Group()
    assert lib.mi_group_workspace_bytes(ctypes.byref(group), ctypes.byref(size)) == -1
    assert lib.mi_normal_rsample(None, 0, None, 0, 1, 1, 0, 0, None, 0, 0, 0, None, None,
                                 None) == -1
    # an element offset that is not a multiple of 4 (one Philox block per element quad)
    buf = ctypes.c_float(0.0)
    assert lib.mi_normal_rsample(ctypes.byref(buf), 0, ctypes.byref(buf), 0, 1, 1, 0, 0, None, 0,
                                 0, 6, None, ctypes.byref(buf), None) == -1
    assert lib.mi_categorical_workspace_bytes(0, 1, ctypes.byref(size)) == -1
    # the peer all-reduce: slot lengths and descriptors are checked before anything is launched
    assert lib.mi_peer_region_bytes(0, ctypes.byref(size)) == -1
    assert lib.mi_peer_region_bytes(nat.PEER_MAX_FLOATS + 1, ctypes.byref(size)) == -1
    assert lib.mi_peer_region_bytes(256, ctypes.byref(size)) == 0
    assert size.value == 2 * nat.PEER_MAX_RANKS * 8 + 2 * nat.PEER_MAX_RANKS * 256 * 4 + 8
    peer = nat.Peer()
    peer.world, peer.rank, peer.max_floats = 2, 0, 256
    word = ctypes.c_uint32(0)
    assert lib.mi_peer_allreduce(ctypes.byref(peer), ctypes.byref(buf), ctypes.byref(buf), 1,
                                 ctypes.byref(word), None) == -1   # (no mapped regions)
    peer.regions[0] = peer.regions[1] = ctypes.addressof(buf)
    assert lib.mi_peer_allreduce(ctypes.byref(peer), ctypes.byref(buf), ctypes.byref(buf), 257,
                                 ctypes.byref(word), None) == -1   # longer than the slots
    peer.rank = 2
    assert lib.mi_peer_allreduce(ctypes.byref(peer), ctypes.byref(buf), ctypes.byref(buf), 1,
                                 ctypes.byref(word), None) == -1   # rank outside the world
    count = ctypes.c_uint64()
    assert lib.mi_peer_call_count(None, ctypes.byref(count)) == -1
    assert lib.mi_peer_call_count(ctypes.byref(peer), None) == -1
    assert lib.mi_peer_call_count(ctypes.byref(peer), ctypes.byref(count)) == -1  # (no region)


def hierarchical(n):
    def model():
        mu = mi.sample("mu", Normal(0, 1))
        z = mi.sample("z", Normal(mu, 1), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))
    return model


def regression(n, p):
    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(10 * n):
            with mi.no_log_prob():
                X = mi.sample("X", Normal(0, 1), sample_shape=(10 * n, p))
            mi.sample("y", Normal(X @ theta, 1))
    return model


def coin(n):
    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])
    return model


@pytest.mark.parametrize("case", ["hierarchical", "regression", "coin"])
def test_specialised_site_programs_compile(case):
    K, n = 16, 257
    if case == "hierarchical":
        mask = torch.rand(n) > 0.2
        model = mi.condition(hierarchical(n), y=torch.masked.as_masked_tensor(torch.randn(n), mask),
                             b=torch.masked.as_masked_tensor((torch.rand(n) < .5).float(), mask))
        samples = {"mu": torch.randn(K, requires_grad=True),
                   "z": torch.randn(K, n, requires_grad=True)}
    elif case == "regression":
        model = mi.condition(regression(n, 4), X=torch.randn(n, 4), y=torch.randn(n))
        samples = {"theta": torch.randn(K, 4, requires_grad=True)}
    else:
        model = mi.condition(coin(n), x=(torch.rand(n) < 0.5).float())
        samples = {"theta": torch.rand(K, requires_grad=True)}
    trace = particles.trace_particles(model, samples, K)
    launchers, _ = engine.plan_groups(trace, -1.0 / K, torch.device("cpu"))
    assert launchers
    for launcher in launchers:
        for grads in (True, False):
            launcher.compile_check(grads)
        source = launcher.source()
        assert "mi_site_program" in source or "BCAST" in source
