"""
oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's ELBO hot path (tillahoffmann/mininf: mininf/nn.py:212-228,
mininf/core.py:207-273) and of the torch.distributions arithmetic it delegates to, used as the
checker for the HIP path:

* ``logprob``   -- per-family log densities and gradients in numpy float64;
* ``elbo``      -- K-particle ELBO values and gradients for configs C1-C5 (numpy float64) with
                   injected guide noise;
* ``philox.c``  -- plain-C Philox-4x32 (7 rounds; 10 for the known-answer vectors) + Box-Muller restatement of the guide generator;
* ``cpu_port``  -- the reference's single-particle torch-CPU semantics, timed as ``cpu_baseline``.

Parity is pinned: every function here is checked against the golden fixtures in ``tests/golden``,
which were produced by running the reference itself (``tests/golden/make_golden.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package. The product (``mininf_amd``) never does.
"""
