"""
Extra distribution families (mirror of the reference's ``mininf/distributions.py``).

``InverseGamma`` (reference ``mininf/distributions.py:5-11``) is not one of the four families the
HIP site kernels implement; in the ELBO engine its sites are evaluated by the generic
``torch.distributions`` site path on the GPU (see ``mininf_amd.particles``).
"""
from torch.distributions import Gamma, PowerTransform, TransformedDistribution


class InverseGamma(TransformedDistribution):
    """
    Inverse gamma distribution: the law of ``1 / X`` for ``X ~ Gamma(concentration, rate)``.
    """
    def __init__(self, concentration, rate, validate_args=None):
        super().__init__(Gamma(concentration, rate), [PowerTransform(-1)], validate_args)
