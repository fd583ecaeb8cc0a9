"""pynngp_amd -- MI355X-native NNGP neighbour sets, B/F sweep and log-likelihood.

Drop-in for the hot path of bwpriest/pyNNGP (``pyNNGP.NNGP``); see DESIGN.md.
The compute runs in ``_build/libnngp_hip.so`` (hand-written gfx950 HIP kernels
behind the C ABI of ``include/nngp.h``); importing this package does not load
it -- the first call that needs it does, and fails loudly if it is missing.
"""
from ._lib import NNGPExtensionError, LIB_PATH, version  # noqa: F401
from .nngp import NNGP, CallableCovariance, Covariance, IsotropicCovariance, NNGPNumericalError  # noqa: F401
from .sweep import ShardedLogLik, shard_range, combine_partials  # noqa: F401
from .gibbs import SeqNNGP, SeqNNGPChains, Priors  # noqa: F401
from .gibbs_sharded import ShardedSeqNNGP  # noqa: F401

__version__ = "0.3.0"


def load_ops():
    """Register ``torch.ops.nngp.*`` (loads the native operator library, libnngp_torch_ops.so)."""
    from . import ops

    ops.load()
    return ops
