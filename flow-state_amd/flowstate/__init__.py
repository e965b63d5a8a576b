"""flowstate — MI355X-native NF-proposed Metropolis-Hastings hot path.

Drop-in mirrors of the reference API surfaces used by
hybrid_NF_MCMC/main_algorithm_1.py:

* ``flowstate.normflows`` — ``NormalizingFlow`` (forward / inverse / log_prob /
  sample), ``flows.CircularCoupledRationalQuadraticSpline``,
  ``Energy.UniformParticle``; state_dict keys identical to the reference.
* ``flowstate.MCMC`` — ``SimulationBox``, ``EnergyCalculator``,
  ``MonteCarlo`` (per-chain ``nf_big_move``), ``BatchedMonteCarlo``
  (C chains, ``step()``), ``initialise_fcc``.

All compute runs in libflowstate.so (hand-written HIP for gfx950) through the
C ABI of include/flowstate.h; there is no CPU fallback.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
