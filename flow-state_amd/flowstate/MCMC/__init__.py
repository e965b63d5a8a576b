"""Drop-in for the reference's ``MCMC`` surface on the hot path
(MCMC/simulation_box.py, energy_calculator.py, monte_carlo.py, initialise.py)."""
from .batched import BatchedMonteCarlo, Physics  # noqa: F401
from .energy_calculator import EnergyCalculator, total_energy  # noqa: F401
from .initialise import initialise_fcc, initialise_low_left, initialise_low_right  # noqa: F401
from .monte_carlo import MonteCarlo  # noqa: F401
from .simulation_box import SimulationBox  # noqa: F401
