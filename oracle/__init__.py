"""ORACLE — test infrastructure only, never the product.

CPU restatement of the reference's NF-proposed Metropolis-Hastings hot path
(Inesalmansa/flow-state).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package, and only as the
checker / the timed CPU baseline.  The product path (``flow-state_amd/``) never
imports it and fails loudly when its HIP library is missing.

Pieces:

* ``oracle.physics`` — ctypes wrapper of ``csrc/physics_oracle.c`` (plain C):
  minimum-image distances, LJ + double-well total energy, numpy PCG64 /
  SeedSequence, the ``nf_big_move`` acceptance rule.
* ``oracle.flow`` — torch-CPU float32 restatement of the circular
  rational-quadratic-spline coupling flow (``NormalizingFlow.log_prob`` /
  ``sample``), written against a reference-format ``state_dict``.
* ``oracle.mh`` — the per-chain reference step (``MonteCarlo.nf_big_move``
  semantics) used for parity traces and for the timed CPU baseline.

Pinning: ``tests/golden/*.npz`` hold vectors produced by importing the
reference itself in the build container (``tests/golden/make_goldens.py``);
``tests/test_oracle_golden.py`` checks this oracle against them.
"""
