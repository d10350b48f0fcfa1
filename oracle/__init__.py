"""CPU oracle for the MMPFN PerFeatureTransformer forward (TEST INFRASTRUCTURE ONLY).

This package is a from-scratch CPU restatement of the reference algorithm
(too-z/MultiModalPFN, ``mmpfn/models/mmpfn/model/*.py``).  It is the *checker*:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it.  The product path (``multimodalpfn_amd``) never
imports, links or calls anything under ``oracle/`` and fails loudly when its HIP
extension is missing.

Parity pinning: the restatement is pinned against golden vectors produced by
running the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``).
"""

from oracle.forward import OracleSpec, oracle_forward, oracle_mixer  # noqa: F401
