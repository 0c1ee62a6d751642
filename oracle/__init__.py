"""CPU oracle for the GP log-likelihood hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain numpy/scipy restatement of the reference
(ameli/gaussian-process-param-estimation v0.0.1) algorithms on the hot path:

* ``oracle.data``      — input generators   (examples/_utilities/data_utilities.py:22-185)
* ``oracle.matern``    — Matérn assembly     (generate_correlation/_kernels.pyx:17-136,
                                               _generate_dense_correlation.pyx:25-162)
* ``oracle.imate_exact`` — the exact ("eigenvalue" / "cholesky") methods of the
  third-party ``imate`` package the reference calls (unpinned, requirements.txt:5,
  absent from this image), restated from their published definitions.
* ``oracle.mixed_correlation`` — the K + eta*I operator (mixed_correlation.py:34-335)
* ``oracle.likelihood`` — Direct / Profile likelihood (_direct_likelihood.py:31-340,
                                                        _profile_likelihood.py:38-192)
* ``oracle.cpu_baseline`` — the reference CPU call pattern, timed by bench.py.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker — never as the product path.
The product (``gaussian_proc`` in ``gaussian-process-param-estimation_amd/``) never
imports it and fails loudly when its HIP library is missing.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference's own Python/Cython code in the development container
(``tests/golden/make_golden.py``; imate's exact methods supplied by
``oracle.imate_exact``) and against the known-answer values of SURVEY.md
Appendix A (``tests/golden/survey_appendix_a.json``).
"""
