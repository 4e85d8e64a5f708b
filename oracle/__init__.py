"""CPU oracle for the RVC v2 48 kHz inference path — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm (the ``rvc/`` PyTorch path of
Acelogic/Retrieval-based-Voice-Conversion-MLX) in plain torch-CPU fp32 /
numpy fp64, one function per reference function, each citing the reference
file:line it follows. It is the checker for the HIP product path:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it;
  * the product package (``rvcx``) never imports it and has no CPU fallback.

Pinning: the restatement is checked against golden vectors produced by running
the reference itself in the survey container (``tests/golden/make_golden.py``,
which imports ``/root/reference`` with module stubs) and against the reference's
own known-answer data (``ios_test_data/rmvpe_hidden.npy`` -> ``rmvpe_f0.npy``).
"""
