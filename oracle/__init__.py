"""CPU oracle for the surgical-phase hot path — TEST INFRASTRUCTURE ONLY.

This package is a functional restatement (torch CPU fp32/fp64 ops over a plain
``{name: tensor}`` state dict, no nn.Module) of the reference's arithmetic:

* ``oracle.mit_evp``   — mix_transformer_evp.py + segformer_head.py forward
* ``oracle.mstcn``     — mstcn.py MultiStageModel_S / SingleStageModel / DilatedResidualLayer
* ``oracle.trans_sv``  — adapter_transformer.py Transformer.original_forward windowing + fc/tanh,
                         and the build's own Transformer2_3_1 (reference source absent:
                         **parity unpinned** for that module only)
* ``oracle.params`` / ``oracle.inputs`` — deterministic parameter and synthetic-input
  generators shared by the golden generator (tests/golden/gen_golden.py, runs only in
  the survey container where /root/reference exists) and the tests on the GPU box.

Pinning: the oracle is checked against golden vectors produced by importing the
reference itself (tests/golden/*.npz, generator script committed next to them).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / the timed CPU baseline — the
product path (the HIP library behind ``models.*``) never calls into it.
"""
