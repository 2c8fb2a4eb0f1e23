"""TEST INFRASTRUCTURE -- CPU oracle for the MCDO gated-attention MIL hot path.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker, never as the measured or shipped path.

  philox_oracle.c  bit-exact definition of the dropout keep-mask stream (C, gcc)
  philox.py        ctypes binding + an independent pure-Python Philox for cross-checks
  mcdo_ref.py      torch-CPU restatement of reference model.py:211-401 with replayed masks

Inputs come from mcgmil.synthetic (the seeded synthetic workload).
Parity of mcdo_ref against the reference module is pinned by tests/golden/*.npz.
"""
