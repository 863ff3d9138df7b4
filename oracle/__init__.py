"""ORACLE PACKAGE — test infrastructure, never product code.

Holds the CPU fp32 restatement of the reference's hot path (the AVMNIST late-fusion
train step of TArsenii/task-specific-pretraining-multimodal, MML_Suite).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from here, and only as the checker / CPU baseline — never as the thing measured or
shipped.  The product path (``tspm_amd``) never imports this package and fails loudly when its
HIP library is missing.

Pinning: ``oracle/avmnist_ref.py`` is checked against golden vectors captured from the real
reference modules (``tests/golden/make_golden.py`` → ``tests/golden/avmnist_step_b4.npz``);
``tests/test_oracle_golden.py`` re-checks that on every CPU test run.
"""
