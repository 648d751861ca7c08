"""ORACLE — TEST INFRASTRUCTURE ONLY.

A clean-room CPU restatement (eager PyTorch, fp32) of the reference's render path
(SuwoongHeo/neurecon @ 2025-02-11).  Every function cites the
reference file:line it restates.

Who may use it: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only
as the *checker* / CPU baseline.  The product (neurecon_amd) never imports it; neurecon_amd
raises if its HIP library is missing instead of falling back to anything here.

Pinning: the restatement is checked against golden vectors produced by importing the real
reference in the build container (tests/golden/gen_golden.py -> tests/golden/*.npz;
tests/test_oracle_golden.py).  Parity is therefore *pinned* (not "unpinned").
"""
