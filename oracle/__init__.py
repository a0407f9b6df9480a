"""CPU restatement of the reference hot path: the PARITY ORACLE and CPU baseline.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import anything from here, and only as the checker or the
timed CPU baseline -- never as the thing measured or shipped.  The product
(eco-dqn_amd/eco_hip + libecohip.so) never imports this package.
"""
