"""CPU oracle for the redistribution path -- TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg (as the checker / CPU baseline).  See redist_oracle.py and mgr_oracle.c.
"""
