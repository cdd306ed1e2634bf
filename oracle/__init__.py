"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  Store-level parity is unpinned; see
oracle/gvs_oracle.h.
"""
