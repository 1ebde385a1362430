"""CPU oracle for the ksched placement hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg import this package; the ksched_amd product never does.
"""
