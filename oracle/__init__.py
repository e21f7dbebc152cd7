"""oracle — CPU restatements of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker / baseline,
never as the thing measured or shipped.
"""
