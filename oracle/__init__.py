"""Test infrastructure: CPU restatements of the reference hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package.  The product (gym_ballenv_amd) never does.
"""
