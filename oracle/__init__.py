"""ORACLE package — CPU restatements of the reference's hot paths, TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg. The product (deepwalk-and-node2vec_amd/) never imports it.
"""
