"""ORACLE / TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference hot path used as parity checkers (tests/, smoke())
and as bench.py's cpu_baseline leg.  The product package never imports this.
"""
