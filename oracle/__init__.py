"""Test oracle package (test infrastructure only; see oracle.py)."""
