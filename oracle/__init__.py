"""ORACLE — test infrastructure only (see oracle.py)."""
