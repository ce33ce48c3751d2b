"""oracle/ -- TEST INFRASTRUCTURE ONLY: CPU parity checker for the shading hot path (see oracle.py)."""
