"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see oracle/oracle.py)."""
