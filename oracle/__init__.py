"""TEST INFRASTRUCTURE ONLY: the CPU oracle (see oracle/pyoracle.py)."""
