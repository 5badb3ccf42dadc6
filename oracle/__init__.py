"""Test-only parity checkers (see oracle/oracle.py).  Never imported by quicknet_amd."""
