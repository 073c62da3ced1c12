"""CPU oracle of the FD mode-sum hot path -- TEST INFRASTRUCTURE ONLY (see fd_oracle.py)."""
