"""CPU oracle for the gsplat hot path (test infrastructure only; see gsplat_oracle.py)."""
