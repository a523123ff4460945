"""TEST INFRASTRUCTURE ONLY: CPU oracle for the hash-join parity tests (see hj_oracle.c header)."""
