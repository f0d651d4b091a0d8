"""TEST INFRASTRUCTURE ONLY: the CPU oracle package (see oracle/refcpu.c)."""
