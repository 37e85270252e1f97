"""CPU oracle for darosior/miningsimulation's per-run loop — TEST INFRASTRUCTURE ONLY (see msim_oracle.c)."""
