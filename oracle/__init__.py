"""Test infrastructure: CPU restatement of the reference ELBO step (see nma_oracle.py).
Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
