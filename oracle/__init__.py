"""ORACLE package — CPU restatements of the reference's hot path, used ONLY as the checker
by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never imported by
the product package `acme_amd`."""
