"""ORACLE package — CPU restatements used ONLY as checkers by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg.  Nothing in the product (vclip_amd) may import this."""
