"""ORACLE package — CPU restatements used only as checkers by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. Nothing in dilabhelmholtzoct_amd/ imports it."""
