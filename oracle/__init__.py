"""ORACLE (test infrastructure only): CPU restatements of the reference path.

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package quantized_vit_amd never imports it.
"""
