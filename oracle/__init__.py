"""ORACLE — test infrastructure only.

CPU restatements of the efls-train forward-encryption path used as the parity checker and as the
timed CPU baseline. Nothing in the product path (`efl` package, libefl_hip.so) may import this.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
