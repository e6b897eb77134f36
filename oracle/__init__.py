"""ORACLE -- test infrastructure only.

CPU restatements of the reference hot path (score net, Langevin update, cross-view
consistency merge), each function citing the reference file:line it follows.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything here, and only as the checker; the product path (``sdp``) never does.
"""
