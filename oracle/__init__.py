"""TEST INFRASTRUCTURE ONLY.

CPU oracle for the DPI label-generation hot path (numpy restatement of the reference,
pinned by reference-generated golden vectors in tests/golden/).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and only
as the checker / CPU baseline — never as the product path.
"""
