"""CPU oracle for the lime_amd parity tests -- TEST INFRASTRUCTURE ONLY.

Imported solely by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / baseline, never as the product.
"""
