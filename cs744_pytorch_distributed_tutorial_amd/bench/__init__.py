"""Benchmarks beyond the headline ``bench.py``: the collective bus-bandwidth sweep
(``busbw``) and the per-sync-mode training throughput sweep (``sync_modes``)."""
