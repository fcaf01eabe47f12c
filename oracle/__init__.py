"""CPU oracle for the RAFT correlation path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product (``dexiraft_amd``) never imports it and has no CPU fallback.

Parity pinning: the restatement is checked against golden vectors produced by
importing the reference ``core/corr.py`` in the build container
(``tests/golden/make_golden.py``; the backward against the reference's
autograd gradients, ``tests/golden/make_backward_golden.py``); see
``tests/test_oracle_golden.py``.
"""
from .corr_oracle import (alt_corr_backward, alt_corr_block, alt_corr_block_queries,
                          alt_corr_forward, avg_pool2x2, avg_pool2x2_backward, bilinear_sample,
                          bilinear_sample_backward, corr_lookup, corr_lookup_backward,
                          corr_lookup_rows, corr_pyramid, corr_pyramid_backward,
                          corr_rows_pyramid, corr_volume, motion_conv1x1, sample_coord)

__all__ = ["alt_corr_backward", "alt_corr_block", "alt_corr_block_queries", "alt_corr_forward",
           "avg_pool2x2", "avg_pool2x2_backward", "bilinear_sample", "bilinear_sample_backward",
           "corr_lookup", "corr_lookup_backward", "corr_lookup_rows", "corr_pyramid",
           "corr_pyramid_backward", "corr_rows_pyramid", "corr_volume", "motion_conv1x1",
           "sample_coord"]
